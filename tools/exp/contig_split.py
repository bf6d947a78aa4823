"""K2 (q + codes) with x in one physically contiguous allocation and q + codes in another,
separated by a contiguous spacer of S GB allocated in between (S = 0 ... 64): does the distance
between the read stream and the write streams in physical memory decide the 1.7 / 2.0 ms mode?
    python tools/exp/contig_split.py"""
import ctypes, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _ok(rc):
    """HIP return code check that python -O does not strip."""
    if rc != 0:
        raise RuntimeError(f"HIP call failed ({rc})")
    return rc


def main():
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    MB, GB = 1 << 20, 1 << 30

    def calloc(nbytes):
        p = ctypes.c_void_p()
        _ok(hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4)))
        return p.value
    src = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.uq_l1_torch_order_f32(src.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
    torch.cuda.synchronize()

    for rep in range(2):
        for S in (0, 4, 16, 64, 1, 32):
            x = calloc(4 * GB)
            sp = calloc(S * GB) if S else None
            q = calloc(5 * GB)
            c = q + 4 * GB
            _ok(hip.hipMemcpy(ctypes.c_void_p(x), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(n * d * 4), 3))
            f = lambda: lib.uq_type_unbiased_codes_f32(x, q, c, ovf.data_ptr(), n, d, m, X.data_ptr(), l1.data_ptr(),
                                                       None, 1, ws.data_ptr(), b.value, st)
            for _ in range(2):
                _lib.check(f(), "k2")
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "spacer_GB": S, "k2_ms": round(e0.elapsed_time(e1) / 5, 4),
                              "q_minus_x_GB": round((q - x) / GB, 3)}), flush=True)
            for p_ in (x, sp, q):
                if p_:
                    hip.hipFree(ctypes.c_void_p(p_))


if __name__ == "__main__":
    main()
