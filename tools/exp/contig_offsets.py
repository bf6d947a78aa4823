"""K2 (q + codes) with x, q and codes carved from ONE physically contiguous allocation
(hipExtMallocWithFlags(hipDeviceMallocContiguous)) at chosen offsets, so their relative
physical placement is set by the offsets alone.  Each offset set is timed twice to see whether
the 1.7 / 2.0 ms modes are a deterministic function of relative physical placement.
    python tools/exp/contig_offsets.py"""
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
    slack = 512 * MB
    total = 9 * GB + 2 * slack
    p = ctypes.c_void_p()
    _ok(hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(total), ctypes.c_uint(0x4)))
    base = p.value
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

    def t(qo, co):
        x = base
        q = base + 4 * GB + qo
        c = base + 8 * GB + slack + co
        if not (qo < slack and co < slack and c + n * d <= base + total):
            raise RuntimeError("carve-out outside the allocation")
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
        return round(e0.elapsed_time(e1) / 5, 4)

    offs = [(0, 0), (0, 2 * MB), (0, 64 * MB), (0, 256 * MB), (2 * MB, 0), (128 * MB, 0), (256 * MB, 256 * MB),
            (4096, 8192), (0, 1 * MB), (0, 384 * MB)]
    for rep in range(2):
        for qo, co in offs:
            print(json.dumps({"rep": rep, "q_off": qo, "c_off": co, "k2_ms": t(qo, co)}), flush=True)
    hip.hipFree(ctypes.c_void_p(base))


if __name__ == "__main__":
    main()
