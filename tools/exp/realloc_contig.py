"""K2 (q + codes) across fresh raw allocations of x, q, codes in ONE process, alternating plain
hipMalloc with hipExtMallocWithFlags(hipDeviceMallocContiguous): does a physically contiguous
allocation avoid K2's slow mode (see tools/exp/realloc.py)?
    python tools/exp/realloc_contig.py"""
import ctypes, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
FLAGS = {"malloc": None, "contig": 0x4}       # hipDeviceMallocContiguous (hip_runtime_api.h)


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

    def alloc(nbytes, flag):
        p = ctypes.c_void_p()
        rc = (hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) if flag is None else
              hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flag)))
        if rc != 0:
            raise RuntimeError(f"alloc rc={rc}")
        return p.value

    for trial in range(16):
        kind = "malloc" if trial % 2 == 0 else "contig"
        try:
            x, q, c = (alloc(n * d * 4, FLAGS[kind]), alloc(n * d * 4, FLAGS[kind]), alloc(n * d, FLAGS[kind]))
        except RuntimeError as e:
            print(json.dumps({"trial": trial, "kind": kind, "error": str(e)}), flush=True)
            continue
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
        print(json.dumps({"trial": trial, "kind": kind, "k2_ms": round(e0.elapsed_time(e1) / 5, 4)}), flush=True)
        for p in (x, q, c):
            hip.hipFree(ctypes.c_void_p(p))


if __name__ == "__main__":
    main()
