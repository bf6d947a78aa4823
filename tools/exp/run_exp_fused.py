"""Times tools/exp/exp_fused.hip (data-flow bound of a fused K1+K2) against K1 + K2 on the
C2 batch (1024 x 2^20).  Build: hipcc ... -o tools/exp/libexp_fused.so (see Makefile line)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    ex = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_fused.so"))
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    dev = torch.device("cuda")
    x = torch.randn(n, d, device=dev)
    q = torch.empty_like(x)
    codes = torch.empty((n, d), dtype=torch.int8, device=dev)
    ovf = torch.zeros(n, dtype=torch.int32, device=dev)
    X = torch.rand(n, device=dev)
    l1 = torch.empty(n, device=dev)
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(max(b.value, 64 << 20), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def base():
        _lib.check(lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
        _lib.check(lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), codes.data_ptr(), ovf.data_ptr(), n, d, m,
                                                  X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st), "k2")

    def fused(segs, grid, phases):
        def f():
            rc = ex.exp_fused(P(x), P(q), P(codes), P(ovf), ctypes.c_int64(n), ctypes.c_int64(d), ctypes.c_int64(m),
                              P(X), P(ws), segs, grid, phases, ctypes.c_void_p(st))
            if (rc) != 0:
                raise RuntimeError('rc' + ' failed')
        return f

    def timeit(f, k=10):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / k, 4)

    res = {"k1+k2": timeit(base)}
    for segs in (16, 32, 64):
        for grid in (1024, 2048):
            res[f"fused s{segs} g{grid}"] = timeit(fused(segs, grid, 7))
    res["only D s32"] = timeit(fused(32, 1024, 4))
    res["A+D s32"] = timeit(fused(32, 1024, 5))
    res["k1+k2 again"] = timeit(base)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
