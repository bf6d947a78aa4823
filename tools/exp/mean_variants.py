"""Driver for tools/exp/exp_mean.hip: the client mean over 1024 x 2^20 q, by variant.
    python tools/exp/mean_variants.py   (GPU box)"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "256 thr x 4 col", 1: "1024 thr x 4 col", 2: "256 thr x 2 col", 3: "64 thr x 4 col", 4: "128 thr x 2 col"}


def main():
    L = ctypes.CDLL(os.path.join(HERE, "libexp_mean.so"))
    L.exp_mean.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_void_p]
    n, d = 1024, 1 << 20
    q = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(9), device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    ref = None
    for v in (0, 1, 2, 3, 4, 0, 1, 2, 3, 4):
        est = torch.empty(d, device="cuda")
        f = lambda: L.exp_mean(q.data_ptr(), n, d, float(n), est.data_ptr(), v, sp)  # noqa: E731
        for _ in range(2):
            if f() != 0:
                raise RuntimeError("launch failed")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        ref = est.clone() if ref is None else ref
        print(json.dumps({"variant": NAMES[v], "ms": round(ms, 4), "TB_s": round(n * d * 4 / ms / 1e9, 3),
                          "est_equal": bool(torch.equal(est, ref))}), flush=True)


if __name__ == "__main__":
    main()
