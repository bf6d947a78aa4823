"""Time uq_client_mean_f32 (K3, the q pipeline's client mean) of every library in
_build/abl/ on one resident 1024 x 2^20 q batch, alternating libraries three times;
each library's est is compared with the first one's (bit-identical expected)."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd", "_build", "abl")
P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
n, d = 1024, 1 << 20
q = torch.randn(n, d, device="cuda")
est = torch.empty(d, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
libs = {}
for f in sorted(os.listdir(OUT)):
    if f.endswith(".so"):
        L = ctypes.CDLL(os.path.join(OUT, f))
        L.uq_client_mean_f32.argtypes = [P, I64, I64, I64, F32, I32, P, P]
        libs[f[:-3]] = L
ref = None
for rep in range(3):
    for name, L in libs.items():
        fn = lambda: L.uq_client_mean_f32(q.data_ptr(), n, d, d, float(n), 0, est.data_ptr(), sp)  # noqa: E731
        if fn() != 0:
            raise RuntimeError(f"{name}: mean failed")
        torch.cuda.synchronize()
        same = None
        if ref is None:
            ref = est.clone()
        else:
            same = bool(torch.equal(ref, est))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(json.dumps({"rep": rep, "lib": name, "ms": round(ms, 4), "TBs": round(4 * n * d / ms / 1e9, 3),
                          "same_as_first": same}), flush=True)
