"""Time the biased quantizer (both tie policies) and the L1 pass of every library in
_build/abl/ on the same resident 1024 x 2^20 N(0,1) batch, alternating libraries; the
outputs of each library are compared with the first one's (bit-identical expected)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import uqdme  # noqa: E402

OUT = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd", "_build", "abl")
P, I64, I32, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
n, d = 1024, 1 << 20
m = uqdme.rate_to_m(1, d)
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(n, d, generator=g, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
libs = {}
for f in sorted(os.listdir(OUT)):
    if f.endswith(".so"):
        L = ctypes.CDLL(os.path.join(OUT, f))
        L.uq_type_biased_f32.argtypes = [P, P, I64, I64, I64, I32, I32, P, P, P, SZ, P]
        L.uq_l1_torch_order_f32.argtypes = [P, I64, I64, I32, P, P, SZ, P]
        b = SZ()
        if L.uq_biased_workspace_bytes(I64(n), I64(d), I32(1), ctypes.byref(b)) != 0:
            raise RuntimeError("workspace query failed")
        libs[f[:-3]] = (L, torch.zeros(b.value, dtype=torch.uint8, device="cuda"), b.value)
out = torch.empty_like(x)
l1 = torch.empty(n, device="cuda")
info = torch.zeros(n, dtype=torch.int32, device="cuda")
ref = {}
for rep in range(int(os.environ.get("REPS", 2))):
    for name, (L, ws, nb) in libs.items():
        for pol in (1, 0):
            f = lambda: L.uq_type_biased_f32(x.data_ptr(), out.data_ptr(), n, d, m, 1, pol, l1.data_ptr(),  # noqa: E731
                                             info.data_ptr(), ws.data_ptr(), nb, sp)
            if f() != 0:
                raise RuntimeError(f"{name}: biased call failed")
            torch.cuda.synchronize()
            same = None
            if rep == 0:
                if pol not in ref:
                    ref[pol] = out.clone()
                else:
                    same = bool(torch.equal(ref[pol], out))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "lib": name, "ties": ["torch", "lowest"][pol],
                              "ms": round(e0.elapsed_time(e1) / 5, 4), "same_as_first": same}), flush=True)
        h = lambda: L.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), nb, sp)  # noqa: E731
        h()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            h()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "lib": name, "l1_ms": round(e0.elapsed_time(e1) / 10, 4)}), flush=True)
