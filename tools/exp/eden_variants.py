"""Time the EDEN 1-bit round trip (uq_eden_f32) of every library in _build/abl/ on one
resident N(0,1) batch (EDEN_N x EDEN_D, default 1024 x 2^20), alternating libraries three times; outputs are compared
with the first library's (bit-identical expected)."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd", "_build", "abl")
P, I64, I32, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
n, d = int(os.environ.get("EDEN_N", 1024)), int(os.environ.get("EDEN_D", 1 << 20))
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(n, d, generator=g, device="cuda")
out = torch.empty_like(x)
scale = torch.empty(n, device="cuda")
seeds = torch.tensor([123], dtype=torch.int32, device="cuda")           # one rotation for all clients (AS:802)
D = 1 << (d - 1).bit_length()                       # padded length (AS:128)
signs = torch.empty((1, D), dtype=torch.int8, device="cuda")
rows = torch.zeros(n, dtype=torch.int32, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
libs = {}
for f in sorted(os.listdir(OUT)):
    if f.endswith(".so"):
        L = ctypes.CDLL(os.path.join(OUT, f))
        L.uq_eden_f32.argtypes = [P, P, I64, I64, I32, P, P, P, P, SZ, P]
        L.uq_rht_signs.argtypes = [P, I64, I64, P, P]
        b = SZ()
        if L.uq_eden_workspace_bytes(I64(n), I64(d), ctypes.byref(b)) != 0:
            raise RuntimeError("workspace query failed")
        libs[f[:-3]] = (L, torch.zeros(b.value, dtype=torch.uint8, device="cuda"), b.value)
first = next(iter(libs.values()))[0]
if first.uq_rht_signs(seeds.data_ptr(), 1, D, signs.data_ptr(), sp) != 0:
    raise RuntimeError("rht signs failed")
ref = None
for rep in range(int(os.environ.get("REPS", 3))):
    for name, (L, ws, nb) in libs.items():
        fn = lambda: L.uq_eden_f32(x.data_ptr(), out.data_ptr(), n, d, 1, signs.data_ptr(), rows.data_ptr(),  # noqa: E731
                                   scale.data_ptr(), ws.data_ptr(), nb, sp)
        if fn() != 0:
            raise RuntimeError(f"{name}: eden failed")
        torch.cuda.synchronize()
        same = None
        if ref is None:
            ref = out.clone()
        else:
            same = bool(torch.equal(ref, out))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "lib": name, "ms": round(e0.elapsed_time(e1) / 5, 4), "same_as_first": same}),
              flush=True)
