"""Time UQR1 encode (uq_tc_encode) of every library in _build/abl/ on one resident batch of
type codes (1024 x 2^20, R = 1, made by the product pipeline), alternating libraries three
times; messages and offsets are compared with the first library's (byte-identical expected)."""
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
x = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(3), device="cuda")
tc = uqdme.quantize_encode(x, 1, X=torch.rand(n, generator=torch.Generator().manual_seed(4)), torch_threads=1)
del x
sp = torch.cuda.current_stream().cuda_stream
libs = {}
for f in sorted(os.listdir(OUT)):
    if f.endswith(".so"):
        L = ctypes.CDLL(os.path.join(OUT, f))
        L.uq_tc_encode.argtypes = [P, P, I64, I64, I64, I32, P, SZ, P, P, SZ, P]
        b, w = SZ(), SZ()
        if L.uq_tc_bound(I64(d), ctypes.byref(b)) != 0 or L.uq_tc_workspace_bytes(I64(n), I64(d), ctypes.byref(w)) != 0:
            raise RuntimeError("size queries failed")
        libs[f[:-3]] = (L, torch.empty(n * b.value, dtype=torch.uint8, device="cuda"),
                        torch.empty(w.value, dtype=torch.uint8, device="cuda"))
off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
ref = None
for rep in range(3):
    for name, (L, data, ws) in libs.items():
        fn = lambda: L.uq_tc_encode(tc.codes.data_ptr(), tc.l1.data_ptr(), n, d, int(tc.m), 0, data.data_ptr(),  # noqa: E731
                                    data.numel(), off.data_ptr(), ws.data_ptr(), ws.numel(), sp)
        if fn() != 0:
            raise RuntimeError(f"{name}: encode failed")
        torch.cuda.synchronize()
        total = int(off[-1])
        same = None
        if ref is None:
            ref = (off.clone(), data[:total].clone())
        else:
            same = bool(torch.equal(ref[0], off)) and bool(torch.equal(ref[1], data[:total]))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "lib": name, "encode_ms": round(e0.elapsed_time(e1) / 5, 4), "same_as_first": same}),
              flush=True)
