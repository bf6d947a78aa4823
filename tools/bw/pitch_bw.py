"""Row-pitch sweep of K2's memory structure (see pitch_bw.hip).  Build:
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/bw/libpitch_bw.so tools/bw/pitch_bw.hip
Prints one JSON line per configuration: ms and GB/s of moved bytes for 1024 rows x 2^20."""
import ctypes
import json
import os
import sys

import torch

so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpitch_bw.so")
L = ctypes.CDLL(so)
L.bw_pitch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
n, d = 1024, 1 << 20
pads = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,64,1024,4160")]
maxpad = max(pads)
xb = torch.randn(n * (d + maxpad), device="cuda")
yb = torch.empty_like(xb)
cb = torch.empty(n * (d + maxpad), dtype=torch.int8, device="cuda")
sink = torch.zeros(n, device="cuda")
sp = torch.cuda.current_stream().cuda_stream


def t(fn, reps=10):
    for _ in range(3):
        r = fn()
        if r != 0:
            raise RuntimeError(f"launch failed {r}")
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for rnd in range(2):
    for pad in pads:
        pitch = d + pad
        for mode, codes, depth in ((0, 0, 1), (0, 0, 2), (0, 1, 1), (1, 0, 1), (1, 0, 2), (2, 0, 1)):
            ms = t(lambda: L.bw_pitch(xb.data_ptr(), yb.data_ptr(), cb.data_ptr(), n, d, pitch, pitch, depth, codes,
                                      mode, sink.data_ptr(), sp))
            nbytes = n * d * ((4 if mode != 2 else 0) + (4 if mode != 1 else 0) + codes)
            print(json.dumps({"round": rnd, "pad_floats": pad, "mode": ["rw", "read", "write"][mode], "codes": codes,
                              "depth": depth, "ms": round(ms, 4), "GBs": round(nbytes / ms / 1e6, 1)}), flush=True)
