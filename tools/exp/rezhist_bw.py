"""KB2 histogram cost (tools/exp/rezhist_bw.hip) on 1024 N(0,1) rows x 2^20 at R = 1 and R = 4:
no histogram / one LDS atomic per element / hot 8-bin windows in registers + atomics for
the rest.  V1 and V2 histograms must be equal.
Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC tools/exp/rezhist_bw.hip -o tools/exp/librezhist_bw.so"""
import ctypes
import json
import os

import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "librezhist_bw.so"))
L.rezhist_bw.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_float,
                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
n, d = 1024, 1 << 20
x = torch.randn(n, d, device="cuda")
rden = 1.0 / (x.abs().sum(1) + 1e-12)
sums = torch.zeros(n * (d // 16384) * 4, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
for R, fm in ((1, 224426.0), (4, 9.0 * 2 ** 20)):
    hs = {}
    for v in (0, 1, 2, 0, 1, 2):
        hist = torch.zeros(n * 2048, dtype=torch.int32, device="cuda")
        f = lambda: L.rezhist_bw(x.data_ptr(), n, d, rden.data_ptr(), fm, sums.data_ptr(), hist.data_ptr(), v, sp)  # noqa: E731
        if f() != 0:
            raise RuntimeError("rezhist_bw failed")
        torch.cuda.synchronize()
        hs[v] = hist.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"R": R, "variant": ["no_hist", "atomic", "windows"][v], "ms": round(ms, 4),
                          "TBs": round(4 * n * d / ms / 1e9, 3)}), flush=True)
    top = torch.topk(hs[1][:2048].float(), 8)
    print(json.dumps({"R": R, "hist_equal": bool(torch.equal(hs[1], hs[2])),
                      "top_bins": [hex(int(i)) for i in top.indices], "top_frac": [round(float(c) / d, 4) for c in top.values]}),
          flush=True)
