"""K2's stream shape without compute (tools/exp/lane_bw.hip): coalesced float4 lanes vs
thread-contiguous 64-byte rows, read x + write q + 1 B codes per element, 1024 x 2^20.
Six output sets (placement modes), every pattern and the product K2 on each.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/exp/lane_bw.hip -o tools/exp/liblane_bw.so"""
import ctypes
import json
import os
import sys

import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblane_bw.so"))
L.lane_bw.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
n, d = 1024, 1 << 20
x = torch.randn(n, d, device="cuda")
q = torch.empty_like(x)
c = torch.empty((n, d), dtype=torch.int8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import uqdme  # noqa: E402
from uqdme_amd import _lib  # noqa: E402
U = _lib.load()
m = uqdme.rate_to_m(1, d)
X = torch.rand(n, device="cuda")
l1 = torch.empty(n, device="cuda")
km = torch.zeros(n, dtype=torch.int32, device="cuda")
b = ctypes.c_size_t()
_lib.check(U.uq_workspace_bytes(n, d, 1, ctypes.byref(b)), "ws")
ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
_lib.check(U.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, sp), "l1")
K2 = lambda: U.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), c.data_ptr(), km.data_ptr(), n, d, m,  # noqa: E731
                                          X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, sp)
sets = [(q, c)] + [(torch.empty_like(x), torch.empty((n, d), dtype=torch.int8, device="cuda")) for _ in range(5)]
for rep, (q, c) in enumerate(sets):          # output placement decides K2's mode: several sets
    for pat in (0, 1, 2):
        f = K2 if pat == 2 else (lambda: L.lane_bw(x.data_ptr(), q.data_ptr(), c.data_ptr(), n, d, pat, sp))  # noqa: E731
        for _ in range(2):
            rc = f()
            if rc != 0:
                raise RuntimeError(f"lane_bw returned {rc}")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        ok = bool(torch.equal(q[:2], x[:2] * 0.5)) if pat < 2 else None
        print(json.dumps({"rep": rep, "pattern": ["coalesced", "thread_rows", "product_K2"][pat], "ms": round(ms, 4),
                          "TBs_9d": round(9 * n * d / ms / 1e9, 3), "q_ok": ok}), flush=True)
