"""Experiment: overlap the L1 pass (K1, HBM-read-bound) of client chunk j+1 with the
quantize pass (K2) of chunk j on a second stream.  C2 batch (1024 x 2^20, R=1), pipelines
encode (K2 writes codes only), codes (q + codes) and q.  Prints one JSON line per case.
Checks that est equals the single-stream est bit for bit."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import uqdme  # noqa: E402
from uqdme_amd import _lib  # noqa: E402

lib = _lib.load()
n, d, T = 1024, 1 << 20, 1
m = uqdme.rate_to_m(1, d)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
x = torch.randn(n, d, generator=g, device=dev)
X = torch.rand(n, generator=torch.Generator().manual_seed(1234)).to(dev)
q = torch.empty_like(x)
codes = torch.empty((n, d), dtype=torch.int8, device=dev)
kmax = torch.zeros(n, dtype=torch.int32, device=dev)
l1 = torch.empty(n, device=dev)
est = torch.empty(d, device=dev)
P = lambda t: t.data_ptr()  # noqa: E731


def wsbytes(nn):
    import ctypes
    b = ctypes.c_size_t()
    _lib.check(lib.uq_workspace_bytes(nn, d, T, ctypes.byref(b)), "ws")
    return int(b.value)


sA = torch.cuda.current_stream(dev)
sB = torch.cuda.Stream(dev)
wsA = torch.zeros(wsbytes(n), dtype=torch.uint8, device=dev)
wsB = torch.zeros(wsbytes(n), dtype=torch.uint8, device=dev)
nbA, nbB = wsA.numel(), wsB.numel()


def step(pipeline, C):
    nc = n // C
    evs = []
    for j in range(C):
        o = j * nc
        _lib.check(lib.uq_l1_torch_order_f32(P(x) + o * d * 4, nc, d, T, P(l1) + o * 4, P(wsA), nbA, sA.cuda_stream), "l1")
        e = torch.cuda.Event()
        e.record(sA)
        evs.append(e)
    sK = sB if C > 1 else sA
    for j in range(C):
        o = j * nc
        if C > 1:
            sK.wait_event(evs[j])
        xo, lo, Xo = P(x) + o * d * 4, P(l1) + o * 4, P(X) + o * 4
        if pipeline == "q":
            _lib.check(lib.uq_type_unbiased_f32(xo, P(q) + o * d * 4, nc, d, m, Xo, lo, None, T, P(wsB), nbB,
                                                sK.cuda_stream), "k2")
            _lib.check(lib.uq_client_mean_f32(P(q) + o * d * 4, nc, d, d, float(n), int(j > 0), P(est), sK.cuda_stream), "mean")
        else:
            _lib.check(lib.uq_type_unbiased_codes_f32(xo, (P(q) + o * d * 4) if pipeline == "codes" else None,
                                                      P(codes) + o * d, P(kmax) + o * 4, nc, d, m, Xo, lo, None, T,
                                                      P(wsB), nbB, sK.cuda_stream), "k2")
            _lib.check(lib.uq_codes_mean_f32(P(codes) + o * d, lo, P(kmax) + o * 4, nc, d, m, float(n), int(j > 0),
                                             P(est), sK.cuda_stream), "mean")
    if C > 1:
        sA.wait_stream(sK)


def timeit(pipeline, C, reps=10):
    for _ in range(3):
        step(pipeline, C)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(sA)
    for _ in range(reps):
        step(pipeline, C)
    b.record(sA)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for pipeline in ("encode", "codes", "q"):
    ref = None
    for C in (1, 2, 4):
        ms = timeit(pipeline, C)
        e = est.clone()
        if ref is None:
            ref = e
        same = bool(torch.equal(e.view(torch.int32), ref.view(torch.int32)))
        print(json.dumps({"pipeline": pipeline, "chunks": C, "ms": round(ms, 4), "Mvec_s": round(n / ms / 1e3, 4),
                          "est_bit_equal": same}), flush=True)
_lib.check(lib.uq_check_status(P(wsA), sA.cuda_stream), "status")
_lib.check(lib.uq_check_status(P(wsB), sA.cuda_stream), "status")
