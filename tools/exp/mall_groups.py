"""Experiment: can K2's read of x hit the 256 MiB Infinity Cache
(MALL) when K2 runs right after K1 on the same group of clients?

C2 batch (1024 x 2^20, R = 1, codes pipeline).  For group sizes G, one step is either
  interleaved:  for each group g:  K1(g) -> K2(g)        (K2 re-reads what K1 just read)
  separate:     K1(all groups)   -> K2(all groups)        (same launches, no reuse possible)
followed by the client mean from the codes.  Groups of >= 256 clients use K2's stream form
(one workgroup per client); smaller groups use the segmented small-batch form (several
workgroups per client, x read three times: tile sums, maps, outputs), whose re-reads of a
group of <= 32 clients (<= 128 MiB) are the ones the cache could serve.  If the cache served
K2's x, interleaved would beat separate at equal G.  Prints one JSON line per case; est is
checked bit-equal across every arrangement.

    python tools/exp/mall_groups.py                 (the timing sweep)
    python tools/exp/mall_groups.py --one G inter K (K steps of one case, for a --pmc pass:
                                                      FETCH_SIZE of K2's kernels per step)"""
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
x = torch.randn(n, d, generator=torch.Generator(device=dev).manual_seed(1234), device=dev)
X = torch.rand(n, generator=torch.Generator().manual_seed(1234)).to(dev)
q = torch.empty_like(x)
codes = torch.empty((n, d), dtype=torch.int8, device=dev)
kmax = torch.zeros(n, dtype=torch.int32, device=dev)
l1 = torch.empty(n, device=dev)
est = torch.empty(d, device=dev)
P = lambda t: t.data_ptr()  # noqa: E731
sp = torch.cuda.current_stream(dev).cuda_stream


def wsbytes(nn):
    import ctypes
    b = ctypes.c_size_t()
    _lib.check(lib.uq_workspace_bytes(nn, d, T, ctypes.byref(b)), "ws")
    return int(b.value)


ws = torch.zeros(wsbytes(n), dtype=torch.uint8, device=dev)
nb = ws.numel()


def k1(o, g):
    _lib.check(lib.uq_l1_torch_order_f32(P(x) + o * d * 4, g, d, T, P(l1) + o * 4, P(ws), nb, sp), "l1")


def k2(o, g):
    _lib.check(lib.uq_type_unbiased_codes_f32(P(x) + o * d * 4, P(q) + o * d * 4, P(codes) + o * d, P(kmax) + o * 4,
                                              g, d, m, P(X) + o * 4, P(l1) + o * 4, None, T, P(ws), nb, sp), "k2")


def step(G, inter):
    groups = range(0, n, G)
    if inter:
        for o in groups:
            k1(o, G)
            k2(o, G)
    else:
        for o in groups:
            k1(o, G)
        for o in groups:
            k2(o, G)
    _lib.check(lib.uq_codes_mean_f32(P(codes), P(l1), P(kmax), n, d, m, float(n), 0, P(est), sp), "mean")


def timeit(G, inter, reps=6):
    for _ in range(2):
        step(G, inter)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        step(G, inter)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


if len(sys.argv) > 1 and sys.argv[1] == "--one":
    G, inter, K = int(sys.argv[2]), bool(int(sys.argv[3])), int(sys.argv[4])
    for _ in range(K):
        step(G, inter)
    torch.cuda.synchronize()
    _lib.check(lib.uq_check_status(P(ws), sp), "status")
    sys.exit(0)

ref = None
for G in (1024, 512, 256, 64, 32, 16):
    for inter in (False, True):
        ms = timeit(G, inter)
        e = est.clone()
        ref = e if ref is None else ref
        print(json.dumps({"group_clients": G, "group_MiB": G * 4, "arrangement": "interleaved" if inter else "separate",
                          "ms_per_step": round(ms, 4), "Mvec_s": round(n / ms / 1e3, 4),
                          "est_bit_equal": bool(torch.equal(e.view(torch.int32), ref.view(torch.int32)))}), flush=True)
_lib.check(lib.uq_check_status(P(ws), sp), "status")
