"""One-shot callers and the output-placement lottery: a loop of fresh
quantize_encode(x, return_q=True) calls (q + codes, the placement-sensitive K2 form) at
1024 x 2^20, timed per call with HIP events, against the same process's DMEPipeline probe
(K1 + the probed K2).  Run it in several fresh processes.

    python tools/exp/oneshot_pool.py [--calls 30] [--no-pool]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--d", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--no-pool", action="store_true")
    a = ap.parse_args()
    import uqdme
    from uqdme_amd.outpool import POOL
    POOL.enabled = not a.no_pool
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(a.n, a.d, device="cuda", generator=g)
    X = torch.rand(a.n, generator=torch.Generator().manual_seed(2))
    Xd = X.cuda()
    times = []
    for i in range(a.calls):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tc, q = uqdme.quantize_encode(x, 1, X=X, torch_threads=1, return_q=True)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
        del tc, q
    # K1 alone and the pipeline's probed K2 in the same process
    k1 = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        uqdme.l1_torch_order(x, torch_threads=1)
        e1.record()
        torch.cuda.synchronize()
        k1.append(e0.elapsed_time(e1))
    pool_rep = {str(k): v for k, v in POOL.report().items()}
    POOL.clear()
    torch.cuda.empty_cache()
    p = uqdme.DMEPipeline(a.n, a.d, 1, torch_threads=1)
    rep = p.probe_outputs(x, Xd, candidates=12, min_candidates=12)
    tail = times[a.calls // 2:]
    best = statistics.median(k1) + rep["k2_ms_chosen"]
    print(json.dumps({"tool": "oneshot_pool", "pool": not a.no_pool, "call_ms": [round(t, 4) for t in times],
                      "steady_median_ms": round(statistics.median(tail), 4), "k1_ms": round(statistics.median(k1), 4),
                      "probe": rep, "k1_plus_probed_k2_ms": round(best, 4),
                      "steady_over_best": round(statistics.median(tail) / best, 4),
                      "pool_sets_ms": pool_rep}), flush=True)


if __name__ == "__main__":
    main()
