"""Time EDEN + RHT (uq_eden_f32) on a resident synthetic batch.

    python tools/bench_eden.py --clients 1024 --dim 1048576 --bits 1"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=1 << 20)
    ap.add_argument("--bits", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import uqdme
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(a.clients, a.dim, generator=g, device="cuda")
    seeds = torch.randint(0, 100, (a.clients,), generator=torch.Generator().manual_seed(5))
    for _ in range(2):
        uqdme.eden_quantize(x, a.bits, seeds=seeds)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        uqdme.eden_quantize(x, a.bits, seeds=seeds)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    print(json.dumps({"tool": "bench_eden", "clients": a.clients, "d": a.dim, "bits": a.bits, "ms_per_call": round(ms, 4),
                      "M_vectors_per_s": round(a.clients / ms / 1e3, 6)}))


if __name__ == "__main__":
    main()
