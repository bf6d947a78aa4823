"""Time the biased type quantizer (uq_type_biased_f32) on resident synthetic batches.

    python tools/bench_biased.py --clients 1024 --dim 1048576 --dist normal --ties torch

dist: normal (no ties at the threshold), smallint (integers in [-3, 3]: every client
ambiguous, KB7 replays torch's topk for each), bernoulli (0/1 with p = 0.7)."""
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
    ap.add_argument("--bits", type=float, default=1)
    ap.add_argument("--dist", default="normal", choices=["normal", "smallint", "bernoulli"])
    ap.add_argument("--ties", default="torch", choices=["torch", "lowest"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--torch-threads", type=int, default=1)
    a = ap.parse_args()
    import uqdme
    bits = int(a.bits) if float(a.bits).is_integer() else a.bits
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    n, d = a.clients, a.dim
    if a.dist == "normal":
        x = torch.randn(n, d, generator=g, device=dev)
    elif a.dist == "smallint":
        x = torch.randint(-3, 4, (n, d), generator=g, device=dev).float()
    else:
        x = (torch.rand(n, d, generator=g, device=dev) < 0.7).float()
    out = torch.empty_like(x)
    m = uqdme.rate_to_m(bits, d)
    for _ in range(2):
        uqdme.biased_quantize(x, m=m, torch_threads=a.torch_threads, ties=a.ties, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        uqdme.biased_quantize(x, m=m, torch_threads=a.torch_threads, ties=a.ties, out=out)
    e1.record()
    torch.cuda.synchronize()
    uqdme.check_status()
    ms = e0.elapsed_time(e1) / a.steps
    _, info = uqdme.biased_quantize(x, m=m, torch_threads=a.torch_threads, ties=a.ties, out=out, return_info=True)
    amb = int(((info[:, 1] & 1) != 0).sum())
    print(json.dumps({"tool": "bench_biased", "clients": n, "d": d, "bits": bits, "dist": a.dist, "ties": a.ties,
                      "ms_per_call": round(ms, 4), "M_vectors_per_s": round(n / ms / 1e3, 6),
                      "GB_per_s_x_plus_out": round(8.0 * n * d / ms / 1e6, 1), "ambiguous_clients": amb}))


if __name__ == "__main__":
    main()
