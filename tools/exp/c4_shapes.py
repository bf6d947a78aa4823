"""Per-batch time of the three quantizers at config C4's shapes (d = 2^22, n in the NMSE
harness's client counts {1, 6, 11, 51, 101} and 256), to find shapes that fall off the
batch kernels' per-client rate.  One JSON line per (scheme, n): ms per batch (HIP events,
5 calls after one warm call) and us per client.

    python tools/exp/c4_shapes.py [d] [schemes, comma-separated]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uqdme  # noqa: E402


def timed(f, reps=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    g = torch.Generator(device="cuda").manual_seed(4)
    qfl = None
    if only is None or "quicfl" in only:        # synthetic sender tables (the published ones are absent)
        import numpy as np
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        gdir = os.path.join(root, "tests", "golden")
        sys.path.insert(0, gdir)
        from quicfl_tables import DATA, sender_tables
        rz = np.load(os.path.join(gdir, "quicfl_recv_vectors.npz"))
        qfl = (uqdme.QuicFLSender(tables={b: (*sender_tables(b), DATA[b]) for b in (1, 2)}),
               uqdme.QuicFLReceiver(tables={b: rz[f"recv{b}"] for b in (1, 2)}))
    for n in (1, 6, 11, 51, 101, 256):
        x = torch.randn(n, d, generator=g, device="cuda")
        X = torch.rand(n, generator=torch.Generator().manual_seed(n))
        seeds = torch.randint(0, 100, (n,), generator=torch.Generator().manual_seed(n))
        m = uqdme.rate_to_m(1, d)
        for name, f in (("unbiased", lambda: uqdme.quantize_dequantize(x, 1, X=X, torch_threads=1)),
                        ("biased", lambda: uqdme.biased_quantize(x, m=m, torch_threads=1, ties="torch")),
                        ("eden", lambda: uqdme.eden_quantize(x, 1, seeds=seeds)),
                        ("quicfl", lambda: uqdme.quicfl_quantize(x, 1, seeds.tolist(), [123] * n, sender=qfl[0],
                                                                 recv_table=qfl[1].recv_table[1],
                                                                 px_seeds=seeds))):
            if only and name not in only:
                continue
            ms = timed(f)
            print(json.dumps({"scheme": name, "d": d, "n": n, "ms": round(ms, 4), "us_per_client": round(ms * 1e3 / n, 2)}),
                  flush=True)
        del x


if __name__ == "__main__":
    main()
