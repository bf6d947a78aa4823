"""Time the QUIC-FL sender (uq_quicfl_compress_f32) and receiver on a resident synthetic batch,
on the synthetic sender tables of tests/golden/quicfl_tables.py and the reference's receiver
tables (tests/golden/quicfl_recv_vectors.npz).  Also times one message per call (the drop-in's
QuicFLSender.compress, host work included).

    python tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def make_sender(uqdme, bits):
    from quicfl_tables import DATA, sender_tables
    X, p = sender_tables(bits)
    return uqdme.QuicFLSender(tables={bits: (X, p, DATA[bits])})


def recv_table(bits):
    return np.load(os.path.join(ROOT, "tests", "golden", "quicfl_recv_vectors.npz"))[f"recv{bits}"]


def digest(msg, out):
    import hashlib
    h = hashlib.sha256()
    for t in (msg.X, msg.exact_mask, msg.exact_dense(), msg.scale, out):
        t = t.contiguous()
        t = t.view(torch.int32) if t.dtype == torch.float32 else t
        w = torch.arange(t.shape[-1], device=t.device, dtype=torch.int64) % 65521 + 1
        rows = (t.to(torch.int64) * w).sum(dim=-1) if t.dim() > 1 else t.to(torch.int64)
        h.update(rows.cpu().numpy().tobytes())
    h.update(np.asarray(msg.exact_count).tobytes())
    return h.hexdigest()[:16]


def timed(f, steps):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=1 << 20)
    ap.add_argument("--bits", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--per-call", type=int, default=5, help="single-message compress calls to time (0: skip)")
    ap.add_argument("--digest", action="store_true", help="add a digest of the messages and the decompressed batch")
    a = ap.parse_args()
    import uqdme
    snd = make_sender(uqdme, a.bits)
    rt = recv_table(a.bits)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(a.clients, a.dim, generator=g, device="cuda")
    seeds = list(range(a.clients))
    rots = [123] * a.clients
    pxs = list(range(1000, 1000 + a.clients))
    holder = {}

    def comp():
        holder["m"] = uqdme.quicfl_compress(x, a.bits, seeds, rots, sender=snd, px_seeds=pxs)

    ms_c = timed(comp, a.steps)
    msg = holder["m"]
    ms_d = timed(lambda: uqdme.quicfl_decompress_messages(msg, rt), a.steps)
    res = {"tool": "bench_quicfl", "clients": a.clients, "d": a.dim, "bits": a.bits, "compress_ms": round(ms_c, 4),
           "decompress_ms": round(ms_d, 4), "exact_per_client": float(msg.exact_count.float().mean()),
           "M_vectors_per_s_compress": round(a.clients / ms_c / 1e3, 6)}
    if a.digest:                           # to compare library variants' outputs (tools/exp/variants.py)
        res["digest"] = digest(msg, uqdme.quicfl_decompress_messages(msg, rt))
    if a.per_call:
        v = x[0].clone()
        data = {"vec": v, "seed": 7, "nbits": a.bits, "rotation_seed": 123}
        snd.compress(data)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.per_call):
            snd.compress(data)
        torch.cuda.synchronize()
        res["compress_per_call_ms"] = round((time.perf_counter() - t0) * 1e3 / a.per_call, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
