"""Where QUICFL_quantize's per-call time goes at the harness's d (host segments, synchronised)."""
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import uqdme
    import uqdme_amd.quicfl as q
    from quicfl_tables import write_tables
    uqdme.set_tables_prefix(write_tables(os.path.join(tempfile.mkdtemp(prefix="qfl_bd_"), "t")))
    res = {}
    for d in (2048, 1 << 20):
        v = torch.randn(d, device="cuda")
        for _ in range(3):
            uqdme.QUICFL_quantize(v, 1)
        torch.cuda.synchronize()
        snd, rcv = q._dropin_pair()
        seg = {"generator_words": 0.0, "compress": 0.0, "decompress": 0.0, "host_copy": 0.0, "total": 0.0}
        k = 20 if d <= 4096 else 5
        for _ in range(k):
            t0 = time.perf_counter()
            st, words = q.generator_words(torch.default_generator)
            t1 = time.perf_counter()
            data = {"vec": v, "seed": int(torch.randint(0, 100, (1,)).item()), "nbits": 1, "rotation_seed": 123}
            msg = snd.compress(data)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out = rcv.decompress(msg)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            host = torch.empty(out.numel(), dtype=torch.float32, pin_memory=True)
            host.copy_(out)
            _ = host.numpy()
            t4 = time.perf_counter()
            seg["generator_words"] += t1 - t0
            seg["compress"] += t2 - t1
            seg["decompress"] += t3 - t2
            seg["host_copy"] += t4 - t3
        t0 = time.perf_counter()
        for _ in range(k):
            uqdme.QUICFL_quantize(v, 1)
        seg["total"] = (time.perf_counter() - t0)
        res[f"d={d}"] = {kk: round(vv / k * 1e3, 4) for kk, vv in seg.items()}
    print(json.dumps({"tool": "qfl_dropin_breakdown", "ms": res}))


if __name__ == "__main__":
    main()
