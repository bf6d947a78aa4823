"""KB-small at the drop-in's sizes: the share of random N(0,1) vectors whose threshold tie needs
torch's choice (flag 1: the drop-in reruns the multi-kernel path), and the per-call time of the
lowest-index launch alone vs the drop-in.  python tools/exp/biased_small_probe.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import uqdme
    RATE_TABLE = sys.modules[uqdme.biased_quantize.__module__].RATE_TABLE
    res = {}
    for d in (1024, 2048, 4096, 16384, 32767):
        vs = [torch.randn(d, device="cuda") for _ in range(64)]
        m = int(RATE_TABLE[1] * d)
        amb = 0
        for v in vs:
            _, info = uqdme.biased_quantize(v.view(1, d), m=m, ties="lowest", return_info=True)
            amb += int(info[0, 1]) & 1
        row = {"ambiguous_of_64": amb}
        for name, f in (("lowest_launch", lambda v: uqdme.biased_quantize(v.view(1, d), m=m, ties="lowest")),
                        ("dropin", lambda v: uqdme.Type_biased_quantize(v, 1))):
            for v in vs[:4]:
                f(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for v in vs:
                f(v)
                torch.cuda.synchronize()
            row[name + "_ms_synced"] = round((time.perf_counter() - t0) / len(vs) * 1e3, 4)
        res[d] = row
        print(d, row, flush=True)
    print(json.dumps({"tool": "biased_small_probe", "rows": res}))


if __name__ == "__main__":
    main()
