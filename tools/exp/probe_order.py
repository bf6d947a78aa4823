"""Is the fast output set a property of the set (placement) or of when it is timed?
Allocates 6 (q, codes) sets after x, then times K2 on them in the order 0..5, 5..0 and
0..5 again (3 timed calls each).  In the bench's probes so far the LAST allocated set was
the fast one every time (r02e, r02g); this separates allocation order from timing order.
    python tools/exp/probe_order.py   (GPU box)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(k=6):
    import uqdme
    n, d = 1024, 1 << 20
    x = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    p = uqdme.DMEPipeline(n, d, 1, torch_threads=1)
    p.l1_norms(x)
    sets = [(p.q, p.codes)] + [p._alloc_outputs() for _ in range(k - 1)]

    def t(q, c, reps=3):
        for _ in range(2):
            p.quantize(x, X, q, c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            p.quantize(x, X, q, c)
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    for name, order in (("forward", range(k)), ("reverse", range(k - 1, -1, -1)), ("forward2", range(k))):
        res = {i: t(*sets[i]) for i in order}
        print(json.dumps({"order": name, "k2_ms_by_set": [res[i] for i in range(k)],
                          "va_GB": [round(sets[i][0].data_ptr() / 2 ** 30, 2) for i in range(k)]}), flush=True)
    # a fresh set allocated now, after all the others
    q, c = p._alloc_outputs()
    print(json.dumps({"order": "new_after", "k2_ms": t(q, c)}), flush=True)
    p.check_status()


if __name__ == "__main__":
    main()
