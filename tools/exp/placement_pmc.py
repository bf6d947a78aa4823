"""is the K2 output-placement lottery a channel imbalance?  One process:
the C2 batch (1024 x 2^20, codes4 pipeline), SETS fresh output sets timed (3 K2 launches each
after 2 warm ones), then the fastest and the slowest set run K2 REPS times each, fast first.
Run under `rocprofv3 --pmc ...`: every K2 dispatch is counted; the last 2 * REPS dispatches are
the comparison.  Prints one JSON line (set times, the two chosen, the dispatch plan).

    python tools/exp/placement_pmc.py [SETS] [REPS]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uqdme  # noqa: E402


def main():
    sets_n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n, d = 1024, 1 << 20
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.randn(n, d, generator=g, device="cuda")
    X = torch.rand(n, generator=torch.Generator().manual_seed(1234)).cuda()
    pipe = uqdme.DMEPipeline(n, d, 1, pipeline="codes4")
    pipe.l1_norms(x)
    sets = [pipe._alloc_outputs() for _ in range(sets_n)]

    def time_set(s, k):
        for _ in range(2):
            pipe.quantize(x, X, *s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            pipe.quantize(x, X, *s)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    times = [time_set(s, 3) for s in sets]
    fast = min(range(sets_n), key=lambda i: times[i])
    slow = max(range(sets_n), key=lambda i: times[i])
    addr = [[int(t.data_ptr()) for t in s] for s in sets]
    torch.cuda.synchronize()
    for _ in range(reps):
        pipe.quantize(x, X, *sets[fast])
    for _ in range(reps):
        pipe.quantize(x, X, *sets[slow])
    torch.cuda.synchronize()
    print(json.dumps({"k2_ms": [round(t, 4) for t in times], "fast": fast, "slow": slow, "reps": reps,
                      "plan": f"last {2 * reps} K2 dispatches: {reps} on the fast set, then {reps} on the slow set",
                      "set_ptrs": addr}), flush=True)


if __name__ == "__main__":
    main()
