"""Timing sweep of the two-bit-code client mean (esc2_mean_kernel) over columns per thread
(UQDME_E2_CPT = 4, 8, 16) against the int8-code mean, on the C2 batch (1024 x 2^20, R = 1).

Experiment, not shipped: the two-bit escape codes (K2 writes 0 / +1 / -1 / "read q" per
coordinate, d/4 bytes per client; the mean reads them and q for counts >= 2) live in
tools/exp/esc2_codes.patch (git apply it to a scratch checkout, rebuild).  They were
bit-exact (tests in the patch) but the mean ran 0.227-0.277 ms against 0.213 ms for the
int8-code mean (profiles/r02l_exp_e2_sweep.jsonl): both means are issue/latency-bound, not
byte-bound, so a quarter of the bytes bought nothing, and K2 did not speed up either in the
fast placement (1.69 ms).
    python tools/exp/e2_sweep.py   (GPU box, patched build)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def timed(f, reps=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def main():
    import uqdme
    n, d = 1024, 1 << 20
    x = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    p2 = uqdme.DMEPipeline(n, d, 1, torch_threads=1, codes="esc2")
    p2.l1_norms(x)
    p2.quantize(x, X)
    ref = None
    for cpt in (4, 8, 16):
        os.environ["UQDME_E2_CPT"] = str(cpt)
        ms = timed(lambda: p2.mean(float(n)))
        e = p2.est.clone()
        ref = e if ref is None else ref
        print(json.dumps({"kernel": "esc2_mean", "cols_per_thread": cpt, "ms": ms,
                          "same_bits": bool(torch.equal(e.view(torch.int32), ref.view(torch.int32)))}), flush=True)
    del p2
    p8 = uqdme.DMEPipeline(n, d, 1, torch_threads=1, codes="int8")
    p8.l1_norms(x)
    p8.quantize(x, X)
    ms = timed(lambda: p8.mean(float(n)))
    print(json.dumps({"kernel": "codes_mean (int8)", "ms": ms,
                      "same_bits": bool(torch.equal(p8.est.view(torch.int32), ref.view(torch.int32)))}), flush=True)
    p8.check_status()


if __name__ == "__main__":
    main()
