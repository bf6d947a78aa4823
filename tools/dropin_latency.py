"""Per-call latency of the drop-ins (one client per call, as the reference's callers use
them): Type_unbiased_quantize, Type_biased_quantize, EDEN_quantize_Hadamard (and with --quicfl QUICFL_quantize).  "ms_per_call":
48 calls back to back (host work overlapping the GPU), "ms_synced": each call waited for.
Sizes: the reference harness's own (d = 1024 in C1, 2048 in Normal_dist.py:40), 4096, the
largest single-launch size (32767) and GRAIN (32768), the FL model (172 554), 2^20, 2^22.

    python tools/dropin_latency.py [--dims 1024,2048]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="1024,2048,4096,32767,32768,172554,1048576,4194304")
    ap.add_argument("--quicfl", action="store_true",
                    help="also QUICFL_quantize, on the synthetic sender tables of tests/golden/quicfl_tables.py")
    a = ap.parse_args()
    import uqdme
    fns = [("Type_unbiased_quantize", uqdme.Type_unbiased_quantize),
           ("Type_biased_quantize", uqdme.Type_biased_quantize),
           ("EDEN_quantize_Hadamard", uqdme.EDEN_quantize_Hadamard)]
    if a.quicfl:
        import tempfile
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
        from quicfl_tables import write_tables
        uqdme.set_tables_prefix(write_tables(os.path.join(tempfile.mkdtemp(prefix="qfl_tabs_"), "t")))
        fns.append(("QUICFL_quantize", uqdme.QUICFL_quantize))
    res, synced = {}, {}
    for d in [int(v) for v in a.dims.split(",")]:
        vs = [torch.randn(d, device="cuda") for _ in range(16)]     # different vectors: some have
        v = vs[0]                                                   # biased-quantizer threshold ties
        for name, f in fns:
            for _ in range(3):
                y = f(v, 1)
            torch.cuda.synchronize()
            k = 48
            t0 = time.perf_counter()
            for i in range(k):
                y = f(vs[i % len(vs)], 1)
            torch.cuda.synchronize()
            res[f"{name}/d={d}"] = round((time.perf_counter() - t0) / k * 1e3, 4)
            t0 = time.perf_counter()
            for i in range(k):
                y = f(vs[i % len(vs)], 1)
                torch.cuda.synchronize()
            synced[f"{name}/d={d}"] = round((time.perf_counter() - t0) / k * 1e3, 4)
            del y
    print(json.dumps({"tool": "dropin_latency", "ms_per_call": res, "ms_synced": synced}))


if __name__ == "__main__":
    main()
