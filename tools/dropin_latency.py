"""Per-call latency of the drop-ins (one client per call, as the reference's callers use
them): Type_unbiased_quantize, Type_biased_quantize, EDEN_quantize_Hadamard.

    python tools/dropin_latency.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import uqdme
    res = {}
    for d in (172554, 1 << 20, 1 << 22):
        vs = [torch.randn(d, device="cuda") for _ in range(16)]     # different vectors: some have
        v = vs[0]                                                   # biased-quantizer threshold ties
        for name, f in (("Type_unbiased_quantize", uqdme.Type_unbiased_quantize),
                        ("Type_biased_quantize", uqdme.Type_biased_quantize),
                        ("EDEN_quantize_Hadamard", uqdme.EDEN_quantize_Hadamard)):
            for _ in range(3):
                y = f(v, 1)
            torch.cuda.synchronize()
            k = 48
            t0 = time.perf_counter()
            for i in range(k):
                y = f(vs[i % len(vs)], 1)
            torch.cuda.synchronize()
            res[f"{name}/d={d}"] = round((time.perf_counter() - t0) / k * 1e3, 4)
            del y
    print(json.dumps({"tool": "dropin_latency", "ms_per_call": res}))


if __name__ == "__main__":
    main()
