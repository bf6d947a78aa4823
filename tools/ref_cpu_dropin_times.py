"""Per-call time of the REFERENCE's drop-ins on this container's CPU (the reference is importable
here, never on the GPU box): Type_unbiased_quantize, Type_biased_quantize, EDEN_quantize_Hadamard
and QUICFL_quantize (its sender tables are absent from the reference, so QuicFLSender's default
prefix is pointed at the synthetic tables of tests/golden/quicfl_tables.py, as the fixture
script does).  The GPU side of the same calls: tools/dropin_latency.py --quicfl.

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_cpu_dropin_times.py --out profiles/r4_ref_cpu_dropin.json"""
import argparse
import json
import os
import platform
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/NMSE_Results/Codes"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="1024,2048,1048576")
    ap.add_argument("--threads", default="1,8")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from quicfl_tables import write_tables
    prefix = write_tables(os.path.join(tempfile.mkdtemp(prefix="qfl_ref_"), "t"))
    sys.path.insert(0, REF)
    import All_Schemes as AS  # noqa: E402  (the reference, this container only)
    AS.QuicFLSender.__init__.__defaults__ = ("cpu", [1, 2, 3, 4], [6, 5, 4, 4], prefix)
    AS.QuicFLReceiver.__init__.__defaults__ = ("cpu", [1, 2, 3, 4], [6, 5, 4, 4], prefix)
    fns = [("Type_unbiased_quantize", AS.Type_unbiased_quantize), ("Type_biased_quantize", AS.Type_biased_quantize),
           ("EDEN_quantize_Hadamard", AS.EDEN_quantize_Hadamard), ("QUICFL_quantize", AS.QUICFL_quantize)]
    res = {"tool": "ref_cpu_dropin_times", "host": platform.processor() or platform.machine(),
           "logical_cpus": os.cpu_count(), "ms_per_call": {}}
    rng = np.random.default_rng(0)
    for T in [int(t) for t in a.threads.split(",")]:
        torch.set_num_threads(T)
        for d in [int(v) for v in a.dims.split(",")]:
            x = torch.from_numpy(rng.standard_normal(d).astype(np.float32))
            for name, f in fns:
                f(x, 1)                                        # warm (QUIC-FL loads its tables here)
                k = 20 if d <= 4096 else 3
                t0 = time.perf_counter()
                for _ in range(k):
                    f(x, 1)
                ms = (time.perf_counter() - t0) / k * 1e3
                res["ms_per_call"][f"{name}/d={d}/threads={T}"] = round(ms, 4)
                print(name, d, T, round(ms, 3), flush=True)
    txt = json.dumps(res)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
