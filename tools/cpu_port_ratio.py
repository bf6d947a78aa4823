"""Restatement/reference CPU speed ratio measured on ONE host.

Times the reference's own Type_unbiased_quantize (imported from /root/reference, this
container only; the GPU box has no reference) and the C restatement oracle/uq_oracle.c
on the same d = 2^20 N(0,1) vectors, R = 1, at 1 thread and at all cores, and checks that
both produce the same bits.  The bench reports this ratio next to its GPU-box CPU
baseline so that the box's port timings can be related to the reference.

    python tools/cpu_port_ratio.py  ->  profiles/r02_cpu_port_vs_reference.json
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference/NMSE_Results/Codes"


def main(nvec=24, d=1 << 20):
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import warnings
    warnings.simplefilter("ignore")
    import All_Schemes as AS  # noqa: E402  (reference, this container only)
    from oracle import uq_oracle_c as C
    from oracle.uq_oracle import rate_to_m

    C.build()
    rng = np.random.default_rng(77)
    xs = rng.standard_normal((nvec, d)).astype(np.float32)
    m = rate_to_m(1, d)
    ncpu = len(os.sched_getaffinity(0))
    res = {"host_cpu": _cpu_model(), "logical_cpus": ncpu, "d": d, "bits": 1, "vectors": nvec,
           "torch": torch.__version__}
    for threads in (1, ncpu):
        torch.set_num_threads(threads)
        gen = torch.Generator().manual_seed(5)
        X = torch.rand(nvec, generator=gen)
        torch.manual_seed(5)
        t0 = time.perf_counter()
        ref = [AS.Type_unbiased_quantize(torch.from_numpy(xs[j]), 1).numpy() for j in range(nvec)]
        t_ref = time.perf_counter() - t0
        # the port, one client per call like the reference (threads = torch's own for the L1 order)
        t0 = time.perf_counter()
        if threads == 1:
            out, _ = C.quantize_batch(xs, m, X.numpy(), threads)
        else:
            out, _, used = C.quantize_batch_mt(xs, m, X.numpy(), threads, threads)
        t_port = time.perf_counter() - t0
        mism = int(sum(np.count_nonzero(out[j].view(np.uint32) != ref[j].view(np.uint32)) for j in range(nvec)))
        res[f"threads_{threads}"] = {
            "reference_ms_per_vector": round(t_ref * 1e3 / nvec, 3),
            "port_ms_per_vector": round(t_port * 1e3 / nvec, 3),
            "port_speedup_over_reference": round(t_ref / t_port, 3),
            "bit_mismatches": mism,
            "how": ("reference: one Type_unbiased_quantize call per vector (torch intra-op threads = "
                    f"{threads}); port: " + ("uqo_quantize_batch, one thread" if threads == 1 else
                                             f"uqo_quantize_batch_mt, clients over {threads} OpenMP threads, "
                                             f"L1 in the torch order of {threads} threads")),
        }
        print(threads, res[f"threads_{threads}"], flush=True)
    out_path = os.path.join(ROOT, "profiles", "r02_cpu_port_vs_reference.json")
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out_path)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


if __name__ == "__main__":
    main()
