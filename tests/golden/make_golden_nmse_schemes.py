"""Known NMSE answers for the multi-scheme DME loop, made by running the REFERENCE's own
functions in the driver's call order (build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_nmse_schemes.py            # d = 2048
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_nmse_schemes.py --dim 4194304  # C4's d = 2^22

ND = NMSE_Results/Codes/Normal_dist.py.  Per client, in order: EDEN_quantize_Hadamard(v, 1),
(v, 2) (ND:135-136), Type_unbiased_quantize(v, 1), (v, 2) (ND:137-138),
Type_biased_quantize(v, 1), (v, 2) (ND:139-140), all drawing from the global torch RNG seeded
42, vectors from np.random seeded 42 (ND:14-15, 88-91), NMSE as ND:151-157.  The other
schemes of the shipped loop are left out (QUIC-FL crashes: its sender tables are missing).
Every EDEN call's rotation seed and scale (EdenSender.compress's output, AS:348: an MKL sdot,
whose summation order is CPU-dependent) are recorded too, so the GPU test can check the rest of
the EDEN path bit for bit with the reference's scale substituted, and the scale itself apart.
Gamma, Bernoulli and Lognormal are the other drivers' generators (Gamma_dist.py:86,
Bernoulli_dist.py:90, Lognormal_dist.py:90).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import warnings

import numpy as np
import torch

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference/NMSE_Results/Codes")
import All_Schemes as AS  # noqa: E402  (the reference module)

SCHEMES = [("eden", 1), ("eden", 2), ("unbiased", 1), ("unbiased", 2), ("biased", 1), ("biased", 2)]
QUICFL = [("quicfl", 1), ("quicfl", 2)]          # ND:141-142, after the biased quantizer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--dists", default="normal,laplace,gamma,bernoulli,lognormal")
    ap.add_argument("--quicfl", action="store_true",
                    help="also QUICFL_quantize (ND:141-142) on the synthetic sender tables of quicfl_tables.py")
    a = ap.parse_args()
    DIM = a.dim
    torch.set_num_threads(1)
    fns = {"eden": AS.EDEN_quantize_Hadamard, "unbiased": AS.Type_unbiased_quantize,
           "biased": AS.Type_biased_quantize, "quicfl": AS.QUICFL_quantize}
    schemes = SCHEMES + (QUICFL if a.quicfl else [])
    if a.quicfl:                                    # the sender reads its tables from a prefix (AS:431)
        import tempfile
        sys.path.insert(0, HERE)
        from make_golden_quicfl_sender import write_prefix
        pre = write_prefix(os.path.join(tempfile.mkdtemp(prefix="qfl_nd_"), "pub"))
        AS.QuicFLSender.__init__.__defaults__ = ("cpu", [1, 2, 3, 4], [6, 5, 4, 4], pre)
    gens = {"normal": lambda: np.random.normal(0, 1, DIM),
            "laplace": lambda: np.random.laplace(loc=1, scale=2, size=DIM),
            "gamma": lambda: np.random.gamma(shape=2, scale=2, size=DIM),
            "bernoulli": lambda: np.random.choice(np.arange(2), size=DIM, p=[0.3, 0.7]),
            "lognormal": lambda: np.random.lognormal(mean=1, sigma=2, size=DIM)}
    seen = []                                       # every EdenSender.compress output, in call order
    orig = AS.EdenSender.compress

    def recording_compress(self, data):
        out = orig(self, data)
        seen.append((int(out["seed"]), int(np.float32(out["scale"].item()).view(np.uint32))))
        return out
    AS.EdenSender.compress = recording_compress
    res, scales = {}, {}
    for dist in a.dists.split(","):
        np.random.seed(42)
        torch.manual_seed(42)
        rows = []
        for n in (1, 6):
            for inst in range(2):
                vecs, norms = [], []
                for _ in range(n):
                    v = np.asarray(gens[dist](), dtype=np.float64)
                    norms.append(np.linalg.norm(v) ** 2)
                    vecs.append(torch.as_tensor(v, dtype=torch.float32))
                vns = sum(norms)
                emp = torch.stack(vecs).sum(dim=0) / n
                est = {k: torch.zeros(DIM) for k in schemes}
                for j, v in enumerate(vecs):
                    for k in schemes:
                        del seen[:]
                        est[k] += torch.as_tensor(fns[k[0]](v, k[1])) / n
                        if k[0] == "eden":
                            assert len(seen) == 1
                            scales.setdefault(dist, []).append([n, inst, j, k[1], seen[0][0], seen[0][1]])
                row = {"n": n, "inst": inst}
                for k in schemes:
                    row[f"{k[0]}{k[1]}"] = float(torch.norm(est[k] - emp).pow(2) / (50 * vns * n))
                rows.append(row)
                print(dist, row, flush=True)
        res[dist] = rows
    name = "nd_nmse_schemes.json" if DIM == 2048 else f"nd_nmse_schemes_d{DIM}.json"
    if a.quicfl:
        name = name.replace(".json", "_quicfl.json")
    with open(os.path.join(HERE, name), "w") as f:
        json.dump({"dim": DIM, "rows": res, "eden_scales_fields": ["n", "inst", "client", "bits", "seed", "scale_bits"],
                   "eden_scales": scales}, f, indent=1)


if __name__ == "__main__":
    main()
