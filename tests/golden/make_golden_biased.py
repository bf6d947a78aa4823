"""Golden fixtures for the biased type quantizer, made by running the REFERENCE itself
(build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_biased.py

Calls `Type_biased_quantize` from /root/reference/NMSE_Results/Codes/All_Schemes.py
(AS:669-687, Reznik AS:644-666) on torch CPU with a given intra-op thread count and
records outputs.  Inputs come from generator specs (tests/golden_data.spec_gen, legacy
RandomState) or, for the hand-made edge cases, are stored.  Outputs are stored for small
vectors and hashed (sha256 of the f32 bytes) for large ones; Delta and whether a tie
straddles the topk threshold (so that torch's tie choice matters) are recorded from the
C++ restatement in oracle/ for the record.
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import torch

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, "/root/reference/NMSE_Results/Codes")
import All_Schemes as AS  # noqa: E402  (the reference module)
from golden_data import sha, spec_gen  # noqa: E402
from oracle import uq_oracle_c as OC  # noqa: E402
from oracle.uq_oracle import rate_to_m  # noqa: E402

f32 = np.float32


def ref(x, R, T):
    torch.set_num_threads(T)
    return AS.Type_biased_quantize(torch.from_numpy(x.copy()), R).numpy().astype(f32)


def main():
    specs, arrs = [], {}

    def add(sp, x, store_x):
        i = len(specs)
        try:
            q = ref(x, sp["R"], sp["threads"])
        except (ValueError, RuntimeError) as e:   # the reference raises (AS:656 / AS:660)
            specs.append(dict(sp, idx=i, raises=type(e).__name__, d=int(x.shape[0]), sha=None))
            arrs[f"x{i}"] = x
            print(i, "raises", type(e).__name__, flush=True)
            return
        _, _, D, A = OC.biased_quantize(x, rate_to_m(sp["R"], x.shape[0]), sp["threads"], 0)
        sp = dict(sp, idx=i, sha=sha(q), delta=D, ambiguous=A, d=int(x.shape[0]))
        if store_x:
            arrs[f"x{i}"] = x
        if x.shape[0] <= 8192:
            arrs[f"q{i}"] = q
        specs.append(sp)
        print(i, sp.get("name", sp.get("dist")), sp["d"], sp["R"], sp["threads"], "Delta", D, "amb", A, flush=True)

    # hand-made edge cases (stored inputs)
    edge = {
        "one": np.array([3.0], f32),
        "zeros": np.zeros(17, f32),
        "single_nonzero": np.eye(1, 33, 7, dtype=f32).reshape(-1) * -2.5,
        "signed_ties": np.array([1, -1, 1, -1, 2, -2, 0, 0, 1, -1, 1, 1] * 9, f32),
        "tiny": (np.arange(1, 50, dtype=f32) * 1e-41).astype(f32),
        "huge": np.array([3e38, -3e38, 1e38, 2.0] * 5, f32)[:19],
        "d7": np.array([0.5, -0.25, 3, 1e-3, -7, 2, 2], f32),
    }
    for name, x in edge.items():
        for R in (0.5, 1, 4):
            with np.errstate(all="ignore"):
                add({"name": name, "R": R, "threads": 1}, x, True)
    # generated vectors
    for dist in ("normal", "laplace", "gamma", "bernoulli", "lognormal", "rounded", "smallint"):
        for d in (100, 1000, 4099):
            for R in (0.5, 1, 2, 4, 8):
                add({"dist": dist, "d": d, "seed": 300 + d % 97, "R": R, "threads": 1}, spec_gen(
                    {"dist": dist, "d": d, "seed": 300 + d % 97}), False)
        for d, T in ((65537, 8), (172554, 1), (1 << 20, 1), (1 << 20, 8)):
            for R in (1, 4):
                sp = {"dist": dist, "d": d, "seed": 400 + T, "R": R, "threads": T}
                add(sp, spec_gen(sp), False)
    np.savez_compressed(os.path.join(HERE, "biased_vectors.npz"), **arrs)
    with open(os.path.join(HERE, "biased_vectors.json"), "w") as f:
        json.dump(specs, f, indent=0)


if __name__ == "__main__":
    main()
