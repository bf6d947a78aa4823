"""Golden fixtures for EDEN + RHT, made by running the REFERENCE itself (build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_eden.py

Calls EdenSender.compress / EdenReceiver.decompress (NMSE_Results/Codes/All_Schemes.py:324-413)
and HadamardSender.randomized_hadamard_transform (AS:123-141) on torch CPU with chosen
rotation seeds, and EDEN_quantize_Hadamard (AS:792-811) after torch.manual_seed for the
drop-in.  Stores: the RHT diagonal for a few seeds (MT19937 known answers), small inputs and
outputs in full, large ones as generator specs + sha256 of the bins + the scale + 4096
sampled outputs.
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
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, "/root/reference/NMSE_Results/Codes")
import All_Schemes as AS  # noqa: E402  (the reference module)
from golden_data import sha, spec_gen  # noqa: E402

f32 = np.float32


def main():
    torch.set_num_threads(1)
    S = AS.EdenSender(device="cpu")
    R = AS.EdenReceiver(device="cpu")
    H = AS.Hadamard(device="cpu")
    arrs, meta = {}, {"diag": [], "cases": [], "dropin": [], "rht": []}
    HS = AS.HadamardSender(device="cpu")
    HR = AS.HadamardReceiver(device="cpu")
    for k, (dim, seed) in enumerate(((1, 3), (5, 0), (1000, 42), (4096, 99), (5000, 7), (1 << 16, 11), (1 << 20, 123))):
        x = spec_gen({"dist": "normal", "d": dim, "seed": 700 + k})
        fwd = HS.randomized_hadamard_transform(torch.from_numpy(x.copy()), seed).numpy().astype(f32)
        inv = HR.randomized_inverse_hadamard_transform(torch.from_numpy(fwd.copy()), seed).numpy().astype(f32)
        meta["rht"].append({"k": k, "dim": dim, "seed": seed, "fwd_sha": sha(fwd), "inv_sha": sha(inv)})
        if dim <= 8192:
            arrs[f"rfwd{k}"] = fwd
            arrs[f"rinv{k}"] = inv
    for seed, D in ((0, 4096), (17, 1000), (99, 624 * 3 + 5), (123, 64)):
        dg = H.random_diagonal(D, seed).numpy().astype(np.int8)
        arrs[f"diag_{seed}_{D}"] = dg
        meta["diag"].append({"seed": seed, "D": D})
    rng = np.random.default_rng(7)
    idx = 0
    for dim, dist, store in ((1, "normal", True), (3, "normal", True), (8, "normal", True), (333, "normal", True),
                             (1000, "laplace", True), (1024, "normal", True), (4096, "lognormal", True),
                             (5000, "bernoulli", True), (65536, "gamma", False), (172554, "normal", False),
                             (1 << 20, "normal", False), (1 << 20, "laplace", False)):
        for nbits in (1, 2):
            for seed in (0, 42, 99):
                sp = {"dist": dist, "d": dim, "seed": 500 + dim % 1000 + seed}
                x = spec_gen(sp) if dim > 1 else np.array([rng.standard_normal()], f32)
                data = S.compress({"vec": torch.from_numpy(x.copy()), "seed": seed, "nbits": nbits})
                out = R.decompress(data).numpy().astype(f32)
                bins = data["bins"].numpy().astype(np.uint8)
                case = dict(sp, idx=idx, nbits=nbits, rseed=seed, scale=float(data["scale"]),
                            bins_sha=sha(bins), out_sha=sha(out), D=int(bins.shape[0]))
                if store:
                    arrs[f"x{idx}"] = x
                    arrs[f"bins{idx}"] = bins
                    arrs[f"out{idx}"] = out
                else:
                    pos = np.random.default_rng(idx).choice(dim, 4096, replace=False).astype(np.int64)
                    arrs[f"pos{idx}"] = pos
                    arrs[f"outs{idx}"] = out[pos]
                meta["cases"].append(case)
                print(idx, dim, dist, nbits, seed, float(data["scale"]), flush=True)
                idx += 1
    # the drop-in: seed drawn from the global generator
    for tseed in (0, 1, 2):
        x = spec_gen({"dist": "normal", "d": 2000, "seed": 900 + tseed})
        for nbits in (1, 2):
            torch.manual_seed(tseed)
            drawn = int(torch.randint(0, 100, (1,)).item())
            torch.manual_seed(tseed)
            out = AS.EDEN_quantize_Hadamard(torch.from_numpy(x.copy()), nbits)
            arrs[f"dx{tseed}_{nbits}"] = x
            arrs[f"dout{tseed}_{nbits}"] = np.asarray(out, f32)
            meta["dropin"].append({"tseed": tseed, "nbits": nbits, "drawn_seed": drawn})
    np.savez_compressed(os.path.join(HERE, "eden_vectors.npz"), **arrs)
    with open(os.path.join(HERE, "eden_vectors.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
