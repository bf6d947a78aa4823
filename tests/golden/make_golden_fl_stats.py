"""Golden fixtures for the FL NMSE statistics, produced by the REFERENCE itself (build
container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fl_stats.py
        -> tests/golden/fl_stats.json, tests/golden/fl_stats.npz

Imports SImulation_Results_datasets/MNIST/Codes/NMSE_Results.py and runs
  * data_format (:7-41) on a spread of values (every branch: nan, [0.01, 1e4), [0.001, 0.01),
    the 5-digit scientific form, integers, values whose mantissa has trailing zeros);
  * compute_nmse_stats_auto (:43-140) on a synthetic NMSE_Results tree in the exact layout the
    client hook writes (Type_unbiased.py:171-197: <scheme>/rate_<R>/NMSE_info_<k>.pkl holding
    [error tensor, float norm]): two schemes x two rates, one rate folder whose file count is
    not 1 + 5*rounds, one with a missing file, one round with zero gradients (nan).
The reference ends by writing an .xlsx through openpyxl, which this image lacks; the
generator replaces pandas.DataFrame.to_excel with a recorder, so the table the reference
would have written is captured as it is, and its printed max / avg values are parsed from
stdout.  The inputs are stored in the npz (error vectors, norms) so the test rebuilds the
same tree."""
from __future__ import annotations

import contextlib
import io
import json
import os
import pickle
import re
import sys
import tempfile
import warnings

import numpy as np
import pandas as pd
import torch

warnings.filterwarnings("ignore")
REF = "/root/reference/SImulation_Results_datasets/MNIST/Codes"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import NMSE_Results as NR  # noqa: E402  (the reference module)

FORMAT_VALUES = [float("nan"), 0.0, 1e-9, 3.14159e-7, 0.000999999, 0.001, 0.0012345678, 0.00999, 0.01, 0.0123456,
                 0.1499999, 0.197, 1.0, 2.5, 9999.9999, 1e4, 123456.789, 5e-5, 1.2e-3, 7.0e-2, 0.02300000001,
                 4.7145409104443203e-11, 1.0085821486427449e-05, 3.9580e-2]

# (scheme, rate folder, number of NMSE_info files, files to drop, zero-gradient round)
TREE = [("Type_unbiased_quantize", "rate_1", 1 + 5 * 4, [], None),
        ("Type_unbiased_quantize", "rate_2", 1 + 5 * 3 + 2, [], None),     # 2 trailing files: not a round
        ("Type_biased_quantize", "rate_1", 1 + 5 * 3, [9], None),          # a missing file
        ("Type_biased_quantize", "rate_2", 1 + 5 * 2, [], 1)]              # round 1: all-zero gradients


def main(d=1000):
    rng = np.random.default_rng(11)
    arrays = {}
    meta = {"format": [], "tree": [], "d": d}
    for v in FORMAT_VALUES:
        meta["format"].append({"value": v, "text": NR.data_format(v)})
    with tempfile.TemporaryDirectory() as top:
        parent = os.path.join(top, "NMSE_Results_MNIST")
        for t, (scheme, rate, nfiles, drop, zround) in enumerate(TREE):
            rd = os.path.join(parent, scheme, rate)
            os.makedirs(rd)
            for k in range(1, nfiles + 1):
                zero = zround is not None and k >= 2 and (k - 2) // 5 == zround
                g = np.zeros(d, np.float32) if zero else (rng.standard_normal(d) * rng.uniform(0.01, 1)).astype(np.float32)
                err = (rng.standard_normal(d) * 0.3 * float(np.abs(g).mean() + (0.1 if zero else 0))).astype(np.float32)
                if zero:
                    err[:] = 0.0
                gn = float(torch.norm(torch.from_numpy(g)).item())
                arrays[f"err_{t}_{k}"] = err
                arrays[f"norm_{t}_{k}"] = np.float64(gn)
                if k in drop:
                    continue
                with open(os.path.join(rd, f"NMSE_info_{k}.pkl"), "wb") as f:
                    pickle.dump([torch.from_numpy(err), gn], f)
            meta["tree"].append({"scheme": scheme, "rate": rate, "files": nfiles, "drop": drop, "zero_round": zround})
        captured = {}

        def record(self, path, index=False, engine=None):
            captured["rows"] = self.to_dict(orient="records")
        out = io.StringIO()
        old = pd.DataFrame.to_excel
        pd.DataFrame.to_excel = record
        cwd = os.getcwd()
        try:
            os.chdir(top)
            with contextlib.redirect_stdout(out):
                NR.compute_nmse_stats_auto(parent, sampled_clients_per_round=5)
        finally:
            os.chdir(cwd)
            pd.DataFrame.to_excel = old
        text = out.getvalue()
        # printed raw values, in the order the reference walked the tree
        walked = []
        cur_scheme = None
        for line in text.splitlines():
            if line.startswith("Scheme: "):
                cur_scheme = line[len("Scheme: "):]
            elif line.startswith("  Rate folder: "):
                walked.append({"scheme": cur_scheme, "rate": line[len("  Rate folder: "):]})
            elif line.startswith("Max NMSE: "):
                walked[-1]["max"] = float(line[len("Max NMSE: "):])
            elif line.startswith("Avg NMSE: "):
                walked[-1]["avg"] = float(line[len("Avg NMSE: "):])
        meta["rows"] = captured["rows"]
        meta["printed"] = walked
        meta["source"] = ("reference SImulation_Results_datasets/MNIST/Codes/NMSE_Results.py "
                          "(data_format, compute_nmse_stats_auto; to_excel recorded)")
    np.savez_compressed(os.path.join(HERE, "fl_stats.npz"), **arrays)
    with open(os.path.join(HERE, "fl_stats.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    print(json.dumps(meta["rows"], indent=1))
    assert re.search(r"Max NMSE", text)


if __name__ == "__main__":
    main()
