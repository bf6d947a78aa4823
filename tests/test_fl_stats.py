"""FL NMSE statistics: fl_stats.compute_nmse_stats_auto / data_format
against the reference's own NMSE_Results.py outputs (tests/golden/fl_stats.*, produced by
tests/golden/make_golden_fl_stats.py), plus one round computed by hand."""
import json
import os
import pickle

import numpy as np
import torch

import uqdme
from tests.golden_data import GOLDEN


def _golden():
    meta = json.load(open(os.path.join(GOLDEN, "fl_stats.json")))
    z = np.load(os.path.join(GOLDEN, "fl_stats.npz"))
    return meta, z


def test_data_format_matches_reference():
    meta, _ = _golden()
    for rec in meta["format"]:
        assert uqdme.data_format(float(rec["value"])) == rec["text"], rec


def _build_tree(top, meta, z):
    parent = os.path.join(top, "NMSE_Results_MNIST")
    for t, tr in enumerate(meta["tree"]):
        rd = os.path.join(parent, tr["scheme"], tr["rate"])
        os.makedirs(rd)
        for k in range(1, tr["files"] + 1):
            if k in tr["drop"]:
                continue
            with open(os.path.join(rd, f"NMSE_info_{k}.pkl"), "wb") as f:      # the hook's format (FLM:171-197)
                pickle.dump([torch.from_numpy(z[f"err_{t}_{k}"]), float(z[f"norm_{t}_{k}"])], f)
    return parent


def test_compute_nmse_stats_auto_matches_reference(tmp_path):
    meta, z = _golden()
    parent = _build_tree(str(tmp_path), meta, z)
    rows = uqdme.compute_nmse_stats_auto(parent, 5, excel_filename=str(tmp_path / "stats.xlsx"), verbose=False)
    key = lambda r: (r["Scheme"], r["Rate Folder"])  # noqa: E731
    got = {key(r): r for r in rows}
    assert len(got) == len(meta["rows"])
    for ref in meta["rows"]:
        g = got[key(ref)]
        for col in ("Total Files", "No of Rounds", "Clients Per Round", "Max NMSE", "Avg NMSE"):
            assert g[col] == ref[col], (key(ref), col, g[col], ref[col])
    for p in meta["printed"]:
        g = got[(p["scheme"], p["rate"])]
        assert g["max_nmse"] == p["max"] and g["avg_nmse"] == p["avg"], (p, g)
    # the table lands beside the requested name (CSV when openpyxl is absent, as here)
    assert os.path.exists(tmp_path / "stats.csv") or os.path.exists(tmp_path / "stats.xlsx")


def test_round_nmse_by_hand():
    rng = np.random.default_rng(3)
    errs = [rng.standard_normal(257).astype(np.float32) for _ in range(5)]
    norms = [float(v) for v in rng.uniform(0.5, 2.0, 5)]
    s = errs[0].copy()
    for e in errs[1:]:
        s = s + e
    avg = s / 5
    want = float(np.sqrt(np.sum(avg.astype(np.float64) ** 2))) ** 2 / (sum(g * g for g in norms) / 5)
    got = uqdme.round_nmse([torch.from_numpy(e) for e in errs], norms)
    assert abs(got - want) <= 1e-6 * want
    assert np.isnan(uqdme.round_nmse([torch.zeros(4)] * 5, [0.0] * 5))
