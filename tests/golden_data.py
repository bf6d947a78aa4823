"""Readers for the committed golden fixtures (tests/golden/, produced by make_golden.py
from the reference itself).  Pure data access: usable on CPU and on the GPU box."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
f32 = np.float32


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def c1():
    return dict(np.load(os.path.join(GOLDEN, "c1_harness.npz")))


def edge_cases():
    z = np.load(os.path.join(GOLDEN, "edge_cases.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "edge_cases.json")))
    for m in meta:
        i = m["idx"]
        yield m["name"], m["R"], np.float32(m["X"]), z[f"x{i}"], z[f"q{i}"]


def spec_gen(sp) -> np.ndarray:
    """Same generators as make_golden.gen (legacy RandomState: stable across numpy)."""
    rs = np.random.RandomState(sp["seed"])
    d, kind = sp["d"], sp["dist"]
    if kind == "normal":
        v = rs.normal(loc=0, scale=1, size=d)
    elif kind == "laplace":
        v = rs.laplace(loc=1, scale=2, size=d)
    elif kind == "gamma":
        v = rs.gamma(shape=2, scale=2, size=d)
    elif kind == "bernoulli":
        v = rs.choice(np.arange(2), size=d, p=[0.3, 0.7]).astype(np.float64)
    elif kind == "lognormal":
        v = rs.lognormal(mean=1, sigma=2, size=d)
    elif kind == "rounded":            # tie-heavy: many equal |x|
        v = np.round(rs.normal(loc=0, scale=1, size=d) * 4) / 4
    elif kind == "smallint":           # signed small integers: massive ties
        v = rs.randint(-3, 4, size=d).astype(np.float64)
    else:
        raise ValueError(kind)
    return v.astype(f32)


def biased_vectors():
    """Fixtures of Type_biased_quantize (AS:669-687) made by make_golden_biased.py.
    Yields (spec, x, expected_or_None, expected_sha)."""
    z = np.load(os.path.join(GOLDEN, "biased_vectors.npz"))
    specs = json.load(open(os.path.join(GOLDEN, "biased_vectors.json")))
    for sp in specs:
        i = sp["idx"]
        x = z[f"x{i}"] if f"x{i}" in z.files else spec_gen(sp)
        q = z[f"q{i}"] if f"q{i}" in z.files else None
        yield sp, x, q, sp.get("sha")


def spec_vectors(large=None):
    z = np.load(os.path.join(GOLDEN, "spec_vectors.npz"))
    specs = json.load(open(os.path.join(GOLDEN, "spec_vectors.json")))
    for sp in specs:
        is_large = bool(sp.get("large"))
        if large is not None and is_large != large:
            continue
        i = sp["idx"]
        if is_large:
            yield sp, None, z[f"pos{i}"], z[f"qs{i}"]
        else:
            yield sp, z[f"q{i}"], None, None


def nd_points():
    return json.load(open(os.path.join(GOLDEN, "nd_nmse_points.json")))


def bits_equal(a, b) -> bool:
    """Bitwise equality, treating any NaN as equal to any NaN at the same position."""
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def n_mismatch(a, b) -> int:
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    na, nb = np.isnan(a), np.isnan(b)
    bad = (na != nb) | (~na & ~nb & (a.view(np.uint32) != b.view(np.uint32)))
    return int(bad.sum())


def eden():
    """EDEN fixtures (make_golden_eden.py): (meta dict, npz)."""
    z = np.load(os.path.join(GOLDEN, "eden_vectors.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "eden_vectors.json")))
    return meta, z


def eden_input(case, z):
    i = case["idx"]
    return z[f"x{i}"] if f"x{i}" in z.files else spec_gen(case)


def l1_threads():
    """torch's AS:624 L1 at many intra-op thread counts (make_golden_threads.py).
    Yields (record, x)."""
    recs = json.load(open(os.path.join(GOLDEN, "l1_threads.json")))["records"]
    cache = {}
    for r in recs:
        key = (r["seed"], r["d"], r["scale"])
        if key not in cache:
            cache.clear()
            cache[key] = (np.random.default_rng(r["seed"]).standard_normal(r["d"]) * r["scale"]).astype(f32)
        yield r, cache[key]
