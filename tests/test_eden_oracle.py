"""CPU: the EDEN + RHT restatement (oracle/uq_eden.py) against the reference's own outputs
(tests/golden/eden_vectors.*, from make_golden_eden.py).  Rotation diagonal and bins are
bit-exact; the scale (and so the output) within 1e-6 relative: the reference's dot product
runs in MKL's CPU-dependent order (AS:335), the restatement accumulates it in fp64."""
import numpy as np
import pytest

from oracle import uq_eden as E
from tests import golden_data as G

RTOL = 1e-6          # north_star floating-point tolerance


@pytest.fixture(scope="module")
def fx():
    return G.eden()


def test_mt19937_diagonal_known_answers(fx):
    meta, z = fx
    for dg in meta["diag"]:
        exp = z[f"diag_{dg['seed']}_{dg['D']}"]
        got = E.random_diagonal(dg["D"], dg["seed"]).astype(np.int8)
        assert np.array_equal(got, exp), dg


def test_tables():
    assert E.boundaries(1).tolist() == [0.0]            # AS:315 overwrites AS:314
    assert len(E.boundaries(2)) == 3 and E.centroids(2).shape == (4,)


def test_eden_oracle_vs_reference(fx):
    meta, z = fx
    for case in meta["cases"]:
        if case["d"] > 200000:
            continue                                   # the GPU tests cover 2^20 against the same fixtures
        x = G.eden_input(case, z)
        bins, scale, _, D = E.eden_compress(x, case["nbits"], case["rseed"])
        assert D == case["D"]
        assert G.sha(bins.astype(np.uint8)) == case["bins_sha"], case["idx"]
        assert abs(float(scale) - case["scale"]) <= RTOL * abs(case["scale"]), case["idx"]
        out = E.eden_decompress(bins, scale, case["nbits"], case["rseed"], case["d"])
        i = case["idx"]
        if f"out{i}" in z.files:
            np.testing.assert_allclose(out, z[f"out{i}"], rtol=RTOL, atol=0)
        else:
            np.testing.assert_allclose(out[z[f"pos{i}"]], z[f"outs{i}"], rtol=RTOL, atol=0)


def test_hadamard_is_an_involution_up_to_rounding():
    rng = np.random.default_rng(0)
    v = rng.standard_normal(1 << 12).astype(np.float32)
    w = E.hadamard(E.hadamard(v))
    np.testing.assert_allclose(w, v, rtol=1e-4, atol=1e-5)


def test_rht_oracle_vs_reference(fx):
    meta, z = fx
    for r in meta["rht"]:
        if r["dim"] > 70000:
            continue
        x = G.spec_gen({"dist": "normal", "d": r["dim"], "seed": 700 + r["k"]})
        f = E.rht(x, r["seed"])
        assert G.sha(f) == r["fwd_sha"], r
        assert G.sha(E.inverse_rht(f, r["seed"])) == r["inv_sha"], r
