"""CPU: the EDEN + RHT restatement (oracle/uq_eden.py) against the reference's own outputs
(tests/golden/eden_vectors.*, from make_golden_eden.py) and the EDEN scales the reference's
driver loop recorded (tests/golden/nd_nmse_schemes*.json): rotation diagonal, bins, scale and
outputs bit for bit.  The scale's torch.dot (AS:335) is restated in MKL sdot's order on the
fixtures' host (oracle/uq_eden.py:torch_dot, pinned in tests/test_dot_oracle.py)."""
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
        assert np.float32(scale) == np.float32(case["scale"]), case["idx"]       # bit for bit
        out = E.eden_decompress(bins, scale, case["nbits"], case["rseed"], case["d"])
        i = case["idx"]
        assert G.sha(out) == case["out_sha"], i
        if f"out{i}" in z.files:
            assert G.bits_equal(out, z[f"out{i}"]), i
        else:
            assert G.bits_equal(out[z[f"pos{i}"]], z[f"outs{i}"]), i


ND_GENS = {"normal": lambda d: np.random.normal(0, 1, d),
           "laplace": lambda d: np.random.laplace(loc=1, scale=2, size=d),
           "gamma": lambda d: np.random.gamma(shape=2, scale=2, size=d),
           "bernoulli": lambda d: np.random.choice(np.arange(2), size=d, p=[0.3, 0.7]),
           "lognormal": lambda d: np.random.lognormal(mean=1, sigma=2, size=d)}


@pytest.mark.parametrize("fixture,per_dist", [("nd_nmse_schemes.json", None), ("nd_nmse_schemes_d4194304.json", 1)])
def test_eden_scales_of_the_reference_loop(fixture, per_dist):
    """Every EDEN scale the reference's driver loop recorded (EdenSender.compress outputs,
    make_golden_nmse_schemes.py): d = 2048, all five distributions; at C4's d = 2^22 the first
    scale of each distribution (the NumPy restatement takes seconds per 2^22 vector; the GPU
    tests check all of them)."""
    import json
    import os
    ref = json.load(open(os.path.join(G.GOLDEN, fixture)))
    dim = ref["dim"]
    checked = 0
    for dist, entries in ref["eden_scales"].items():
        st = np.random.get_state()
        try:
            np.random.seed(42)                      # ND:14-15, vectors in the loop's order
            vecs = {(n, inst, j): np.asarray(ND_GENS[dist](dim), np.float64).astype(np.float32)
                    for n in (1, 6) for inst in range(2) for j in range(n)}
        finally:
            np.random.set_state(st)
        for n, inst, client, bits, seed, sbits in entries[:per_dist]:
            _, sc, _, _ = E.eden_compress(vecs[(n, inst, client)], bits, seed)
            assert int(np.float32(sc).view(np.uint32)) == sbits, (dist, n, inst, client, bits)
            checked += 1
    assert checked == (140 if per_dist is None else 5)


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
