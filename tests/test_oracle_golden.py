"""Pin the CPU oracle (oracle/) against fixtures produced by the reference itself.

These run on CPU.  They are what makes the oracle trustworthy as the checker for the
GPU parity tests (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C
from tests import golden_data as G

f32 = np.float32


def test_c1_harness_outputs_and_nmse():
    z = G.c1()
    x = z["x"]
    q1 = np.stack([O.type_unbiased_quantize(x[j], 1, z["X1"][j]) for j in range(16)])
    q2 = np.stack([O.type_unbiased_quantize(x[j], 2, z["X2"][j]) for j in range(16)])
    assert G.bits_equal(q1, z["q1"])
    assert G.bits_equal(q2, z["q2"])
    e1 = O.client_mean(q1, 16)
    e2 = O.client_mean(q2, 16)
    assert G.bits_equal(e1, z["est1"])
    assert G.bits_equal(e2, z["est2"])
    n1 = O.script_nmse(e1, z["emp"], float(z["vec_norm_squared"]), 16)
    n2 = O.script_nmse(e2, z["emp"], float(z["vec_norm_squared"]), 16)
    # bit for bit: script_nmse restates torch.norm's f32 order (north_star allows 1e-6 relative)
    assert n1 == float(z["nmse1"]) and n2 == float(z["nmse2"]), (n1, n2)
    # survey known answers
    assert float(z["nmse1"]) == 1.0085821486427449e-05
    assert float(z["nmse2"]) == 1.197929691443278e-06


def test_c_oracle_matches_c1():
    z = G.c1()
    m1 = O.rate_to_m(1, 1024)
    q1, l1 = C.quantize_batch(z["x"], m1, z["X1"], 1)
    assert G.bits_equal(q1, z["q1"])
    assert G.bits_equal(C.client_mean(q1, 16), z["est1"])


@pytest.mark.parametrize("impl", ["py", "c"])
def test_edge_cases(impl):
    n = 0
    for name, R, X, x, q in G.edge_cases():
        if impl == "py":
            got = O.type_unbiased_quantize(x, R, X)
        else:
            got = C.quantize_batch(x[None], O.rate_to_m(R, x.shape[0]), [X])[0][0]
        assert G.bits_equal(got, q), (name, R, G.n_mismatch(got, q))
        n += 1
    assert n > 40


def test_spec_vectors_mid():
    n = 0
    for sp, q, _, _ in G.spec_vectors(large=False):
        x = G.spec_gen(sp)
        assert G.sha(x) == sp["x_sha256"]
        assert O.l1_torch_order(x, sp["threads"]) == f32(sp["l1"])
        got = C.quantize_batch(x[None], O.rate_to_m(sp["R"], sp["d"]), [sp["X"]], sp["threads"])[0][0]
        assert G.bits_equal(got, q), (sp, G.n_mismatch(got, q))
        n += 1
    assert n >= 40


def test_spec_vectors_large_c_oracle():
    for sp, _, pos, qs in G.spec_vectors(large=True):
        x = G.spec_gen(sp)
        assert G.sha(x) == sp["x_sha256"]
        got = C.quantize_batch(x[None], O.rate_to_m(sp["R"], sp["d"]), [sp["X"]], sp["threads"])[0][0]
        assert C.l1_torch_order(x, sp["threads"]) == f32(sp["l1"])
        assert G.bits_equal(got[pos], qs)
        assert G.sha(got) == sp["q_sha256"], sp


def test_python_oracle_large_l1():
    # the vectorised Python cascade at full size, both thread counts
    for sp, _, _, _ in G.spec_vectors(large=True):
        if sp["d"] != 1 << 20:
            continue
        x = G.spec_gen(sp)
        assert O.l1_torch_order(x, sp["threads"]) == f32(sp["l1"])


def test_nd_harness_points():
    """ND loop (dim=2048, n in {1,6,11}) restated on the oracle reproduces the reference
    NMSE per instance (seed 42 numpy + torch draws reproduced with torch's CPU generator)."""
    import torch
    pts = G.nd_points()
    for dist, rows in pts.items():
        np.random.seed(42)
        gen = torch.Generator().manual_seed(42)
        k = 0
        for n in (1, 6, 11):
            for inst in range(4):
                vecs, norms = [], []
                for _ in range(n):
                    v = (np.random.normal(0, 1, 2048) if dist == "normal"
                         else np.random.laplace(loc=1, scale=2, size=2048))
                    norms.append(np.linalg.norm(v) ** 2)
                    vecs.append(v.astype(f32))
                vns = sum(norms)
                emp = (torch.stack([torch.from_numpy(v) for v in vecs]).sum(dim=0) / n).numpy()   # ND:95
                q1, q2 = [], []
                for v in vecs:
                    X1 = torch.rand(1, generator=gen).item()
                    X2 = torch.rand(1, generator=gen).item()
                    q1.append(O.type_unbiased_quantize(v, 1, X1))
                    q2.append(O.type_unbiased_quantize(v, 2, X2))
                n1 = O.script_nmse(O.client_mean(q1, n), emp, vns, n)
                n2 = O.script_nmse(O.client_mean(q2, n), emp, vns, n)
                row = rows[k]
                assert row["n"] == n and row["inst"] == inst
                # bit for bit (emp by the reference's own torch op; the norm in torch's order)
                assert n1 == row["nmse1"], (dist, n, inst, n1, row)
                assert n2 == row["nmse2"], (dist, n, inst, n2, row)
                k += 1


def test_random_py_vs_c_oracle():
    rng = np.random.default_rng(11)
    for d in (1, 2, 3, 7, 8, 9, 31, 32, 33, 257, 1000, 4099, 40000, 70001):
        for T in (1, 3, 8):
            x = (rng.standard_normal(d) * rng.choice([1e-3, 1.0, 1e3])).astype(f32)
            assert O.l1_torch_order(x, T) == C.l1_torch_order(x, T), (d, T)
            for R in (0.5, 1, 4):
                X = rng.random()
                m = O.rate_to_m(R, d)
                a = O.quantize_with_m(x, m, X, T)
                b = C.quantize_batch(x[None], m, [X], T)[0][0]
                assert G.bits_equal(a, b), (d, T, R)


def test_rate_table_matches_survey_m():
    assert O.rate_to_m(1, 1024) == 219 and O.rate_to_m(2, 1024) == 652
    assert O.rate_to_m(1, 1 << 20) == 224426 and O.rate_to_m(2, 1 << 20) == 668488
    assert O.rate_to_m(1, 1 << 22) == 897706 and O.rate_to_m(2, 1 << 22) == 2673952
    assert O.rate_to_m(1, 172554) == 36931 and O.rate_to_m(2, 172554) == 110006
    with pytest.raises(KeyError):
        O.rate_to_m(3.3, 10)


def test_l1_thread_counts_match_torch_fixture():
    """AS:624 at T = 1..256 torch threads: torch reduces in two passes (per-thread chunk
    sums into a T-element buffer, then the same cascade over the buffer), pinned by
    tests/golden/l1_threads.json (torch's own results).  C oracle everywhere, the NumPy
    restatement on the sizes it finishes quickly."""
    n = 0
    for r, x in G.l1_threads():
        want = np.uint32(r["l1_bits"]).view(f32)
        assert C.l1_torch_order(x, r["threads"]) == want, (r["d"], r["threads"])
        if r["d"] <= 65537:
            assert O.l1_torch_order(x, r["threads"]) == want, (r["d"], r["threads"])
        n += 1
    assert n >= 140
