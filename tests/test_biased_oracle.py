"""CPU: the C++ restatement of Type_biased_quantize / Reznik (oracle/uq_biased.cpp) against
the reference's own outputs (tests/golden/biased_vectors.*, made by make_golden_biased.py),
ties included: torch.topk's choice among equal delta' values is libstdc++'s
nth_element / partial_sort, which the oracle replays."""
import numpy as np
import pytest

from oracle import uq_oracle_c as C
from oracle.uq_oracle import rate_to_m
from tests import golden_data as G


@pytest.fixture(scope="module")
def cases():
    C.build()
    return list(G.biased_vectors())


def test_fixture_count(cases):
    assert len(cases) >= 150
    assert sum(1 for sp, *_ in cases if sp.get("ambiguous")) >= 50     # ties do straddle the threshold
    assert sum(1 for sp, *_ in cases if sp.get("raises")) >= 3


def test_oracle_torch_ties_bit_exact(cases):
    bad = []
    for sp, x, q, h in cases:
        m = rate_to_m(sp["R"], x.shape[0])
        if sp.get("raises"):
            with pytest.raises(RuntimeError):
                C.biased_quantize(x, m, sp["threads"], 0)
            continue
        with np.errstate(all="ignore"):
            out, _, D, A = C.biased_quantize(x, m, sp["threads"], 0)
        ok = G.bits_equal(out, q) if q is not None else G.sha(out) == h
        if not ok or D != sp["delta"] or A != sp["ambiguous"]:
            bad.append(sp["idx"])
    assert not bad, f"oracle differs from the reference on fixtures {bad}"


def test_lowest_index_rule_only_differs_on_ambiguous(cases):
    """tie_mode 1 (the GPU's cheap rule) equals the reference whenever no tie straddles the
    threshold; where one does, only threshold-tied coordinates move and sum(k) == m holds."""
    for sp, x, q, h in cases:
        if sp.get("raises") or x.shape[0] > 8192:
            continue
        m = rate_to_m(sp["R"], x.shape[0])
        with np.errstate(all="ignore"):
            out1, L, D, A = C.biased_quantize(x, m, sp["threads"], 1)
            out0, *_ = C.biased_quantize(x, m, sp["threads"], 0)
        if not A:
            assert G.bits_equal(out1, out0), sp["idx"]
        elif np.isfinite(L) and L > 0 and m > 0:
            k0 = np.rint(np.abs(out0.astype(np.float64)) * m / float(L))
            k1 = np.rint(np.abs(out1.astype(np.float64)) * m / float(L))
            assert k0.sum() == k1.sum() == m, sp["idx"]


def test_biased_sum_is_m_when_adjusted():
    """Reznik's point: after the adjustment sum(k'') == m exactly (AS:657-666)."""
    C.build()
    rng = np.random.default_rng(5)
    for d in (10, 333, 5000):
        for R in (0.5, 1, 2, 4):
            x = rng.standard_normal(d).astype(np.float32)
            m = rate_to_m(R, d)
            if m == 0:          # k'/0: the reference's output is NaN
                continue
            out, L, D, A = C.biased_quantize(x, m, 1, 0)
            k = np.rint(np.abs(out.astype(np.float64)) * m / float(L))
            assert k.sum() == m
