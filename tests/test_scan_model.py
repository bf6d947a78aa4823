"""CPU: the arithmetic behind K2's exact scan reproduces torch's
sequential fp64 cumsum (AS:635) bit for bit, on inputs where a plain parallel tree scan
does not (tests/scan_models.py)."""
import numpy as np
import pytest

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C
from tests import scan_models as S

f64 = np.float64


def fractions(x, m):
    _, _, fr = O.fractional_parts(x, m, C.l1_torch_order(x, 1))
    return fr


@pytest.mark.parametrize("seed,d,mix,scale", [(1, 1 << 16, 0.5, 1e-4), (2, 1 << 16, 0.95, 1e-5),
                                              (3, 100003, 0.0, 1.0), (4, 50001, 0.9, 1e-3)])
def test_exact_scheme_matches_sequential_cumsum(seed, d, mix, scale):
    x = S.tiny_mix(seed, d, mix, scale)
    fr = fractions(x, O.rate_to_m(1, d))
    seq = np.cumsum(fr.astype(f64))
    ex = S.exact_prefix(fr)
    assert np.array_equal(seq.view(np.uint64), ex.view(np.uint64))


def test_tree_scan_differs_on_the_gpu_test_inputs():
    d = 1 << 20
    X, i = S.exposing_X(S.tiny_mix(6, d), O.rate_to_m(1, d))
    assert X is not None and i > 0
