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


def _compose_scan(d0, d1):
    """The small-batch fold's wave scan (exact_fold_kernel): maps P -> P + d[P & 1] in
    integer units of G, Hillis-Steele over 64 lanes with (F then g).d[p] =
    F.d[p] + g.d[p ^ (F.d[p] & 1)]; returns the inclusive composed maps."""
    d0, d1 = d0.copy(), d1.copy()
    o = 1
    while o < 64:
        f0 = np.concatenate([np.zeros(o, np.uint64), d0[:-o]])
        f1 = np.concatenate([np.zeros(o, np.uint64), d1[:-o]])
        n0 = f0 + np.where(f0 & 1, d1, d0)
        n1 = f1 + np.where(f1 & 1, d0, d1)
        lane = np.arange(64)
        d0 = np.where(lane >= o, n0, d0).astype(np.uint64)
        d1 = np.where(lane >= o, n1, d1).astype(np.uint64)
        o <<= 1
    return d0, d1


def test_tile_map_composition_equals_serial_fold():
    """Regular tile maps of one binade composed by the wave scan give the same exact tile
    starts as the serial fold P_{t+1} = P_t + m[parity(P_t)] (and as the sequential cumsum)."""
    d = 400 * S.TILE
    x = S.tiny_mix(11, d, 0.3, 1e-3)
    fr = fractions(x, O.rate_to_m(1, d)).astype(f64)
    seq = np.concatenate([[0.0], np.cumsum(fr)])
    tiles = d // S.TILE
    P = seq[np.arange(tiles) * S.TILE]                     # exact tile starts
    checked = 0
    t = 1
    while t + 64 <= tiles:
        E = S.binade(P[t])
        G = np.ldexp(1.0, E - 52)
        if P[t] < 32.0 or S.binade(P[t + 64]) != E:
            t += 1
            continue
        # maps of tiles t .. t+63 from an even and an odd start inside the binade
        m0 = np.empty(64, np.uint64)
        m1 = np.empty(64, np.uint64)
        for u in range(64):
            v = fr[(t + u) * S.TILE:(t + u + 1) * S.TILE].reshape(S.BLOCK, S.ITEMS)
            pe = P[t + u] if S.par(P[t + u]) == 0 else P[t + u] - G
            po = pe + G
            m0[u] = np.uint64(round((S.exact_tile(pe, v)[1] - pe) / G))
            m1[u] = np.uint64(round((S.exact_tile(po, v)[1] - po) / G))
        i0, i1 = _compose_scan(m0, m1)
        Pi0 = np.uint64(round(P[t] / G))                     # P / G (with the implicit bit)
        odd = int(Pi0) & 1
        excl = np.concatenate([[np.uint64(0)], (i1 if odd else i0)[:-1]])
        starts = (Pi0 + excl).astype(np.float64) * G
        assert np.array_equal(starts.view(np.uint64), P[t:t + 64].view(np.uint64))
        end = float(Pi0 + (i1 if odd else i0)[-1]) * G
        assert end == P[t + 64]
        checked += 64
        t += 64
    assert checked >= 128
