"""MT19937 jump-ahead (uq_mt_poly.cpp, the host half of the QUIC-FL sender's jump path KQ0j):
the state b blocks ahead computed from t^(624 (b - 1)) mod phi and the correlation with the
stream's first words must equal b direct twists (oracle/uq_quicfl.py's ATen restatement) for
seeded states and arbitrary torch generator states.  Host-only: no GPU."""
import ctypes

import numpy as np
import pytest
import torch

import uqdme  # noqa: F401  (registers the uqdme_amd package alias)
from oracle import uq_quicfl as Q
from uqdme_amd._lib import load


def jump(state: np.ndarray, b: int) -> np.ndarray:
    st = np.ascontiguousarray(state, np.uint32)
    out = np.zeros(624, np.uint32)
    rc = load().uq_mt_jump_host(st.ctypes.data_as(ctypes.c_void_p), b, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


def twisted(state: np.ndarray, b: int) -> np.ndarray:
    mt = state.astype(np.uint32)
    for _ in range(b):
        mt = Q._twist(mt)
    return mt


@pytest.mark.parametrize("b", [0, 1, 2, 31, 32, 33, 34, 100, 1681])
def test_jump_equals_twists_seeded(b):
    for seed in (0, 5489, 65535):
        st = Q.seeded_state(seed)[2]
        assert np.array_equal(jump(st, b), twisted(st, b)), (seed, b)


def test_jump_from_torch_generator_states():
    """Arbitrary states of torch's CPU generator (the global stream of AS:489), not only fresh
    seeds: the jump works on any 624-word array, including its word 0 (only its top bit is
    state) -- the result's every word is exact."""
    import uqdme_amd.quicfl as q
    rng = np.random.default_rng(7)
    g = torch.Generator()
    for k in range(3):
        g.manual_seed(int(rng.integers(0, 2**31)))
        torch.rand(int(rng.integers(1, 5000)), generator=g)
        st = np.asarray(q.generator_words(g)[1][2:], np.uint32)
        for b in (1, 7, 300):
            assert np.array_equal(jump(st, b), twisted(st, b)), (k, b)


def test_jump_far_matches_stream():
    """A long jump (a 2^22-coordinate message reaches ~13 500 blocks into its local stream):
    the jumped block's tempered words are torch's own draws at that position
    (randint(0, 100) takes one word per element, word % 100, as h at AS:465)."""
    g = torch.Generator()
    g.manual_seed(4242)
    b = 13_447
    got = torch.randint(0, 100, (624 * b + 624,), generator=g)[624 * b:].numpy()
    blk = jump(Q.seeded_state(4242)[2], b + 1)      # block b + 1 holds draws 624 b .. 624 b + 623
    assert np.array_equal(got, (Q._temper(blk) % np.uint32(100)).astype(np.int64))
