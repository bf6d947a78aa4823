"""uq_legacy_draw_f32 (csrc/uq_legacy_rng.cpp): the drivers' input vectors,
byte-identical to numpy's legacy RandomState -- the reference's own generator, run here as the
oracle -- for every distribution the NMSE drivers draw (ND:89, Laplace_dist.py:89,
Gamma_dist.py:86, Bernoulli_dist.py:90, Lognormal_dist.py:90), across consecutive calls, at the
drivers' d = 2048 and C4's d = 2^22, with the state (key, pos, gauss cache) left exactly where
RandomState leaves it, in one thread and many, and through the parallel form's chunk meetings
(including forced misses)."""
import ctypes

import numpy as np
import pytest

import uqdme  # noqa: F401
from uqdme_amd import _lib
from uqdme_amd.dme import DISTRIBUTIONS, legacy_draw

DISTS = ("normal", "laplace", "gamma", "bernoulli", "lognormal", "uniform")


def _want(rs, dist, n, d):
    vs = np.stack([np.asarray(DISTRIBUTIONS[dist](rs, d), np.float64) for _ in range(n)])
    return vs, np.array([np.linalg.norm(v) ** 2 for v in vs])


def _same_state(a, b):
    sa, sb = a.get_state(), b.get_state()
    return np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]


def _check(dist, shapes, threads, seed=42):
    ra, rb = np.random.RandomState(seed), np.random.RandomState(seed)
    for n, d in shapes:
        want, wn = _want(ra, dist, n, d)
        got, gn = legacy_draw(rb, dist, n, d, threads=threads)
        assert np.array_equal(got, want.astype(np.float32)), (dist, n, d)
        assert np.allclose(gn, wn, rtol=1e-12, atol=0), (dist, n, d)
        assert _same_state(ra, rb), (dist, n, d)


@pytest.fixture
def chunking():
    """Small chunks / overlap for one test, restored after (and the counters read)."""
    lib = _lib.load()
    w, m = ctypes.c_int64(), ctypes.c_int64()

    def set_(min_chunk, overlap):
        lib.uq_legacy_test_params(min_chunk, overlap, ctypes.addressof(w), ctypes.addressof(m))

    def counters():
        lib.uq_legacy_test_params(0, 0, ctypes.addressof(w), ctypes.addressof(m))
        return w.value, m.value

    yield set_, counters
    set_(1 << 21, 1 << 14)


@pytest.mark.parametrize("dist", DISTS)
def test_drivers_d2048_consecutive_calls(dist):
    # the drivers' d = 2048: n = 1, 6, 11 successive vectors, as three instances would draw them
    _check(dist, [(1, 2048), (6, 2048), (11, 2048), (1, 2048)], threads=8)


@pytest.mark.parametrize("dist", DISTS)
def test_c4_d4194304(dist):
    # C4's d = 2^22: two consecutive single-vector calls and a 2-vector one, many chunks
    _check(dist, [(1, 1 << 22), (1, 1 << 22), (2, 1 << 22)], threads=8)


@pytest.mark.parametrize("dist", ("normal", "gamma", "lognormal"))
def test_gauss_cache_carries_across_calls(dist):
    # odd sizes leave a cached gauss in the state; the next call (of any sampler) starts from it
    _check(dist, [(1, 1), (1, 3), (3, 5), (1, 1001), (2, 4097)], threads=4)


def test_threads_do_not_change_values():
    for dist in DISTS:
        a, _ = legacy_draw(np.random.RandomState(7), dist, 3, 300_001, threads=1)
        b, _ = legacy_draw(np.random.RandomState(7), dist, 3, 300_001, threads=8)
        assert np.array_equal(a, b), dist


def test_mixed_samplers_share_one_stream():
    ra, rb = np.random.RandomState(3), np.random.RandomState(3)
    for dist, d in (("normal", 5), ("laplace", 1000), ("gamma", 777), ("normal", 3), ("bernoulli", 64),
                    ("lognormal", 9), ("uniform", 11), ("gamma", 20001)):
        want, _ = _want(ra, dist, 1, d)
        got, _ = legacy_draw(rb, dist, 1, d, threads=4)
        assert np.array_equal(got, want.astype(np.float32)), dist
        assert _same_state(ra, rb), dist


@pytest.mark.parametrize("dist", DISTS)
def test_many_chunk_meetings(dist, chunking):
    set_, counters = chunking
    set_(4096, 512)                      # ~100 chunks per call: every boundary must meet
    counters()
    _check(dist, [(3, 40_000), (1, 123_457)], threads=8)
    waves, misses = counters()
    assert waves >= 2
    if dist != "gamma":
        assert misses == 0, (dist, misses)


@pytest.mark.parametrize("dist", ("normal", "gamma"))
def test_missed_meetings_still_exact(dist, chunking):
    set_, counters = chunking
    set_(2048, 2)                        # an overlap of 2 words: most meetings are missed
    counters()
    _check(dist, [(2, 30_000)], threads=8)
    _, misses = counters()
    assert misses > 0


def test_bad_arguments():
    lib = _lib.load()
    key = np.zeros(624, np.uint32)
    pos, hg, g = ctypes.c_int32(625), ctypes.c_int32(0), ctypes.c_double(0.0)
    out = np.empty(4, np.float32)
    nrm = np.empty(1, np.float64)
    args = (key.ctypes.data, ctypes.addressof(pos), ctypes.addressof(hg), ctypes.addressof(g))
    assert lib.uq_legacy_draw_f32(*args, 0, 0.0, 1.0, 1, 4, out.ctypes.data, nrm.ctypes.data, 1) == -1   # pos > 624
    pos.value = 624
    assert lib.uq_legacy_draw_f32(*args, 9, 0.0, 1.0, 1, 4, out.ctypes.data, nrm.ctypes.data, 1) == -1   # dist
    assert lib.uq_legacy_draw_f32(*args, 2, 0.5, 1.0, 1, 4, out.ctypes.data, nrm.ctypes.data, 1) == -1   # shape <= 1
    assert lib.uq_legacy_draw_f32(*args, 0, 0.0, 1.0, 1, 4, None, nrm.ctypes.data, 1) == -1
    with pytest.raises(KeyError):
        legacy_draw(np.random.RandomState(0), "no-such", 1, 4)


def test_empty_draws_leave_the_state():
    for n, d in ((0, 16), (3, 0), (0, 0)):
        rs, ref = np.random.RandomState(11), np.random.RandomState(11)
        rs.normal(size=3)
        ref.normal(size=3)                        # a cached gauss in both
        b, nrm = legacy_draw(rs, "normal", n, d, threads=4)
        assert b.shape == (n, d) and b.dtype == np.float32 and nrm.shape == (n,) and not nrm.any()
        assert _same_state(rs, ref)


def test_out_buffer_checked():
    rs = np.random.RandomState(0)
    with pytest.raises(ValueError):
        legacy_draw(rs, "normal", 2, 8, out=np.empty((2, 9), np.float32))
    with pytest.raises(ValueError):
        legacy_draw(rs, "normal", 2, 8, out=np.empty((2, 8), np.float64))
    with pytest.raises(ValueError):
        legacy_draw(rs, "normal", 2, 8, out=np.empty((8, 2), np.float32).T)
    buf = np.empty((2, 8), np.float32)
    got, _ = legacy_draw(np.random.RandomState(5), "laplace", 2, 8, out=buf)
    assert got is buf
    want, _ = _want(np.random.RandomState(5), "laplace", 2, 8)
    assert np.array_equal(buf, want.astype(np.float32))
