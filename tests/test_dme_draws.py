"""The NMSE harness's draw-ahead thread gives the drivers' legacy np.random stream (ND:88-95):
the batches, sum ||v||^2 and the CPU empirical mean, in the drivers' order."""
import numpy as np
import torch

import uqdme  # noqa: F401  (registers the uqdme_amd package)


def test_draw_ahead_matches_inline_draws():
    from uqdme_amd.dme import _draw_ahead, draw_vectors
    users, inst, dim = (1, 3, 2), 2, 257
    for dist in ("normal", "laplace", "gamma", "bernoulli", "lognormal"):
        rs = np.random.RandomState(42)
        want = []
        for n in users:
            for _ in range(inst):
                vecs, vns = draw_vectors(dist, n, dim, rs)
                b = np.stack([v.astype(np.float32) for v in vecs])
                want.append((b, vns, torch.from_numpy(b).sum(dim=0) / n))
        got = list(_draw_ahead(dist, users, inst, dim, np.random.RandomState(42), threads=4))
        assert len(got) == len(want)
        for (gb, gv, ge, _), (wb, wv, we) in zip(got, want):
            assert gb.dtype == torch.float32 and np.array_equal(gb.numpy(), wb)
            assert abs(gv - wv) <= 1e-13 * wv
            assert torch.equal(ge, we)


def test_draw_ahead_reports_the_state_before_each_batch():
    from uqdme_amd.dme import _draw_ahead, draw_vectors
    rs = np.random.RandomState(42)
    for x, _, _, st in _draw_ahead("gamma", (1, 2), 2, 301, np.random.RandomState(42), threads=2):
        mine = np.random.RandomState(0)
        mine.set_state(st)
        assert mine.get_state()[2:] == rs.get_state()[2:] and np.array_equal(mine.get_state()[1], rs.get_state()[1])
        vecs, _ = draw_vectors("gamma", x.shape[0], 301, rs)
        assert np.array_equal(x.numpy(), np.stack(vecs).astype(np.float32))


def test_draw_ahead_stops_early_and_raises():
    from uqdme_amd.dme import _draw_ahead
    it = _draw_ahead("normal", (1, 2), 3, 16, np.random.RandomState(0))
    next(it)
    it.close()                                    # the thread is told to stop
    bad = _draw_ahead("no-such", (1,), 1, 16, np.random.RandomState(0))
    try:
        next(bad)
    except KeyError:
        pass
    else:
        raise AssertionError("expected KeyError")


def test_parallel_client_draws_equal_the_sequential_loop():
    """The harness's torch draws per instance (ND:133-140: EDEN's seed, unbiased's X, QUIC-FL's
    seed, generator state and D skipped words per client and rate), computed client by client in
    threads from jumped starts, equal the sequential loop's values and leave the generator in the
    same state -- with a short D (jumps inside a block) and C4's padded D = 2^22 (real jumps)."""
    from concurrent.futures import ThreadPoolExecutor
    from uqdme_amd.dme import _client_draws, _client_draws_parallel
    from uqdme_amd.quicfl import generator_words
    order = ("eden", "unbiased", "biased", "quicfl")
    with ThreadPoolExecutor(4) as pool:
        for n, qD in ((5, 300), (4, 1 << 22), (1, 1 << 22), (0, 64)):
            ga, gb = torch.Generator().manual_seed(42), torch.Generator().manual_seed(42)
            torch.rand(777, generator=ga)
            torch.rand(777, generator=gb)                 # off a block edge
            want = _client_draws(ga, n, order, (1, 2), qD)
            got = _client_draws_parallel(gb, n, order, (1, 2), qD, pool)
            assert got.keys() == want.keys()
            for k in want:
                if k[0] == "quicfl":
                    assert [s for s, _ in got[k]] == [s for s, _ in want[k]], (n, qD, k)
                    assert all(np.array_equal(a, b) for (_, a), (_, b) in zip(got[k], want[k])), (n, qD, k)
                else:
                    assert got[k] == want[k], (n, qD, k)
            assert np.array_equal(generator_words(ga)[1], generator_words(gb)[1]), (n, qD)
            assert float(torch.rand(1, generator=ga)) == float(torch.rand(1, generator=gb))
