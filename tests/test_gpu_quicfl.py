"""GPU: the QUIC-FL receiver (AS:507-535) against the reference's QuicFLReceiver.decompress
outputs (tests/golden/make_golden_quicfl.py) and the oracle, bit for bit, through the C ABI
(uq_quicfl_receive_f32 + uq_rht_f32)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import uq_eden as E

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def fx(gpu_ready):
    meta = json.load(open(os.path.join(HERE, "quicfl_recv_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    return meta, z


def test_receiver_matches_reference(fx):
    import uqdme
    meta, z = fx
    rx = uqdme.QuicFLReceiver(tables={b: z[f"recv{b}"] for b in (1, 2, 3, 4)})
    for c in meta["cases"]:
        i = c["idx"]
        mask = torch.from_numpy(z[f"mask{i}"])
        msg = {"X": torch.from_numpy(z[f"X{i}"].astype(np.int64)), "exact_values": torch.from_numpy(z[f"vals{i}"]),
               "exact_indeces": mask, "prng_seed": c["prng_seed"], "rotation_seed": c["rotation_seed"],
               "dim": c["dim"], "scale": torch.tensor(c["scale"], dtype=torch.float32), "nbits": c["nbits"],
               "h_len": c["h_len"]}
        out = rx.decompress(msg).cpu().numpy()
        assert out.shape == (c["dim"],)
        assert out.view(np.uint32).tolist() == z[f"out{i}"].view(np.uint32).tolist(), i


def test_batched_receiver_matches_oracle(fx):
    import uqdme
    meta, z = fx
    rng = np.random.default_rng(5)
    nbits, n, dim = 2, 6, 3000
    D = 4096
    tab = z[f"recv{nbits}"]
    X = rng.integers(0, 1 << nbits, size=(n, D))
    mask = rng.random((n, D)) < 0.01
    vals = np.where(mask, rng.standard_normal((n, D)) * 4, 0).astype(np.float32)
    ps = rng.integers(0, 1 << 16, size=n)
    rs = rng.integers(0, 100, size=n)
    sc = (rng.random(n) * 3 + 0.5).astype(np.float32)
    out = uqdme.quicfl_decompress(torch.from_numpy(X), nbits, ps, rs, sc, dim, tab, tab.shape[1],
                                  torch.from_numpy(mask), torch.from_numpy(vals)).cpu().numpy()
    for j in range(n):
        exp = E.quicfl_decompress(X[j], tab, tab.shape[1], int(ps[j]), mask[j], vals[j][mask[j]], sc[j], int(rs[j]), dim)
        assert out[j].view(np.uint32).tolist() == exp.view(np.uint32).tolist(), j
    with pytest.raises(IndexError):
        uqdme.quicfl_decompress(torch.full((1, D), 1 << nbits), nbits, [1], [1], [1.0], dim, tab)


def test_receiver_x_kinds_layouts_and_errors(fx):
    """uq_quicfl_receive_f32: X read in place as int64 / uint8 / int32; exact values dense or
    compact (index order, quicfl_compress's layout); the take index -numel <= i < numel with
    negatives wrapping (AS:530) -- all bit-equal to the oracle; a compact row whose count
    disagrees with its mask raises like AS:531, an index past the table raises IndexError."""
    import uqdme
    meta, z = fx
    rng = np.random.default_rng(11)
    nbits, n, dim, D = 3, 5, 5000, 8192
    tab = z[f"recv{nbits}"]
    rows = tab.shape[0]
    X = rng.integers(0, rows, size=(n, D))
    X[1, :50] = -1                                   # -h_len + h: wraps to the last row (take semantics)
    X[2, 7] = -rows                                  # the lowest index take accepts
    mask = rng.random((n, D)) < 0.004
    mask[3] = False                                  # a row without exact coordinates
    dense = np.where(mask, rng.standard_normal((n, D)) * 5, 0).astype(np.float32)
    compact = np.zeros((n, D), np.float32)
    cnt = mask.sum(1)
    for j in range(n):
        compact[j, :cnt[j]] = dense[j][mask[j]]
    ps = rng.integers(0, 1 << 16, size=n)
    rs = rng.integers(0, 100, size=n)
    sc = (rng.random(n) * 3 + 0.5).astype(np.float32)
    exp = [E.quicfl_decompress(X[j], tab, tab.shape[1], int(ps[j]), mask[j], dense[j][mask[j]], sc[j], int(rs[j]), dim)
           for j in range(n)]
    md = torch.from_numpy(mask).cuda()
    for dt in (torch.int64, torch.int32):
        Xd = torch.from_numpy(X).to(dt).cuda()
        for vals, c in ((dense, None), (compact, cnt)):
            out = uqdme.quicfl_decompress(Xd, nbits, ps, rs, sc, dim, tab, tab.shape[1], md, torch.from_numpy(vals).cuda(),
                                          c).cpu().numpy()
            for j in range(n):
                assert out[j].view(np.uint32).tolist() == exp[j].view(np.uint32).tolist(), (dt, c is None, j)
    Xu = np.where(X < 0, 0, X)                        # uint8 rows: the non-negative part
    exp_u = E.quicfl_decompress(Xu[0], tab, tab.shape[1], int(ps[0]), mask[0], dense[0][mask[0]], sc[0], int(rs[0]), dim)
    out = uqdme.quicfl_decompress(torch.from_numpy(Xu[:1]).to(torch.uint8).cuda(), nbits, ps[:1], rs[:1], sc[:1], dim, tab,
                                  None, md[:1], torch.from_numpy(compact[:1]).cuda(), cnt[:1]).cpu().numpy()
    assert out[0].view(np.uint32).tolist() == exp_u.view(np.uint32).tolist()
    bad = cnt.copy()
    bad[4] += 1
    with pytest.raises(RuntimeError):
        uqdme.quicfl_decompress(torch.from_numpy(X).cuda(), nbits, ps, rs, sc, dim, tab, None, md,
                                torch.from_numpy(compact).cuda(), bad)
    Xb = X.copy()
    Xb[0, 3] = -rows - 1                             # below -numel for every h
    with pytest.raises(IndexError):
        uqdme.quicfl_decompress(torch.from_numpy(Xb).cuda(), nbits, ps, rs, sc, dim, tab)


def test_receiver_team_equals_wave(fx):
    """A few messages (one workgroup each: the h stream's scout hands the runs their first
    blocks; compact slots start after the earlier runs' exact coordinates) give the bits the
    batch kernel (one wave per message) gives, for every X kind and both exact layouts."""
    import uqdme
    meta, z = fx
    rng = np.random.default_rng(21)
    nbits, n, D = 2, 70, 1 << 15
    tab = z[f"recv{nbits}"]
    X = rng.integers(0, tab.shape[0], size=(n, D))
    mask = rng.random((n, D)) < 0.004
    dense = np.where(mask, rng.standard_normal((n, D)), 0).astype(np.float32)
    compact = np.zeros((n, D), np.float32)
    cnt = mask.sum(1)
    for j in range(n):
        compact[j, :cnt[j]] = dense[j][mask[j]]
    ps = rng.integers(0, 1 << 16, size=n)
    rs = rng.integers(0, 100, size=n)
    sc = (rng.random(n) * 3 + 0.5).astype(np.float32)
    md = torch.from_numpy(mask).cuda()
    for dt in (torch.uint8, torch.int32, torch.int64):
        Xd = torch.from_numpy(X).to(dt).cuda()
        for vals, c in ((dense, None), (compact, cnt)):
            vd = torch.from_numpy(vals).cuda()
            full = uqdme.quicfl_decompress(Xd, nbits, ps, rs, sc, D, tab, None, md, vd, c)
            few = uqdme.quicfl_decompress(Xd[:5], nbits, ps[:5], rs[:5], sc[:5], D, tab, None, md[:5], vd[:5],
                                          None if c is None else c[:5])
            assert torch.equal(full[:5].view(torch.int32), few.view(torch.int32)), (dt, c is None)
    exp = E.quicfl_decompress(X[3], tab, tab.shape[1], int(ps[3]), mask[3], dense[3][mask[3]], sc[3], int(rs[3]), D)
    assert few[3].cpu().numpy().view(np.uint32).tolist() == exp.view(np.uint32).tolist()


@pytest.mark.parametrize("n,D", [(3, 1 << 16), (3, 1 << 20), (300, 1 << 16), (342, 1 << 18)])
def test_receiver_jump_equals_team_and_wave(fx, n, D):
    """A few messages of 2^16 / 2^20 coordinates take the receiver's jump path (KQ0s + KQ0j on
    the h stream, every run at once, compact slots from KQ2c's counts): the same bits as the
    team kernel (test hook 4) and the one-wave kernel (hook 2), both exact layouts, and the
    oracle on one message.  300 messages: the jump path past the team kernel's 256 (hook 4
    falls back to the one-wave kernel there); 342 x 2^18: 5 runs per message, 1710 run waves,
    two per SIMD."""
    import uqdme
    from uqdme_amd._lib import load
    meta, z = fx
    rng = np.random.default_rng(D % 977 + n)
    nbits = 1
    tab = z[f"recv{nbits}"]
    X = rng.integers(0, tab.shape[0], size=(n, D))
    mask = rng.random((n, D)) < 0.004
    dense = np.where(mask, rng.standard_normal((n, D)), 0).astype(np.float32)
    compact = np.zeros((n, D), np.float32)
    cnt = mask.sum(1)
    for j in range(n):
        compact[j, :cnt[j]] = dense[j][mask[j]]
    ps = rng.integers(0, 1 << 16, size=n)
    rs = rng.integers(0, 100, size=n)
    sc = (rng.random(n) * 3 + 0.5).astype(np.float32)
    md = torch.from_numpy(mask).cuda()
    Xd = torch.from_numpy(X).to(torch.uint8).cuda()
    outs = {}
    for hooks in (0, 2, 4):
        prev = load().uq_test_set_quicfl_hooks(hooks)
        try:
            for vals, c in ((dense, None), (compact, cnt)):
                outs[(hooks, c is None)] = uqdme.quicfl_decompress(Xd, nbits, ps, rs, sc, D, tab, None, md,
                                                                   torch.from_numpy(vals).cuda(), c)
        finally:
            load().uq_test_set_quicfl_hooks(prev)
    for k, v in outs.items():
        assert torch.equal(v.view(torch.int32), outs[(0, True)].view(torch.int32)), k
    exp = E.quicfl_decompress(X[1], tab, tab.shape[1], int(ps[1]), mask[1], dense[1][mask[1]], sc[1], int(rs[1]), D)
    assert outs[(0, False)][1].cpu().numpy().view(np.uint32).tolist() == exp.view(np.uint32).tolist()
    # a wrong exact count is still reported (the jump path's KQ2f)
    bad = cnt.copy()
    bad[2] += 1
    with pytest.raises(RuntimeError, match="shape mismatch"):
        uqdme.quicfl_decompress(Xd, nbits, ps, rs, sc, D, tab, None, md, torch.from_numpy(compact).cuda(), bad)


def test_timeout_flag_raises_in_sender_and_receiver(fx):
    """A run of a team kernel whose wait ran out (UQ_QFL_TIMEOUT, forced through the test hook
    uq_test_set_quicfl_hooks) never writes its coordinates: the sender, the receiver and the
    drop-in's deferred check all raise instead of returning them."""
    import sys
    import uqdme
    from uqdme_amd import quicfl as q
    from uqdme_amd._lib import load
    sys.path.insert(0, HERE)
    from quicfl_tables import DATA, sender_tables
    meta, z = fx
    snd = uqdme.QuicFLSender(tables={1: (*sender_tables(1), DATA[1])})
    rx = uqdme.QuicFLReceiver(tables={1: z["recv1"]})
    x = torch.randn(1, 1 << 14)
    msg = q.quicfl_compress(x, 1, [3], [123], sender=snd, px_seeds=[5])
    assert load().uq_test_set_quicfl_hooks(1) == 0
    try:
        with pytest.raises(RuntimeError, match="wait ran out"):
            q.quicfl_compress(x, 1, [3], [123], sender=snd, px_seeds=[5])
        with pytest.raises(RuntimeError, match="wait ran out"):
            q.quicfl_decompress_messages(msg, z["recv1"])
        d = {"X": msg.X[0].long(), "exact_values": msg.exact_vals[0, :int(msg.exact_count[0])],
             "exact_indeces": msg.exact_mask[0], "prng_seed": int(msg.prng_seeds[0]), "rotation_seed": 123,
             "dim": 1 << 14, "scale": msg.scale[0], "nbits": 1, "h_len": msg.h_len}
        with pytest.raises(RuntimeError, match="wait ran out"):
            rx.decompress(d)
        _, info = rx.decompress(d, _defer_check=True)
        with pytest.raises(RuntimeError, match="wait ran out"):
            q._raise_recv_flags(int(info.cpu()[0]))
    finally:
        assert load().uq_test_set_quicfl_hooks(0) == 1
    rx.decompress(d)                                   # hook off: the same message decodes


def test_receiver_broadcasts_one_exact_value(fx):
    """AS:531 vec[exact_indeces] = exact_values with a one-element exact_values broadcasts it
    over every masked coordinate (and over none): the dict receiver accepts it like the
    reference (vs the receiver oracle, whose numpy assignment broadcasts the same way)."""
    import uqdme
    meta, z = fx
    rng = np.random.default_rng(11)
    tab = z["recv2"]
    rx = uqdme.QuicFLReceiver(tables={2: tab})
    D, dim = 8192, 8000
    X = rng.integers(0, 4, size=D)
    for nmask in (0, 1, 37):
        mask = np.zeros(D, bool)
        mask[rng.choice(D, nmask, replace=False)] = True
        val = np.array([2.75], np.float32)
        msg = {"X": torch.from_numpy(X), "exact_values": torch.from_numpy(val), "exact_indeces": torch.from_numpy(mask),
               "prng_seed": 4242, "rotation_seed": 17, "dim": dim, "scale": torch.tensor(1.5, dtype=torch.float32),
               "nbits": 2, "h_len": tab.shape[1]}
        out = rx.decompress(msg).cpu().numpy()
        exp = E.quicfl_decompress(X, tab, tab.shape[1], 4242, mask, val, np.float32(1.5), 17, dim)
        assert out.view(np.uint32).tolist() == exp.view(np.uint32).tolist(), nmask
