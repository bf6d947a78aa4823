"""GPU: the QUIC-FL sender (AS:429-503) and the QUICFL_quantize drop-in (AS:814-832) through the
C ABI (uq_quicfl_compress_f32), bit for bit against the reference's own outputs on synthetic
sender tables (tests/golden/make_golden_quicfl_sender.py) and against the oracle
(oracle/uq_quicfl.py) on batches; sender -> GPU receiver round trips."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

from oracle import uq_eden as E
from oracle import uq_quicfl as Q

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
from quicfl_tables import DATA, SR_BITS, data_txt, sender_tables  # noqa: E402


def gen(kind, seed, dim):
    rs = np.random.RandomState(seed)
    if kind == "normal":
        v = rs.normal(0, 1, dim)
    elif kind == "laplace":
        v = rs.laplace(1, 2, dim)
    elif kind == "zeros":
        v = np.zeros(dim)
    elif kind == "spike":
        v = rs.normal(0, 1, dim)
        v[dim // 3] = 3000.0
    return v.astype(np.float32)


@pytest.fixture(scope="module")
def fx(gpu_ready):
    meta = json.load(open(os.path.join(HERE, "quicfl_sender_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_sender_vectors.npz"))
    rmeta = json.load(open(os.path.join(HERE, "quicfl_recv_vectors.json")))
    rz = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    return meta, z, rmeta, rz


def senders(meta):
    import uqdme
    out = {}
    for tag in ("pub", "small", "oor"):
        tabs = {}
        for b in (1, 2, 3, 4):
            dd = dict(DATA[b])
            x_len = None
            if tag != "pub":
                x_len = meta[tag]["x_len"]
                dd.update(x_len=x_len, delta=meta[tag]["delta"])
            X, p = sender_tables(b, x_len=x_len)
            tabs[b] = (X, p, dd)
        out[tag] = uqdme.QuicFLSender(tables=tabs)
    return out


def set_global(gseed, pre):
    torch.manual_seed(gseed)
    if pre:
        torch.rand(pre)


def state_words():
    import uqdme_amd.quicfl as q
    return q.generator_words(torch.default_generator)[1]


def test_sender_matches_reference(fx):
    import uqdme
    meta, z, rmeta, rz = fx
    snd = senders(meta)
    rx = uqdme.QuicFLReceiver(tables={b: rz[f"recv{b}"] for b in (1, 2, 3, 4)})
    checked = 0
    for c in meta["cases"]:
        k = c["idx"]
        x = z[f"x{k}"] if c.get("x_stored") else gen(c["kind"], c["vseed"], c["dim"])
        set_global(c["gseed"], c["pre"])
        before = state_words()
        data = {"vec": torch.from_numpy(x), "seed": c["seed"], "nbits": c["nbits"], "rotation_seed": c["rotation_seed"]}
        if "error" in c:
            exc = {"RuntimeError": RuntimeError, "IndexError": IndexError}[c["error"]]
            with pytest.raises(exc):
                snd[c["tables"]].compress(data)
            assert np.array_equal(state_words(), before), k          # nothing drawn: the reference raised first
            continue
        msg = snd[c["tables"]].compress(data)
        assert msg["prng_seed"] == c["prng_seed"] and msg["dim"] == c["dim"] and msg["h_len"] == c["h_len"]
        assert msg["X"].dtype == torch.int64 and msg["X"].is_cuda
        assert np.array_equal(msg["X"].cpu().numpy(), z[f"X{k}"].astype(np.int64)), k
        assert msg["exact_indeces"].dtype == torch.bool
        assert np.array_equal(np.flatnonzero(msg["exact_indeces"].cpu().numpy()), z[f"ei{k}"]), k
        assert msg["exact_values"].cpu().numpy().view(np.uint32).tolist() == z[f"ev{k}"].view(np.uint32).tolist(), k
        assert msg["scale"].dim() == 0 and int(msg["scale"].cpu().numpy().view(np.uint32)) == c["scale_bits"], k
        after = state_words()
        assert (after[0], after[1]) == (c["left1"], c["next1"]) and np.array_equal(after[2:], z[f"st1_{k}"]), k
        if c["tables"] == "pub":                                    # sender -> GPU receiver
            out = rx.decompress(msg).cpu().numpy()
            if f"rx{k}" in z.files:
                assert out.view(np.uint32).tolist() == z[f"rx{k}"].view(np.uint32).tolist(), k
            else:
                assert hashlib.sha256(out.tobytes()).hexdigest() == c["rx_sha"], k
                assert np.array_equal(out[z[f"rxpos{k}"]].view(np.uint32), z[f"rxs{k}"].view(np.uint32))
        checked += 1
    assert checked == 27


def test_dropin_matches_reference(fx, tmp_path):
    """QUICFL_quantize twice in a row from manual_seed(g), the tables under a prefix as the
    reference reads them (sender tables synthetic, receiver tables the reference's)."""
    import uqdme
    meta, z, rmeta, rz = fx
    for b in (1, 2, 3, 4):
        fn = str(tmp_path / f"{b}_X_{SR_BITS[b]}_h_256_q_")
        X, p = sender_tables(b)
        torch.save(torch.from_numpy(X), fn + "sender_table_X.pt")
        torch.save(torch.from_numpy(p), fn + "sender_table_p.pt")
        torch.save(torch.from_numpy(rz[f"recv{b}"]), fn + "recv_table.pt")
        open(fn + "data.txt", "w").write(data_txt(b))
    uqdme.set_tables_prefix(str(tmp_path))
    try:
        for c in meta["dropin"]:
            j = c["idx"]
            torch.manual_seed(c["gseed"])
            for t in range(2):
                out = uqdme.QUICFL_quantize(z[f"dx{j}"], c["nbits"])
                assert isinstance(out, np.ndarray) and out.dtype == np.float32 and out.shape == (c["dim"],)
                assert out.view(np.uint32).tolist() == z[f"dout{j}_{t}"].view(np.uint32).tolist(), (j, t)
            w = state_words()
            assert (w[0], w[1]) == (c["left1"], c["next1"]) and np.array_equal(w[2:], z[f"dst1_{j}"])
    finally:
        uqdme.set_tables_prefix(None)


def test_missing_tables_raise_like_the_reference(tmp_path):
    import uqdme
    with pytest.raises(FileNotFoundError):
        uqdme.QuicFLSender(prefix=str(tmp_path) + "/")


def _oracle_row(x, nbits, seed, rot, tX, tp, dd, gstate):
    return Q.compress(x, nbits, seed, rot, tX, tp, dd["delta"], dd["h_len"], gstate)


@pytest.mark.parametrize("nbits,n,dim", [(1, 6, 3000), (2, 3, 1 << 14), (4, 5, 4096), (3, 2, 70000)])
def test_batch_matches_oracle(fx, nbits, n, dim):
    """quicfl_compress over n rows (seeded generators per row for the bernoulli(p_X) draws),
    uint8 X; and the batch receiver on its messages vs the receiver oracle."""
    import uqdme
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    rng = np.random.default_rng(nbits * 100 + n)
    x = (rng.standard_normal((n, dim)) * rng.uniform(0.5, 3, (n, 1))).astype(np.float32)
    seeds = [int(s) for s in rng.integers(0, 100, n)]
    rots = [int(s) for s in rng.integers(0, 200, n)]
    pxs = [int(s) for s in rng.integers(0, 2 ** 31, n)]
    msg = uqdme.quicfl_compress(torch.from_numpy(x), nbits, seeds, rots, sender=snd, px_seeds=pxs)
    assert msg.X.dtype == torch.uint8
    tX, tp = sender_tables(nbits)
    out = uqdme.quicfl_decompress_messages(msg, rz[f"recv{nbits}"]).cpu().numpy()
    for j in range(n):
        exp, _ = _oracle_row(x[j], nbits, seeds[j], rots[j], tX, tp, DATA[nbits], Q.seeded_state(pxs[j]))
        assert np.array_equal(msg.X[j].cpu().numpy().astype(np.int64), exp["X"]), j
        assert np.array_equal(msg.exact_mask[j].cpu().numpy(), exp["exact_indeces"]), j
        cnt = int(msg.exact_count[j])
        assert msg.exact_vals[j, :cnt].cpu().numpy().view(np.uint32).tolist() == exp["exact_values"].view(np.uint32).tolist()
        assert np.float32(msg.scale[j].item()).view(np.uint32) == np.float32(exp["scale"]).view(np.uint32)
        rec = E.quicfl_decompress(exp["X"], rz[f"recv{nbits}"], rmeta["tables"][str(nbits)]["h_len"], exp["prng_seed"],
                                  exp["exact_indeces"], exp["exact_values"], exp["scale"], rots[j], dim)
        assert out[j].view(np.uint32).tolist() == rec.view(np.uint32).tolist(), j


def test_batch_states_and_many_messages(fx):
    """px_states from generators at arbitrary positions (left/next off the block edge), and a
    batch above 256 messages (the sequential-chain norm instead of the segmented one)."""
    import uqdme
    import uqdme_amd.quicfl as q
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    n, dim, nbits = 300, 16384, 2
    rng = np.random.default_rng(7)
    x = rng.laplace(1, 2, (n, dim)).astype(np.float32)
    seeds = [int(s) for s in rng.integers(0, 10 ** 6, n)]
    states = np.empty((n, 626), np.uint32)
    g = torch.Generator()
    for j in range(n):
        g.manual_seed(int(j * 7919 + 1))
        pre = int(rng.integers(0, 2000))
        if pre:
            torch.rand(pre, generator=g)
        states[j] = q.generator_words(g)[1]
    msg, new = q.quicfl_compress(torch.from_numpy(x), nbits, seeds, [123] * n, sender=snd, px_states=states,
                                 _state_out=True)
    # the first 20 messages again as a few-message call (the jump path: every run's generator
    # blocks by jump-ahead, KQ0j): the same bits and end states as the batch's one-wave-per-
    # message kernel
    few, fnew = q.quicfl_compress(torch.from_numpy(x[:20]), nbits, seeds[:20], [123] * 20, sender=snd,
                                  px_states=states[:20], _state_out=True)
    assert torch.equal(few.X, msg.X[:20]) and torch.equal(few.exact_mask, msg.exact_mask[:20])
    assert torch.equal(few.scale, msg.scale[:20]) and torch.equal(few.exact_count, msg.exact_count[:20])
    for j in range(20):
        cnt = int(few.exact_count[j])
        assert torch.equal(few.exact_vals[j, :cnt], msg.exact_vals[j, :cnt]), j
    assert np.array_equal(fnew, new[:20])
    # and through the team kernel (scouts + runs, test hook 4): the same again
    from uqdme_amd._lib import load
    prev = load().uq_test_set_quicfl_hooks(4)
    try:
        team, tnew = q.quicfl_compress(torch.from_numpy(x[:20]), nbits, seeds[:20], [123] * 20, sender=snd,
                                       px_states=states[:20], _state_out=True)
    finally:
        load().uq_test_set_quicfl_hooks(prev)
    assert torch.equal(team.X, few.X) and torch.equal(team.exact_count, few.exact_count) and np.array_equal(tnew, fnew)
    for j in range(20):
        cnt = int(few.exact_count[j])
        assert torch.equal(team.exact_vals[j, :cnt], few.exact_vals[j, :cnt]), j
    tX, tp = sender_tables(nbits)
    for j in list(range(0, n, 37)) + [n - 1]:
        st = (int(states[j, 0]), int(states[j, 1]), states[j, 2:])
        exp, gst = _oracle_row(x[j], nbits, seeds[j], 123, tX, tp, DATA[nbits], st)
        assert np.array_equal(msg.X[j].cpu().numpy().astype(np.int64), exp["X"]), j
        assert np.float32(msg.scale[j].item()).view(np.uint32) == np.float32(exp["scale"]).view(np.uint32), j
        assert (new[j, 0], new[j, 1]) == (gst[0], gst[1]) and np.array_equal(new[j, 2:], gst[2]), j


@pytest.mark.parametrize("hooks", [0, 2, 4])
def test_fused_quantize_equals_compress_then_decompress(fx, hooks):
    """quicfl_quantize (uq_quicfl_quantize_f32: the receiver fused into the sender's stage 2 with
    the sender's own h, AS:526-532) gives the bits of compress -> decompress and the same end
    generator states, through the jump path (hooks 0: KQ0j + KQ1j), the one-wave kernels
    (hooks 2) and the team kernels (hooks 4)."""
    import uqdme
    import uqdme_amd.quicfl as q
    from uqdme_amd._lib import load
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    rng = np.random.default_rng(40 + hooks)
    prev = load().uq_test_set_quicfl_hooks(hooks)
    try:
        for nbits, n, dim in ((1, 3, 20000), (2, 2, 4099), (4, 1, 1 << 16), (3, 4, 700)):
            x = (rng.standard_normal((n, dim)) * 2).astype(np.float32)
            x[0, 5] = 500.0                                          # exact coordinates too
            seeds = [int(s) for s in rng.integers(0, 100, n)]
            rots = [int(s) for s in rng.integers(0, 100, n)]
            g = torch.Generator()
            states = []
            for j in range(n):
                g.manual_seed(1000 + j)
                torch.rand(int(rng.integers(0, 700)), generator=g)
                states.append(q.generator_words(g)[1])
            states = np.stack(states)
            msg, new = q.quicfl_compress(torch.from_numpy(x), nbits, seeds, rots, sender=snd, px_states=states,
                                         x_dtype=torch.int64, _state_out=True)
            ref = uqdme.quicfl_decompress_messages(msg, rz[f"recv{nbits}"]).cpu().numpy()
            out, fnew, sc = uqdme.quicfl_quantize(torch.from_numpy(x), nbits, seeds, rots, sender=snd,
                                                  recv_table=rz[f"recv{nbits}"], px_states=states)
            assert out.cpu().numpy().view(np.uint32).tolist() == ref.view(np.uint32).tolist(), (nbits, n, dim)
            assert np.array_equal(fnew, new) and torch.equal(sc, msg.scale)
    finally:
        load().uq_test_set_quicfl_hooks(prev)


def test_fused_receiver_index_error_after_sender(fx, tmp_path):
    """A receiver table too short for X * h_len + h: the reference's receiver raises IndexError
    after its sender returned (the global generator advanced by the sender's draws); the fused
    drop-in raises the same and leaves the generator where the reference does."""
    import uqdme
    meta, z, rmeta, rz = fx
    for b in (1, 2, 3, 4):
        fn = str(tmp_path / f"{b}_X_{SR_BITS[b]}_h_256_q_")
        X, p = sender_tables(b)
        torch.save(torch.from_numpy(X), fn + "sender_table_X.pt")
        torch.save(torch.from_numpy(p), fn + "sender_table_p.pt")
        torch.save(torch.from_numpy(rz[f"recv{b}"][:1]), fn + "recv_table.pt")    # one row only
        open(fn + "data.txt", "w").write(data_txt(b))
    uqdme.set_tables_prefix(str(tmp_path))
    try:
        x = np.random.default_rng(3).standard_normal(5000).astype(np.float32)
        torch.manual_seed(77)
        snd = uqdme.QuicFLSender(prefix=str(tmp_path) + "/")
        data = {"vec": torch.from_numpy(x), "seed": int(torch.randint(0, 100, (1,)).item()), "nbits": 2,
                "rotation_seed": 123}
        snd.compress(data)                                   # what the reference's sender draws
        expect = state_words()
        torch.manual_seed(77)
        with pytest.raises(IndexError):
            uqdme.QUICFL_quantize(x, 2)
        assert np.array_equal(state_words(), expect)
    finally:
        uqdme.set_tables_prefix(None)


def test_packed_table_same_bits(fx, monkeypatch):
    """The sender's 4-byte packed table ((X << 25) | ceil(p * 2^24): one gather per coordinate)
    and the (X, p) pairs give the same messages and end states, in batches (one wave per
    message) and few-message calls (team kernels); a table with a non-integer X is not packed."""
    import uqdme
    import uqdme_amd.quicfl as q
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    rng = np.random.default_rng(21)
    for n, dim, nbits in ((300, 4096, 1), (3, 1 << 16, 2), (2, 20000, 4)):
        x = rng.standard_normal((n, dim)).astype(np.float32)
        seeds = [int(s) for s in rng.integers(0, 100, n)]
        pxs = [int(s) for s in rng.integers(0, 2 ** 31, n)]
        res = []
        for packed in (True, False):
            monkeypatch.setattr(q, "_USE_PACKED", packed)
            m = q.quicfl_compress(torch.from_numpy(x), nbits, seeds, [123] * n, sender=snd, px_seeds=pxs)
            res.append(m)
        assert snd.table_packed(nbits, torch.device("cuda", 0)) is not None
        a, b = res
        assert torch.equal(a.X, b.X) and torch.equal(a.exact_mask, b.exact_mask) and torch.equal(a.scale, b.scale)
        assert torch.equal(a.exact_count, b.exact_count)
    tX, tp = sender_tables(1)
    tX = tX.copy()
    tX[0, 0] = 0.5
    odd = uqdme.QuicFLSender(tables={1: (tX, tp, DATA[1])})
    assert odd.table_packed(1, torch.device("cuda", 0)) is None


@pytest.mark.parametrize("n,dim", [(1, 4096), (1, 5000), (3, 9000), (17, 1 << 15), (128, 1 << 14), (2, (1 << 21) + 7),
                                   (1, 3 << 18), (5, 1 << 20), (300, 1 << 16), (342, 1 << 18)])
def test_jump_path_equals_one_wave_across_shapes(fx, n, dim):
    """The jump path (its run count and length come from a cost model of (n, D), so every shape
    cuts the streams differently) against the one-wave kernel (test hook 2) on the same
    messages: X, mask, exact values, scales, generator end states; px states off the block
    edge and fresh px seeds.  (300, 2^16): 3 runs per message past the team kernel's 256;
    (342, 2^18): 5 runs, 1710 run waves, the two-waves-per-SIMD runs kernel."""
    import uqdme_amd.quicfl as q
    from uqdme_amd._lib import load
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    rng = np.random.default_rng(n * 1000 + dim % 997)
    x = (rng.standard_normal((n, dim)) * rng.uniform(0.5, 4, (n, 1))).astype(np.float32)
    x[0, 1] = 1e4                                                 # an exact coordinate at least
    seeds = [int(s) for s in rng.integers(0, 100, n)]
    rots = [int(s) for s in rng.integers(0, 100, n)]
    g = torch.Generator()
    states = np.empty((n, 626), np.uint32)
    for j in range(n):
        g.manual_seed(int(rng.integers(0, 2 ** 31)))
        pre = int(rng.integers(0, 1300))
        if pre:
            torch.rand(pre, generator=g)
        states[j] = q.generator_words(g)[1]
    for nbits in (1, 3):
        for kw in ({"px_states": states}, {"px_seeds": [int(s) for s in rng.integers(0, 2 ** 31, n)]}):
            out = {}
            for hooks in (0, 2):
                prev = load().uq_test_set_quicfl_hooks(hooks)
                try:
                    out[hooks] = q.quicfl_compress(torch.from_numpy(x), nbits, seeds, rots, sender=snd,
                                                   _state_out=True, **kw)
                finally:
                    load().uq_test_set_quicfl_hooks(prev)
            (a, sa), (b, sb) = out[0], out[2]
            assert torch.equal(a.X, b.X) and torch.equal(a.exact_mask, b.exact_mask), (nbits, kw.keys())
            assert torch.equal(a.exact_count, b.exact_count) and torch.equal(a.scale, b.scale)
            for j in range(n):
                c = int(a.exact_count[j])
                assert torch.equal(a.exact_vals[j, :c], b.exact_vals[j, :c]), j
            assert (sa is None and sb is None) or np.array_equal(sa, sb)


def test_two_runs_per_message_at_900_messages(fx):
    """900 messages of 2^18: the cost model takes the jump path with two runs per message (1800
    run waves, two per SIMD: the lean KQ1j) for the sender and the receiver; X, mask, exact
    values, scales and the decompressed batch equal the one-wave kernels' (test hook 2) on the
    same messages, from GPU-resident input; the fused quantize (the receiver inside the
    two-wave runs) equals compress -> decompress."""
    import uqdme_amd.quicfl as q
    from uqdme_amd._lib import load
    meta, z, rmeta, rz = fx
    snd = senders(meta)["pub"]
    n, dim, nbits = 900, 1 << 18, 1
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(n, dim, generator=g, device="cuda") * 2.0
    x[0, 1] = 1e4
    seeds = list(range(n))
    rots = [int(s) for s in np.random.default_rng(9).integers(0, 100, n)]
    pxs = list(range(5000, 5000 + n))
    rt = rz[f"recv{nbits}"]
    out = {}
    for hooks in (0, 2):
        prev = load().uq_test_set_quicfl_hooks(hooks)
        try:
            m = q.quicfl_compress(x, nbits, seeds, rots, sender=snd, px_seeds=pxs)
            out[hooks] = (m, q.quicfl_decompress_messages(m, rt))
        finally:
            load().uq_test_set_quicfl_hooks(prev)
    (a, da), (b, db) = out[0], out[2]
    assert torch.equal(a.X, b.X) and torch.equal(a.exact_mask, b.exact_mask)
    assert torch.equal(a.exact_count, b.exact_count) and torch.equal(a.scale, b.scale)
    assert torch.equal(a.exact_dense(), b.exact_dense())
    assert torch.equal(da.view(torch.int32), db.view(torch.int32))
    # the receiver fused into the two-wave runs (QUICFL_quantize's path) gives the same batch
    fo, _, fsc = q.quicfl_quantize(x, nbits, seeds, rots, sender=snd, recv_table=rt, px_seeds=pxs)
    assert torch.equal(fo.view(torch.int32), da.view(torch.int32)) and torch.equal(fsc, a.scale)
