"""CPU: the QUIC-FL sender restatement (oracle/uq_quicfl.py, AS:429-503 and AS:814-832) against
the reference's own QuicFLSender.compress / QUICFL_quantize outputs on synthetic sender tables
(tests/golden/make_golden_quicfl_sender.py), bit for bit; and the generator pieces it relies on
against torch itself."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

from oracle import uq_eden as E
from oracle import uq_quicfl as Q

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
from quicfl_tables import sender_tables  # noqa: E402


@pytest.fixture(scope="module")
def fx():
    meta = json.load(open(os.path.join(HERE, "quicfl_sender_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_sender_vectors.npz"))
    return meta, z


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


def case_input(c, z):
    return z[f"x{c['idx']}"] if c.get("x_stored") else gen(c["kind"], c["vseed"], c["dim"])


def case_tables(meta, c):
    b = c["nbits"]
    x_len = None if c["tables"] == "pub" else meta[c["tables"]]["x_len"]
    delta = meta["data"][str(b)]["delta"] if c["tables"] == "pub" else meta[c["tables"]]["delta"]
    X, p = sender_tables(b, x_len=x_len)
    return X, p, delta, meta["data"][str(b)]["h_len"]


def test_xxh64_matches_xxhash():
    xxhash = pytest.importorskip("xxhash")
    for s in list(range(0, 200)) + [10 ** 6, 2 ** 40 + 3, -5]:
        assert Q.xxh64(str(s).encode()) == xxhash.xxh64(str(s)).intdigest()
    for n in range(0, 80):
        b = bytes(range(n))
        assert Q.xxh64(b) == xxhash.xxh64(b).intdigest()


def test_generator_state_round_trip_matches_torch():
    g = torch.Generator().manual_seed(1234)
    for pre in (0, 1, 622, 623, 624, 1000):
        g.manual_seed(1234 + pre)
        if pre:
            torch.rand(pre, generator=g)
        st = g.get_state().numpy()
        state = Q.torch_state_unpack(st)
        w, new = Q.mt_draw(state, 3001)
        g2 = torch.Generator()
        g2.set_state(torch.from_numpy(Q.torch_state_pack(st, state)))
        p = torch.rand(3001, generator=g2).numpy()
        assert np.array_equal(((w & 0xFFFFFF).astype(np.float64) * 2.0 ** -24).astype(np.float32), p)
        g3 = torch.Generator()
        g3.set_state(torch.from_numpy(Q.torch_state_pack(st, new)))
        g4 = torch.Generator()
        g4.set_state(torch.from_numpy(st))
        torch.rand(3001, generator=g4)
        assert torch.equal(torch.rand(700, generator=g3), torch.rand(700, generator=g4))


def test_oracle_matches_reference_sender(fx):
    meta, z = fx
    assert len(meta["cases"]) == 29
    done = 0
    for c in meta["cases"]:
        k = c["idx"]
        x = case_input(c, z)
        tX, tp, delta, h_len = case_tables(meta, c)
        gstate = (c["left0"], c["next0"], z[f"st0_{k}"]) if f"st0_{k}" in z.files else None
        if "error" in c:
            gstate = Q.seeded_state(c["gseed"])
            if c["pre"]:
                _, gstate = Q.mt_draw(gstate, c["pre"])
            exc = {"RuntimeError": RuntimeError, "IndexError": IndexError}[c["error"]]
            with pytest.raises(exc):
                Q.compress(x, c["nbits"], c["seed"], c["rotation_seed"], tX, tp, delta, h_len, gstate)
            continue
        msg, gst = Q.compress(x, c["nbits"], c["seed"], c["rotation_seed"], tX, tp, delta, h_len, gstate)
        assert msg["prng_seed"] == c["prng_seed"]
        assert int(np.float32(msg["scale"]).view(np.uint32)) == c["scale_bits"], k
        assert np.array_equal(msg["X"], z[f"X{k}"].astype(np.int64)), k
        assert np.array_equal(np.flatnonzero(msg["exact_indeces"]), z[f"ei{k}"]), k
        assert msg["exact_values"].view(np.uint32).tolist() == z[f"ev{k}"].view(np.uint32).tolist(), k
        assert (gst[0], gst[1]) == (c["left1"], c["next1"]) and np.array_equal(gst[2], z[f"st1_{k}"]), k
        done += 1
    assert done == 27


def test_reference_receiver_outputs_follow_from_the_message(fx):
    """The committed decompress outputs are the receiver oracle applied to the message."""
    meta, z = fx
    tabs = json.load(open(os.path.join(HERE, "quicfl_recv_vectors.json")))
    rz = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    n = 0
    for c in meta["cases"]:
        k = c["idx"]
        if "error" in c or c["tables"] != "pub" or c["D"] > 1 << 17:
            continue
        b = c["nbits"]
        mask = np.zeros(c["D"], bool)
        mask[z[f"ei{k}"]] = True
        out = E.quicfl_decompress(z[f"X{k}"], rz[f"recv{b}"], tabs["tables"][str(b)]["h_len"], c["prng_seed"], mask,
                                  z[f"ev{k}"], np.float32(np.uint32(c["scale_bits"]).view(np.float32)),
                                  c["rotation_seed"], c["dim"])
        assert out.view(np.uint32).tolist() == z[f"rx{k}"].view(np.uint32).tolist(), k
        n += 1
    assert n >= 20


def test_dropin_sequence_matches_reference(fx):
    """QUICFL_quantize (AS:814-832) twice in a row from manual_seed(g): seed draw (randint
    word % 100), compress (global generator: D bernoulli words), decompress."""
    meta, z = fx
    tabs = json.load(open(os.path.join(HERE, "quicfl_recv_vectors.json")))
    rz = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    for c in meta["dropin"]:
        j, b = c["idx"], c["nbits"]
        x = z[f"dx{j}"]
        tX, tp = sender_tables(b)
        st = Q.seeded_state(c["gseed"])
        for t in range(2):
            w, st = Q.mt_draw(st, 1)
            seed = int(w[0] % 100)
            msg, st = Q.compress(x, b, seed, 123, tX, tp, meta["data"][str(b)]["delta"], meta["data"][str(b)]["h_len"],
                                 st)
            out = E.quicfl_decompress(msg["X"], rz[f"recv{b}"], tabs["tables"][str(b)]["h_len"], msg["prng_seed"],
                                      msg["exact_indeces"], msg["exact_values"], msg["scale"], 123, c["dim"])
            assert out.view(np.uint32).tolist() == z[f"dout{j}_{t}"].view(np.uint32).tolist(), (j, t)
        assert (st[0], st[1]) == (c["left1"], c["next1"]) and np.array_equal(st[2], z[f"dst1_{j}"])


def test_large_message_sha(fx):
    meta, z = fx
    big = [c for c in meta["cases"] if c.get("rx_sha")]
    assert big and all(c["D"] == 1 << 20 for c in big)
    for c in big:
        k = c["idx"]
        assert z[f"rxs{k}"].size == 4096 and len(c["rx_sha"]) == 64
    assert hashlib  # the sha itself is checked on the GPU (tests/test_gpu_quicfl_sender.py)


@pytest.mark.parametrize("k", [1, 2])
def test_oracle_matches_reference_sender_2pow22(k):
    """Config C4's size (tests/golden/make_golden_quicfl_c4.py): the reference's messages at
    D = 2^22 (padded dim 2^22 - 5 at 1 bit; 2^22 at 2 bits, generator one block in) by SHA-256
    of X, the mask and the exact values, the scale and the generator's end state."""
    from quicfl_tables import DATA
    meta = json.load(open(os.path.join(HERE, "quicfl_c4_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_c4_vectors.npz"))
    c = meta["cases"][k]
    x = gen(c["kind"], c["vseed"], c["dim"])
    st = Q.seeded_state(c["gseed"])
    if c["pre"]:
        _, st = Q.mt_draw(st, c["pre"])
    tX, tp = sender_tables(c["nbits"])
    msg, gst = Q.compress(x, c["nbits"], c["seed"], 123, tX, tp, DATA[c["nbits"]]["delta"], DATA[c["nbits"]]["h_len"], st)
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    assert sha(msg["X"].astype(np.int64)) == c["X_sha"]
    assert sha(msg["exact_indeces"].astype(np.bool_)) == c["mask_sha"]
    assert sha(msg["exact_values"].astype(np.float32)) == c["ev_sha"]
    assert int(np.float32(msg["scale"]).view(np.uint32)) == c["scale_bits"]
    assert (gst[0], gst[1]) == (c["left1"], c["next1"]) and np.array_equal(gst[2], z[f"st1_{k}"])
