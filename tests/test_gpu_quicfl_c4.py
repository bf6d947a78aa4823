"""GPU: QUIC-FL at config C4's size, D = 2^22 (AS:429-535, AS:814-832), bit for bit against the
reference's own sender, receiver and drop-in run on the synthetic sender tables
(tests/golden/make_golden_quicfl_c4.py): dim = 2^22 and 2^22 - 5 (padded), 1 and 2 bits,
through the few-message paths (the sender's jump path KQ0j + KQ1j, the receiver's team kernel
KQ2t) and, by the test hooks, the one-wave kernels (KQ1 / KQ2) and the sender's team kernel KQ1t -- X, mask, exact values, scale, the global generator's end state and the
receiver's output; QUICFL_quantize at 2^22 through the fused receiver."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
from quicfl_tables import DATA, SR_BITS, data_txt, sender_tables  # noqa: E402


def gen(kind, seed, dim):
    rs = np.random.RandomState(seed)
    v = rs.normal(0, 1, dim) if kind == "normal" else rs.laplace(1, 2, dim)
    return v.astype(np.float32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def fx(gpu_ready):
    meta = json.load(open(os.path.join(HERE, "quicfl_c4_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_c4_vectors.npz"))
    rz = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    return meta, z, rz


def state_words():
    import uqdme_amd.quicfl as q
    return q.generator_words(torch.default_generator)[1]


@pytest.mark.parametrize("hooks", [0, 2, 4])
def test_sender_receiver_2pow22_vs_reference(fx, hooks):
    import uqdme
    from uqdme_amd._lib import load
    meta, z, rz = fx
    snd = uqdme.QuicFLSender(tables={b: (*sender_tables(b), DATA[b]) for b in (1, 2, 3, 4)})
    rx = uqdme.QuicFLReceiver(tables={b: rz[f"recv{b}"] for b in (1, 2, 3, 4)})
    prev = load().uq_test_set_quicfl_hooks(hooks)
    try:
        for c in meta["cases"]:
            k = c["idx"]
            x = gen(c["kind"], c["vseed"], c["dim"])
            torch.manual_seed(c["gseed"])
            if c["pre"]:
                torch.rand(c["pre"])
            msg = snd.compress({"vec": torch.from_numpy(x), "seed": c["seed"], "nbits": c["nbits"], "rotation_seed": 123})
            X = msg["X"].cpu().numpy()
            mask = msg["exact_indeces"].cpu().numpy()
            ev = msg["exact_values"].cpu().numpy()
            pos = z[f"pos{k}"]
            assert np.array_equal(X[pos], z[f"Xs{k}"].astype(np.int64)), k
            assert np.array_equal(mask[pos], z[f"ms{k}"]), k
            assert sha(X.astype(np.int64)) == c["X_sha"] and sha(mask.astype(np.bool_)) == c["mask_sha"], k
            assert ev.size == c["n_exact"] and sha(ev) == c["ev_sha"], k
            assert int(msg["scale"].cpu().numpy().view(np.uint32)) == c["scale_bits"], k
            w = state_words()
            assert (w[0], w[1]) == (c["left1"], c["next1"]) and np.array_equal(w[2:], z[f"st1_{k}"]), k
            out = rx.decompress(msg).cpu().numpy()
            assert np.array_equal(out[z[f"opos{k}"]].view(np.uint32), z[f"rxs{k}"].view(np.uint32)), k
            assert sha(out) == c["rx_sha"], k
    finally:
        load().uq_test_set_quicfl_hooks(prev)


def test_dropin_2pow22_vs_reference(fx, tmp_path):
    import uqdme
    meta, z, rz = fx
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
            x = gen(c["kind"], c["vseed"], c["dim"])
            torch.manual_seed(c["gseed"])
            out = uqdme.QUICFL_quantize(x, c["nbits"])
            assert np.array_equal(out[z[f"dpos{j}"]].view(np.uint32), z[f"douts{j}"].view(np.uint32))
            assert sha(out) == c["out_sha"]
            w = state_words()
            assert (w[0], w[1]) == (c["left1"], c["next1"]) and np.array_equal(w[2:], z[f"dst1_{j}"])
    finally:
        uqdme.set_tables_prefix(None)
