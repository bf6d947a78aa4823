"""CPU: the QUIC-FL receiver restatement (oracle/uq_eden.py quicfl_decompress, AS:526-535)
against the reference's QuicFLReceiver.decompress outputs (tests/golden/make_golden_quicfl.py),
bit for bit.  The sender (AS:429-505) has no golden vectors: its tables are not in the
reference, so it is not built."""
import json
import os

import numpy as np

from oracle import uq_eden as E

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    meta = json.load(open(os.path.join(HERE, "quicfl_recv_vectors.json")))
    z = np.load(os.path.join(HERE, "quicfl_recv_vectors.npz"))
    return meta, z


def test_randint_is_mt19937_word_mod_range():
    import torch
    g = torch.Generator().manual_seed(4242)
    h = torch.randint(0, 32, (3000,), generator=g).numpy()
    assert np.array_equal(h, (E.mt19937(4242, 3000) % np.uint32(32)).astype(np.int64))


def test_oracle_matches_reference_receiver():
    meta, z = load()
    assert len(meta["cases"]) == 12
    for c in meta["cases"]:
        i, b = c["idx"], c["nbits"]
        tab = z[f"recv{b}"]
        assert tab.shape == tuple(meta["tables"][str(b)]["shape"]) and tab.shape[1] == c["h_len"]
        out = E.quicfl_decompress(z[f"X{i}"], tab, c["h_len"], c["prng_seed"], z[f"mask{i}"], z[f"vals{i}"],
                                  np.float32(c["scale"]), c["rotation_seed"], c["dim"])
        assert out.view(np.uint32).tolist() == z[f"out{i}"].view(np.uint32).tolist(), i
