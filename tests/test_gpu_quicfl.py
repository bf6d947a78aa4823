"""GPU: the QUIC-FL receiver (AS:507-535) against the reference's QuicFLReceiver.decompress
outputs (tests/golden/make_golden_quicfl.py) and the oracle, bit for bit, through the C ABI
(uq_quicfl_prepare_f32 + uq_rht_f32)."""
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
