"""Synthetic QUIC-FL sender tables (test data; the published ones are not in the reference).

The reference's QuicFLSender (NMSE_Results/Codes/All_Schemes.py:429-451) loads, per bit width,
`{b}_X_{s}_h_256_q_sender_table_X.pt`, `..._sender_table_p.pt` and `..._data.txt` from its
`prefix`.  The .pt files are missing from the reference, so the sender's
semantics are pinned on tables made here.  They follow the shape rule of AS:443
(numel = (2K + 1) * h_len, half_table_size = K * h_len, K = (x_len - 1) / 2) with the
reference's own data.txt parameters (delta, T, h_len, x_len), and their values are exact
binary fractions built from integers, so every host produces the same bits:

    X[r, h] = clip(((r * (L - 1)) * h_len + h * (x_len - 1)) // ((x_len - 1) * h_len), 0, L - 1)
    p[r, h] = ((r * 2654435761 + h * 40503 + b * 97) mod 2^24) / 2^24, and 0 where X = L - 1

with L = 2^b, so X + bernoulli(p) stays a valid receiver row (AS:530).
"""
from __future__ import annotations

import numpy as np

# data.txt of the reference's tables/ directory (NMSE_Results/Codes/tables/*_data.txt), as data
DATA = {
    1: {'delta': 0.0006194538156387708, 'T': 3.0972690781930625, 'h_len': 64, 'x_len': 10001},
    2: {'delta': 0.0006194538156392149, 'T': 3.097269078196875, 'h_len': 32, 'x_len': 10001},
    3: {'delta': 0.0006194538156414353, 'T': 3.09726907820625, 'h_len': 16, 'x_len': 10001},
    4: {'delta': 0.0006194538156414353, 'T': 3.0972690782062497, 'h_len': 16, 'x_len': 10001},
}
SR_BITS = {1: 6, 2: 5, 3: 4, 4: 4}           # AS:431 sr_bits=[6, 5, 4, 4]


def sender_tables(b: int, x_len: int | None = None, h_len: int | None = None):
    """(X, p) float32 [x_len, h_len] for bit width b."""
    x_len = int(x_len if x_len is not None else DATA[b]['x_len'])
    h_len = int(h_len if h_len is not None else DATA[b]['h_len'])
    L = 1 << b
    r = np.arange(x_len, dtype=np.int64)[:, None]
    h = np.arange(h_len, dtype=np.int64)[None, :]
    X = ((r * (L - 1)) * h_len + h * (x_len - 1)) // ((x_len - 1) * h_len)
    X = np.clip(X, 0, L - 1)
    p = ((r * 2654435761 + h * 40503 + b * 97) % (1 << 24)).astype(np.float64) / float(1 << 24)
    p = np.where(X == L - 1, 0.0, p)
    return X.astype(np.float32), p.astype(np.float32)


def data_txt(b: int, **override) -> str:
    d = dict(DATA[b])
    d.update(override)
    return repr(d)


def write_tables(root: str) -> str:
    """A complete table prefix as QuicFLSender / QuicFLReceiver read it: the synthetic sender
    tables above, data.txt, and the reference's receiver tables from the committed fixture
    (quicfl_recv_vectors.npz).  Returns the prefix (root + '/')."""
    import os
    import torch
    os.makedirs(root, exist_ok=True)
    rz = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "quicfl_recv_vectors.npz"))
    for b in (1, 2, 3, 4):
        fn = os.path.join(root, f"{b}_X_{SR_BITS[b]}_h_256_q_")
        X, p = sender_tables(b)
        torch.save(torch.from_numpy(X), fn + "sender_table_X.pt")
        torch.save(torch.from_numpy(p), fn + "sender_table_p.pt")
        torch.save(torch.from_numpy(rz[f"recv{b}"]), fn + "recv_table.pt")
        with open(fn + "data.txt", "w") as f:
            f.write(data_txt(b))
    return root + "/"
