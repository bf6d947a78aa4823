"""QUIC-FL receiver on the GPU — SURVEY §8(f) row 2 (baseline), the half the reference pins.

    QuicFLReceiver(device=..., bits=[1, 2, 3, 4], sr_bits=[6, 5, 4, 4], prefix=.../tables/)
        mirrors NMSE_Results/Codes/All_Schemes.py:507-535: receiver tables loaded from the
        reference's tables/ directory (torch.load(weights_only=True)), decompress(data) takes
        the sender's message dict and returns vec[:dim].
    quicfl_decompress(X[n, D], nbits, prng_seeds, rotation_seeds, scale[n], dim, recv_table)
        the same for a batch: (exact ? exact value : recv_table[X * h_len + h]) / scale, inverse
        RHT, [:dim], with h = torch.randint(0, h_len, (D,)) of a CPU generator seeded with
        prng_seed (MT19937 word % h_len).

Bit-identical to the reference's QuicFLReceiver.decompress (tests/golden/quicfl_recv_vectors.*).
The sender (QuicFLSender, AS:429-505) is not provided: its tables
(tables/*_sender_table_X.pt, *_sender_table_p.pt) are missing from the reference, whose drivers
crash at their first QUIC-FL call (Normal_dist.py:141), so no sender output can be pinned.
"""
from __future__ import annotations

import ast
import os

import torch

from . import _lib
from .eden import padded_dim, randomized_inverse_hadamard_transform
from .quantizer import _device, _ptr, _stream_ptr

__all__ = ["QuicFLReceiver", "quicfl_decompress"]


def quicfl_decompress(X, nbits: int, prng_seeds, rotation_seeds, scale, dim: int, recv_table, h_len: int | None = None,
                      exact_mask=None, exact_vals=None) -> torch.Tensor:
    """Batched QuicFLReceiver.decompress (AS:526-535).  X [n, D] integers in [0, rows) with D a
    power of two; recv_table [rows, h_len]; exact_mask bool [n, D] with exact_vals f32 [n, D]
    (dense: the value where the mask is set) or both None; scale [n]; returns [n, dim] f32."""
    dev = _device()
    X = torch.as_tensor(X)
    if X.dim() == 1:
        X = X.view(1, -1)
    n, D = X.shape
    if D != padded_dim(D):
        raise ValueError("X rows are the padded (power-of-two) dimension (AS:461-467)")
    if not 0 < dim <= D:
        raise ValueError("dim must be in 1..D")
    tab = torch.as_tensor(recv_table, dtype=torch.float32).to(dev).contiguous()
    rows, hl = (tab.shape[0], tab.shape[1]) if tab.dim() == 2 else (1, tab.numel())
    if h_len is not None and int(h_len) != hl:
        raise ValueError("h_len does not match the receiver table")
    if X.numel() and (int(X.min()) < 0 or int(X.max()) >= rows):
        raise IndexError("X outside the receiver table (torch.take raises, AS:530)")
    Xd = X.to(device=dev, dtype=torch.int32).contiguous()
    ps = torch.as_tensor(prng_seeds, dtype=torch.int64).reshape(-1)
    rs = torch.as_tensor(rotation_seeds, dtype=torch.int64).reshape(-1)
    sc = torch.as_tensor(scale, dtype=torch.float32).reshape(-1).to(dev)
    if ps.numel() != n or rs.numel() != n or sc.numel() != n:
        raise ValueError("one prng seed, rotation seed and scale per message")
    if (exact_mask is None) != (exact_vals is None):
        raise ValueError("exact_mask and exact_vals go together")
    m = v = None
    if exact_mask is not None:
        m = torch.as_tensor(exact_mask).to(device=dev, dtype=torch.uint8).reshape(n, D).contiguous()
        v = torch.as_tensor(exact_vals, dtype=torch.float32).to(dev).reshape(n, D).contiguous()
    pre = torch.empty((n, D), dtype=torch.float32, device=dev)
    if n:
        seeds32 = (ps & 0xFFFFFFFF).to(torch.int64)
        seeds32 = torch.where(seeds32 >= 1 << 31, seeds32 - (1 << 32), seeds32).to(torch.int32).to(dev)
        _lib.check(_lib.load().uq_quicfl_prepare_f32(_ptr(Xd), n, D, _ptr(tab), rows, hl, _ptr(seeds32),
                                                      _ptr(m) if m is not None else None,
                                                      _ptr(v) if v is not None else None, _ptr(sc), _ptr(pre),
                                                      _stream_ptr(dev)), "uq_quicfl_prepare_f32")
    return randomized_inverse_hadamard_transform(pre, rs)[:, :dim]


class QuicFLReceiver:
    """AS:507-535 with the same constructor arguments and decompress(data) contract."""

    def __init__(self, device=None, bits=(1, 2, 3, 4), sr_bits=(6, 5, 4, 4), prefix=None, tables=None):
        self.device = device if device is not None else _device()
        self.recv_table = {}
        if tables is not None:                      # {nbits: [rows, h_len] tensor or array}
            for b, t in tables.items():
                self.recv_table[int(b)] = torch.as_tensor(t, dtype=torch.float32)
        else:
            if prefix is None:
                raise ValueError("prefix: the reference's tables/ directory (AS:509)")
            for b, s in zip(bits, sr_bits):
                fn = os.path.join(prefix, f"{b}_X_{s}_h_256_q_")
                self.recv_table[b] = self.receiver_table(fn, self.device)

    @staticmethod
    def receiver_table(prefix, device):
        """AS:520-523, loading with weights_only=True (no code from the file runs)."""
        return torch.load(prefix + "recv_table.pt", weights_only=True).to(torch.float32)

    @staticmethod
    def table_params(prefix):
        """The data.txt dictionary next to a table (parsed with ast.literal_eval, not eval)."""
        with open(prefix + "data.txt") as f:
            return ast.literal_eval(f.read())

    def decompress(self, data):
        """AS:526-535: the message dict of QuicFLSender.compress -> vec[:dim] (on the GPU)."""
        X = torch.as_tensor(data["X"]).reshape(1, -1)
        D = X.shape[1]
        mask = vals = None
        ei = data.get("exact_indeces")
        if ei is not None and bool(torch.as_tensor(ei).any()):
            mask = torch.as_tensor(ei).reshape(1, D).to(torch.bool)
            vals = torch.zeros((1, D), dtype=torch.float32)
            vals[mask] = torch.as_tensor(data["exact_values"], dtype=torch.float32).reshape(-1).cpu()
        out = quicfl_decompress(X, data["nbits"], [int(data["prng_seed"])], [int(data["rotation_seed"])],
                                [float(torch.as_tensor(data["scale"]))], int(data["dim"]),
                                self.recv_table[int(data["nbits"])], int(data["h_len"]), mask, vals)
        return out.view(-1)
