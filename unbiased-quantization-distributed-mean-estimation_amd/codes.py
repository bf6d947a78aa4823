"""Type codes: a wire format for the unbiased L1-ball type quantizer.

The reference never encodes: `Type_unbiased_quantize` (All_Schemes.py:609-641) returns the
dequantized vector L1 * sign(v) * k / m with k = fl + r the lattice counts (sum ~= m).  A
client message is fully described by (L1, m, signed k), so a DME client can send that
instead of d floats, and the server rebuilds q bit-for-bit:

    code_i = k_i          if sign(v_i) >= 0      (k_i in [0, 127])
    code_i = -k_i - 1     if sign(v_i) <  0      (so a negative coordinate with k = 0,
                                                  which the reference outputs as -0.0,
                                                  round-trips exactly)
    q_i    = +-RN(RN(L1 * k_i) / f32(m))                      (== AS:640 bit-for-bit)

Counts above 127 (high rates / heavy tails) saturate and set the client's overflow flag;
such clients must be sent as floats (or re-encoded at a lower rate).  At R <= 2 with the
reference's distributions no overflow occurs.  One byte per coordinate vs four: the bench's
"codes" pipeline folds the mean from codes (reading d bytes per client instead of 4d).
The nominal rate R is an entropy figure (log2 of the number of signed types / d); this v1
format is fixed-length and does not reach it -- parity unpinned (the reference has no codec).

Serialized message (little endian):
    b"UQT1" | u32 version=1 | i64 n | i64 d | i64 m | f32 l1[n] | i8 codes[n*d]
(the per-client max count is recomputed from the codes on receipt)
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np
import torch

MAGIC = b"UQT1"
VERSION = 1
_HDR = struct.Struct("<4sIqqq")


@dataclass
class TypeCodes:
    codes: torch.Tensor      # int8 [n, d] (device or host)
    l1: torch.Tensor         # f32 [n]
    m: int                   # lattice sum (AS:623)
    overflow: torch.Tensor   # int32 [n]: the client's largest count k; 128 = a count > 127 saturated

    @property
    def n(self) -> int:
        return int(self.codes.shape[0])

    @property
    def d(self) -> int:
        return int(self.codes.shape[1])

    def check(self) -> None:
        """Raise if any client's counts did not fit the 8-bit code (synchronises)."""
        bad = int(torch.count_nonzero(self.overflow > 127).item())
        if bad:
            raise OverflowError(f"{bad} client(s) have lattice counts > 127; send them as floats")

    def to_bytes(self) -> bytes:
        self.check()
        hdr = _HDR.pack(MAGIC, VERSION, self.n, self.d, int(self.m))
        l1 = self.l1.detach().to("cpu", torch.float32).contiguous().numpy().astype("<f4").tobytes()
        c = self.codes.detach().to("cpu").contiguous().numpy().astype(np.int8).tobytes()
        return hdr + l1 + c

    @classmethod
    def from_bytes(cls, buf: bytes, device=None) -> "TypeCodes":
        magic, ver, n, d, m = _HDR.unpack_from(buf, 0)
        if magic != MAGIC or ver != VERSION:
            raise ValueError("not a UQT1 type-codes message")
        off = _HDR.size
        l1 = np.frombuffer(buf, dtype="<f4", count=n, offset=off).astype(np.float32)
        off += 4 * n
        codes = np.frombuffer(buf, dtype=np.int8, count=n * d, offset=off).reshape(n, d)
        if off + n * d != len(buf):
            raise ValueError("truncated or oversized UQT1 message")
        dev = device or "cpu"
        k = np.where(codes < 0, -(codes.astype(np.int32)) - 1, codes.astype(np.int32))
        kmax = k.max(axis=1) if d else np.zeros(n, np.int32)
        return cls(codes=torch.from_numpy(codes.copy()).to(dev), l1=torch.from_numpy(l1).to(dev), m=int(m),
                   overflow=torch.from_numpy(kmax.astype(np.int32)).to(dev))
