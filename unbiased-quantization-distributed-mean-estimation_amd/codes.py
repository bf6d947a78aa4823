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
The nominal rate R is an entropy figure (log2 of the number of signed types / d); these
int8 codes are fixed-length and do not reach it.  `encode_messages` / `decode_messages`
entropy-code them on the GPU ("UQR1", rANS with a per-client static model, see
include/uq_dme.h uq_tc_*): ~R bits per coordinate (0.99 at R = 1, 1.92 at R = 2 for
d = 2^20 Gaussian clients).  Parity unpinned: the reference has no codec; decode(encode) is
checked against AS:640's output (values, and bits with exact_zero_signs).

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


@dataclass
class TypeMessages:
    """A batch of UQR1 messages packed back to back on the device: client j's message is
    data[offsets[j]:offsets[j+1]] (include/uq_dme.h, uq_tc_encode)."""
    data: torch.Tensor       # uint8 [capacity] (device)
    offsets: torch.Tensor    # int64 [n+1] (device; u64 in the C ABI)
    n: int
    d: int
    m: int
    exact_zero_signs: bool

    def sizes(self) -> np.ndarray:
        o = self.offsets.cpu().numpy().astype(np.int64)
        return o[1:] - o[:-1]

    def total_bytes(self) -> int:
        return int(self.offsets[self.n].item())

    def bits_per_dim(self) -> float:
        return 8.0 * self.total_bytes() / max(1, self.n * self.d)

    def message(self, j: int) -> bytes:
        o = self.offsets.cpu().numpy()
        return self.data[int(o[j]):int(o[j + 1])].cpu().numpy().tobytes()

    def messages(self) -> list:
        o = self.offsets.cpu().numpy()
        host = self.data[:int(o[self.n])].cpu().numpy()
        return [host[int(o[j]):int(o[j + 1])].tobytes() for j in range(self.n)]

    @classmethod
    def from_messages(cls, msgs, d: int, device=None) -> "TypeMessages":
        """Pack host messages (bytes) of one batch for decode_messages.  Every header must
        carry the same m and flags (one batch is decoded and averaged with one m; ValueError
        otherwise); the decoder then checks each message in full, and flags (status bit 4) any
        whose m differs from the batch's."""
        for j, b in enumerate(msgs):
            if len(b) < 40 or b[:4] != b"UQR1":
                raise ValueError(f"message {j} is not a UQR1 message")
        ms = {struct.unpack_from("<Q", b, 16)[0] for b in msgs}
        fl = {struct.unpack_from("<H", b, 6)[0] & 1 for b in msgs}
        if len(ms) > 1 or len(fl) > 1:
            raise ValueError(f"messages of one batch must share m and flags (m: {sorted(ms)[:4]}, flags: {sorted(fl)})")
        # each message starts 4-byte aligned (the decoder reads 32-bit words); sizes are
        # multiples of 4 by construction (tc_align4), others are padded here
        sizes = np.array([(len(b) + 3) & ~3 for b in msgs], np.int64)
        off = np.zeros(len(msgs) + 1, np.int64)
        np.cumsum(sizes, out=off[1:])
        buf = (np.frombuffer(b"".join(b + bytes(-len(b) % 4) for b in msgs), np.uint8) if msgs
               else np.zeros(0, np.uint8))
        m = ms.pop() if msgs else 0
        exact = bool(fl.pop()) if msgs else False
        dev = device or "cuda"
        return cls(data=torch.from_numpy(buf.copy()).to(dev), offsets=torch.from_numpy(off).to(dev), n=len(msgs),
                   d=int(d), m=int(m), exact_zero_signs=exact)


def _tc_sizes(lib, n, d):
    import ctypes
    from . import _lib
    b = ctypes.c_size_t()
    _lib.check(lib.uq_tc_bound(d, ctypes.byref(b)), "uq_tc_bound")
    w = ctypes.c_size_t()
    _lib.check(lib.uq_tc_workspace_bytes(n, d, ctypes.byref(w)), "uq_tc_workspace_bytes")
    return int(b.value), int(w.value)


STAGING_BYTES = 256 << 20     # encode_messages: worst-case message bytes staged per client chunk


def encode_messages(tc: "TypeCodes", exact_zero_signs: bool = False,
                    staging_bytes: int = STAGING_BYTES) -> TypeMessages:
    """Entropy-code a batch of type codes on the GPU (one UQR1 message per client).

    The encoder writes into a buffer sized for the worst case (uq_tc_bound: ~2 B per
    coordinate) with ~2 B per coordinate of workspace scratch, against ~R/8 B per coordinate
    of actual message.  A batch whose worst case exceeds `staging_bytes` is encoded in client
    chunks through one staging buffer and workspace of that size, each chunk's exact bytes
    kept (one synchronisation per chunk): at 1024 x 2^20 the transient is ~0.5 GB instead of
    ~4.3 GB, and the returned buffer holds exactly the messages."""
    from . import _lib
    from .quantizer import _device, _ptr, _stream_ptr
    dev = _device()
    lib = _lib.load()
    codes = tc.codes.to(dev).contiguous()
    l1 = tc.l1.to(device=dev, dtype=torch.float32).contiguous()
    n, d = codes.shape
    tc.check()
    flags = 1 if exact_zero_signs else 0
    bound, _ = _tc_sizes(lib, n, d)
    chunk = n if n * bound <= staging_bytes else max(1, staging_bytes // max(1, bound))

    def encode(j0, nj, data, offsets, ws):
        _lib.check(lib.uq_tc_encode(_ptr(codes[j0:j0 + nj]), _ptr(l1[j0:j0 + nj]), nj, d, int(tc.m), flags,
                                    _ptr(data), data.numel(), _ptr(offsets), _ptr(ws), ws.numel(), _stream_ptr(dev)),
                   "uq_tc_encode")

    if chunk >= n:
        _, wsb = _tc_sizes(lib, n, d)
        data = torch.empty(max(1, n * bound), dtype=torch.uint8, device=dev)
        offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
        encode(0, n, data, offsets, torch.empty(max(1, wsb), dtype=torch.uint8, device=dev))
        return TypeMessages(data=data, offsets=offsets, n=n, d=d, m=int(tc.m), exact_zero_signs=bool(exact_zero_signs))
    _, wsb = _tc_sizes(lib, chunk, d)
    stage = torch.empty(chunk * bound, dtype=torch.uint8, device=dev)
    soff = torch.empty(chunk + 1, dtype=torch.int64, device=dev)
    ws = torch.empty(max(1, wsb), dtype=torch.uint8, device=dev)
    parts, offs, base = [], [torch.zeros(1, dtype=torch.int64, device=dev)], 0
    for j0 in range(0, n, chunk):
        nj = min(chunk, n - j0)
        encode(j0, nj, stage, soff[:nj + 1], ws)
        tot = int(soff[nj].item())
        parts.append(stage[:tot].clone())
        offs.append(soff[1:nj + 1] + base)
        base += tot
    return TypeMessages(data=torch.cat(parts), offsets=torch.cat(offs), n=n, d=d, m=int(tc.m),
                        exact_zero_signs=bool(exact_zero_signs))


def decode_messages(msgs: TypeMessages) -> "TypeCodes":
    """UQR1 messages -> TypeCodes (device); raises if any message is malformed (synchronises)."""
    from . import _lib
    from .quantizer import _device, _ptr, _stream_ptr
    dev = _device()
    lib = _lib.load()
    n, d = msgs.n, msgs.d
    codes = torch.empty((n, d), dtype=torch.int8, device=dev)
    l1 = torch.empty(n, dtype=torch.float32, device=dev)
    kmax = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    data = msgs.data.to(dev)
    offsets = msgs.offsets.to(dev)
    _lib.check(lib.uq_tc_decode(_ptr(data), data.numel(), _ptr(offsets), n, d, int(msgs.m), _ptr(codes), _ptr(l1),
                                _ptr(kmax), _ptr(status), _stream_ptr(dev)), "uq_tc_decode")
    bad = int(torch.count_nonzero(status[:n]).item()) if n else 0
    if bad:
        raise ValueError(f"{bad} malformed UQR1 message(s) (status {status[:n].cpu().numpy().tolist()[:8]})")
    return TypeCodes(codes=codes, l1=l1, m=msgs.m, overflow=kmax)
