"""CPU ORACLE — test infrastructure only, never the product path.

NumPy restatement of the reference's QUIC-FL sender and of the pieces
of torch's CPU generator it draws from.  AS = NMSE_Results/Codes/All_Schemes.py:
  AS:429-451  QuicFLSender: per bit width a sender table X, a table p and data.txt
              (delta, h_len, ...); half_table_size = ((numel // h_len) - 1) * h_len // 2
  AS:455-503  compress
  AS:814-832  QUICFL_quantize (seed = torch.randint(0, 100) from the global generator)

Float / generator semantics (each checked against torch 2.10 CPU by
tests/test_quicfl_sender_oracle.py and pinned by the reference's own outputs,
tests/golden/make_golden_quicfl_sender.py):
  * prng_seed = xxh64(str(seed)) % 2^16 (AS:457; xxHash64 restated below, seed 0).
  * the rotation is the EDEN sender's RHT (oracle/uq_eden.py: rht), the norm torch.norm's
    8 fma lanes (uq_eden.torch_norm2).
  * scale = np.sqrt(D) / norm goes through Tensor.__rtruediv__ = reciprocal(norm) * other:
    f32(f32(1 / norm) * f32(sqrt(D))).
  * v = rot * scale (f32); exact = v > f32(T) | v < -f32(T), T = norm.ppf(1 - 2^-9) (torch
    compares against the scalar cast to f32).
  * q = v / f32(delta) (IEEE division), q[exact] = 0; p = q - floor(q).
  * h = randint(0, h_len, (D,)) from the local generator (word % h_len), then
    bernoulli(p, local) continues that stream: one word per element, 1 iff
    (w & 0xFFFFFF) * 2^-24 < p (p outside [0, 1], e.g. NaN, raises RuntimeError).
  * index = ((f32(floor(q) + b) * f32(h_len)) + f32(h)) + f32(half) in f32, .long() truncates;
    torch.take wraps negative indices and raises IndexError outside [-numel, numel).
  * X = f32(table_X[idx] + bernoulli(table_p[idx])) with the GLOBAL generator (one word per
    element), .long().
  * the global generator's state (left, next, 624 words) follows ATen's mt19937: a call
    decrements left, twists when it reaches 0, returns state[next++] tempered.
"""
from __future__ import annotations

import struct

import numpy as np

from . import uq_eden as E

f32 = np.float32
M64 = (1 << 64) - 1
T_EXACT = 2.8856349124267573             # scipy.stats.norm.ppf(1 - 2**-9) (AS:475-478)


# ---- xxHash64 (AS:457 xxhash.xxh64(str(seed)).intdigest()) --------------------------------
_P1, _P2, _P3, _P4, _P5 = (0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9, 0x85EBCA77C2B2AE63,
                           0x27D4EB2F165667C5)


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _round(acc, lane):
    acc = (acc + lane * _P2) & M64
    return (_rotl(acc, 31) * _P1) & M64


def _merge(acc, val):
    acc ^= _round(0, val)
    return (acc * _P1 + _P4) & M64


def xxh64(data: bytes, seed: int = 0) -> int:
    n = len(data)
    i = 0
    if n >= 32:
        v = [(seed + _P1 + _P2) & M64, (seed + _P2) & M64, seed & M64, (seed - _P1) & M64]
        while i + 32 <= n:
            for k in range(4):
                v[k] = _round(v[k], struct.unpack_from("<Q", data, i + 8 * k)[0])
            i += 32
        h = (_rotl(v[0], 1) + _rotl(v[1], 7) + _rotl(v[2], 12) + _rotl(v[3], 18)) & M64
        for k in range(4):
            h = _merge(h, v[k])
    else:
        h = (seed + _P5) & M64
    h = (h + n) & M64
    while i + 8 <= n:
        h ^= _round(0, struct.unpack_from("<Q", data, i)[0])
        h = (_rotl(h, 27) * _P1 + _P4) & M64
        i += 8
    if i + 4 <= n:
        h ^= (struct.unpack_from("<I", data, i)[0] * _P1) & M64
        h = (_rotl(h, 23) * _P2 + _P3) & M64
        i += 4
    while i < n:
        h ^= (data[i] * _P5) & M64
        h = (_rotl(h, 11) * _P1) & M64
        i += 1
    h ^= h >> 33
    h = (h * _P2) & M64
    h ^= h >> 29
    h = (h * _P3) & M64
    h ^= h >> 32
    return h


def prng_seed(seed) -> int:
    """AS:457."""
    return xxh64(str(seed).encode()) % (1 << 16)


# ---- torch CPU generator (ATen mt19937) from an arbitrary state ------------------------------
def seeded_state(seed: int):
    """(left, next, words[624]) right after manual_seed(seed) (init_genrand; left = 1)."""
    mt = np.zeros(624, np.uint64)
    mt[0] = seed & 0xFFFFFFFF
    for i in range(1, 624):
        mt[i] = (1812433253 * (int(mt[i - 1]) ^ (int(mt[i - 1]) >> 30)) + i) & 0xFFFFFFFF
    return 1, 0, mt.astype(np.uint32)


def _twist(mt: np.ndarray) -> np.ndarray:
    mt = mt.copy()
    for lo, hi in ((0, 227), (227, 454), (454, 623)):
        i = np.arange(lo, hi)
        y = (mt[i] & 0x80000000) | (mt[i + 1] & 0x7FFFFFFF)
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ np.where(y & 1, 0x9908B0DF, 0).astype(np.uint32)
    y = (mt[623] & 0x80000000) | (mt[0] & 0x7FFFFFFF)
    mt[623] = mt[396] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
    return mt


def _temper(y: np.ndarray) -> np.ndarray:
    y = y.copy()
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    y ^= y >> 18
    return y


def mt_draw(state, n: int):
    """n successive 32-bit outputs of ATen's mt19937 from state (left, next, words);
    returns (words, new state)."""
    left, nxt, mt = int(state[0]), int(state[1]), np.asarray(state[2], np.uint32).copy()
    out = np.empty(n, np.uint32)
    k = 0
    while k < n:
        if left == 1:                          # this call's --left reaches 0: twist
            mt = _twist(mt)
            left, nxt = 625, 0
        take = min(n - k, left - 1)            # calls served from the current block
        out[k:k + take] = _temper(mt[nxt:nxt + take])
        nxt += take
        left -= take
        k += take
    return out, (left, nxt, mt)


def torch_state_unpack(st: np.ndarray):
    """torch.Generator.get_state() bytes -> (left, next, words)."""
    st = np.asarray(st, np.uint8)
    _, left, _, nxt = struct.unpack_from("<QiiQ", st.tobytes(), 0)
    words = np.frombuffer(st[24:24 + 624 * 8].tobytes(), dtype=np.uint64).astype(np.uint32)
    return int(left), int(nxt), words


def torch_state_pack(st: np.ndarray, state) -> np.ndarray:
    """A copy of get_state() bytes with (left, next, words) replaced."""
    b = bytearray(np.asarray(st, np.uint8).tobytes())
    struct.pack_into("<i", b, 8, int(state[0]))
    struct.pack_into("<Q", b, 16, int(state[1]))
    b[24:24 + 624 * 8] = np.asarray(state[2], np.uint32).astype(np.uint64).tobytes()
    return np.frombuffer(bytes(b), np.uint8).copy()


# ---- QuicFLSender.compress ----------------------------------------------------------------------
def half_table_size(numel: int, h_len: int) -> int:
    """AS:443."""
    return ((numel // h_len) - 1) * h_len // 2


def _bern(words: np.ndarray, p: np.ndarray) -> np.ndarray:
    p = np.asarray(p, f32)
    if not np.all((p >= 0) & (p <= 1)):      # NaN included: at::bernoulli_distribution's check
        raise RuntimeError("Expected p_in >= 0 && p_in <= 1 to be true, but got false.")
    return ((words & 0xFFFFFF).astype(np.float64) * 2.0 ** -24 < p.astype(np.float64)).astype(f32)


def compress(x, nbits: int, seed, rotation_seed: int, table_X, table_p, delta: float, h_len: int, gstate):
    """QuicFLSender.compress (AS:455-503) on the CPU.  gstate: the global generator's
    (left, next, words) before the call.  Returns (message dict, new gstate)."""
    x = np.asarray(x, f32).reshape(-1)
    dim = x.shape[0]
    ps = prng_seed(seed)
    vec = E.rht(x, rotation_seed)                                    # AS:460-468
    D = vec.shape[0]
    loc, lst = mt_draw(seeded_state(ps), D)                          # AS:465/469 randint
    h = (loc % np.uint32(h_len)).astype(np.int64)
    nrm = E.torch_norm2(vec)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        scale = f32(f32(f32(1) / nrm) * f32(np.sqrt(D)))              # AS:466/470 via __rtruediv__
        v = (vec * scale).astype(f32)                                # AS:472
        t = f32(T_EXACT)
        exact = (v > t) | (v < -t)                                   # AS:478
        q = (v / f32(delta)).astype(f32)                             # AS:480
        q[exact] = 0                                                 # AS:481
        fl = np.floor(q).astype(f32)
        p = (q - fl).astype(f32)                                     # AS:483
    bw, _ = mt_draw(lst, D)                                          # AS:484 bernoulli(p, local)
    iq = (fl + _bern(bw, p)).astype(f32)
    tX = np.asarray(table_X, f32).reshape(-1)
    tp = np.asarray(table_p, f32).reshape(-1)
    numel = tX.size
    half = half_table_size(numel, h_len)
    idxf = ((iq * f32(h_len)).astype(f32) + h.astype(f32)).astype(f32)
    idxf = (idxf + f32(half)).astype(f32)                            # AS:486-487 (f32 arithmetic)
    idx = np.trunc(idxf).astype(np.int64)
    bad = (idx < -numel) | (idx >= numel)
    if bad.any():
        j = int(idx[bad][0])
        raise IndexError(f"out of range: tried to access index {j} on a tensor of {numel} elements.")
    idx = np.where(idx < 0, idx + numel, idx)
    gw, gst = mt_draw(gstate, D)                                     # AS:489 bernoulli(p_X), global
    Xf = (tX[idx] + _bern(gw, tp[idx])).astype(f32)
    X = np.trunc(Xf).astype(np.int64)                                # AS:490
    msg = {"X": X, "exact_values": v[exact], "exact_indeces": exact, "seed": seed, "prng_seed": ps,
           "rotation_seed": rotation_seed, "dim": dim, "scale": scale, "nbits": nbits, "h_len": h_len}
    return msg, gst
