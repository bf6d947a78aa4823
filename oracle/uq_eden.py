"""CPU ORACLE — test infrastructure only, never the product path.

NumPy restatement of the reference's EDEN baseline with the randomized Hadamard
transform.  Citations are relative to the reference root,
AS = NMSE_Results/Codes/All_Schemes.py:
  AS:95-120   Hadamard.hadamard (butterfly a' = a + b, b' = a' - 2b, then / sqrt(d)),
              random_diagonal (seeded CPU generator, torch.bernoulli(1/2))
  AS:123-141  HadamardSender.randomized_hadamard_transform (zero-pad to 2^p, * diag, H)
  AS:146-153  HadamardReceiver.randomized_inverse_hadamard_transform (H, then * diag)
  AS:300-316  gen_normal_centoirds_and_boundries (1- and 2-bit tables)
  AS:324-376  EdenSender.quantize / compress (integer nbits, delta=None path)
  AS:378-413  EdenReceiver.decompress
  AS:792-811  EDEN_quantize_Hadamard (seed = torch.randint(0, 100) per call)

Float semantics pinned here against torch 2.10 CPU (tools in tests/golden/make_golden_eden.py):
  * torch's CPU generator is MT19937 (init_genrand(seed)); bernoulli(p) on a float
    tensor draws one 32-bit word per element: u = (w & 0xFFFFFF) * 2^-24, value = u < p.
    randint(0, 100) = w % 100.
  * torch.norm(v, 2) (f32): 8 interleaved lanes, acc = fma(v, v, acc) sequentially,
    lanes added 0..7 in order, tail, f32 sqrt.
  * torch.dot (AS:335) goes to MKL's cblas sdot (torch 2.10's BLAS, oneMKL 2024.2, one
    thread: torch.set_num_threads(1) also sets MKL's).  Its AVX-512 path on the fixtures'
    host, found by summation-order probing (tools/dot_order_probe.py) and pinned by
    tests/golden/dot_vectors.* (torch.dot's own bits, n = 1 .. 2^22) and by every EDEN scale the
    reference recorded: 4 accumulators of 16 lanes, element i -> accumulator (i / 16) % 4,
    lane i % 16 of 64-element blocks, each lane a sequential fma chain; then
    (acc0 + acc1) + (acc2 + acc3) lane-wise; then the 16 lanes as i + (i + 8), i + (i + 4),
    (0 + 1) + (2 + 3).  Of a remainder below 64, a 32-element block goes into acc0 and acc1,
    then 16-element chunks into acc0, the last one masked.  torch_dot below.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32

# AS:302-306 (only 1 and 2 bits are defined in the reference)
CENTROIDS_POS = {1: [0.7978845608028654], 2: [0.4527800398860679, 1.5104176087114887]}


def centroids(nbits: int) -> np.ndarray:
    c = CENTROIDS_POS[nbits]
    return np.array([-v for v in c[::-1]] + c, dtype=f32)          # AS:309 torch.Tensor -> f32


def boundaries(nbits: int) -> np.ndarray:
    # AS:314 sets boundries[1] = centroids[1][0] ** 2, but the update on AS:315 overwrites
    # it with the midpoints for every table (1 bit: [0.0]).
    c = centroids(nbits)
    return np.array([f32((float(a) + float(b)) / 2) for a, b in zip(c[:-1], c[1:])], dtype=f32)   # AS:311-315


def mt19937(seed: int, n: int) -> np.ndarray:
    """n 32-bit outputs of MT19937 seeded with init_genrand(seed) (torch CPU generator)."""
    mt = np.zeros(624, np.uint64)
    mt[0] = seed & 0xFFFFFFFF
    for i in range(1, 624):
        mt[i] = (1812433253 * (int(mt[i - 1]) ^ (int(mt[i - 1]) >> 30)) + i) & 0xFFFFFFFF
    mt = mt.astype(np.uint32)
    out = np.empty(n, np.uint32)
    k = 0
    while k < n:
        # twist (vectorized in the three dependency phases of the in-place update)
        for lo, hi in ((0, 227), (227, 454), (454, 623)):
            i = np.arange(lo, hi)
            y = (mt[i] & 0x80000000) | (mt[i + 1] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ np.where(y & 1, 0x9908B0DF, 0).astype(np.uint32)
        y = (mt[623] & 0x80000000) | (mt[0] & 0x7FFFFFFF)
        mt[623] = mt[396] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        y = mt.copy()
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        take = min(624, n - k)
        out[k:k + take] = y[:take]
        k += take
    return out


def random_diagonal(size: int, seed: int) -> np.ndarray:
    """AS:117-120: 2 * bernoulli(1/2) - 1 from a generator seeded with `seed`."""
    w = mt19937(seed, size)
    b = ((w & 0xFFFFFF) < (1 << 23)).astype(f32)        # u < 0.5 <=> low 24 bits < 2^23
    return (f32(2) * b - f32(1)).astype(f32)


def hadamard(v: np.ndarray) -> np.ndarray:
    """AS:100-115 in f32: stages h = 2..d, a' = a + b, b' = a' - 2b, then v / f32(sqrt(d))."""
    v = np.array(v, dtype=f32, copy=True)
    d = v.shape[0]
    assert d & (d - 1) == 0
    h = 2
    while h <= d:
        hf = h // 2
        w = v.reshape(d // h, h)
        a = (w[:, :hf] + w[:, hf:]).astype(f32)
        w[:, hf:] = (a - (f32(2) * w[:, hf:]).astype(f32)).astype(f32)
        w[:, :hf] = a
        h *= 2
    return (v / f32(np.sqrt(d))).astype(f32)


def padded_dim(dim: int) -> int:
    return dim if dim & (dim - 1) == 0 else int(2 ** (np.ceil(np.log2(dim))))


def rht(x: np.ndarray, seed: int) -> np.ndarray:
    """AS:123-141: zero-pad, multiply by the diagonal, Hadamard."""
    x = np.asarray(x, f32)
    D = padded_dim(x.shape[0])
    p = np.zeros(D, f32)
    p[:x.shape[0]] = x
    return hadamard((p * random_diagonal(D, seed)).astype(f32))


def inverse_rht(v: np.ndarray, seed: int) -> np.ndarray:
    """AS:146-153: Hadamard, then multiply by the diagonal."""
    return (hadamard(v) * random_diagonal(v.shape[0], seed)).astype(f32)


def torch_norm2(v: np.ndarray) -> f32:
    """torch.norm(v, 2) on CPU f32: 8 lanes of fma accumulation, lanes in order, tail, sqrt."""
    v = np.asarray(v, f32)
    n = v.shape[0] - v.shape[0] % 8
    acc = np.zeros(8, np.float64)
    blk = v[:n].reshape(-1, 8).astype(np.float64)
    accf = np.zeros(8, f32)
    for r in blk:                                  # fma: exact product + acc, one rounding
        accf = (accf.astype(np.float64) + r * r).astype(f32)
    del acc
    s = accf[0]
    for j in range(1, 8):
        s = f32(s + accf[j])
    # below one 8-wide vector torch takes other paths (measured, torch 2.10): |x| for one
    # element, fma for two, mul + add for four
    if v.shape[0] == 1:
        return f32(abs(v[0]))
    if v.shape[0] == 2:
        return f32(np.sqrt(f32(np.float64(f32(np.float64(v[0]) * v[0])) + np.float64(v[1]) * v[1])))
    for t in v[n:]:
        s = f32(s + f32(t * t))
    return f32(np.sqrt(s))


def torch_dot(x: np.ndarray, y: np.ndarray) -> f32:
    """torch.dot(x, y) of two f32 vectors on CPU (MKL sdot, see the module header).  fma is
    evaluated in extended precision (64-bit significand: a 48-bit product plus a 24-bit
    accumulator) and rounded once to f32 except in the rare case where the exact sum needs
    more than 64 bits (oracle/uq_oracle.c uqo_torch_dot uses fmaf)."""
    if np.finfo(np.longdouble).nmant < 63:     # fma stand-in needs x87's 64-bit significand
        raise RuntimeError("torch_dot oracle needs an 80-bit long double (x86); use uq_oracle_c.torch_dot")
    x = np.asarray(x, f32).reshape(-1)
    y = np.asarray(y, f32).reshape(-1)
    n = x.shape[0]
    L = np.longdouble
    acc = np.zeros(64, f32)                        # accumulator k lane l at 16 k + l
    nb = n // 64
    if nb:
        xb = x[:nb * 64].reshape(nb, 64).astype(L)
        yb = y[:nb * 64].reshape(nb, 64).astype(L)
        pr = xb * yb                               # exact products
        for b in range(nb):
            acc = (acc.astype(L) + pr[b]).astype(f32)
    i0 = nb * 64
    if n - i0 >= 32:                               # remainder: a 32-element block into acc0, acc1
        acc[:32] = (acc[:32].astype(L) + x[i0:i0 + 32].astype(L) * y[i0:i0 + 32].astype(L)).astype(f32)
        i0 += 32
    for i0 in range(i0, n, 16):                    # then 16-element chunks into acc0 (last masked)
        m = min(16, n - i0)
        acc[:m] = (acc[:m].astype(L) + x[i0:i0 + m].astype(L) * y[i0:i0 + m].astype(L)).astype(f32)
        acc[m:16] = (acc[m:16] + f32(0)).astype(f32)                          # masked lanes: + 0 * 0
    v = ((acc[0:16] + acc[16:32]).astype(f32) + (acc[32:48] + acc[48:64]).astype(f32)).astype(f32)
    v = (v[:8] + v[8:]).astype(f32)
    v = (v[:4] + v[4:]).astype(f32)
    return f32(f32(v[0] + v[1]) + f32(v[2] + v[3]))


def bucketize(x: np.ndarray, b: np.ndarray) -> np.ndarray:
    """torch.bucketize(x, b) (right=False): number of boundaries strictly below x."""
    return np.searchsorted(b, x, side="left").astype(np.int64)


def eden_compress(x: np.ndarray, nbits: int, seed: int):
    """AS:324-376 (integer nbits, cscale=False): returns (bins, scale, vec, D)."""
    vec = rht(x, seed)
    D = vec.shape[0]
    nrm = torch_norm2(vec)
    sq = f32(np.sqrt(D))                                   # vec.numel() ** 0.5 -> f32 operand
    bins = bucketize(((vec * sq).astype(f32) / nrm).astype(f32), boundaries(nbits))
    c = centroids(nbits)[bins]
    dot = torch_dot(c, vec)                                # AS:335 torch.dot (MKL sdot order)
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = f32(f32(nrm * nrm) / dot)
    return bins, scale, vec, D


def eden_decompress(bins: np.ndarray, scale, nbits: int, seed: int, dim: int) -> np.ndarray:
    """AS:378-413 (integer nbits, no drop): scale * inverse_rht(centroids[bins])[:dim]."""
    v = inverse_rht(centroids(nbits)[bins], seed)
    return (f32(scale) * v).astype(f32)[:dim]


def eden_quantize(x: np.ndarray, nbits: int, seed: int) -> np.ndarray:
    """EDEN_quantize_Hadamard (AS:792-811) with the per-call seed given."""
    x = np.asarray(x, f32)
    bins, scale, _, _ = eden_compress(x, nbits, seed)
    return eden_decompress(bins, scale, nbits, seed, x.shape[0])


def quicfl_decompress(X: np.ndarray, recv_table: np.ndarray, h_len: int, prng_seed: int, exact_mask, exact_values,
                      scale, rotation_seed: int, dim: int) -> np.ndarray:
    """QuicFLReceiver.decompress (AS:526-535): h = torch.randint(0, h_len, (D,)) from a CPU
    generator seeded with prng_seed (= MT19937 word % h_len), v = recv_table.take(X * h_len + h),
    exact coordinates overwritten in index order, v / scale (f32), inverse RHT, [:dim]."""
    X = np.asarray(X, np.int64).reshape(-1)
    h = (mt19937(int(prng_seed), X.size) % np.uint32(h_len)).astype(np.int64)
    v = np.asarray(recv_table, f32).reshape(-1)[X * h_len + h].copy()
    if exact_mask is not None:
        m = np.asarray(exact_mask, bool).reshape(-1)
        v[m] = np.asarray(exact_values, f32).reshape(-1)
    v = (v / f32(scale)).astype(f32)
    return inverse_rht(v, rotation_seed)[:dim]
