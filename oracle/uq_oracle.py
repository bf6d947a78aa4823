"""CPU ORACLE — test infrastructure only, never the product path.

A from-scratch NumPy restatement of the reference's unbiased L1-ball type
quantizer and of the DME harness around it.  It is imported only by `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg, where it serves
as the checker.  The shipped path (`uqdme` -> HIP kernels) never calls it.

Pinning: this restatement was checked bit-for-bit against the reference
function itself (`NMSE_Results/Codes/All_Schemes.py:609-641`, imported in the
build container) and against `torch.sum` / `torch.cumsum` for the two torch
primitives whose float semantics define every output bit; the committed
fixtures under `tests/golden/` were produced by the reference and are re-checked
against this file by `tests/test_oracle_golden.py`.

Citations are `path:line` relative to the reference root:
  AS = NMSE_Results/Codes/All_Schemes.py
  ND = NMSE_Results/Codes/Normal_dist.py
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
f64 = np.float64

# AS:614-620 — rate table R (bits/dim) -> l_R, with m = int(l_R * d) (AS:622-623).
RATE_TABLE = {
    0.5: 0.08282, 1: 0.21403, 1.5: 0.39443, 2: 0.63752,
    2.5: 0.96656, 3: 1.41725, 3.5: 2.04187, 4: 2.91504,
    4.5: 4.14217, 5: 5.87195, 5.5: 8.31416, 6: 11.76507,
    6.5: 16.64332, 7: 23.54075, 7.5: 33.29414, 8: 47.0868,
    8.5: 66.59204, 9: 94.17625, 9.5: 133.18596, 10: 188.35383,
}

# torch CPU reduction constants (ATen SumKernel cascade_sum, torch 2.10 CPU):
TORCH_GRAIN = 32768   # at::internal::GRAIN_SIZE: threads split a reduction above this
VEC_LANES = 8         # Vectorized<float> width used by the sum kernel (AVX2 build)
ILP = 4               # row_sum ilp_factor
NUM_LEVELS = 4        # multi_row_sum num_levels


def rate_to_m(bits_per_dimension, d: int) -> int:
    """AS:614-623: `m = int(table[bits] * d)`; unknown keys raise KeyError."""
    return int(RATE_TABLE[bits_per_dimension] * d)


def _ceil_log2(x: int) -> int:
    return 0 if x <= 1 else (int(x) - 1).bit_length()


def _cascade(rows: np.ndarray) -> np.ndarray:
    """ATen `multi_row_sum` over `rows` (shape [R, W]) -> [W], f32 accumulate.

    Level 0 sums `step` rows sequentially; level j>0 accumulates level j-1 and
    flushes upward when the row counter is a multiple of step**j.  All adds are
    f32, per column, in exactly that order (data-independent tree)."""
    R, W = rows.shape
    lp = max(4, _ceil_log2(R) // NUM_LEVELS)
    step = 1 << lp
    nleaf = R // step
    zero = np.zeros(W, f32)
    # level 0: leaves of `step` rows, summed sequentially from 0
    leaves = zero[None, :].repeat(nleaf, 0)
    if nleaf:
        blk = rows[: nleaf * step].reshape(nleaf, step, W)
        for r in range(step):
            leaves = (leaves + blk[:, r]).astype(f32)
    # tail rows (< step) land in acc0 after the last reset
    acc0 = zero.copy()
    for r in range(nleaf * step, R):
        acc0 = (acc0 + rows[r]).astype(f32)

    def seq_groups(vals):
        """Sequential sums of full groups of `step` and of the trailing partial group."""
        ng = vals.shape[0] // step
        full = zero[None, :].repeat(ng, 0)
        if ng:
            g = vals[: ng * step].reshape(ng, step, W)
            for k in range(step):
                full = (full + g[:, k]).astype(f32)
        part = zero.copy()
        for k in range(ng * step, vals.shape[0]):
            part = (part + vals[k]).astype(f32)
        return full, part

    b1, acc1 = seq_groups(leaves)      # level-1 blocks (step^2 rows) + open level-1 acc
    b2, acc2 = seq_groups(b1)          # level-2 blocks (step^3 rows) + open level-2 acc
    acc3 = zero.copy()                 # level 3 never flushes further
    for k in range(b2.shape[0]):
        acc3 = (acc3 + b2[k]).astype(f32)
    out = acc0
    for a in (acc1, acc2, acc3):
        out = (out + a).astype(f32)
    return out


def _row_sum_scalar(x: np.ndarray) -> f32:
    """ATen `row_sum` with the scalar load policy (inner size < 8 lanes)."""
    s = x.shape[0]
    nilp = s // ILP
    p = _cascade(x[: nilp * ILP].reshape(nilp, ILP)) if nilp else np.zeros(ILP, f32)
    p = p.copy()
    for k in range(nilp * ILP, s):
        p[0] = f32(p[0] + x[k])
    for k in range(1, ILP):
        p[0] = f32(p[0] + p[k])
    return f32(p[0])


def _chunk_sum(x: np.ndarray) -> f32:
    """ATen `vectorized_inner_sum` for one contiguous chunk of f32 values."""
    s = x.shape[0]
    if s < VEC_LANES:
        return _row_sum_scalar(x)
    vs = s // VEC_LANES
    nilp = vs // ILP
    W = VEC_LANES * ILP
    if nilp:
        p = _cascade(x[: nilp * W].reshape(nilp, W)).reshape(ILP, VEC_LANES)
    else:
        p = np.zeros((ILP, VEC_LANES), f32)
    p0 = p[0].copy()
    for v in range(nilp * ILP, vs):                        # leftover 8-wide vectors
        p0 = (p0 + x[v * VEC_LANES:(v + 1) * VEC_LANES]).astype(f32)
    for k in range(1, ILP):
        p0 = (p0 + p[k]).astype(f32)
    acc = f32(0)
    for k in range(vs * VEC_LANES, s):                     # scalar tail first
        acc = f32(acc + x[k])
    for l in range(VEC_LANES):                             # then the 8 lanes in order
        acc = f32(acc + p0[l])
    return acc


def l1_torch_order(x: np.ndarray, torch_threads: int = 1) -> f32:
    """AS:624 `input_vector.abs().sum()` with torch CPU's exact f32 summation order.

    With T intra-op threads and d >= GRAIN, ATen's two_pass_reduction
    (TensorIteratorBase::parallel_reduce) splits the vector into
    nt = min(T, ceil(d/GRAIN)) chunks of ceil(d/nt); thread t adds its chunk's sum
    into buffer[t] of a T-element zero buffer, and the result is 0 + the same cascade
    sum over that buffer.  Checked against torch 2.10 for T = 1..39, 47, 63..65, 96,
    128, 200, 256 at five sizes (tests/golden/l1_threads.json); the chunk sums are not
    added sequentially unless T is 1, 2, 3, 4 or 8."""
    return torch_sum(np.abs(np.asarray(x, dtype=f32)), torch_threads)


def torch_sum(a: np.ndarray, torch_threads: int = 1) -> f32:
    """torch CPU f32 `Tensor.sum()` of a contiguous vector (see l1_torch_order)."""
    a = np.asarray(a, dtype=f32)
    d = a.shape[0]
    if d == 0:
        return f32(0)
    T = max(1, int(torch_threads))
    if d < TORCH_GRAIN or T == 1:
        return f32(f32(0) + _chunk_sum(a))
    nt = min(T, -(-d // TORCH_GRAIN))
    cs = -(-d // nt)
    buf = np.zeros(T, f32)
    for c in range(nt):
        if c * cs < d:
            buf[c] = f32(f32(0) + _chunk_sum(a[c * cs:(c + 1) * cs]))
    return f32(f32(0) + _chunk_sum(buf))


def fractional_parts(x: np.ndarray, m: int, l1: f32):
    """AS:625-631: den = L1 + 1e-12 (f32), v = x/den (IEEE f32), p=|v|,
    mp = f32(m)*p, fl = floor(mp), fr = mp - fl."""
    x = np.asarray(x, dtype=f32)
    den = f32(f32(l1) + f32(1e-12))
    with np.errstate(all="ignore"):
        v = (x / den).astype(f32)
        p = np.abs(v)
        mp = (f32(m) * p).astype(f32)
        fl = np.floor(mp).astype(f32)
        fr = (mp - fl).astype(f32)
    return v, fl, fr


def prefix_c(fr: np.ndarray) -> np.ndarray:
    """AS:635 `cat([0], fr.cumsum(0))`: torch CPU cumsum of f32 accumulates
    sequentially in fp64 and rounds each prefix to f32."""
    c = np.empty(fr.shape[0] + 1, f32)
    c[0] = 0
    c[1:] = np.cumsum(fr.astype(f64)).astype(f32)
    return c


def type_unbiased_quantize(x, bits_per_dimension=1, X=None, torch_threads: int = 1,
                           l1=None) -> np.ndarray:
    """Restatement of `Type_unbiased_quantize` (AS:609-641); returns the
    dequantized f32 vector.  `X` is the single U[0,1) draw of AS:634 (passed in)."""
    x = np.asarray(x, dtype=f32).reshape(-1)
    d = x.shape[0]
    m = rate_to_m(bits_per_dimension, d)
    return quantize_with_m(x, m, X, torch_threads, l1)


def quantize_with_m(x: np.ndarray, m: int, X, torch_threads: int = 1, l1=None) -> np.ndarray:
    x = np.asarray(x, dtype=f32).reshape(-1)
    L = l1_torch_order(x, torch_threads) if l1 is None else f32(l1)
    v, fl, fr = fractional_parts(x, m, L)
    c = prefix_c(fr)
    Xf = f32(X)
    with np.errstate(all="ignore"):
        # AS:636-637 crossing test; AS:640 output, left-to-right f32
        diff = np.floor((c[1:] - Xf).astype(f32)) - np.floor((c[:-1] - Xf).astype(f32))
        r = (diff == 1).astype(f32)
        sgn = np.sign(v).astype(f32)
        sgn[np.isnan(v)] = 0           # torch.sign(NaN) == 0
        sgn = sgn + f32(0)             # sign(-0.0) == +0.0 in torch
        out = ((f32(L) * sgn).astype(f32) * (fl + r).astype(f32)).astype(f32) / f32(m)
    return out.astype(f32)


def client_mean(q_rows, n_div) -> np.ndarray:
    """ND:137-138: est = 0; for each client in order: est += q / n (f32 IEEE div, f32 add)."""
    q_rows = [np.asarray(q, dtype=f32) for q in q_rows]
    est = np.zeros_like(q_rows[0])
    nf = f32(n_div)
    for q in q_rows:
        est = (est + (q / nf).astype(f32)).astype(f32)
    return est


def script_nmse(est: np.ndarray, emp_mean: np.ndarray, vec_norm_squared: float,
                num_users: int, num_trials: int = 50) -> float:
    """ND:151-157: torch.norm(est - emp).pow(2) / (num_trials * sum||x||^2 * n), all in f32
    as torch CPU evaluates it: the norm in torch's order (8 interleaved lanes of fma
    accumulation, lanes added in order, tail, f32 sqrt; oracle/uq_eden.py:torch_norm2),
    pow(2) as one f32 multiply, the Python-float denominator rounded to f32."""
    from .uq_eden import torch_norm2
    diff = (np.asarray(est, f32) - np.asarray(emp_mean, f32)).astype(f32)
    nrm = torch_norm2(diff)
    return float(f32(nrm * nrm) / f32(num_trials * vec_norm_squared * num_users))


def quantize_dequantize_batch(x2d: np.ndarray, m: int, X: np.ndarray, torch_threads: int = 1):
    """Batched form: row j uses X[j]."""
    return np.stack([quantize_with_m(x2d[j], m, X[j], torch_threads) for j in range(x2d.shape[0])])


def type_codes(x, m: int, X, torch_threads: int = 1, l1=None):
    """Wire codes of the reference's output (see codes.py): k = fl + r per coordinate
    (AS:630-637), code = k if sign(v) >= 0 else -k-1; overflow if any k > 127 or NaN."""
    x = np.asarray(x, dtype=f32).reshape(-1)
    L = l1_torch_order(x, torch_threads) if l1 is None else f32(l1)
    v, fl, fr = fractional_parts(x, m, L)
    c = prefix_c(fr)
    Xf = f32(X)
    with np.errstate(all="ignore"):
        diff = np.floor((c[1:] - Xf).astype(f32)) - np.floor((c[:-1] - Xf).astype(f32))
        r = (diff == 1).astype(f32)
        k = (fl + r).astype(f32)
    ok = k <= 127
    kk = np.where(ok, k, 127).astype(np.int64)
    code = np.where(v < 0, -kk - 1, kk).astype(np.int8)
    return code, L, bool((~ok).any())
