"""Vectors for torch.norm's 8-lane fma order (AS:329, the EDEN sender's norm) that stress the
segmented chains of KE2s (uq_eden_kernels.h): binade crossings at every scale, exact ties
(few mantissa bits), subnormal and overflowing sums, zero runs (EDEN's padding), spikes,
NaN / Inf.  Shared by the oracle test (CPU) and the GPU parity test."""
from __future__ import annotations

import numpy as np

f32 = np.float32


def norm_cases(D: int, seed: int = 0):
    rng = np.random.default_rng(seed + D)
    z = lambda: np.zeros(D, f32)  # noqa: E731
    g = rng.standard_normal(D).astype(f32)
    cases = [("normal", g)]
    cases.append(("normal_1e-18", (g * f32(1e-18)).astype(f32)))      # squares subnormal / tiny sums
    cases.append(("normal_1e15", (g * f32(1e15)).astype(f32)))        # large, finite sums
    cases.append(("normal_3e18", (g * f32(3e18)).astype(f32)))        # the sum overflows to inf
    odd = ((2 * rng.integers(0, 1024, D) + 1) * rng.choice([-1, 1], D)).astype(f32)
    cases.append(("odd_ties", (odd * f32(2.0 ** -10)).astype(f32)))   # x^2 has bits at 2^-20: ties from acc >= 16
    cases.append(("half_ints", (rng.integers(-40, 40, D) + f32(0.5)).astype(f32)))
    cases.append(("ones", np.where(rng.random(D) < 0.5, f32(1), f32(-1)).astype(f32)))
    cases.append(("subnormal", (rng.standard_normal(D) * 1e-40).astype(f32)))
    cases.append(("zeros", z()))
    pad = g.copy()
    pad[D // 3:] = 0                                                 # EDEN's zero padding
    cases.append(("zero_tail", pad))
    lead = g.copy()
    lead[:D // 2] = 0
    cases.append(("zero_head", lead))
    one = z()
    one[(D // 2 + 3) % D] = f32(1.75)
    cases.append(("single", one))
    sp = g.copy()
    sp[rng.integers(0, D, 6)] = f32(1e10)                             # abrupt jumps across binades
    cases.append(("spikes", sp))
    ramp = (np.arange(D, dtype=np.float64) / D * rng.standard_normal(D)).astype(f32)
    cases.append(("ramp", ramp))
    nan = g.copy()
    nan[D // 5] = np.nan
    cases.append(("nan", nan))
    inf = g.copy()
    inf[max(0, D - 9)] = -np.inf
    cases.append(("inf", inf))
    return cases


def same_bits(a, b) -> bool:
    a, b = np.float32(a), np.float32(b)
    return bool((np.isnan(a) and np.isnan(b)) or a.view(np.uint32) == b.view(np.uint32))
