"""DME NMSE harness: the unbiased-type-quantizer slice of the reference drivers
NMSE_Results/Codes/{Normal,Laplace,Gamma,Bernoulli,Lognormal}_dist.py (ND:77-221),
running every quantization and client mean on the HIP path.

Semantics kept from the reference (ND = Normal_dist.py):
  ND:14-15    np.random.seed(seed); torch.manual_seed(seed)   (here: a private CPU
              torch.Generator, so the caller's global RNG is untouched)
  ND:88-91    per instance, n vectors drawn with legacy np.random (f64) -> f32
  ND:94-95    vec_norm_squared = sum ||v||^2 (f64); emp = stack(v).sum(0) / n (f32, torch CPU)
  ND:133-138  per client, in order, every rate: est_R += Q(v, R) / n; one U[0,1) draw per
              call in call order (client-major, rate-minor)
  ND:151-157  NMSE = ||est - emp||^2 / (num_trials * vec_norm_squared * n)   ("script" NMSE,
              scales as 1/n^3); the standard NMSE = script * num_trials * n^2 is also returned
  ND:193-221  max / mean over instances
The reference also calls 12 other schemes in the same loop; they consume the global torch
RNG, so the shipped drivers' X stream differs from this unbiased-only loop (results agree
statistically).
"""
from __future__ import annotations

import numpy as np
import torch

from .quantizer import client_mean, quantize_dequantize

__all__ = ["DISTRIBUTIONS", "draw_vectors", "nmse_simulation", "USERS_ND"]

# ND:43 (also Lognormal_dist.py:43): num_users_list = arange(1, 102, 5); Laplace/Gamma/
# Bernoulli drivers use arange(1, 101, 5).
USERS_ND = tuple(range(1, 102, 5))

# ND:89, Laplace_dist.py:89, Gamma_dist.py:86, Bernoulli_dist.py:90, Lognormal_dist.py:90;
# "uniform" is build-defined (BASELINE.json config C3), not in the reference.
DISTRIBUTIONS = {
    "normal": lambda rs, d: rs.normal(loc=0, scale=1, size=d),
    "laplace": lambda rs, d: rs.laplace(loc=1, scale=2, size=d),
    "gamma": lambda rs, d: rs.gamma(shape=2, scale=2, size=d),
    "bernoulli": lambda rs, d: rs.choice(np.arange(2), size=d, p=[0.3, 0.7]),
    "lognormal": lambda rs, d: rs.lognormal(mean=1, sigma=2, size=d),
    "uniform": lambda rs, d: rs.uniform(low=-1.0, high=1.0, size=d),
}


def draw_vectors(dist: str, n: int, dim: int, rs=np.random):
    """n f64 vectors in the reference's draw order, their ||v||^2 sum, and the f32 batch."""
    gen = DISTRIBUTIONS[dist]
    vecs, norms = [], []
    for _ in range(n):
        v = np.asarray(gen(rs, dim), dtype=np.float64)
        norms.append(np.linalg.norm(v) ** 2)
        vecs.append(v)
    return vecs, float(sum(norms))


def nmse_simulation(dist: str = "normal", dim: int = 2048, users=USERS_ND, num_instances: int = 50,
                    num_trials: int = 50, rates=(1, 2), seed: int = 42, torch_threads: int = 1,
                    device=None):
    """Returns {rate: {"script": [len(users), num_instances] array, "avg", "max",
    "standard_avg", "standard_max"}} with the reference's normalisation."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    rs = np.random.RandomState(seed)                 # legacy stream == np.random.seed(seed)
    gen = torch.Generator().manual_seed(seed)        # == torch.manual_seed(seed) CPU stream
    R = len(rates)
    script = {r: np.zeros((len(users), num_instances), np.float64) for r in rates}
    for ui, n in enumerate(users):
        for inst in range(num_instances):
            vecs, vns = draw_vectors(dist, n, dim, rs)
            xs = torch.stack([torch.as_tensor(v, dtype=torch.float32) for v in vecs])     # ND:91
            emp = xs.sum(dim=0) / n                                                        # ND:95 (CPU)
            X = torch.rand(R * n, generator=gen)                                           # AS:634 draws
            xd = xs.to(device)
            for k, r in enumerate(rates):
                q = quantize_dequantize(xd, r, X=X[k::R], torch_threads=torch_threads)
                est = client_mean(q, n).cpu()
                script[r][ui, inst] = float(torch.norm(est - emp).pow(2) / (num_trials * vns * n))   # ND:155
    out = {}
    for r in rates:
        s = script[r].astype(np.float32)              # the reference stores NMSE in f32 tensors
        std = s.astype(np.float64) * num_trials * np.asarray(users, np.float64)[:, None] ** 2
        out[r] = {"script": s, "avg": s.mean(axis=1), "max": s.max(axis=1),
                  "standard_avg": std.mean(axis=1), "standard_max": std.max(axis=1)}
    return out
