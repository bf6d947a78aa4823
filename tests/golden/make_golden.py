"""Generate golden fixtures by running the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports `Type_unbiased_quantize` from /root/reference/NMSE_Results/Codes/All_Schemes.py
(AS:609-641) on torch CPU and records inputs / draws / outputs.  The reference is
never needed afterwards: the fixtures are plain data (npz + json) and the tests only
read them.  Inputs that are large are stored as a generator spec (legacy
np.random.RandomState, stable across numpy versions) plus their sha256.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import warnings

import numpy as np
import torch

warnings.filterwarnings("ignore")
REF = "/root/reference/NMSE_Results/Codes"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import All_Schemes as AS  # noqa: E402  (the reference module)

f32 = np.float32


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gen(spec: dict) -> np.ndarray:
    """Synthetic inputs, mirroring the reference's generators (ND:89, Laplace_dist.py:89,
    Gamma_dist.py:86, Bernoulli_dist.py:90, Lognormal_dist.py:90)."""
    rs = np.random.RandomState(spec["seed"])
    d, kind = spec["d"], spec["dist"]
    if kind == "normal":
        v = rs.normal(loc=0, scale=1, size=d)
    elif kind == "laplace":
        v = rs.laplace(loc=1, scale=2, size=d)
    elif kind == "gamma":
        v = rs.gamma(shape=2, scale=2, size=d)
    elif kind == "bernoulli":
        v = rs.choice(np.arange(2), size=d, p=[0.3, 0.7]).astype(np.float64)
    elif kind == "lognormal":
        v = rs.lognormal(mean=1, sigma=2, size=d)
    else:
        raise ValueError(kind)
    return v.astype(f32)


def ref_call(x: np.ndarray, R, seed: int, threads: int):
    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    X = float(torch.rand(1).item())
    torch.manual_seed(seed)
    out = AS.Type_unbiased_quantize(torch.from_numpy(x.copy()), R).numpy().copy()
    l1 = float(torch.from_numpy(x).abs().sum().item())
    return X, l1, out


def c1_harness():
    """C1: the Normal_dist.py loop (ND:14-15, 88-95, 133-138, 151-157) reduced to the
    unbiased scheme: seed 42, n=16 clients, d=1024, per client R=1 then R=2, 1 thread."""
    torch.set_num_threads(1)
    np.random.seed(42)
    torch.manual_seed(42)
    n, d = 16, 1024
    vecs, norms = [], []
    for _ in range(n):
        v = np.random.normal(loc=0, scale=1, size=d)
        norms.append(np.linalg.norm(v) ** 2)
        vecs.append(torch.as_tensor(v, dtype=torch.float32))
    vec_norm_squared = sum(norms)
    emp = torch.stack(vecs).sum(dim=0) / n
    est1 = torch.zeros(d)
    est2 = torch.zeros(d)
    q1, q2, X1, X2 = [], [], [], []
    for v in vecs:
        st = torch.get_rng_state()
        X1.append(float(torch.rand(1).item()))
        torch.set_rng_state(st)
        a = AS.Type_unbiased_quantize(v, 1)
        st = torch.get_rng_state()
        X2.append(float(torch.rand(1).item()))
        torch.set_rng_state(st)
        b = AS.Type_unbiased_quantize(v, 2)
        q1.append(a.numpy().copy())
        q2.append(b.numpy().copy())
        est1 += torch.as_tensor(a) / n
        est2 += torch.as_tensor(b) / n
    nmse1 = float(torch.norm(est1 - emp).pow(2) / (50 * vec_norm_squared * n))
    nmse2 = float(torch.norm(est2 - emp).pow(2) / (50 * vec_norm_squared * n))
    np.savez_compressed(
        os.path.join(HERE, "c1_harness.npz"),
        x=torch.stack(vecs).numpy(), X1=np.array(X1, f32), X2=np.array(X2, f32),
        q1=np.stack(q1), q2=np.stack(q2), est1=est1.numpy(), est2=est2.numpy(),
        emp=emp.numpy(), vec_norm_squared=np.float64(vec_norm_squared),
        nmse1=np.float64(nmse1), nmse2=np.float64(nmse2))
    print("c1: nmse", nmse1, nmse2)


def edge_cases():
    """Small hand-made vectors exercising the float edge semantics of AS:609-641."""
    tiny = np.float32(1e-30)
    den = np.float32(1e-41)  # subnormal
    cases = {
        "zeros8": np.zeros(8, f32),
        "one_elem": np.array([3.5], f32),
        "one_neg": np.array([-2.0], f32),
        "two": np.array([1.0, -1.0], f32),
        "signed_zeros": np.array([0.0, -0.0, 1.0, -0.0, -2.0, 0.0, 0.5, -0.25], f32),
        "tiny": (np.arange(1, 65, dtype=f32) * tiny),
        "subnormal": np.array([den, -den, 2 * den, 0.0, -3 * den, den], f32),
        "mixed_scale": np.array([1e30, -1e-30, 1.0, -1e10, 3e-5, 0.0, 7.0], f32),
        "nan": np.array([1.0, np.nan, -2.0, 3.0], f32),
        "inf": np.array([1.0, np.inf, -2.0], f32),
        "const_ones": np.ones(1000, f32),
        "bern_like": (np.arange(257) % 3 == 0).astype(f32),
        "ramp": np.linspace(-5, 5, 777).astype(f32),
    }
    rng = np.random.RandomState(1234)
    for d in (5, 9, 31, 33, 63, 65, 127, 129, 513, 1023, 4097):
        cases[f"normal_{d}"] = rng.normal(size=d).astype(f32)
    rates = sorted(AS_rates())
    out = {}
    seed = 1000
    for name, x in cases.items():
        for R in rates if name in ("normal_129", "ramp") else (1, 2):
            seed += 1
            X, l1, q = ref_call(x, R, seed, 1)
            out[f"{name}|{R}"] = (x, R, X, q)
    arrs, meta = {}, []
    for i, (k, (x, R, X, q)) in enumerate(out.items()):
        arrs[f"x{i}"] = x
        arrs[f"q{i}"] = q
        meta.append({"name": k, "R": R, "X": X, "idx": i})
    np.savez_compressed(os.path.join(HERE, "edge_cases.npz"), **arrs)
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print("edge cases:", len(meta))


def AS_rates():
    return [0.5, 1, 1.5, 2, 2.5, 3, 3.5, 4, 4.5, 5, 5.5, 6, 6.5, 7, 7.5, 8, 8.5, 9, 9.5, 10]


def spec_vectors():
    """Mid/large vectors: inputs regenerated from a spec; outputs stored (mid) or hashed (large)."""
    specs = []
    s = 0
    for dist in ("normal", "laplace", "gamma", "bernoulli", "lognormal"):
        for d in (1000, 4099, 65537, 172554):
            for R in (1, 2):
                s += 1
                specs.append({"dist": dist, "d": d, "seed": 100 + s, "R": R, "threads": 1})
    for d, T in ((65537, 8), (172554, 8), (122626, 4)):
        s += 1
        specs.append({"dist": "normal", "d": d, "seed": 100 + s, "R": 1, "threads": T})
    for dist in ("normal", "laplace"):
        for R in (1, 2):
            for T in (1, 8):
                s += 1
                specs.append({"dist": dist, "d": 1 << 20, "seed": 100 + s, "R": R, "threads": T, "large": True})
    s += 1
    specs.append({"dist": "normal", "d": 1 << 22, "seed": 100 + s, "R": 1, "threads": 1, "large": True})
    arrs = {}
    for i, sp in enumerate(specs):
        x = gen(sp)
        X, l1, q = ref_call(x, sp["R"], 5000 + i, sp["threads"])
        sp.update({"X": X, "l1": l1, "x_sha256": sha(x), "q_sha256": sha(q), "idx": i})
        if not sp.get("large"):
            arrs[f"q{i}"] = q
        else:
            rs = np.random.RandomState(i)
            pos = np.sort(rs.choice(sp["d"], 4096, replace=False))
            arrs[f"pos{i}"] = pos.astype(np.int64)
            arrs[f"qs{i}"] = q[pos]
        print("spec", i, sp["dist"], sp["d"], sp["R"], sp["threads"], flush=True)
    np.savez_compressed(os.path.join(HERE, "spec_vectors.npz"), **arrs)
    with open(os.path.join(HERE, "spec_vectors.json"), "w") as f:
        json.dump(specs, f, indent=0)


def nd_nmse_points():
    """Known answers from the full ND loop restricted to the unbiased scheme (dim=2048,
    num_trials=50), n in {1, 6, 11}, 4 instances each, seed 42 for numpy and torch."""
    torch.set_num_threads(1)
    res = {}
    for dist in ("normal", "laplace"):
        np.random.seed(42)
        torch.manual_seed(42)
        rows = []
        for n in (1, 6, 11):
            for inst in range(4):
                vecs, norms = [], []
                for _ in range(n):
                    v = (np.random.normal(0, 1, 2048) if dist == "normal"
                         else np.random.laplace(loc=1, scale=2, size=2048))
                    norms.append(np.linalg.norm(v) ** 2)
                    vecs.append(torch.as_tensor(v, dtype=torch.float32))
                vns = sum(norms)
                emp = torch.stack(vecs).sum(dim=0) / n
                e1 = torch.zeros(2048)
                e2 = torch.zeros(2048)
                for v in vecs:
                    e1 += torch.as_tensor(AS.Type_unbiased_quantize(v, 1)) / n
                    e2 += torch.as_tensor(AS.Type_unbiased_quantize(v, 2)) / n
                rows.append({"n": n, "inst": inst,
                             "nmse1": float(torch.norm(e1 - emp).pow(2) / (50 * vns * n)),
                             "nmse2": float(torch.norm(e2 - emp).pow(2) / (50 * vns * n))})
        res[dist] = rows
    with open(os.path.join(HERE, "nd_nmse_points.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("nd points done")


if __name__ == "__main__":
    c1_harness()
    edge_cases()
    nd_nmse_points()
    spec_vectors()
