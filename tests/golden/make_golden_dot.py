"""Golden vectors for torch.dot on CPU f32 (AS:335, EDEN's scale = ||v||^2 / dot(c[bins], v)):
torch.dot's own output bits here (torch 2.10, oneMKL 2024.2 sdot, one thread), for the oracle's
order model (oracle/uq_eden.py torch_dot, oracle/uq_oracle.c uqo_torch_dot) and the GPU's
(eden_dot_kernel).  Inputs are regenerated from seeds (numpy PCG64) and their SHA-256 is
recorded so a change of the generator is caught.

    python tests/golden/make_golden_dot.py
"""
import hashlib
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def inputs(kind, n, seed):
    """(x, y) f32: 'normal' N(0,1) pairs; 'eden' centroid-like x = +-0.798 by sign of y, the
    products of EDEN's 1-bit scale; 'wide' magnitudes over 2^-20 .. 2^20 (roundings in every
    add); 'cancel' alternating large +-, small values between (order-sensitive)."""
    rng = np.random.default_rng(seed)
    y = rng.standard_normal(n)
    if kind == "normal":
        x = rng.standard_normal(n)
    elif kind == "eden":
        x = np.where(y > 0, 0.7978845608028654, -0.7978845608028654)
    elif kind == "wide":
        x = rng.standard_normal(n) * np.exp2(rng.integers(-20, 21, n))
    elif kind == "cancel":
        x = np.where(np.arange(n) % 2 == 0, 1e6, -1e6) * (1 + rng.standard_normal(n) * 1e-3)
        x[rng.random(n) < 0.3] *= 1e-8
    else:
        raise ValueError(kind)
    return x.astype(np.float32), y.astype(np.float32)


def cases():
    out = []
    s = 100
    for k in range(0, 23):
        for kind in (("normal", "eden", "wide", "cancel") if k <= 20 else ("normal", "eden")):
            out.append((kind, 1 << k, s))
            s += 1
    for n in list(range(1, 130)) + [191, 200, 255, 1000, 4097, 65537 + 33, 100003]:
        out.append(("normal", n, s))
        s += 1
    return out


def main():
    torch.set_num_threads(1)
    res = []
    for kind, n, seed in cases():
        x, y = inputs(kind, n, seed)
        r = np.float32(torch.dot(torch.from_numpy(x), torch.from_numpy(y)).item())
        res.append({"kind": kind, "n": n, "seed": seed, "dot_bits": int(r.view(np.uint32)),
                    "in_sha": hashlib.sha256(x.tobytes() + y.tobytes()).hexdigest()[:16]})
    json.dump({"torch": torch.__version__, "threads": 1, "cases": res},
              open(os.path.join(HERE, "dot_vectors.json"), "w"), indent=0)
    print(len(res), "cases")


if __name__ == "__main__":
    main()
