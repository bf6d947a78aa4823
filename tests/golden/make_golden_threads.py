"""Golden L1 values for AS:624 (`input_vector.abs().sum()`) at many torch intra-op thread
counts, produced by torch itself (the primitive the reference calls; torch 2.10 CPU).

    python tests/golden/make_golden_threads.py   ->  tests/golden/l1_threads.json

Each record holds the generator of x (numpy default_rng(seed).standard_normal(d) * scale,
f32), the thread count T and the f32 bits of torch's result.  torch reduces a vector
with d >= 32768 and T > 1 in two passes (ATen two_pass_reduction): per-thread chunk sums
into a T-element buffer, then the same cascade over that buffer -- these records pin that
second pass for T up to 256 (SURVEY.md §8(a3) covered T = 1, 2, 4, 8)."""
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SIZES = [(1 << 20, 1.0), (1 << 22, 1.0), (3000017, 3.0), (172554, 0.01), (40000, 1e3), (32768, 1.0), (65537, 1.0)]
THREADS = [1, 2, 3, 5, 6, 7, 8, 9, 13, 16, 21, 32, 37, 63, 64, 65, 100, 128, 200, 256]


def gen(seed, d, scale):
    return (np.random.default_rng(seed).standard_normal(d) * scale).astype(np.float32)


def main():
    recs = []
    for i, (d, scale) in enumerate(SIZES):
        seed = 9000 + i
        t = torch.from_numpy(gen(seed, d, scale))
        for T in THREADS:
            torch.set_num_threads(T)
            assert torch.get_num_threads() == T
            v = np.float32(t.abs().sum().item())
            recs.append({"seed": seed, "d": d, "scale": scale, "threads": T,
                         "l1": float(v), "l1_bits": int(v.view(np.uint32))})
    out = {"source": f"torch {torch.__version__} CPU, Tensor.abs().sum() (AS:624)", "records": recs}
    with open(os.path.join(HERE, "l1_threads.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(len(recs), "records")


if __name__ == "__main__":
    main()
