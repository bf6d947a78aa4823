"""How torch.dot (AS:335, EDEN's scale) sums on this host's CPU: summation-order probing.

    python tools/dot_order_probe.py [n]

torch 2.10's CPU dot goes to MKL's sdot.  With x_i = M, x_j = -M (M = 2^60) and every other
x = 1, y = 1, the ones added into a partial sum holding M before M meets -M are absorbed, so
n - dot(x, y) is the number of leaves under the lowest common ancestor of i and j in the
summation tree (the method of FPRev).  Printed for i = 0 and i = n - 1 against every j; for
n = 64 / 65 / 128 the pattern reads: 64-element blocks split into 4 accumulators of 16
lanes, (acc0 + acc1) + (acc2 + acc3), then lanes i + (i + 8), i + (i + 4), (0 + 1) + (2 + 3);
blocks accumulate sequentially (fma); a ragged tail goes into acc0.  oracle/uq_eden.py
torch_dot restates it; tests/golden/dot_vectors.* pins it on random vectors up to 2^22.
"""
import sys

import numpy as np
import torch

torch.set_num_threads(1)
M = np.float32(2.0 ** 60)


def lca_size(n, i, j):
    x = np.ones(n, np.float32)
    x[i], x[j] = M, -M
    return n - int(torch.dot(torch.from_numpy(x), torch.from_numpy(np.ones(n, np.float32))).item())


def main():
    for n in ([int(sys.argv[1])] if len(sys.argv) > 1 else [64, 65, 128]):
        print(n, "S(0, j), j = 1..:", [lca_size(n, 0, j) for j in range(1, n)])
        print(n, "S(n-1, j), j = 0..:", [lca_size(n, n - 1, j) for j in range(n - 1)])


if __name__ == "__main__":
    main()
