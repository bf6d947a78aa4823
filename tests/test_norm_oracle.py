"""The C oracle's torch.norm (oracle/uq_oracle.c: uqo_torch_norm2, the checker of the GPU's
KE2 / KE2s) against torch.norm itself on CPU and the NumPy restatement (oracle/uq_eden.py),
on the adversarial vectors of tests/norm_cases.py."""
import numpy as np
import torch

from oracle import uq_eden as E
from oracle import uq_oracle_c as C
from tests.norm_cases import norm_cases, same_bits


def test_c_norm_matches_torch_and_numpy_oracle():
    for D in (1, 2, 4, 8, 64, 1024, 16384):   # EDEN pads to powers of two
        for name, v in norm_cases(D):
            t = np.float32(torch.norm(torch.from_numpy(v), 2).item())
            c = C.torch_norm2(v)
            assert same_bits(c, t), (D, name, c, t)
            if D <= 1024:
                assert same_bits(c, E.torch_norm2(v)), (D, name)
