"""Kernel trace of the per-client drop-in (n = 1) at a given d, for rocprofv3 --stats:
    python tools/dropin_prof.py 172554"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import uqdme  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 172554
v = torch.randn(d, device="cuda")
for _ in range(30):
    y = uqdme.Type_unbiased_quantize(v, 1)
torch.cuda.synchronize()
