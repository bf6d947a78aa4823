"""Kernel trace of a per-client drop-in (n = 1) at a given d, for rocprofv3 --stats:
    python tools/dropin_prof.py 172554 [Type_unbiased_quantize | Type_biased_quantize | EDEN_quantize_Hadamard]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import uqdme  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 172554
f = getattr(uqdme, sys.argv[2] if len(sys.argv) > 2 else "Type_unbiased_quantize")
v = torch.randn(d, device="cuda")
for _ in range(30):
    y = f(v, 1)
torch.cuda.synchronize()
