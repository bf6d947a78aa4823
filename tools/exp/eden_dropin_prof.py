"""Kernel trace of the per-call EDEN drop-in (n = 1, d = 2^20), for rocprofv3 --stats."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uqdme  # noqa: E402
v = torch.randn(1 << 20, device="cuda")
for _ in range(20):
    y = uqdme.EDEN_quantize_Hadamard(v, 1)
torch.cuda.synchronize()
