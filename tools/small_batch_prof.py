"""Kernel-by-kernel timing of the small-batch K2 forms (run under rocprofv3 --kernel-trace
--stats): n clients x d = 2^20, q + codes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import uqdme
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
d = 1 << 20
x = torch.randn(n, d, device="cuda")
X = uqdme.draw_uniforms(n, torch.Generator().manual_seed(1))
for _ in range(20):
    tc = uqdme.quantize_encode(x, 1, X=X, torch_threads=1, return_q=True)
torch.cuda.synchronize()
