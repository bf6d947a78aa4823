"""cProfile of EDEN_quantize_Hadamard and Type_biased_quantize at d = 2048 (host-side cost per call)."""
import cProfile
import os
import pstats
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import uqdme  # noqa: E402
from quicfl_tables import write_tables  # noqa: E402

v = torch.randn(2048, device="cuda")
for F in (uqdme.EDEN_quantize_Hadamard, uqdme.Type_biased_quantize):
  print("=====", F.__name__)
  for _ in range(5):
      F(v, 1)
  torch.cuda.synchronize()
  pr = cProfile.Profile()
  pr.enable()
  for _ in range(200):
      F(v, 1)
  pr.disable()
  pstats.Stats(pr).sort_stats("tottime").print_stats(18)
