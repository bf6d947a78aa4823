"""Search seeds of tests.scan_models.tiny_mix on which the round-1 tree scan would give
different outputs (run offline; the seeds go into tests/test_gpu_exact_scan.py)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import uq_oracle as O, uq_oracle_c as C
from tests import scan_models as S
d = int(sys.argv[1]); R = float(sys.argv[2]); nseeds = int(sys.argv[3]); mix = float(sys.argv[4]) if len(sys.argv) > 4 else 0.5
m = O.rate_to_m(R if R != int(R) else int(R), d)
found = []
for seed in range(nseeds):
    x = S.tiny_mix(seed, d, mix)
    X, i = S.exposing_X(x, m)
    if X is None:
        continue
    q, _ = C.quantize_batch(x[None], m, np.array([X], np.float32), 1)
    print(f"seed {seed}: prefix {i} differs, X = {float(X)!r}", flush=True)
    found.append((seed, float(X), i))
print(found)
