"""cProfile of QUICFL_quantize's host path (one client per call), for the per-call overhead.

    python tools/exp/qfl_host_prof.py [d] [calls]"""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    import uqdme
    from quicfl_tables import write_tables
    uqdme.set_tables_prefix(write_tables(os.path.join(tempfile.mkdtemp(prefix="qfl_tabs_"), "t")))
    v = torch.randn(d, device="cuda")
    for _ in range(5):
        uqdme.QUICFL_quantize(v, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        uqdme.QUICFL_quantize(v, 1)
    print(f"ms_per_call {1e3 * (time.perf_counter() - t0) / k:.4f}")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(k):
        uqdme.QUICFL_quantize(v, 1)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
