"""QUICFL_quantize at one size, K calls (for rocprofv3 kernel traces / PMC passes).

    python tools/exp/qfl_dropin_loop.py [d] [K]"""
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import uqdme
    from quicfl_tables import write_tables
    uqdme.set_tables_prefix(write_tables(os.path.join(tempfile.mkdtemp(prefix="qfl_tabs_"), "t")))
    v = torch.randn(d, device="cuda")
    for _ in range(k):
        uqdme.QUICFL_quantize(v, 1)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
