"""GPU, several processes: the client-sharded product path (distributed.py)
with the HIP quantizer and the HIP client-ordered fold in every rank.

2, 4 or 8 ranks share cuda:0 over gloo (tests/dist_worker.py; RCCL refuses two ranks on one
device, and the driver's 8-GPU bench covers RCCL).  Against the single-process path on the
same clients (quantize_dequantize + client_mean, ND:133-138):
  * every rank's q block is bit-identical to the single-process rows;
  * mode "ordered" gives est bit-identical to the sequential client-ordered sum;
  * mode "reduce" (one reduce of per-rank partial means) gives the script NMSE within 1e-6
    relative (north_star tolerance).
Cases: C1 (16 x 1024, the reference fixture's clients and draws) and Laplace(1, 2) clients at
d = 2^20 (config C3's distribution, Laplace_dist.py:89)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from tests.dist_worker import case_inputs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(case, world, out):
    port = _port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, "-m", "tests.dist_worker", "--rank", str(r), "--world", str(world),
                               "--port", str(port), "--case", case, "--out", out], cwd=ROOT, env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs


# (case, world): world 4 splits C1's 16 clients 4 ways; world 8 rehearses the 8-GPU node's
# sharding with 6 Laplace clients, so two ranks hold no client (their partial mean is zeros
# and the ordered chain passes their blocks through unchanged)
@pytest.mark.parametrize("case,world", [("c1", 2), ("laplace", 2), ("c1", 4), ("laplace", 8)])
def test_ranks_share_gpu_product_path(gpu_ready, tmp_path, case, world):
    import uqdme
    from uqdme_amd.distributed import shard_range
    _launch(case, world, str(tmp_path))
    x, Xs = case_inputs(case)
    n = x.shape[0]
    emp = (x.sum(axis=0, dtype=np.float32) / np.float32(n)).astype(np.float32)
    vns = float(np.sum(x.astype(np.float64) ** 2))
    xt = torch.from_numpy(x).cuda()
    for R in (1, 2):
        q_ref = uqdme.quantize_dequantize(xt, R, X=Xs[R], torch_threads=1)
        est_ref = uqdme.client_mean(q_ref, float(n)).cpu().numpy()
        q_ref = q_ref.cpu().numpy()
        nmse_ref = O.script_nmse(est_ref, emp, vns, n)
        for mode in ("ordered", "reduce"):
            for r in range(world):
                lo, hi = shard_range(n, world, r)
                q = np.load(tmp_path / f"q_{R}_{mode}_{r}.npy")
                assert np.array_equal(q.view(np.uint32), q_ref[lo:hi].view(np.uint32)), (case, R, mode, r)
            est = np.load(tmp_path / f"est_{R}_{mode}.npy")
            if mode == "ordered":
                assert np.array_equal(est.view(np.uint32), est_ref.view(np.uint32)), (case, R)
            else:
                nmse = O.script_nmse(est, emp, vns, n)
                assert abs(nmse - nmse_ref) <= 1e-6 * nmse_ref, (case, R, nmse, nmse_ref)
