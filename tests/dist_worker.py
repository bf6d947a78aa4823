"""One rank of the GPU multi-process test (tests/test_gpu_distributed.py).

    python -m tests.dist_worker --rank R --world W --port P --case c1|laplace --out DIR

Every rank builds the same client batch, takes its contiguous block (shard_range), runs the
product path sharded_quantize_mean (HIP quantize + HIP client-ordered fold, distributed.py)
for R = 1 and 2 in modes "ordered" and "reduce", and saves its q block and, on rank 0, est.
The ranks share cuda:0 through the gloo backend (RCCL refuses two ranks on one device);
distributed.py stages gloo's exchanges through host memory."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def case_inputs(case):
    """(x[n, d] f32, X[n] f32): C1 from the reference fixture, or Laplace(1, 2) clients as
    Laplace_dist.py:89 draws them (legacy np.random, seed 42) at d = 2^20 (config C3)."""
    from tests import golden_data as G
    if case == "c1":
        z = G.c1()
        return z["x"].astype(np.float32), {1: z["X1"].astype(np.float32), 2: z["X2"].astype(np.float32)}
    rs = np.random.RandomState(42)
    n, d = 6, 1 << 20
    x = np.stack([rs.laplace(loc=1, scale=2, size=d) for _ in range(n)]).astype(np.float32)
    X = {1: np.random.RandomState(7).random_sample(n).astype(np.float32),
         2: np.random.RandomState(8).random_sample(n).astype(np.float32)}
    return x, X


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--case", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--torch-threads", type=int, default=1)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port))
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    try:
        torch.cuda.set_device(0)
        import uqdme
        x, Xs = case_inputs(a.case)
        n = x.shape[0]
        lo, hi = uqdme.shard_range(n, a.world, a.rank)
        xl = torch.from_numpy(x[lo:hi]).cuda()
        for R in (1, 2):
            for mode in ("ordered", "reduce"):
                est, q = uqdme.sharded_quantize_mean(xl, R, Xs[R][lo:hi], n, mode=mode, dst=0,
                                                     torch_threads=a.torch_threads, return_q=True)
                torch.cuda.synchronize()
                uqdme.check_status()
                np.save(os.path.join(a.out, f"q_{R}_{mode}_{a.rank}.npy"), q.cpu().numpy())
                if a.rank == 0:
                    np.save(os.path.join(a.out, f"est_{R}_{mode}.npy"), est.cpu().numpy())
                dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
