"""Multi-process (gloo, CPU) tests of the client-sharded mean protocol used on GPUs
(distributed.py).  The per-rank fold is a plain torch-CPU restatement of ND:137-138
here (test infrastructure); on GPUs it is the HIP client-mean kernel."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import uqdme  # noqa: F401  (registers uqdme_amd)
from uqdme_amd.distributed import shard_range, sharded_client_mean


def cpu_fold(q, n_div, est):
    """est (+)= q[j] / n_div for rows in order, f32 (ND:137-138)."""
    out = torch.zeros(q.shape[1], dtype=torch.float32) if est is None else est
    nd = torch.tensor(n_div, dtype=torch.float32)
    for j in range(q.shape[0]):
        out.add_(q[j] / nd)
    return out


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, d, mode, dst, block, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(5)
        q_all = torch.randn(n_total, d, generator=g)
        lo, hi = shard_range(n_total, world, rank)
        est = sharded_client_mean(q_all[lo:hi].contiguous(), float(n_total), mode=mode, dst=dst,
                                  block=block, fold=cpu_fold)
        if rank == dst:
            np.save(os.path.join(outdir, "est.npy"), est.numpy())
    finally:
        dist.destroy_process_group()


def run(world, n_total, d, mode, dst=0, block=64):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, free_port(), n_total, d, mode, dst, block, td), nprocs=world, join=True)
        return np.load(os.path.join(td, "est.npy"))


def reference(n_total, d):
    g = torch.Generator().manual_seed(5)
    q_all = torch.randn(n_total, d, generator=g)
    return cpu_fold(q_all, float(n_total), None).numpy()


def test_shard_range_partitions_in_order():
    for n in (0, 1, 7, 1024, 8192, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


@pytest.mark.parametrize("world,dst", [(2, 0), (3, 0), (3, 2)])
def test_ordered_mean_is_bit_identical_to_sequential(world, dst):
    n_total, d = 7, 300
    got = run(world, n_total, d, "ordered", dst=dst, block=64)
    ref = reference(n_total, d)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_reduce_mean_matches_within_f32_rounding():
    n_total, d = 9, 500
    got = run(2, n_total, d, "reduce")
    ref = reference(n_total, d)
    np.testing.assert_allclose(got, ref, rtol=0, atol=8 * np.finfo(np.float32).eps * np.abs(ref).max())
