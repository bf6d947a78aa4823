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


class CpuPipe:
    """torch-CPU stand-in for DMEPipeline (test infrastructure): q = a fixed function of x
    (the quantizer is not what these tests check), est (+)= q[j] / n_div in client order."""

    def __init__(self, n, d):
        self.q = torch.zeros(n, d)
        self.est = torch.zeros(d)
        self.fold = cpu_fold

    def step(self, x, X, n_div, accumulate=False, *, est=None, events=None, pipeline=None):
        self.q.copy_(torch.round(x * 4) / 4 + X[:, None])
        out = self.est if est is None else est
        out.copy_(cpu_fold(self.q, n_div, None))
        return out

    def probe_outputs(self, *a, **k):
        return None

    def check_status(self):
        pass


def _sharded_dme_worker(rank, world, port, n_total, d, mode, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from uqdme_amd.distributed import ShardedDME
        lo, hi = shard_range(n_total, world, rank)
        sh = ShardedDME(hi - lo, d, n_total, mode=mode, pipe=CpuPipe(hi - lo, d), block=64)
        assert not sh.overlap and sh.world == world
        for k in range(3):                                   # three rounds, new clients each
            g = torch.Generator().manual_seed(100 + k)
            x = torch.randn(n_total, d, generator=g)
            X = torch.rand(n_total, generator=g)
            est = sh.step(x[lo:hi].contiguous(), X[lo:hi].contiguous())
            sh.drain()
            if rank == 0:
                np.save(os.path.join(outdir, f"est_{k}.npy"), est.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,n_total", [(2, "reduce", 11), (2, "ordered", 11), (3, "ordered", 11),
                                                (3, "reduce", 2), (3, "ordered", 2)])
def test_sharded_dme_protocol_multi_rank(world, mode, n_total):
    """ShardedDME (the object bench.py --gpus N drives) at world 2-3 over gloo on CPU: each
    rank folds its contiguous client block, then one reduce (f32 re-association only) or the
    ordered chain (bit-identical to the sequential client-ordered mean), over three steps;
    with fewer clients than ranks a rank holds none."""
    d = 300
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_sharded_dme_worker, args=(world, free_port(), n_total, d, mode, td), nprocs=world, join=True)
        for k in range(3):
            got = np.load(os.path.join(td, f"est_{k}.npy"))
            g = torch.Generator().manual_seed(100 + k)
            x = torch.randn(n_total, d, generator=g)
            X = torch.rand(n_total, generator=g)
            ref = cpu_fold(torch.round(x * 4) / 4 + X[:, None], float(n_total), None).numpy()
            if mode == "ordered":
                assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
            else:
                np.testing.assert_allclose(got, ref, rtol=0, atol=8 * np.finfo(np.float32).eps * np.abs(ref).max())
