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

    def __init__(self, n, d, pipeline="codes"):
        self.q = torch.zeros(n, d)
        self.est = torch.zeros(d)
        self.fold = cpu_fold
        self.pipeline = pipeline
        self.means = 0

    def step(self, x, X, n_div, accumulate=False, *, est=None, events=None, pipeline=None, mean=True):
        self.q.copy_(torch.round(x * 4) / 4 + X[:, None])
        if not mean:
            return None
        self.means += 1
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
        if mode == "ordered":
            assert sh.pipe.means == 0                         # the chain folds q; no wasted mean kernel
            with pytest.raises(ValueError):                  # an encode step writes no q to fold
                sh.step(x[lo:hi].contiguous(), X[lo:hi].contiguous(), pipeline="encode")
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


def _overlap_worker(rank, world, port, n_total, d, steps, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from uqdme_amd.distributed import ShardedDME
        lo, hi = shard_range(n_total, world, rank)
        got = {}
        sh = ShardedDME(hi - lo, d, n_total, mode="reduce", pipe=CpuPipe(hi - lo, d), overlap=True,
                        on_complete=lambda k, est: got.__setitem__(k, est.clone()))
        ref = ShardedDME(hi - lo, d, n_total, mode="reduce", pipe=CpuPipe(hi - lo, d), overlap=False)
        assert sh.overlap and len(sh.est_bufs) == 2 and not ref.overlap
        sync = []
        bufs = []
        for k in range(steps):                              # step k >= 2 reuses step k-2's buffer
            g = torch.Generator().manual_seed(300 + k)
            x = torch.randn(n_total, d, generator=g)
            X = torch.rand(n_total, generator=g)
            est = sh.step(x[lo:hi].contiguous(), X[lo:hi].contiguous())
            bufs.append(est.data_ptr())
            if k >= 2:
                assert k - 2 in got                         # reduce k-2 completed before its buffer was reused
            sync.append(ref.step(x[lo:hi].contiguous(), X[lo:hi].contiguous()).clone())
        sh.drain()
        assert sorted(got) == list(range(steps)) and all(s is None for s in sh.pending)
        assert bufs[0] == bufs[2] and bufs[1] == bufs[3] and bufs[0] != bufs[1]
        if rank == 0:
            for k in range(steps):
                np.save(os.path.join(outdir, f"ov_{k}.npy"), got[k].numpy())
                np.save(os.path.join(outdir, f"sy_{k}.npy"), sync[k].numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 9), (3, 10)])
def test_sharded_dme_overlapped_reduce_multi_rank(world, n_total):
    """The two-buffer asynchronous reduce ShardedDME uses over RCCL (bench --gpus N), run with
    gloo's async reduce on host tensors at world 2-3 over five steps: every step's est on dst
    (taken by on_complete when its reduce is waited for, before step k+2 reuses the buffer)
    equals the synchronous path's bit for bit (Normal_dist.py:137-138 per round)."""
    d, steps = 257, 5
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_overlap_worker, args=(world, free_port(), n_total, d, steps, td), nprocs=world, join=True)
        for k in range(steps):
            ov = np.load(os.path.join(td, f"ov_{k}.npy"))
            sy = np.load(os.path.join(td, f"sy_{k}.npy"))
            assert np.array_equal(ov.view(np.uint32), sy.view(np.uint32)), k
