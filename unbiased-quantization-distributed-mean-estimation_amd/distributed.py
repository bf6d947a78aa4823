"""Client-sharded DME across the GPUs of one node (one process per GPU).

The reference runs single-process: est += Q(v)/n over clients in order
(NMSE_Results/Codes/Normal_dist.py:133-138).  Clients are independent up to that
mean, so they shard across ranks with no data-path collective; the only exchange
is the final mean:

  mode="reduce"   each rank folds its clients (a contiguous block, in client order)
                  into a partial est, then ONE reduce(SUM) of d floats to `dst`
                  (RCCL over xGMI with the nccl backend).  The cross-rank sum
                  re-associates f32 adds, so est differs from the single-process
                  sequential sum in the last bits (NMSE impact ~1e-8 relative).
  mode="ordered"  bit-identical to the single-process sequential sum: ranks form a
                  chain over column blocks of est.  Rank r receives block b from
                  rank r-1, continues the client-ordered sum with its own clients,
                  forwards it to rank r+1; blocks pipeline, so every rank works on
                  a different block at once.  The last rank ends up with the whole
                  est and sends it to `dst`.

The per-rank compute is injected (`fold`), so the protocol runs unchanged on the
gloo backend in CPU tests; on GPUs `fold` defaults to the HIP client-mean kernel.
With a non-RCCL backend (gloo) and device tensors, every exchange is staged through host
memory (gloo's point-to-point ops take host tensors); that is how several ranks sharing
one GPU test the HIP path, while the product path on a node is RCCL with no staging.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

Fold = Callable[[torch.Tensor, float, Optional[torch.Tensor]], torch.Tensor]


def shard_range(n_total: int, world: int, rank: int) -> tuple:
    """Contiguous client block of `rank`: sizes differ by at most one, in rank order."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) != "nccl"


def _reduce(est, dst, group):
    if _staged(est, group):
        h = est.cpu()
        dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM, group=group)
        if dist.get_rank(group) == dst:
            est.copy_(h)
    else:
        dist.reduce(est, dst=dst, op=dist.ReduceOp.SUM, group=group)


def _recv(t, src, group):
    if _staged(t, group):
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.recv(t, src=src, group=group)


def _isend(t, dst, group):
    """Returns (work, buffer): the buffer must live until the work completes."""
    buf = t.cpu() if _staged(t, group) else t
    return dist.isend(buf, dst=dst, group=group), buf


def _default_fold(q: torch.Tensor, n_div: float, est: Optional[torch.Tensor]) -> torch.Tensor:
    from .quantizer import client_mean
    if est is None:
        return client_mean(q, n_div)
    return client_mean(q, n_div, est=est, accumulate=True)


def sharded_client_mean(q_local: torch.Tensor, n_div: float, *, mode: str = "reduce", dst: int = 0,
                        block: int = 1 << 18, group=None, fold: Optional[Fold] = None) -> Optional[torch.Tensor]:
    """Global client mean of the per-rank quantized blocks q_local[n_local, d].

    Returns est[d] on `dst` (and the partial/None elsewhere)."""
    fold = fold or _default_fold
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_local, d = q_local.shape
    if mode == "reduce":
        if n_local:
            est = fold(q_local, n_div, None)
        else:
            est = torch.zeros(d, dtype=torch.float32, device=q_local.device)
        if world > 1:
            _reduce(est, dst, group)
        return est if rank == dst else None
    if mode != "ordered":
        raise ValueError("mode must be 'reduce' or 'ordered'")
    est = torch.zeros(d, dtype=torch.float32, device=q_local.device)
    pending = []
    for c0 in range(0, d, block):
        c1 = min(d, c0 + block)
        blk = est[c0:c1]
        if rank > 0:
            _recv(blk, rank - 1, group)
        if n_local:
            fold(q_local[:, c0:c1], n_div, blk)       # continues the client-ordered sum in place
        if rank < world - 1:
            pending.append(_isend(blk, rank + 1, group))
    for work, _buf in pending:
        work.wait()
    last = world - 1
    if dst != last:
        if rank == last:
            dist.send(est.cpu() if _staged(est, group) else est, dst=dst, group=group)
        elif rank == dst:
            _recv(est, last, group)
    return est if rank == dst else None


class ShardedDME:
    """One rank's share of the client-sharded DME step on a node (the path bench.py times).

        sh = ShardedDME(n_local, d, n_total, bits_per_dimension=1, mode="reduce")
        sh.probe_outputs(x_local, X_local)          # optional, once (pipeline.py)
        est = sh.step(x_local, X_local)             # K1 -> K2 (q + codes) -> K3c -> reduce
        sh.drain()                                  # every pending reduce done; est valid on dst

    The rank quantizes its contiguous client block with a resident DMEPipeline (no data-path
    collective) and folds it into a partial mean over n_total, then:
      mode "reduce":  ONE reduce(SUM) of d floats to `dst` (RCCL over xGMI).  With RCCL and
                      overlap=True (the default there) the reduce of step k is issued
                      asynchronously and runs beside step k+1's kernels: two estimate buffers
                      alternate, and step k+2 waits (stream-ordered, the host does not block)
                      for reduce k before it overwrites that buffer.  est of step k is valid on
                      `dst` once reduce k is waited for: at step k+2, or drain().  on_complete(k,
                      est) is called right then (before the buffer is reused), so a caller can
                      take every step's estimate (copies enqueued there are stream-ordered after
                      the reduce).
      mode "ordered": the bit-exact chain of sharded_client_mean over q's column blocks
                      (the pipeline must write q; its own mean kernel is skipped).
    With gloo and device tensors (ranks sharing one GPU) the reduce is host-staged and
    synchronous; with gloo and host tensors (the CPU tests' stand-in pipeline) overlap=True runs
    the same two-buffer protocol with gloo's async reduce.
    `pipe` replaces the HIP pipeline by any object with its interface (est, q, step(x, X,
    n_div, est=, events=, pipeline=), probe_outputs, check_status): the CPU multi-process
    tests run this protocol with a torch-CPU stand-in."""

    def __init__(self, n_local: int, d: int, n_total: int, bits_per_dimension=1, *, m: int | None = None,
                 torch_threads: int = 1, pipeline: str = "codes", mode: str = "reduce", dst: int = 0, group=None,
                 overlap: Optional[bool] = None, block: int = 1 << 18, device=None, pipe=None,
                 on_complete: Optional[Callable[[int, torch.Tensor], None]] = None):
        if mode not in ("reduce", "ordered"):
            raise ValueError("mode must be 'reduce' or 'ordered'")
        if mode == "ordered" and pipeline == "encode":
            raise ValueError("mode 'ordered' folds q: use pipeline 'codes' or 'q'")
        if pipe is None:
            from .pipeline import DMEPipeline
            pipe = DMEPipeline(n_local, d, bits_per_dimension, m=m, torch_threads=torch_threads, pipeline=pipeline,
                               device=device)
        self.pipe = pipe
        self.n_total, self.mode, self.dst, self.group, self.block = int(n_total), mode, int(dst), group, int(block)
        self.dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist_on else 1
        self.rank = dist.get_rank(group) if self.dist_on else 0
        rccl = self.dist_on and dist.get_backend(group) == "nccl"
        host_gloo = self.dist_on and not rccl and not self.pipe.est.is_cuda      # async gloo on host tensors
        self.overlap = bool(rccl and mode == "reduce" and self.world > 1 if overlap is None else overlap)
        if self.overlap and not ((rccl or host_gloo) and mode == "reduce"):
            raise ValueError("overlap needs mode 'reduce' and RCCL (or gloo with host tensors)")
        self.est_bufs = [self.pipe.est, torch.empty_like(self.pipe.est)] if self.overlap else [self.pipe.est]
        self.fold = getattr(pipe, "fold", None)          # ordered chain's per-rank fold (default: HIP)
        self.pending = [None] * len(self.est_bufs)
        self.pending_step = [None] * len(self.est_bufs)
        self.on_complete = on_complete
        self.nstep = 0

    def _complete(self, slot):
        self.pending[slot].wait()
        self.pending[slot] = None
        k, self.pending_step[slot] = self.pending_step[slot], None
        if self.on_complete is not None:
            self.on_complete(k, self.est_bufs[slot])

    def probe_outputs(self, x_local, X_local, **kw):
        return self.pipe.probe_outputs(x_local, X_local, **kw)

    def step(self, x_local, X_local, *, events=None, pipeline: Optional[str] = None):
        """Returns this step's est buffer (the global mean on `dst` once its reduce is done:
        immediately unless overlap; None off `dst` in mode "ordered")."""
        pl = pipeline or getattr(self.pipe, "pipeline", None)
        if self.mode == "ordered" and self.world > 1 and pl == "encode":
            raise ValueError("mode 'ordered' folds q: an 'encode' step writes no q")
        slot = self.nstep % len(self.est_bufs)
        k = self.nstep
        self.nstep += 1
        est = self.est_bufs[slot]
        if self.pending[slot] is not None:            # reduce of step k-2 still owns this buffer
            self._complete(slot)
        ev = list(events or (None,) * 5)
        ordered = self.mode == "ordered" and self.world > 1
        self.pipe.step(x_local, X_local, float(self.n_total), est=est, events=ev[:4], pipeline=pipeline,
                       mean=not ordered)
        if self.world > 1 or self.overlap:            # (overlap at world 1: RCCL's no-op reduce, tests)
            if self.mode == "reduce":
                if self.overlap:
                    self.pending[slot] = dist.reduce(est, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group,
                                                     async_op=True)
                    self.pending_step[slot] = k
                else:
                    _reduce(est, self.dst, self.group)
            else:
                est = sharded_client_mean(self.pipe.q, float(self.n_total), mode="ordered", dst=self.dst,
                                          block=self.block, group=self.group, fold=self.fold)
        if ev[4] is not None:
            ev[4].record()
        return est if (self.rank == self.dst or self.mode == "reduce") else None

    def drain(self):
        """Wait (stream-ordered) for every pending reduce."""
        order = sorted((k, i) for i, k in enumerate(self.pending_step) if k is not None)
        for _, i in order:                            # oldest first, so on_complete sees steps in order
            self._complete(i)

    def check_status(self):
        self.pipe.check_status()


def sharded_quantize_mean(x_local: torch.Tensor, bits_per_dimension, X_local, n_total: int, *,
                          mode: str = "reduce", dst: int = 0, torch_threads: int = 1, group=None,
                          return_q: bool = False):
    """Quantize this rank's clients (HIP) and form the global client mean: one ShardedDME
    step (K1 -> K2 writing q -> client mean of q -> one reduce, or the ordered chain), with
    buffers allocated for this call (no placement probe; the same est bits as the codes
    pipeline, without writing codes a one-shot caller never reads).

    x_local = the rank's contiguous client block (see shard_range); X_local = its
    slice of the per-client uniforms drawn once for all clients."""
    from .quantizer import _as_device_f32_2d, _device
    dev = _device()
    x_local = _as_device_f32_2d(x_local, dev)
    n_local, d = x_local.shape
    X_local = torch.as_tensor(X_local, dtype=torch.float32).reshape(-1).to(dev)
    sh = ShardedDME(n_local, d, n_total, bits_per_dimension, torch_threads=torch_threads, pipeline="q", mode=mode,
                    dst=dst, group=group, overlap=False, device=dev)
    est = sh.step(x_local, X_local)
    if est is not None and mode == "reduce" and sh.rank != dst:
        est = None
    return (est, sh.pipe.q) if return_q else est
