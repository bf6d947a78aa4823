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


def sharded_quantize_mean(x_local: torch.Tensor, bits_per_dimension, X_local, n_total: int, *,
                          mode: str = "reduce", dst: int = 0, torch_threads: int = 1, group=None,
                          return_q: bool = False):
    """Quantize this rank's clients (HIP) and form the global client mean.

    x_local = the rank's contiguous client block (see shard_range); X_local = its
    slice of the per-client uniforms drawn once for all clients."""
    from .quantizer import quantize_dequantize
    q = quantize_dequantize(x_local, bits_per_dimension, X=X_local, torch_threads=torch_threads)
    est = sharded_client_mean(q, float(n_total), mode=mode, dst=dst, group=group)
    return (est, q) if return_q else est
