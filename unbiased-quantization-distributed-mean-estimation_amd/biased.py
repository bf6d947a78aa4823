"""Biased type quantizer (Reznik rounding) on the GPU — SURVEY §8(f) row 1.

Drop-in:
    Type_biased_quantize(input_vector, bits_per_dimension=1)
        == NMSE_Results/Codes/All_Schemes.py:669-687 (with Reznik, AS:644-666): same name,
        argument meaning, return type (new f32 tensor of shape (d,) on the GPU), no RNG,
        KeyError for an unknown rate (AS:684).

Batched:
    biased_quantize(x[n, d], bits | m=, ties="torch" | "lowest") -> out[n, d]

Numerics (all f32, as torch CPU): k' = floor(m*p + 0.5), m' = k'.sum() in torch CPU order
for `torch_threads`, Delta = int(m' - m), the |Delta| extreme delta' = k' - m*p adjusted by
-+1, out = (L1 * sign(x)) * (k' / m).  torch.topk picks among equal delta' values by what
libstdc++'s nth_element / partial_sort leave in front; ties="lowest" takes the lowest
indices instead (identical whenever info flag 1 is clear; see include/uq_dme.h).
"""
from __future__ import annotations

import ctypes
import functools
import threading

import numpy as np
import torch

from . import _lib
from .quantizer import (_as_device_f32_2d, _device, _ptr, _resolve_m, _stream_ptr, _workspace,
                        check_status, get_torch_threads)
from .rates import RATE_TABLE

__all__ = ["Type_biased_quantize", "biased_quantize", "TIES_TORCH", "TIES_LOWEST_INDEX",
           "FLAG_AMBIGUOUS", "FLAG_NONFINITE", "FLAG_RANGE", "FLAG_TORCH_TIES"]

TIES_TORCH = 0            # UQ_TIES_TORCH
TIES_LOWEST_INDEX = 1     # UQ_TIES_LOWEST_INDEX
_HOST_CHECK = 4           # UQ_TIES_HOST_CHECK
_SMALL_MAX = 32767        # kSmallBiasedMax: one-launch vectors (shorter than torch's GRAIN)
_tls = threading.local()
FLAG_AMBIGUOUS = 1
FLAG_NONFINITE = 2
FLAG_RANGE = 4
FLAG_TORCH_TIES = 8

_TIES = {"torch": TIES_TORCH, "lowest": TIES_LOWEST_INDEX, TIES_TORCH: TIES_TORCH,
         TIES_LOWEST_INDEX: TIES_LOWEST_INDEX}


@functools.lru_cache(maxsize=256)
def _biased_ws_bytes(n: int, d: int, T: int) -> int:
    out = ctypes.c_size_t(0)
    _lib.check(_lib.load().uq_biased_workspace_bytes(n, d, T, ctypes.byref(out)), "uq_biased_workspace_bytes")
    return int(out.value)


def biased_quantize(x, bits_per_dimension=1, *, m: int | None = None, torch_threads: int | None = None,
                    ties="torch", out=None, return_l1: bool = False, return_info: bool = False,
                    host_check: bool = False):
    """Batched Type_biased_quantize over the rows of x [n, d].

    return_info adds an int32 [n, 2] tensor {Delta, flags} per row (flags: 1 a tie
    straddled the threshold, 2 m' not finite, 4 |Delta| > d, 8 torch tie choice replayed).
    host_check (torch ties): the call may wait once for the number of rows whose tie choice
    needs the replay and skips the replay's kernels when there are none (UQ_TIES_HOST_CHECK:
    for synchronous few-row callers; the same bits either way)."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    mm = _resolve_m(bits_per_dimension, m, d)
    T = get_torch_threads() if torch_threads is None else int(torch_threads)
    if ties not in _TIES:
        raise ValueError("ties must be 'torch' or 'lowest'")
    if out is None:
        out = torch.empty_like(x)
    elif out.shape != x.shape or out.dtype != torch.float32 or out.device != x.device or not out.is_contiguous():
        raise ValueError("out must be a contiguous f32 tensor like x")
    l1_out = torch.empty(n, dtype=torch.float32, device=dev) if return_l1 else None
    info = torch.empty((n, 2), dtype=torch.int32, device=dev) if return_info else None
    ws = _workspace(dev, _biased_ws_bytes(n, d, T))
    policy = _TIES[ties] | (_HOST_CHECK if host_check and _TIES[ties] == TIES_TORCH else 0)
    _lib.check(_lib.load().uq_type_biased_f32(_ptr(x), _ptr(out), n, d, mm, T, policy, _ptr(l1_out),
                                              _ptr(info), _ptr(ws), ws.numel(), _stream_ptr(dev)),
               "uq_type_biased_f32")
    res = [out]
    if return_l1:
        res.append(l1_out)
    if return_info:
        res.append(info)
    return res[0] if len(res) == 1 else tuple(res)


def _flags_and_status(dev, d: int, info) -> int:
    """One synchronisation for row 0's flags and this workspace's status word (uq_check_status's
    word at byte 8; check_status() would read every cached workspace of the stream)."""
    ws = _workspace(dev, _biased_ws_bytes(1, d, get_torch_threads()))
    hw = getattr(_tls, "pinned", None)
    if hw is None:
        hw = _tls.pinned = torch.empty(2, dtype=torch.int32, pin_memory=True)
    hw[0:1].copy_(info[0, 1:2], non_blocking=True)
    hw[1:2].copy_(ws[8:12].view(torch.int32), non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    flags, status = int(hw[0]), int(hw[1])
    if status:
        check_status()                            # raises with the library's message, clears the word
    return flags


def Type_biased_quantize(input_vector, bits_per_dimension=1):
    """Drop-in for NMSE_Results/Codes/All_Schemes.py:669 (same name for FLM:177's
    directory naming).  KeyError for an unknown rate (AS:684), bit-identical to the
    reference on torch CPU with the same intra-op thread count, ties included.  The
    reference raises when m' is not finite (AS:656); so does this.  AS:671 copies the input
    so as not to alias it; here the kernels only read it and the result is always a new
    tensor (d == 0 returns a clone), so no device-side copy is made."""
    dev = _device()
    l_rate = RATE_TABLE[bits_per_dimension]
    if torch.is_tensor(input_vector):
        v = input_vector.detach().to(device=dev, dtype=torch.float32)
    else:
        v = torch.tensor(np.asarray(input_vector), dtype=torch.float32, device=dev)
    if v.dim() != 1:
        raise RuntimeError("Type_biased_quantize expects a 1-D vector")
    d = v.numel()
    m = int(l_rate * d)
    if d == 0:
        return v.clone()
    if not v.is_contiguous():
        v = v.contiguous()
    # below GRAIN the lowest-index rule runs as one launch (KB-small) and gives torch's bits
    # unless a threshold tie straddles the selection (flag 1): read the flags once and rerun
    # with the replay only then, so a tie-free call synchronises once
    small = d <= _SMALL_MAX
    out, info = biased_quantize(v.view(1, d), m=m, ties="lowest" if small else "torch", return_info=True,
                                host_check=not small)
    flags = _flags_and_status(dev, d, info)
    if small and flags & FLAG_AMBIGUOUS:
        out, info = biased_quantize(v.view(1, d), m=m, ties="torch", return_info=True, host_check=True)
        flags = _flags_and_status(dev, d, info)
    if flags & FLAG_NONFINITE:
        raise ValueError("cannot convert float NaN to integer (m' is not finite, AS:656)")
    if flags & FLAG_RANGE:
        raise RuntimeError("selected index k out of range (AS:660)")
    return out.view(d)
