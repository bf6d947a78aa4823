"""Host-side mirror of the reference's quantizer interface, backed by HIP kernels.

Drop-in:
    Type_unbiased_quantize(input_vector, bits_per_dimension=1)
        == NMSE_Results/Codes/All_Schemes.py:609-641, same name, argument meaning,
        return type (new f32 tensor of shape (d,) on the GPU), RNG use (one draw from
        torch's global CPU generator per call, AS:634) and errors (KeyError for an
        unknown rate, AS:622; RuntimeError for non-1-D input, AS:635).

Batched APIs (what the DME harness and the bench use):
    quantize_dequantize(x[n, d], bits | m=, X[n])       -> q[n, d]
    client_mean(q[n, d], n_div, est=None)                 -> est[d]   (ND:137-138)
    quantize_mean(x[n, d], bits, X[n], n_div, est=None)   -> est[d]
    l1_torch_order(x[n, d], torch_threads)                -> l1[n]    (AS:624)

Every path calls the C-ABI in include/uq_dme.h; nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

import numpy as np
import torch

from . import _lib
from .outpool import POOL
from .rates import RATE_TABLE, rate_to_m

__all__ = [
    "Type_unbiased_quantize", "quantize_dequantize", "client_mean", "quantize_mean", "quantize_encode", "decode",
    "codes_mean",
    "l1_torch_order", "draw_uniforms", "set_torch_threads", "get_torch_threads",
]

_ws_lock = threading.Lock()
_ws_cache: dict = {}
_torch_threads_override = None


def set_torch_threads(t):
    """Pin the torch-CPU summation order used for L1 (AS:624).  None -> follow
    torch.get_num_threads() at call time, i.e. what the CPU reference would do in
    this process."""
    global _torch_threads_override
    _torch_threads_override = None if t is None else int(t)


def get_torch_threads() -> int:
    if _torch_threads_override is not None:
        return _torch_threads_override
    env = os.environ.get("UQDME_TORCH_THREADS")
    if env:
        return int(env)
    return int(torch.get_num_threads())


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("uqdme requires a ROCm GPU (no CPU fallback by design)")
    return torch.device("cuda", torch.cuda.current_device())


def _stream_ptr(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """Per (device, stream) workspace, grown on demand (stream-ordered reuse)."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    with _ws_lock:
        ws = _ws_cache.get(key)
        if ws is None or ws.numel() < nbytes:
            # zero-filled once: the C-ABI requires a zeroed control block on first use
            ws = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
            _ws_cache[key] = ws
        return ws


@functools.lru_cache(maxsize=256)
def _ws_bytes(n: int, d: int, T: int) -> int:
    out = ctypes.c_size_t(0)
    _lib.check(_lib.load().uq_workspace_bytes(n, d, T, ctypes.byref(out)), "uq_workspace_bytes")
    return int(out.value)


def draw_uniforms(n: int, generator: torch.Generator | None = None) -> torch.Tensor:
    """n draws of AS:634's X from a CPU generator; torch.rand(n) equals n successive
    torch.rand(1) calls, so this reproduces a per-client loop of the reference."""
    return torch.rand(n, generator=generator, dtype=torch.float32)


def _as_device_f32_2d(x, dev) -> torch.Tensor:
    if not torch.is_tensor(x):
        x = torch.as_tensor(np.asarray(x), dtype=torch.float32)
    if x.dim() != 2:
        raise ValueError("expected a 2-D [n, d] batch")
    return x.to(device=dev, dtype=torch.float32).contiguous()


def _resolve_m(bits, m, d):
    if m is not None:
        return int(m)
    return rate_to_m(bits, d)


def l1_torch_order(x, torch_threads: int | None = None) -> torch.Tensor:
    """AS:624 `|x|.sum()` per row, bit-identical to torch CPU with `torch_threads` threads."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    T = get_torch_threads() if torch_threads is None else int(torch_threads)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    nb = _ws_bytes(n, d, T)
    ws = _workspace(dev, nb)
    _lib.check(_lib.load().uq_l1_torch_order_f32(_ptr(x), n, d, T, _ptr(out), _ptr(ws), ws.numel(),
                                                  _stream_ptr(dev)), "uq_l1_torch_order_f32")
    return out


def quantize_dequantize(x, bits_per_dimension=1, X=None, *, m: int | None = None,
                        torch_threads: int | None = None, l1=None, out=None,
                        return_l1: bool = False, generator: torch.Generator | None = None):
    """Batched `Type_unbiased_quantize`: row j of `x` is quantized with uniform X[j].

    X defaults to n fresh draws from the CPU generator (global one unless given)."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    mm = _resolve_m(bits_per_dimension, m, d)
    T = get_torch_threads() if torch_threads is None else int(torch_threads)
    if X is None:
        X = draw_uniforms(n, generator)
    X = torch.as_tensor(X, dtype=torch.float32).reshape(-1)
    if X.numel() != n:
        raise ValueError("X must have one draw per row")
    token = None
    if out is None:
        (out,), token = POOL.acquire(dev, [((n, d), torch.float32)])     # probed placement for big batches
    elif out.shape != x.shape or out.dtype != torch.float32 or out.device != x.device or not out.is_contiguous():
        raise ValueError("out must be a contiguous f32 tensor like x")
    if n == 1 and d > 0 and l1 is None and not return_l1 and X.device.type == "cpu":
        # one vector with its draw on the host: the drop-in's entry (X by value, no copy of
        # X to the device, no workspace fill; same kernels, same bits): 0.20 -> 0.15 ms at 2^22
        ws = _workspace(dev, _ws_bytes(1, d, T))
        _lib.check(_lib.load().uq_type_unbiased_vec_f32(_ptr(x), _ptr(out), d, mm, float(X[0]), T, _ptr(ws),
                                                        ws.numel(), _stream_ptr(dev)), "uq_type_unbiased_vec_f32")
        return out
    X = X.to(dev)
    if l1 is not None:
        l1 = torch.as_tensor(l1, dtype=torch.float32).reshape(-1).to(dev).contiguous()
        if l1.numel() != n:
            raise ValueError("l1 must have one value per row")
    l1_out = torch.empty(n, dtype=torch.float32, device=dev) if return_l1 else None
    nb = _ws_bytes(n, d, T)
    ws = _workspace(dev, nb)
    POOL.timed(token, lambda: _lib.check(_lib.load().uq_type_unbiased_f32(
        _ptr(x), _ptr(out), n, d, mm, _ptr(X), _ptr(l1), _ptr(l1_out), T, _ptr(ws), ws.numel(), _stream_ptr(dev)),
        "uq_type_unbiased_f32"))
    return (out, l1_out) if return_l1 else out


def quantize_encode(x, bits_per_dimension=1, X=None, *, m: int | None = None, torch_threads: int | None = None,
                    l1=None, return_q: bool = False, generator: torch.Generator | None = None):
    """Quantize a batch and emit type codes (codes.TypeCodes); optionally also q.

    Same numerics as quantize_dequantize: decode(codes) == q bit-for-bit."""
    from .codes import TypeCodes
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    mm = _resolve_m(bits_per_dimension, m, d)
    T = get_torch_threads() if torch_threads is None else int(torch_threads)
    if X is None:
        X = draw_uniforms(n, generator)
    X = torch.as_tensor(X, dtype=torch.float32).reshape(-1).to(dev)
    if X.numel() != n:
        raise ValueError("X must have one draw per row")
    if l1 is not None:
        l1 = torch.as_tensor(l1, dtype=torch.float32).reshape(-1).to(dev).contiguous()
    specs = [((n, d), torch.int8)] + ([((n, d), torch.float32)] if return_q else [])
    bufs, token = POOL.acquire(dev, specs)                      # probed placement for big batches
    codes = bufs[0]
    q = bufs[1] if return_q else None
    overflow = torch.zeros(n, dtype=torch.int32, device=dev)     # per-client kmax (128 = overflow)
    l1_out = torch.empty(n, dtype=torch.float32, device=dev)
    nb = _ws_bytes(n, d, T)
    ws = _workspace(dev, nb)
    POOL.timed(token, lambda: _lib.check(_lib.load().uq_type_unbiased_codes_f32(
        _ptr(x), _ptr(q), _ptr(codes), _ptr(overflow), n, d, mm, _ptr(X), _ptr(l1), _ptr(l1_out), T, _ptr(ws),
        ws.numel(), _stream_ptr(dev)), "uq_type_unbiased_codes_f32"))
    tc = TypeCodes(codes=codes, l1=l1_out, m=mm, overflow=overflow)
    return (tc, q) if return_q else tc


def decode(tc) -> torch.Tensor:
    """Rebuild the dequantized batch from type codes (bit-identical to quantize_dequantize)."""
    dev = _device()
    codes = tc.codes.to(dev).contiguous()
    l1 = tc.l1.to(device=dev, dtype=torch.float32).contiguous()
    n, d = codes.shape
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().uq_codes_decode_f32(_ptr(codes), _ptr(l1), n, d, int(tc.m), _ptr(out), _stream_ptr(dev)),
               "uq_codes_decode_f32")
    return out


def codes_mean(tc, n_div, est=None, accumulate: bool = False) -> torch.Tensor:
    """ND:137-138 from type codes: est (+)= decode(codes)[j] / n_div over clients j in order,
    bit-identical to client_mean(decode(tc), n_div)."""
    dev = _device()
    codes = tc.codes.to(dev).contiguous()
    l1 = tc.l1.to(device=dev, dtype=torch.float32).contiguous()
    n, d = codes.shape
    if est is None:
        est = torch.empty(d, dtype=torch.float32, device=dev)
        accumulate = False
    kmax = tc.overflow.to(device=dev, dtype=torch.int32).contiguous()
    _lib.check(_lib.load().uq_codes_mean_f32(_ptr(codes), _ptr(l1), _ptr(kmax), n, d, int(tc.m), float(n_div),
                                             int(bool(accumulate)), _ptr(est), _stream_ptr(dev)), "uq_codes_mean_f32")
    return est


def client_mean(q, n_div, est=None, accumulate: bool = False) -> torch.Tensor:
    """ND:137-138: est (+)= q[j] / n_div over rows j in order (f32).

    `q` may be a column block of a wider row-major batch (unit column stride, any row
    stride); with accumulate=True the sum continues from `est` bit-for-bit."""
    dev = _device()
    if not torch.is_tensor(q):
        q = torch.as_tensor(np.asarray(q), dtype=torch.float32)
    if q.dim() != 2:
        raise ValueError("expected a 2-D [n, d] batch")
    q = q.to(device=dev, dtype=torch.float32)
    if q.shape[1] > 0 and (q.stride(1) != 1 or q.stride(0) < q.shape[1]):
        q = q.contiguous()
    n, d = q.shape
    ld = q.stride(0) if n > 0 else d
    if est is None:
        est = torch.empty(d, dtype=torch.float32, device=dev)
        accumulate = False
    elif est.shape != (d,) or est.dtype != torch.float32 or est.device != q.device or not est.is_contiguous():
        raise ValueError("est must be a contiguous f32 vector of length d on the same device")
    _lib.check(_lib.load().uq_client_mean_f32(_ptr(q), n, d, max(ld, d), float(n_div), int(bool(accumulate)),
                                              _ptr(est), _stream_ptr(dev)), "uq_client_mean_f32")
    return est


def quantize_mean(x, bits_per_dimension=1, X=None, n_div=None, *, m: int | None = None,
                  torch_threads: int | None = None, est=None, accumulate: bool = False, out=None):
    """Quantize every row and fold it into the client-ordered mean (ND:133-138)."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    mm = _resolve_m(bits_per_dimension, m, d)
    T = get_torch_threads() if torch_threads is None else int(torch_threads)
    if X is None:
        X = draw_uniforms(n)
    X = torch.as_tensor(X, dtype=torch.float32).reshape(-1).to(dev)
    if n_div is None:
        n_div = n
    if est is None:
        est = torch.empty(d, dtype=torch.float32, device=dev)
        accumulate = False
    token = None
    if out is None:
        (out,), token = POOL.acquire(dev, [((n, d), torch.float32)])     # scratch q: probed placement
    nb = _ws_bytes(n, d, T)
    ws = _workspace(dev, nb)
    POOL.timed(token, lambda: _lib.check(_lib.load().uq_type_unbiased_mean_f32(
        _ptr(x), _ptr(out), n, d, mm, _ptr(X), _ptr(None), T, float(n_div), int(bool(accumulate)), _ptr(est),
        _ptr(ws), ws.numel(), _stream_ptr(dev)), "uq_type_unbiased_mean_f32"))
    return est


def check_status() -> None:
    """Synchronise the current stream and raise if an in-kernel wait timed out."""
    dev = _device()
    for (idx, sp), ws in list(_ws_cache.items()):
        if idx == dev.index and sp == torch.cuda.current_stream(dev).cuda_stream:
            _lib.check(_lib.load().uq_check_status(_ptr(ws), _stream_ptr(dev)), "uq_check_status")


def Type_unbiased_quantize(input_vector, bits_per_dimension=1):
    """Drop-in for NMSE_Results/Codes/All_Schemes.py:609 (same name: the Flower client
    derives directory names from `__name__`, FLM:177).

    AS:611  takes `input_vector` as f32 on the device (the input is only read; the result
            is always a new tensor, as the reference's copy guarantees)
    AS:622  unknown `bits_per_dimension` -> KeyError (checked before any work)
    AS:634  consumes exactly one draw of torch's global CPU generator
    Returns a new f32 tensor of shape (d,) on the GPU."""
    dev = _device()
    l_rate = RATE_TABLE[bits_per_dimension]          # KeyError like the reference
    if torch.is_tensor(input_vector):
        # no device-side copy (AS:611 copies so as not to alias the input; here the kernels
        # only read v and write a new output, and d == 0 returns a clone below)
        v = input_vector.detach().to(device=dev, dtype=torch.float32)
    else:
        v = torch.tensor(np.asarray(input_vector), dtype=torch.float32, device=dev)
    if v.dim() != 1:
        raise RuntimeError("Type_unbiased_quantize expects a 1-D vector "
                           "(the reference fails at torch.cat for other ranks)")
    d = v.numel()
    m = int(l_rate * d)
    X = torch.rand(1)                                   # AS:634 (global CPU generator)
    if d == 0:
        return v.clone()
    if not v.is_contiguous():
        v = v.contiguous()
    # one vector per call: X goes to the kernels by value (uq_type_unbiased_vec_f32), so the
    # call is the kernel chain alone -- no host-to-device copy of X, no workspace fill
    T = get_torch_threads()
    out = torch.empty_like(v)
    ws = _workspace(dev, _ws_bytes(1, d, T))
    _lib.check(_lib.load().uq_type_unbiased_vec_f32(_ptr(v), _ptr(out), d, m, float(X[0]), T, _ptr(ws),
                                                    ws.numel(), _stream_ptr(dev)), "uq_type_unbiased_vec_f32")
    return out
