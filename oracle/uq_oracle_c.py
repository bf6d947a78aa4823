"""ctypes handle on the C oracle (oracle/uq_oracle.c).  Test infrastructure only:
used by tests/ and bench.py's cpu_baseline leg as the checker, never shipped."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libuq_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        i64, f, p = ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
        L.uqo_l1_torch_order.restype = f
        L.uqo_l1_torch_order.argtypes = [p, i64, ctypes.c_int, p]
        L.uqo_quantize.restype = f
        L.uqo_quantize.argtypes = [p, p, i64, i64, f, ctypes.c_int, ctypes.c_int, f, p]
        L.uqo_quantize_batch.restype = None
        L.uqo_quantize_batch.argtypes = [p, p, i64, i64, i64, p, ctypes.c_int, p, p]
        L.uqo_quantize_batch_mt.restype = ctypes.c_int
        L.uqo_quantize_batch_mt.argtypes = [p, p, i64, i64, i64, p, ctypes.c_int, p, ctypes.c_int]
        L.uqo_client_mean.restype = None
        L.uqo_client_mean.argtypes = [p, i64, i64, f, p]
        L.uqo_client_mean_acc.restype = None
        L.uqo_client_mean_acc.argtypes = [p, i64, i64, f, p]
        L.uqo_torch_sum.restype = f
        L.uqo_torch_sum.argtypes = [p, i64, ctypes.c_int]
        L.uqo_torch_norm2.restype = f
        L.uqo_torch_norm2.argtypes = [p, i64]
        L.uqo_torch_dot.restype = f
        L.uqo_torch_dot.argtypes = [p, p, i64]
        L.uqc_bound.restype = ctypes.c_uint64
        L.uqc_bound.argtypes = [i64]
        L.uqc_encode.restype = ctypes.c_uint64
        L.uqc_encode.argtypes = [p, i64, i64, f, ctypes.c_int, p]
        L.uqc_decode.restype = ctypes.c_int
        L.uqc_decode.argtypes = [p, ctypes.c_uint64, p, i64, p, p]
        L.uqo_biased_quantize.restype = ctypes.c_int
        L.uqo_biased_quantize.argtypes = [p, p, i64, i64, ctypes.c_int, ctypes.c_int, p, p, p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def l1_torch_order(x, torch_threads: int = 1) -> np.float32:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    scratch = np.empty(max(1, x.shape[0]), np.float32)
    return np.float32(lib().uqo_l1_torch_order(_ptr(x), x.shape[0], torch_threads, _ptr(scratch)))


def quantize_batch(x2d, m: int, X, torch_threads: int = 1):
    x2d = np.ascontiguousarray(x2d, dtype=np.float32)
    n, d = x2d.shape
    X = np.ascontiguousarray(X, dtype=np.float32).reshape(n)
    out = np.empty_like(x2d)
    l1 = np.empty(n, np.float32)
    scratch = np.empty(max(1, d), np.float32)
    lib().uqo_quantize_batch(_ptr(x2d), _ptr(out), n, d, m, _ptr(X), torch_threads, _ptr(l1), _ptr(scratch))
    return out, l1


def quantize_batch_mt(x2d, m: int, X, torch_threads: int = 1, nthreads: int = 1):
    """quantize_batch with clients spread over OpenMP threads; returns (out, l1, threads used)."""
    x2d = np.ascontiguousarray(x2d, dtype=np.float32)
    n, d = x2d.shape
    X = np.ascontiguousarray(X, dtype=np.float32).reshape(n)
    out = np.empty_like(x2d)
    l1 = np.empty(n, np.float32)
    used = lib().uqo_quantize_batch_mt(_ptr(x2d), _ptr(out), n, d, m, _ptr(X), torch_threads, _ptr(l1), nthreads)
    return out, l1, int(used)


def quantize_with_l1(x, m: int, X: float, l1: float):
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    out = np.empty_like(x)
    scratch = np.empty(1, np.float32)
    lib().uqo_quantize(_ptr(x), _ptr(out), x.shape[0], m, np.float32(X), 1, 1, np.float32(l1), _ptr(scratch))
    return out


def client_mean(q2d, n_div):
    q2d = np.ascontiguousarray(q2d, dtype=np.float32)
    n, d = q2d.shape
    est = np.empty(d, np.float32)
    lib().uqo_client_mean(_ptr(q2d), n, d, np.float32(n_div), _ptr(est))
    return est


def client_mean_acc(q2d, n_div, est):
    """est += q2d[j] / n_div for rows in order, in place (continues a client-ordered mean)."""
    q2d = np.ascontiguousarray(q2d, dtype=np.float32)
    n, d = q2d.shape
    assert est.dtype == np.float32 and est.flags.c_contiguous and est.shape == (d,)
    lib().uqo_client_mean_acc(_ptr(q2d), n, d, np.float32(n_div), _ptr(est))
    return est


def torch_norm2(v) -> np.float32:
    """torch.norm(v, 2) in torch's CPU f32 order (8 fma lanes; oracle/uq_eden.py:torch_norm2)."""
    v = np.ascontiguousarray(v, dtype=np.float32).reshape(-1)
    return np.float32(lib().uqo_torch_norm2(_ptr(v), v.shape[0]))


def torch_dot(x, y) -> np.float32:
    """torch.dot(x, y) in MKL sdot's CPU f32 order (oracle/uq_eden.py:torch_dot), exact fmaf."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    y = np.ascontiguousarray(y, dtype=np.float32).reshape(-1)
    assert x.shape == y.shape
    return np.float32(lib().uqo_torch_dot(_ptr(x), _ptr(y), x.shape[0]))


def torch_sum(v, torch_threads: int = 1):
    v = np.ascontiguousarray(v, dtype=np.float32).reshape(-1)
    return np.float32(lib().uqo_torch_sum(_ptr(v), v.shape[0], torch_threads))


def biased_quantize(x, m: int, torch_threads: int = 1, tie_mode: int = 0):
    """Type_biased_quantize (AS:669-687).  tie_mode 0: torch's topk choice among equal
    values at the threshold; 1: lowest indices.  Returns (out, L1, Delta, ambiguous);
    raises like the reference (ValueError / RuntimeError)."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    out = np.empty_like(x)
    L = np.zeros(1, np.float32)
    D = np.zeros(1, np.int64)
    A = np.zeros(1, np.int32)
    rc = lib().uqo_biased_quantize(_ptr(x), _ptr(out), x.shape[0], m, torch_threads, tie_mode, _ptr(L), _ptr(D),
                                   _ptr(A))
    if rc == -1:
        raise ValueError("cannot convert float NaN to integer (m' not finite, AS:656)")
    if rc == -2:
        raise RuntimeError("selected index k out of range (AS:660)")
    return out, np.float32(L[0]), int(D[0]), bool(A[0])


def codec_encode(codes, m: int, l1: float, exact: bool = False) -> bytes:
    """One client's int8 type codes -> a UQR1 message (oracle/uq_codec.c)."""
    c = np.ascontiguousarray(codes, dtype=np.int8).reshape(-1)
    out = np.empty(int(lib().uqc_bound(c.shape[0])), np.uint8)
    n = lib().uqc_encode(_ptr(c), c.shape[0], int(m), np.float32(l1), int(bool(exact)), _ptr(out))
    if n == 0 and c.shape[0] > 0:
        raise ValueError("uqc_encode failed")
    return out[:n].tobytes()


def codec_decode(msg: bytes, d: int):
    """UQR1 message -> (codes int8 [d], l1 f32, m); raises on a malformed message."""
    buf = np.frombuffer(msg, np.uint8).copy()
    codes = np.empty(max(1, d), np.int8)
    l1 = np.zeros(1, np.float32)
    m = np.zeros(1, np.int64)
    rc = lib().uqc_decode(_ptr(buf), buf.shape[0], _ptr(codes), int(d), _ptr(l1), _ptr(m))
    if rc != 0:
        raise ValueError(f"malformed UQR1 message ({rc})")
    return codes[:d], np.float32(l1[0]), int(m[0])
