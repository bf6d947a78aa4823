"""EDEN with the randomized Hadamard transform on the GPU — SURVEY §8(f) row 2 (baseline).

Drop-in:
    EDEN_quantize_Hadamard(input_vector, bits_per_dimension=1)
        == NMSE_Results/Codes/All_Schemes.py:792-811: one torch.randint(0, 100) draw of the
        global CPU generator per call (the rotation seed, AS:797), EdenSender.compress then
        EdenReceiver.decompress, returns a NumPy f32 array of length d (AS:811).

Batched:
    eden_quantize(x[n, d], bits, seeds[n])              -> out[n, d]
    eden_compress(x[n, d], bits, seeds[n])              -> EdenMessage(bins u8 [n, D], scale[n], seeds, d)
    eden_decompress(msg)                                -> out[n, d]

Numerics: rotation (MT19937 diagonal, f32 butterflies a+b / (a+b)-2b, / f32(sqrt(D))), the
norm (torch CPU order) and the bins are bit-identical to the reference; the scale's dot
product is accumulated in fp64 because the reference's (MKL sdot) order is CPU-dependent,
so outputs agree to 1e-6 relative.  Only the 1- and 2-bit tables exist in the reference.
"""
from __future__ import annotations

import ctypes
import threading
import weakref
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .quantizer import _as_device_f32_2d, _device, _ptr, _stream_ptr, _workspace

__all__ = ["EDEN_quantize_Hadamard", "eden_quantize", "eden_compress", "eden_decompress", "EdenMessage",
           "rht_signs", "padded_dim", "randomized_hadamard_transform", "randomized_inverse_hadamard_transform"]

_SEEDS = 100                       # AS:797 torch.randint(0, 100)
_cache_lock = threading.Lock()


class _SignCache:
    """Device sign tables kept between calls, bounded by BYTES (least recently used first out):
    the shared table of seeds 0..99 per (device, D) and the rows of other seeds (single seeds
    of the drop-ins, sets of <= 4 seeds such as QUIC-FL's fixed 123).  The newest entry always
    stays, so a table larger than the budget is still reused by the next call with that key.
    The per-call row-index tensors (4 bytes each) are cached apart, by count."""

    def __init__(self, budget_bytes: int = 2 << 30, max_rows: int = 4096):
        from collections import OrderedDict
        self.budget, self.max_rows = budget_bytes, max_rows
        self.tabs = OrderedDict()      # key -> (tensor, nbytes)
        self.rows = OrderedDict()      # key -> small int32 device tensor
        self.bytes = 0

    def get(self, key):
        hit = self.tabs.get(key)
        if hit is None:
            return None
        self.tabs.move_to_end(key)
        return hit[0]

    def put(self, key, tab):
        nb = tab.numel() * tab.element_size()
        old = self.tabs.pop(key, None)
        if old is not None:
            self.bytes -= old[1]
        self.tabs[key] = (tab, nb)
        self.bytes += nb
        while self.bytes > self.budget and len(self.tabs) > 1:
            _, (_, b) = self.tabs.popitem(last=False)
            self.bytes -= b

    def row(self, key, make):
        r = self.rows.get(key)
        if r is None:
            r = make()
            self.rows[key] = r
            while len(self.rows) > self.max_rows:
                self.rows.popitem(last=False)
        else:
            self.rows.move_to_end(key)
        return r

    def clear(self):
        self.tabs.clear()
        self.rows.clear()
        self.bytes = 0


_signs = _SignCache()


def padded_dim(d: int) -> int:
    """AS:128 / AS:359: the next power of two (d itself when it is one)."""
    return 1 if d <= 1 else 1 << (int(d) - 1).bit_length()


def rht_signs(seeds, D: int, device=None) -> torch.Tensor:
    """int8 [len(seeds), D] RHT diagonals (AS:117-120) generated on the GPU."""
    dev = device or _device()
    s = torch.as_tensor(seeds, dtype=torch.int32).reshape(-1).to(dev)
    out = torch.empty((s.numel(), D), dtype=torch.int8, device=dev)
    _lib.check(_lib.load().uq_rht_signs(_ptr(s), s.numel(), D, _ptr(out), _stream_ptr(dev)), "uq_rht_signs")
    return out


def _shared_table(D: int, dev):
    key = (dev.index, D, "ref")
    with _cache_lock:
        tab = _signs.get(key)
        if tab is None:
            tab = rht_signs(torch.arange(_SEEDS), D, dev)
            _signs.put(key, tab)
        return tab


def _sign_rows(seeds: torch.Tensor, D: int, dev):
    """(table, row index per client).  Seeds 0..99 (the reference's range) share one cached
    table per (device, D); other seeds get rows of their own (cached for single seeds and sets
    of up to four, within the cache's byte budget)."""
    seeds_cpu = seeds.to("cpu", torch.int64).reshape(-1)
    in_range = bool(((seeds_cpu >= 0) & (seeds_cpu < _SEEDS)).all())
    if seeds_cpu.numel() == 1:                       # the per-vector drop-ins
        sd = int(seeds_cpu[0])
        if in_range:
            tab = _shared_table(D, dev)
            with _cache_lock:
                return tab, _signs.row((dev.index, sd), lambda: torch.tensor([sd], dtype=torch.int32, device=dev))
        key = (dev.index, D, "one", sd)
        with _cache_lock:
            tab = _signs.get(key)
            if tab is None:
                tab = rht_signs(seeds_cpu, D, dev)
                _signs.put(key, tab)
            return tab, _signs.row((dev.index, "zero"), lambda: torch.zeros(1, dtype=torch.int32, device=dev))
    if in_range:
        return _shared_table(D, dev), seeds_cpu.to(torch.int32).to(dev)
    uniq, inv = torch.unique(seeds_cpu, return_inverse=True)
    if uniq.numel() <= 4:                 # a few other seeds (e.g. QUIC-FL's fixed 123, AS:822): cached too
        key = (dev.index, D, tuple(uniq.tolist()))
        with _cache_lock:
            tab = _signs.get(key)
            if tab is None:
                tab = rht_signs(uniq, D, dev)
                _signs.put(key, tab)
        return tab, inv.to(torch.int32).to(dev)
    return rht_signs(uniq, D, dev), inv.to(torch.int32).to(dev)


def rht_sign_bits(tab: torch.Tensor) -> torch.Tensor:
    """int32 [rows, ceil(D / 32)]: the diagonal rows of `tab` as bits (bit set where the sign is
    -1), which the EDEN passes that apply the diagonal read instead of the int8 rows."""
    rows, D = tab.shape
    out = torch.empty((rows, (D + 31) // 32), dtype=torch.int32, device=tab.device)
    _lib.check(_lib.load().uq_rht_sign_bits(_ptr(tab), rows, D, _ptr(out), _stream_ptr(tab.device)),
               "uq_rht_sign_bits")
    return out


_bits_of: dict = {}          # id(table) -> (weak reference to the table, its bit rows)


def _bits_for(tab: torch.Tensor) -> torch.Tensor:
    """The bit rows of a sign table, kept exactly as long as the table itself lives."""
    with _cache_lock:
        e = _bits_of.get(id(tab))
        if e is not None and e[0]() is tab:
            return e[1]
    bits = rht_sign_bits(tab)
    k = id(tab)
    with _cache_lock:
        _bits_of[k] = (weakref.ref(tab, lambda _r, k=k: _bits_of.pop(k, None)), bits)
    return bits


def _sign_rows_bits(seeds: torch.Tensor, D: int, dev):
    """(table, row index per client, the table's rows as bits)."""
    tab, rows = _sign_rows(seeds, D, dev)
    return tab, rows, _bits_for(tab)


def _ws(n, d, dev):
    b = ctypes.c_size_t(0)
    _lib.check(_lib.load().uq_eden_workspace_bytes(n, d, ctypes.byref(b)), "uq_eden_workspace_bytes")
    return _workspace(dev, int(b.value))


def _seeds(seeds, n, generator=None):
    if seeds is None:
        return torch.randint(0, _SEEDS, (n,), generator=generator)     # n successive AS:797 draws
    s = torch.as_tensor(seeds, dtype=torch.int64).reshape(-1)
    if s.numel() != n:
        raise ValueError("one seed per row")
    return s


def _bits(bits):
    if bits not in (1, 2):
        raise ValueError("EDEN supports 1 and 2 bits (the reference's centroid tables, AS:302-306)")
    return int(bits)


@dataclass
class EdenMessage:
    bins: torch.Tensor      # u8 [n, D]
    scale: torch.Tensor     # f32 [n]
    seeds: torch.Tensor     # int64 [n] (rotation seeds)
    nbits: int
    dim: int


def eden_compress(x, bits_per_dimension=1, seeds=None, *, generator=None) -> EdenMessage:
    """EdenSender.compress (AS:355-376) for every row of x [n, d]."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    nb = _bits(bits_per_dimension)
    s = _seeds(seeds, n, generator)
    D = padded_dim(d)
    bins = torch.empty((n, D), dtype=torch.uint8, device=dev)
    scale = torch.empty(n, dtype=torch.float32, device=dev)
    if n and d:
        tab, rows, sb = _sign_rows_bits(s, D, dev)
        ws = _ws(n, d, dev)
        _lib.check(_lib.load().uq_eden_compress_f32_sb(_ptr(x), n, d, nb, _ptr(tab), _ptr(rows), _ptr(sb), _ptr(bins),
                                                       _ptr(scale), _ptr(ws), ws.numel(), _stream_ptr(dev)),
                   "uq_eden_compress_f32_sb")
    return EdenMessage(bins=bins, scale=scale, seeds=s, nbits=nb, dim=d)


def eden_decompress(msg: EdenMessage) -> torch.Tensor:
    """EdenReceiver.decompress (AS:383-413) for every row."""
    dev = _device()
    bins = msg.bins.to(dev).contiguous()
    scale = msg.scale.to(device=dev, dtype=torch.float32).contiguous()
    n = bins.shape[0]
    d = msg.dim
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    if n and d:
        tab, rows, sb = _sign_rows_bits(torch.as_tensor(msg.seeds), bins.shape[1], dev)
        ws = _ws(n, d, dev)
        _lib.check(_lib.load().uq_eden_decompress_f32_sb(_ptr(bins), _ptr(scale), n, d, msg.nbits, _ptr(tab),
                                                         _ptr(rows), _ptr(sb), _ptr(out), _ptr(ws), ws.numel(),
                                                         _stream_ptr(dev)), "uq_eden_decompress_f32_sb")
    return out


def eden_quantize(x, bits_per_dimension=1, seeds=None, *, return_scale: bool = False, generator=None):
    """EDEN_quantize_Hadamard for every row of x [n, d] (rotation seed per row)."""
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    nb = _bits(bits_per_dimension)
    s = _seeds(seeds, n, generator)
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    scale = torch.empty(n, dtype=torch.float32, device=dev)
    if n and d:
        tab, rows, sb = _sign_rows_bits(s, padded_dim(d), dev)
        ws = _ws(n, d, dev)
        _lib.check(_lib.load().uq_eden_f32_sb(_ptr(x), _ptr(out), n, d, nb, _ptr(tab), _ptr(rows), _ptr(sb),
                                              _ptr(scale), _ptr(ws), ws.numel(), _stream_ptr(dev)), "uq_eden_f32_sb")
    return (out, scale) if return_scale else out


def _rht(x, seeds, inverse: bool):
    dev = _device()
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    D = padded_dim(d)
    if inverse and d != D:
        raise ValueError("the inverse transform takes power-of-two rows (AS:146-153)")
    s = torch.as_tensor(seeds, dtype=torch.int64).reshape(-1)
    if s.numel() != n:
        raise ValueError("one seed per row")
    out = torch.empty((n, D), dtype=torch.float32, device=dev)
    if n and d:
        tab, rows = _sign_rows(s, D, dev)
        ws = _ws(n, D, dev)
        _lib.check(_lib.load().uq_rht_f32(_ptr(x), _ptr(out), n, d, int(inverse), _ptr(tab), _ptr(rows), _ptr(ws),
                                          ws.numel(), _stream_ptr(dev)), "uq_rht_f32")
    return out


def randomized_hadamard_transform(x, seeds) -> torch.Tensor:
    """HadamardSender.randomized_hadamard_transform (AS:123-141) per row: zero-pad to a
    power of two, multiply by the seeded diagonal, normalized Walsh-Hadamard transform."""
    return _rht(x, seeds, False)


def randomized_inverse_hadamard_transform(x, seeds) -> torch.Tensor:
    """HadamardReceiver.randomized_inverse_hadamard_transform (AS:146-153) per row."""
    return _rht(x, seeds, True)


def EDEN_quantize_Hadamard(input_vector, bits_per_dimension=1):
    """Drop-in for AS:792 (same name for the drivers' result keys).  Draws the rotation
    seed from torch's global CPU generator like the CPU reference (AS:797) and returns a
    NumPy f32 array (AS:811)."""
    dev = _device()
    if torch.is_tensor(input_vector):
        v = input_vector.detach().to(device=dev, dtype=torch.float32).reshape(-1)
    else:
        v = torch.tensor(np.asarray(input_vector), dtype=torch.float32, device=dev).reshape(-1)
    seed = int(torch.randint(0, _SEEDS, (1,)).item())
    out = eden_quantize(v.view(1, -1), bits_per_dimension, seeds=[seed])
    # the NumPy result comes back through pinned memory (torch's caching host allocator):
    # a pageable 4 MB copy costs ~1 ms, about twice the whole GPU work at d = 2^20
    host = torch.empty(out.numel(), dtype=torch.float32, pin_memory=True)
    host.copy_(out.view(-1))
    return host.numpy()
