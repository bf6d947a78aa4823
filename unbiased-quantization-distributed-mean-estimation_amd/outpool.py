"""Output pool for the one-shot batched APIs (quantize_dequantize, quantize_encode,
quantize_mean): K2's speed depends on where its OUTPUT buffers sit in physical memory
(DESIGN.md §8 and NOTES.md §4, "two speeds": q + codes 1.66-1.76 ms or 1.93-2.03 ms per 1024 x 2^20 batch,
a property of the buffer set, not of the moment).  DMEPipeline probes its resident outputs
once; a caller that asks for fresh outputs on every call would draw a new placement each
time.  For large batches the one-shot APIs therefore take their outputs from this pool:

  * per (device, shapes, dtypes) a few output sets are kept; a set is handed out as fresh
    views only when nothing outside the pool references its storage (torch's storage use
    count: views, slices and NumPy aliases of an earlier result all count), so a result the
    caller still holds is never overwritten;
  * each call is timed with HIP events on its stream; the elapsed time is read lazily
    (event already complete, no synchronisation), and after `explore` sets have each been
    used the slowest free ones are released, so the loop settles on the fastest placements
    (at least two, since a caller typically holds the previous result while asking for the
    next);
  * small batches (< `min_bytes`) bypass the pool: their placement does not matter; the pool
    holds at most `max_frac` of device memory (then a call gets a plain allocation), and
    `POOL.clear()` releases everything it holds.

The pool is OPT-IN (`uqdme.set_output_pool(True)` or UQDME_OUTPUT_POOL=1): it keeps device
memory (up to explore + keep sets per shape, at most `max_frac` of the device) after the call
returns, which a caller that goes on to allocate for other work may not expect.  Off, every
call allocates plainly through torch's caching allocator (and draws a random placement).  On,
sets left unused for `idle_s` seconds are released at the pool's next call, and `clear()`
releases everything at once.

Results are the same bits whichever set is used; only the time differs.
"""
from __future__ import annotations

import os
import threading
import time

import torch

__all__ = ["OutputPool", "POOL", "set_output_pool"]


def _use_count(t: torch.Tensor) -> int:
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


class _Set:
    def __init__(self, bufs):
        self.bufs = bufs                       # base tensors (the pool's own references)
        self.idle = [_use_count(b) for b in bufs]
        self.ms_sum, self.ms_n = 0.0, 0
        self.pending = []                      # (start event, end event) not read yet
        self.stream = None                     # stream of the last launch writing the set
        self.last_use = time.monotonic()

    def free(self, stream=None) -> bool:
        """Nothing outside the pool holds the set, and a launch on another stream than
        `stream` has completed (same-stream reuse is ordered by the stream itself)."""
        if not all(_use_count(b) == c for b, c in zip(self.bufs, self.idle)):
            return False
        return stream is None or self.stream is None or self.stream == stream or not self.pending

    def harvest(self):
        keep = []
        for e0, e1 in self.pending:
            if e1.query():
                self.ms_sum += e0.elapsed_time(e1)
                self.ms_n += 1
            else:
                keep.append((e0, e1))
        self.pending = keep

    def mean(self):
        return self.ms_sum / self.ms_n if self.ms_n else None


class OutputPool:
    def __init__(self, explore: int = 6, keep: int = 2, min_bytes: int = 1 << 28, reserve_frac: float = 0.25,
                 max_frac: float = 0.125, idle_s: float = 30.0, enabled: bool | None = None):
        # max_frac: the pool never holds more than this share of device memory (36 GB of an
        # MI355X's 288 GB); beyond it a call gets a plain allocation
        self.explore, self.keep, self.min_bytes, self.reserve_frac = explore, keep, min_bytes, reserve_frac
        self.max_frac = max_frac
        self._lock = threading.Lock()
        self._sets: dict = {}
        self.idle_s = idle_s
        self.enabled = (os.environ.get("UQDME_OUTPUT_POOL", "0") == "1") if enabled is None else enabled

    def _alloc(self, dev, specs):
        return _Set([torch.empty(shape, dtype=dt, device=dev) for shape, dt in specs])

    def acquire(self, dev, specs):
        """specs: [(shape, dtype), ...] -> (list of fresh views, token) or (new tensors, None)
        for batches below min_bytes.  Pass the token to timed() around the launch."""
        nbytes = sum(torch.Size(s).numel() * torch.empty((), dtype=dt).element_size() for s, dt in specs)
        if not self.enabled or nbytes < self.min_bytes:
            return [torch.empty(s, dtype=dt, device=dev) for s, dt in specs], None
        key = (dev.index, tuple((tuple(s), dt) for s, dt in specs))
        with self._lock:
            self._release_idle()
            ent = self._sets.setdefault(key, {"sets": [], "explored": False})
            sets = ent["sets"]
            for st in sets:
                st.harvest()
            if not ent["explored"] and sum(1 for st in sets if st.ms_n) >= self.explore:
                ent["explored"] = True
            if ent["explored"]:
                self._prune(sets)
            sid = torch.cuda.current_stream(dev).cuda_stream
            free = [st for st in sets if st.free(sid)]
            chosen = None
            untried = [st for st in free if st.ms_n == 0]
            if untried:
                chosen = untried[0]
            elif not ent["explored"] or not free:
                # exploring: a new placement; explored but every kept set is held: one more
                if len(sets) < self.explore + self.keep:
                    fm, tot = torch.cuda.mem_get_info(dev)
                    pooled = sum(sum(b.numel() * b.element_size() for b in st.bufs)
                                 for e in self._sets.values() for st in e["sets"] if e is not None)
                    if fm - nbytes >= self.reserve_frac * tot and pooled + nbytes <= self.max_frac * tot:
                        chosen = self._alloc(dev, specs)
                        sets.append(chosen)
            if chosen is None and free:
                chosen = min(free, key=lambda st: st.mean() if st.ms_n else float("inf"))
            if chosen is None:                 # everything held and no room: a plain allocation
                return [torch.empty(s, dtype=dt, device=dev) for s, dt in specs], None
            chosen.last_use = time.monotonic()
            return [b.view(b.shape) for b in chosen.bufs], chosen

    def _release_idle(self):
        """Drop sets nobody holds that have not been handed out for idle_s seconds."""
        now = time.monotonic()
        for k in list(self._sets):
            sets = self._sets[k]["sets"]
            for st in list(sets):
                st.harvest()
                if now - st.last_use > self.idle_s and st.free() and not st.pending:
                    sets.remove(st)
            if not sets:
                del self._sets[k]

    def _prune(self, sets):
        """Keep the `keep` fastest timed sets (and any set still held); release the rest."""
        ranked = sorted([st for st in sets if st.ms_n], key=lambda st: st.mean())
        for st in ranked[self.keep:]:
            if st.free() and not st.pending:         # (pending: a launch may still write it)
                sets.remove(st)

    def timed(self, token, launch):
        """Run launch() between two events on the current stream, recorded for `token`."""
        if token is None:
            return launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = launch()
        e1.record()
        with self._lock:
            token.pending.append((e0, e1))
            token.stream = torch.cuda.current_stream().cuda_stream
        return out

    def report(self):
        """{key: [mean ms per set]} (sets timed so far)."""
        with self._lock:
            out = {}
            for k, ent in self._sets.items():
                for st in ent["sets"]:
                    st.harvest()
                out[k] = [st.mean() for st in ent["sets"]]
            return out

    def clear(self):
        with self._lock:
            self._sets.clear()


POOL = OutputPool()


def set_output_pool(on: bool) -> None:
    """Turn the one-shot APIs' output pool on or off (off releases what it holds)."""
    POOL.enabled = bool(on)
    if not on:
        POOL.clear()
