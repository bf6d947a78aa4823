"""Host logic of the one-shot output pool (outpool.py) on CPU tensors, with HIP events and the
device-memory query replaced by scripted fakes: a held result is never handed out again, the
pool explores `explore` placements, then keeps the `keep` fastest and serves the fastest free
one, and it never grows past its memory cap."""
import pytest
import torch

import uqdme  # noqa: F401  (registers the package as uqdme_amd)
from uqdme_amd import outpool


class FakeEvent:

    def __init__(self, enable_timing=True):
        self.t = None

    def record(self):
        pass

    def query(self):
        return True

    def elapsed_time(self, other):
        return other.ms


class Clock:
    """timed() records (e0, e1); e1.ms is the scripted time of that launch."""

    def __init__(self, monkeypatch, total=1 << 40):
        self.next_ms = 1.0
        clock = self

        class Ev(FakeEvent):
            def record(self):
                self.ms = clock.next_ms

        class Stream:
            cuda_stream = 1

        monkeypatch.setattr(torch.cuda, "Event", Ev)
        monkeypatch.setattr(torch.cuda, "current_stream", lambda dev=None: Stream())
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (total, total))


DEV = torch.device("cpu")
SPEC = [((4, 1024), torch.float32)]        # 16 KiB: above the pool's min_bytes below


def call(pool, clock, ms):
    (out,), tok = pool.acquire(DEV, SPEC)
    clock.next_ms = ms
    pool.timed(tok, lambda: out.fill_(ms))
    return out, tok


def test_small_batches_bypass(monkeypatch):
    Clock(monkeypatch)
    pool = outpool.OutputPool(enabled=True, min_bytes=1 << 20)
    (out,), tok = pool.acquire(DEV, SPEC)
    assert tok is None and out.shape == (4, 1024)


def test_held_results_are_never_reused(monkeypatch):
    clock = Clock(monkeypatch)
    pool = outpool.OutputPool(enabled=True, explore=3, keep=2, min_bytes=1)
    held = []
    for i in range(12):
        out, tok = call(pool, clock, 1.0 + i)
        for h in held:                            # a fresh set, not one a caller still holds
            assert out.data_ptr() != h.data_ptr()
        held.append(out)
        if len(held) > 2:                         # the caller drops all but its last two results
            held.pop(0)
    # aliases keep a set held too: a slice or a NumPy view of an old result
    a, _ = call(pool, clock, 1.0)
    sl = a[1:]
    npv = a.numpy()
    del a
    b, _ = call(pool, clock, 1.0)
    assert b.data_ptr() != sl.data_ptr() - 1024 * 4 and b.data_ptr() != npv.ctypes.data


def test_explores_then_serves_fastest(monkeypatch):
    clock = Clock(monkeypatch)
    pool = outpool.OutputPool(enabled=True, explore=4, keep=2, min_bytes=1)
    times = [3.0, 1.0, 4.0, 2.0]
    ptrs = {}
    for ms in times:                              # results held one call at a time: the pool
        out, _ = call(pool, clock, ms)            # cycles through new placements while exploring
        ptrs[out.data_ptr()] = ms
        del out
    # the slowest two are released once exploration ends; every later free pick is the fastest
    seen = []
    for _ in range(5):
        out, _ = call(pool, clock, 1.0)
        seen.append(ptrs.get(out.data_ptr()))
        del out
    assert seen == [1.0] * 5
    means = list(pool.report().values())[0]
    assert len(means) == 2


def test_fastest_held_falls_back_to_second(monkeypatch):
    clock = Clock(monkeypatch)
    pool = outpool.OutputPool(enabled=True, explore=3, keep=2, min_bytes=1)
    ptrs = {}
    for ms in (2.0, 1.0, 3.0):
        out, _ = call(pool, clock, ms)
        ptrs[out.data_ptr()] = ms
        del out
    first, _ = call(pool, clock, 1.0)              # the fastest, held by the caller
    second, _ = call(pool, clock, 2.0)
    assert ptrs[first.data_ptr()] == 1.0 and ptrs[second.data_ptr()] == 2.0


def test_memory_cap(monkeypatch):
    clock = Clock(monkeypatch, total=64 * 1024)    # 64 KiB "device": max_frac 1/4 -> one 16 KiB set
    pool = outpool.OutputPool(enabled=True, explore=6, keep=2, min_bytes=1, max_frac=0.25, reserve_frac=0.0)
    a, ta = call(pool, clock, 1.0)
    b, tb = call(pool, clock, 1.0)                 # a is held and the cap is reached: plain tensor
    assert ta is not None and tb is None and b.data_ptr() != a.data_ptr()
    pool.clear()
    assert pool.report() == {}


def test_opt_in_and_idle_release(monkeypatch):
    clock = Clock(monkeypatch)
    monkeypatch.delenv("UQDME_OUTPUT_POOL", raising=False)
    off = outpool.OutputPool(min_bytes=1)
    (o,), tok = off.acquire(DEV, SPEC)
    assert not off.enabled and tok is None          # default: off, plain allocations
    monkeypatch.setenv("UQDME_OUTPUT_POOL", "1")
    assert outpool.OutputPool(min_bytes=1).enabled
    pool = outpool.OutputPool(enabled=True, explore=3, keep=2, min_bytes=1, idle_s=0.05)
    out, _ = call(pool, clock, 1.0)
    held = out
    out2, _ = call(pool, clock, 2.0)
    del out2
    import time
    time.sleep(0.1)
    (o,), _ = pool.acquire(DEV, [((2, 8), torch.float32)])  # any call releases idle free sets
    sets = [st for e in pool._sets.values() for st in e["sets"]]
    assert len(sets) == 2                           # the held set stays, the idle free one went
    assert any(st.bufs[0].data_ptr() == held.data_ptr() for st in sets)


if __name__ == "__main__":
    raise SystemExit(pytest.main([__file__, "-q"]))
