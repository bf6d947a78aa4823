"""DME NMSE harness: the unbiased-type-quantizer slice of the reference drivers
NMSE_Results/Codes/{Normal,Laplace,Gamma,Bernoulli,Lognormal}_dist.py (ND:77-221),
running every quantization and client mean on the HIP path.

Semantics kept from the reference (ND = Normal_dist.py):
  ND:14-15    np.random.seed(seed); torch.manual_seed(seed)   (here: a private CPU
              torch.Generator, so the caller's global RNG is untouched)
  ND:88-91    per instance, n vectors drawn with legacy np.random (f64) -> f32
  ND:94-95    vec_norm_squared = sum ||v||^2 (f64); emp = stack(v).sum(0) / n (f32, torch CPU)
  ND:133-138  per client, in order, every rate: est_R += Q(v, R) / n; one U[0,1) draw per
              call in call order (client-major, rate-minor)
  ND:151-157  NMSE = ||est - emp||^2 / (num_trials * vec_norm_squared * n)   ("script" NMSE,
              scales as 1/n^3); the standard NMSE = script * num_trials * n^2 is also returned
  ND:193-221  max / mean over instances
The reference also calls other schemes in the same loop (ND:133-147), consuming the
global torch RNG in client-major, scheme-minor order.  `schemes` selects which of the
implemented ones run, in the reference's call order: EDEN_quantize_Hadamard (ND:135-136,
one randint(0, 100) per call), Type_unbiased_quantize (ND:137-138, one rand(1) per call),
Type_biased_quantize (ND:139-140, no draws), QUICFL_quantize (ND:141-142: one randint(0, 100)
for the message seed, then D words of the same generator for bernoulli(p_X), AS:489 -- the host
advances a copy of the CPU generator past those words and hands each message its generator
state, so the batched sender draws exactly the reference's words; tables from `quicfl=(sender,
receiver)` or the drop-in's prefix).  DRIVE / Kashin / Scalar are not built, so the draw stream
equals that of a driver calling only the selected schemes.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import torch

from . import _lib
from .biased import biased_quantize
from .eden import eden_compress, eden_decompress, eden_quantize
from .quantizer import client_mean, quantize_dequantize
from .quicfl import quicfl_quantize

SCHEME_ORDER = ("eden", "unbiased", "biased", "quicfl")     # ND:135-142 call order

__all__ = ["DISTRIBUTIONS", "draw_vectors", "legacy_draw", "nmse_simulation", "Suspended", "USERS_ND"]

# ND:43 (also Lognormal_dist.py:43): num_users_list = arange(1, 102, 5); Laplace/Gamma/
# Bernoulli drivers use arange(1, 101, 5).
USERS_ND = tuple(range(1, 102, 5))

# ND:89, Laplace_dist.py:89, Gamma_dist.py:86, Bernoulli_dist.py:90, Lognormal_dist.py:90;
# "uniform" is build-defined (BASELINE.json config C3), not in the reference.
DISTRIBUTIONS = {
    "normal": lambda rs, d: rs.normal(loc=0, scale=1, size=d),
    "laplace": lambda rs, d: rs.laplace(loc=1, scale=2, size=d),
    "gamma": lambda rs, d: rs.gamma(shape=2, scale=2, size=d),
    "bernoulli": lambda rs, d: rs.choice(np.arange(2), size=d, p=[0.3, 0.7]),
    "lognormal": lambda rs, d: rs.lognormal(mean=1, sigma=2, size=d),
    "uniform": lambda rs, d: rs.uniform(low=-1.0, high=1.0, size=d),
}


def draw_vectors(dist: str, n: int, dim: int, rs=np.random):
    """n f64 vectors in the reference's draw order, their ||v||^2 sum, and the f32 batch."""
    gen = DISTRIBUTIONS[dist]
    vecs, norms = [], []
    for _ in range(n):
        v = np.asarray(gen(rs, dim), dtype=np.float64)
        norms.append(np.linalg.norm(v) ** 2)
        vecs.append(v)
    return vecs, float(sum(norms))


def _cdf2(p):
    """choice(arange(2), p=p)'s cdf as legacy RandomState.choice builds it (cumsum, / last)."""
    c = np.asarray(p, np.float64).cumsum()
    c /= c[-1]
    return float(c[0]), float(c[1])


# dist -> (uq_legacy_draw_f32 code, a, b): the arguments of DISTRIBUTIONS above
LEGACY = {
    "normal": (0, 0.0, 1.0),
    "laplace": (1, 1.0, 2.0),
    "gamma": (2, 2.0, 2.0),
    "bernoulli": (3, *_cdf2([0.3, 0.7])),
    "lognormal": (4, 1.0, 2.0),
    "uniform": (5, -1.0, 2.0),
}


def host_threads() -> int:
    """Host threads for the draws: the CPUs this process may run on, capped by
    $UQDME_DRAW_THREADS or $OMP_NUM_THREADS (the GPU box sets 16, its share of the host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    for var in ("UQDME_DRAW_THREADS", "OMP_NUM_THREADS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            return max(1, min(n, int(v)))
    return max(1, min(n, 64))


def legacy_draw(rs: np.random.RandomState, dist: str, n: int, dim: int, threads: int | None = None,
                out: np.ndarray | None = None):
    """n successive rs.<dist>(size=dim) draws of the drivers (DISTRIBUTIONS), bit-identical to
    RandomState's own, on host threads (uq_legacy_draw_f32, csrc/uq_legacy_rng.cpp); rs is left
    exactly where the n calls leave it.  Returns (f32 batch [n, dim] -- ND:91's cast --, [n] f64
    ||v||^2 as np.linalg.norm(v) ** 2, to the last bits of its summation order)."""
    code, a, b = LEGACY[dist]
    name, key, pos, has_gauss, gauss = rs.get_state(legacy=True)
    if name != "MT19937":
        raise ValueError("legacy MT19937 RandomState required")
    key = np.array(key, dtype=np.uint32)
    pos_, hg_, g_ = ctypes.c_int32(int(pos)), ctypes.c_int32(int(has_gauss)), ctypes.c_double(float(gauss))
    if out is None:
        out = np.empty((n, dim), np.float32)
    elif out.dtype != np.float32 or out.shape != (n, dim) or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous f32 [n, dim] array")
    norms = np.zeros(n, np.float64)
    rc = _lib.load().uq_legacy_draw_f32(key.ctypes.data, ctypes.addressof(pos_), ctypes.addressof(hg_),
                                        ctypes.addressof(g_), code, a, b, n, dim, out.ctypes.data,
                                        norms.ctypes.data, int(threads or host_threads()))
    if rc != 0:
        raise RuntimeError(f"uq_legacy_draw_f32 failed ({rc})")
    rs.set_state(("MT19937", key, pos_.value, hg_.value, g_.value))
    return out, norms


def _draw_ahead(dist: str, users, num_instances: int, dim: int, rs, device=None, threads=None):
    """The instances' batches in the drivers' order, in a three-stage pipeline ahead of the
    caller: yields (x [n, dim] f32 -- on `device`, a CPU tensor if None --, sum ||v||^2 (ND:94,
    summed in the drivers' order), emp (ND:95: the batch's f32 sum over clients / n on the CPU,
    as torch computes it), the legacy state before this batch was drawn).
      * drawer thread: legacy_draw (host threads, the drivers' exact stream; rs is used by this
        thread alone) straight into one of three reusable (pinned, with a device) host buffers;
      * prep thread: emp, and the host-to-device copy on a side stream (ready when yielded;
        the caller records its own stream on the tensor before using it);
      * the caller quantizes the previous batch meanwhile.
    Host memory: three buffers of max(users) * dim f32, plus the draw's f64 values of the batch
    being drawn (8 n * dim bytes, pooled inside the library)."""
    import queue
    import threading

    total = len(users) * num_instances
    stop = threading.Event()
    nmax = max(users) if len(users) else 0
    ring: queue.Queue = queue.Queue()
    for _ in range(3 if total else 0):
        ring.put(torch.empty((nmax, dim), dtype=torch.float32, pin_memory=device is not None))
    q1: queue.Queue = queue.Queue(maxsize=1)
    q2: queue.Queue = queue.Queue(maxsize=1)
    side = torch.cuda.Stream(device) if device is not None else None

    def put(q, item):
        while not stop.is_set():
            try:
                q.put(item, timeout=0.5)
                return True
            except queue.Full:
                pass
        return False

    def get(q):
        while not stop.is_set():
            try:
                return q.get(timeout=0.5)
            except queue.Empty:
                pass
        return None

    def draw():
        try:
            for n in users:
                for _ in range(num_instances):
                    buf = get(ring)
                    if buf is None:
                        return
                    st = rs.get_state(legacy=True)
                    _, norms = legacy_draw(rs, dist, n, dim, threads, out=buf[:n].numpy())   # ND:88-91
                    vns = 0
                    for v in norms.tolist():                                               # ND:94 sum(list)
                        vns += v
                    if not put(q1, (buf, n, float(vns), st)):
                        return
        except BaseException as e:                                            # re-raised by the consumer
            put(q1, e)

    def prep():
        try:
            for _ in range(total):
                item = get(q1)
                if item is None:
                    return
                if isinstance(item, BaseException):
                    put(q2, item)
                    return
                buf, n, vns, st = item
                xs = buf[:n]
                emp = xs.sum(dim=0) / n                                            # ND:95 (CPU)
                if side is not None:
                    with torch.cuda.stream(side):
                        x = xs.to(device, non_blocking=True)
                    side.synchronize()
                else:
                    x = xs.clone()
                ring.put(buf)
                if not put(q2, (x, vns, emp, st)):
                    return
        except BaseException as e:
            put(q2, e)

    workers = [threading.Thread(target=f, daemon=True) for f in (draw, prep)]
    for w in workers:
        w.start()
    try:
        for _ in range(total):
            item = q2.get()
            if isinstance(item, BaseException):
                raise item
            yield item
    finally:
        stop.set()


class Suspended(Exception):
    """nmse_simulation stopped at a user-count boundary (time_limit_s); its checkpoint file
    holds everything needed to resume there."""


def _save_checkpoint(path, meta, ui, rs_state, gen_state, script):
    tmp = path + ".tmp.npz"
    _, key, pos, hg, g = rs_state
    np.savez(tmp, meta=np.frombuffer(repr(meta).encode(), np.uint8), ui=ui, key=np.asarray(key, np.uint32),
             pos=pos, has_gauss=hg, gauss=g, gen=gen_state.numpy(),
             **{f"script_{sc}_{r}": v for (sc, r), v in script.items()})
    os.replace(tmp, path)


def _client_draws(gen, n, order, rates, qD):
    """ND:133-140's torch draws of n clients, client-major and scheme / rate-minor, from `gen`
    (which ends where the reference's loop leaves torch's global generator): EDEN's rotation
    seed (AS:797), unbiased's X (AS:634), QUIC-FL's prng seed (AS:820), its generator state, and
    its D bernoulli(p_X) words skipped by jump-ahead (AS:489)."""
    from .quicfl import advance_generator, generator_words
    draws = {(sc, r): [] for sc in order for r in rates}
    for _ in range(n):
        for sc in order:
            for r in rates:
                if sc == "eden":
                    draws[(sc, r)].append(int(torch.randint(0, 100, (1,), generator=gen)))   # AS:797
                elif sc == "unbiased":
                    draws[(sc, r)].append(float(torch.rand(1, generator=gen)))               # AS:634
                elif sc == "quicfl":
                    seed = int(torch.randint(0, 100, (1,), generator=gen))                    # AS:820
                    draws[(sc, r)].append((seed, generator_words(gen)[1]))
                    advance_generator(gen, qD)             # past the D bernoulli(p_X) words (AS:489)
    return draws


def _client_words(order, rates, qD):
    """32-bit words of torch's CPU generator one client takes in _client_draws: randint(0, 100)
    and rand(1) one each (ATen's random() for a range below 2^32 / a float), QUIC-FL's seed plus its
    D words."""
    per = {"eden": 1, "unbiased": 1, "biased": 0, "quicfl": 1 + (qD or 0)}
    return sum(per[sc] for sc in order) * len(rates)


def _client_draws_parallel(gen, n, order, rates, qD, pool):
    """_client_draws with each client's share of the stream in its own thread: a client takes a
    fixed number of words (_client_words), so client j starts where j of them leave the stream
    -- one jump-ahead from the instance's first state -- and its QUIC-FL skips are jumps too;
    the jumps (uq_mt_jump_host, ~0.6 ms each, outside the GIL) overlap.  Same values and the same
    end state as the sequential loop (tests/test_dme_draws.py)."""
    from .quicfl import advance_generator, generator_words, set_generator_words
    if n == 0:
        return {(sc, r): [] for sc in order for r in rates}
    st, w0 = generator_words(gen)
    W = _client_words(order, rates, qD)

    def one(j):
        g = torch.Generator()
        set_generator_words(g, st, w0)
        if j:
            advance_generator(g, j * W)
        d = _client_draws(g, 1, order, rates, qD)
        return d, (generator_words(g) if j == n - 1 else None)

    res = list(pool.map(one, range(n))) if pool is not None else [one(j) for j in range(n)]
    draws = {(sc, r): [x for d, _ in res for x in d[(sc, r)]] for sc in order for r in rates}
    end_st, end_w = res[-1][1]
    set_generator_words(gen, end_st, end_w)
    return draws


def nmse_simulation(dist: str = "normal", dim: int = 2048, users=USERS_ND, num_instances: int = 50,
                    num_trials: int = 50, rates=(1, 2), seed: int = 42, torch_threads: int = 1,
                    device=None, schemes=("unbiased",), progress=None, eden_scales=None, eden_scales_out=None,
                    quicfl=None, threads=None, stats=None, checkpoint=None, time_limit_s=None):
    """NMSE curves of the selected schemes with the reference's normalisation.

    Returns {rate: {...}} for the default unbiased-only run, else {(scheme, rate): {...}};
    each value holds "script" ([len(users), num_instances]), "avg", "max", "standard_avg",
    "standard_max".  `progress(n, inst)` is called after each instance (long runs).
    eden_scales {(n, inst, rate): [scale per client]} replaces EDEN's scale (AS:348) by the
    given values (the receiver then runs on them); eden_scales_out, a dict, receives the
    scales computed here under the same keys.  threads: host threads for the draws
    (legacy_draw; default host_threads()).  stats, a dict, receives "wait_s": the time spent
    waiting for drawn batches (the part of the run the host draws did not hide).
    checkpoint: a file path; at the start of every user count the run saves there the legacy and
    torch generator states and the finished rows, and a call with an existing checkpoint of the
    same configuration resumes from it (the streams continue exactly).  time_limit_s: stop at
    the first user-count boundary after that many seconds, raising Suspended (checkpoint saved)."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    schemes = tuple(schemes)
    for sc in schemes:
        if sc not in SCHEME_ORDER:
            raise ValueError(f"unknown scheme {sc!r}")
    order = [sc for sc in SCHEME_ORDER if sc in schemes]
    if "quicfl" in order:
        from .eden import padded_dim
        from .quicfl import _dropin_pair
        qsend, qrecv = quicfl if quicfl is not None else _dropin_pair()
        qD = padded_dim(dim)
    rs = np.random.RandomState(seed)                 # legacy stream == np.random.seed(seed)
    gen = torch.Generator().manual_seed(seed)        # == torch.manual_seed(seed) CPU stream
    keys = [(sc, r) for sc in order for r in rates]
    script = {k: np.zeros((len(users), num_instances), np.float64) for k in keys}
    users = tuple(int(u) for u in users)
    meta = (dist, dim, users, num_instances, num_trials, tuple(rates), seed, torch_threads, tuple(order))
    start_ui = 0
    if checkpoint is not None and os.path.exists(checkpoint):
        with np.load(checkpoint, allow_pickle=False) as ck:
            if bytes(ck["meta"]).decode() != repr(meta):
                raise ValueError(f"checkpoint {checkpoint} is of another configuration")
            start_ui = int(ck["ui"])
            rs.set_state(("MT19937", ck["key"], int(ck["pos"]), int(ck["has_gauss"]), float(ck["gauss"])))
            gen.set_state(torch.from_numpy(ck["gen"].copy()))
            for sc, r in keys:
                script[(sc, r)][:] = ck[f"script_{sc}_{r}"]
    t_start = time.perf_counter()
    from concurrent.futures import ThreadPoolExecutor
    jump_pool = None
    if "quicfl" in order:
        jump_pool = ThreadPoolExecutor(max_workers=max(1, min(8, host_threads() // 2)))
    host_pool = ThreadPoolExecutor(max_workers=4) if len(keys) > 1 else None   # the NMSE norms on the host
    batches = _draw_ahead(dist, users[start_ui:], num_instances, dim, rs, device=device, threads=threads)
    for ui in range(start_ui, len(users)):
        n = users[ui]
        for inst in range(num_instances):
            t_wait = time.perf_counter()
            xd, vns, emp, rs_before = next(batches)                                        # ND:88-95
            if stats is not None:
                stats["wait_s"] = stats.get("wait_s", 0.0) + time.perf_counter() - t_wait
            if inst == 0 and checkpoint is not None:       # both streams as they stand before this user count
                _save_checkpoint(checkpoint, meta, ui, rs_before, gen.get_state(), script)
                if time_limit_s is not None and ui > start_ui and time.perf_counter() - t_start > time_limit_s:
                    batches.close()
                    for pool in (jump_pool, host_pool):
                        if pool is not None:
                            pool.shutdown()
                    raise Suspended(f"suspended before user count {n} (index {ui}); resume from {checkpoint}")
            if xd.is_cuda:
                xd.record_stream(torch.cuda.current_stream(device))   # copied on the side stream, used here
            if "quicfl" in order:                     # the clients' torch draws in parallel (exact)
                draws = _client_draws_parallel(gen, n, order, rates, qD, jump_pool)
            else:
                draws = _client_draws(gen, n, order, rates, None)
            ests = {}
            for sc, r in keys:
                if sc == "unbiased":
                    q = quantize_dequantize(xd, r, X=torch.tensor(draws[(sc, r)], dtype=torch.float32),
                                            torch_threads=torch_threads)
                elif sc == "biased":
                    q = biased_quantize(xd, r, torch_threads=torch_threads)
                elif sc == "quicfl":
                    seeds = [s_ for s_, _ in draws[(sc, r)]]
                    states = np.stack([w for _, w in draws[(sc, r)]])
                    q, _, _ = quicfl_quantize(xd, r, seeds, [123] * n, sender=qsend,                 # AS:814-832
                                              recv_table=qrecv.recv_table[r], px_states=states)
                elif eden_scales is None and eden_scales_out is None:
                    q = eden_quantize(xd, r, seeds=draws[(sc, r)])
                else:                                 # compress, (record / replace the scale), decompress
                    msg = eden_compress(xd, r, seeds=draws[(sc, r)])
                    if eden_scales_out is not None:
                        eden_scales_out[(n, inst, r)] = msg.scale.cpu().numpy().copy()
                    if eden_scales is not None:
                        msg.scale = torch.as_tensor(np.asarray(eden_scales[(n, inst, r)], np.float32)).to(device)
                    q = eden_decompress(msg)
                ests[(sc, r)] = client_mean(q, n)
                del q

            def nmse(k):                              # ND:155, on the host as the reference computes it
                return float(torch.norm(ests[k].cpu() - emp).pow(2) / (num_trials * vns * n))
            # every scheme's estimate queued first: the copies and the CPU norms overlap each other
            # and the GPU work still running (same values: each norm is the same call on the same data)
            vals = list(host_pool.map(nmse, keys)) if host_pool is not None else [nmse(k) for k in keys]
            for k, v in zip(keys, vals):
                script[k][ui, inst] = v
            if progress is not None:
                progress(n, inst)
    for pool in (jump_pool, host_pool):
        if pool is not None:
            pool.shutdown()
    if checkpoint is not None:                        # finished: a rerun returns the same rows
        _save_checkpoint(checkpoint, meta, len(users), rs.get_state(legacy=True), gen.get_state(), script)
    out = {}
    for k in keys:
        sv = script[k].astype(np.float32)             # the reference stores NMSE in f32 tensors
        std = sv.astype(np.float64) * num_trials * np.asarray(users, np.float64)[:, None] ** 2
        out[k] = {"script": sv, "avg": sv.mean(axis=1), "max": sv.max(axis=1),
                  "standard_avg": std.mean(axis=1), "standard_max": std.max(axis=1)}
    if schemes == ("unbiased",):
        return {r: out[("unbiased", r)] for r in rates}
    return out
