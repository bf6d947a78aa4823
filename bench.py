"""Throughput bench for the unbiased L1-ball type quantizer (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
Without an external launcher, --gpus N > 1 starts the N rank processes itself (spawn_ranks:
child processes with the launcher's environment, rank 0's JSON line forwarded, non-zero exit
if any rank fails); under a launcher --gpus must equal WORLD_SIZE.

Workload (BASELINE.json configs[1], "C2"): per GPU, n=1024 client vectors of d=2^20
i.i.d. N(0,1) f32, resident in HBM before timing; rate R=1 (m = 224426); L1 in the
torch-CPU order of 1 thread.  One step = one pass of the hot path over the batch:
    K1 torch-order L1 (AS:624)  ->  K2 fused quantize/dequantize (AS:625-640; writes the
    dequantized q and the type codes as 4-bit fields)  ->  K3n client-ordered mean from the
    codes (ND:137-138, bit-identical to the mean of q)  ->  [N>1] one RCCL reduce of est to rank 0.
(--pipeline auto = codes4 where its counts fit (R <= 2, n >= 256, d % 4096 == 0), else codes:
int8 codes; q: K2 writes q only and K3 reads q; encode: int8 codes only.)
Clients shard across GPUs with no data-path collective except that final reduce
(weak scaling: 1024 clients per GPU).  value = all clients processed / max-over-ranks
time, in M-vectors/s.

Rank 0 prints ONE JSON line.  `roofline` is computed for K2 from HIP events recorded
around its launches inside the timed region.  Algorithmic bytes follow SURVEY.md §8(d):
8*d per vector for quantize+dequantize (read x, write q); the code stream K2 also writes
(0.5*d as 4-bit fields, 1*d as int8) is implementation traffic, reported apart (`impl_bytes_per_launch`) and never
counted as achieved bandwidth; --pipeline encode (no q) counts 4*d.  `roofline.step` prices
the whole step the same way (8*d per vector / ms_per_step) and sets the PMC traffic of all
the step's kernels against it.  W warmup steps run first.  `cpu_baseline` times the C
restatement of the reference path (oracle/, the checker) on this host: the whole batch
with clients over all the host's allotted cores (OpenMP) and a bounded single-thread
sample; the batch doubles as a bit-parity and NMSE check of the GPU output.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "quantize+dequantize M-vectors/sec at d=2^20 (1/2/4/8 GPU) + NMSE vs reference"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without an external launcher (WORLD_SIZE unset) N > 1 "
                         "starts N rank processes itself; under torch.distributed.run it must equal "
                         "WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clients", type=int, default=1024, help="clients per GPU")
    ap.add_argument("--dim", type=int, default=1 << 20)
    ap.add_argument("--bits", type=float, default=1)
    ap.add_argument("--torch-threads", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--dist", choices=["normal", "laplace", "uniform"], default="normal",
                    help="client vectors: N(0,1) (C2), Laplace(1,2) as Laplace_dist.py:89 or U(-1,1) (C3 sweeps)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="budget of the single-thread CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None, help="PMC traffic summary (default: newest profiles/pmc_*.json)")
    ap.add_argument("--mean-mode", choices=["reduce", "ordered"], default="reduce",
                    help="N>1: one RCCL reduce of per-rank partial means, or the bit-exact ordered chain")
    ap.add_argument("--pipeline", choices=["auto", "q", "codes", "codes4", "encode"], default="auto",
                    help="q: K2 writes the dequantized q, mean reads q (the reference's drop-in semantics); "
                         "codes: K2 writes q AND type codes, mean decodes codes; "
                         "encode: K2 writes codes only, the mean kernel dequantizes (DME wire pipeline)")
    ap.add_argument("--probe-candidates", type=int, default=16,
                    help="at most this many output-buffer sets probed once before warmup, until both "
                         "speeds are seen (pipeline.py); <= 1: no probe")
    ap.add_argument("--probe-min", type=int, default=16,
                    help="output sets the placement probe always times (16 x 5 GB at C2, freed after): the "
                         "fastest of all 16 ran K2 1.69-1.71 ms in three processes, the spread-stop rule "
                         "1.70-1.74 ms (profiles/r05b_exp_probe_all.jsonl)")
    ap.add_argument("--side-pipelines", action="store_true", default=True,
                    help="also time the other pipelines (reported under 'pipelines')")
    ap.add_argument("--no-side-pipelines", dest="side_pipelines", action="store_false")
    return ap.parse_args(argv)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, cmd, env=None, port=None, out=None, grace_s: float = 30.0) -> int:
    """`bench.py --gpus N` without an external launcher: start N rank processes of `cmd` (fresh
    interpreters, no exec; this parent never touches the GPU) with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as torch.distributed.run would, forward rank
    0's stdout (the JSON line) to `out`, send the other ranks' stdout to stderr, and return
    0 only if every rank exits 0.  When one rank fails the others get `grace_s` seconds to end
    (a peer blocked in a collective would otherwise wait forever) and are then terminated."""
    import subprocess
    import threading
    out = out if out is not None else sys.stdout
    port = port or free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))

    def pump():
        for line in procs[0].stdout:
            out.write(line)
            out.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    failed_at = None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            break
        if failed_at is None and any(c not in (None, 0) for c in codes):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.05)
    th.join(5)
    codes = [p.wait() for p in procs]
    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
    if bad:
        print(f"bench.py: rank(s) failed: {bad}", file=sys.stderr, flush=True)
        return 1
    return 0


def world_from_env(args) -> int:
    """The launcher's WORLD_SIZE must agree with --gpus (SystemExit otherwise)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:
        args.gpus = world
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (the launcher started "
                         f"{world} rank(s)); pass the same N to both")
    return world


# RCCL (backend "nccl") is the product path.  UQDME_BENCH_BACKEND=gloo is a rehearsal knob
# that lets several ranks share one GPU; it stages the one reduce through host memory.
BACKEND = os.environ.get("UQDME_BENCH_BACKEND", "nccl")


def dist_init(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())    # one rank per GPU; wraps if fewer GPUs
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:    # rehearsal only: ranks sharing one GPU (RCCL refuses duplicate devices)
            dist.init_process_group("gloo")
        return dist, rank, world, local
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def rank_record(rank, local, seg_ms, probe, elapsed_s, reduce_alone=None):
    """One rank's own timings for the per_rank list of rank 0's line: each rank draws its own
    output placement (pipeline.py probe), so a slow rank must be visible next to rank 0."""
    return {"rank": int(rank), "local_rank": int(local),
            "l1_ms": round(float(seg_ms[0]), 4), "quantize_ms": round(float(seg_ms[1]), 4),
            "client_mean_ms": round(float(seg_ms[2]), 4), "reduce_segment_ms": round(float(seg_ms[3]), 4),
            "quantize_ms_probed": probe["k2_ms_chosen"] if probe else None,
            "quantize_ms_median_unprobed": probe["k2_ms_median_unprobed"] if probe else None,
            "probe_spread_ms": (round(max(probe["k2_ms"]) - min(probe["k2_ms"]), 4) if probe and probe.get("k2_ms")
                                else None),
            "elapsed_s": round(float(elapsed_s), 6), "reduce_alone_ms": reduce_alone}


def gather_per_rank(dist, rank, record):
    """Every rank's record on rank 0 (a list ordered by rank), None on the others; [record]
    without a process group."""
    if dist is None:
        return [record]
    objs = [None] * dist.get_world_size() if rank == 0 else None
    dist.gather_object(record, objs, dst=0)
    return objs


def load_traffic(path, d, n, pipeline):
    """Per-launch HBM bytes of the quantize kernel from a committed PMC summary of the
    same workload and pipeline (profiles/pmc_*.json, written by tools/summarize_profile.py)."""
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    for p in reversed(cands):
        try:
            j = json.load(open(p))
        except Exception:
            continue
        if (j.get("d") == d and j.get("clients") == n and j.get("pipeline", "q") == pipeline
                and "quantize_bytes_per_launch" in j):
            # one launch each of the step's kernels (input generation and fills excluded)
            step = sum(v["hbm_bytes"] for k, v in j.get("kernels", {}).items()
                       if any(s in k for s in STEP_KERNELS)) or None
            return float(j["quantize_bytes_per_launch"]), os.path.relpath(p, ROOT), step
    return None, None, None


PIPELINE_WHAT = {
    "q": "drop-in equivalent: K2 writes the dequantized q only (what Type_unbiased_quantize returns), "
         "the client mean reads q (ND:137-138)",
    "codes": "K2 writes q and int8 type codes, the client mean decodes the codes (same est bits)",
    "encode": "K2 writes int8 type codes only (no per-client q), the mean kernel dequantizes them",
    "codes4": "K2 writes q and 4-bit type codes, the client mean decodes them (same est bits; kmax > 7 from q)",
}

# kernels launched once per bench step (tools/summarize_profile.py keeps one entry per name)
STEP_KERNELS = ("l1_partial_kernel", "l1_finalize_kernel", "quantize_stream_kernel", "codes_mean_kernel",
                "nibbles_mean_kernel", "client_mean_kernel")


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no external launcher: one child process per rank (started before anything here
        # initialises the GPU; children are new processes, never an exec of this one)
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world_from_env(args)
    dist, rank, world, local = dist_init(args)
    import uqdme

    dev = torch.device("cuda", torch.cuda.current_device())
    n, d = args.clients, args.dim
    m = uqdme.rate_to_m(args.bits, d)
    T = args.torch_threads
    if args.pipeline == "auto":         # 4-bit codes where every count fits (pipeline.py)
        args.pipeline = "codes4" if uqdme.codes4_fits(n, d, args.bits) else "codes"
    n_total = n * world

    # ---- synthetic inputs resident in HBM (generation is outside the timed region) ----
    g = torch.Generator(device=dev).manual_seed(args.seed + 7919 * rank)
    if args.dist == "normal":
        x = torch.randn(n, d, generator=g, device=dev, dtype=torch.float32)
    elif args.dist == "laplace":        # loc 1, scale 2 by inversion of a uniform draw
        # u in (-1/2, 1/2) strictly (|u| = 1/2 would invert to -inf): clamp to 1/2 - 2^-25
        lim = 0.5 - 2.0 ** -25
        u = (torch.rand(n, d, generator=g, device=dev, dtype=torch.float32) - 0.5).clamp_(-lim, lim)
        x = 1.0 - 2.0 * torch.sign(u) * torch.log1p(-2.0 * u.abs())
        del u
    else:
        x = torch.rand(n, d, generator=g, device=dev, dtype=torch.float32) * 2.0 - 1.0
    X_cpu = torch.rand(n_total, generator=torch.Generator().manual_seed(args.seed))[rank * n:(rank + 1) * n]
    X = X_cpu.to(dev)
    # the library's multi-GPU product API (distributed.ShardedDME): a resident DMEPipeline
    # (K1 -> K2 -> K3c) per rank, then ONE RCCL reduce of est to rank 0 (N > 1; with RCCL the
    # reduce of step k runs beside step k+1's kernels, see ShardedDME).  The output placement
    # is probed once (pipeline.py: K2's speed follows where q and the codes land).
    if args.mean_mode == "ordered" and args.pipeline == "encode" and world > 1:
        raise SystemExit("--mean-mode ordered folds q across ranks: use --pipeline codes or q")
    sh = uqdme.ShardedDME(n, d, n_total, m=m, torch_threads=T, pipeline="codes4" if args.pipeline == "codes4" else "codes",
                          mode=args.mean_mode)
    pipe = sh.pipe
    probe = sh.probe_outputs(x, X, candidates=args.probe_candidates, min_candidates=args.probe_min) \
        if args.probe_candidates > 1 else None
    q, ovf = pipe.q, pipe.kmax
    stream = torch.cuda.current_stream(dev)
    overlap = sh.overlap

    def time_pipeline(pipeline, steps):
        for _ in range(2):
            sh.step(x, X, pipeline=pipeline)
        sh.drain()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            sh.step(x, X, pipeline=pipeline)
        sh.drain()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    for _ in range(args.warmup):                  # W untimed warmup steps
        sh.step(x, X, pipeline=args.pipeline)
    sh.drain()
    torch.cuda.synchronize()
    pipe.check_status()                           # status after warmup
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        sh.step(x, X, events=evs[k], pipeline=args.pipeline)
    sh.drain()                                    # every reduce inside the timed region
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    pipe.check_status()                           # status after the timed steps
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    reduce_alone = None
    if dist is not None and args.mean_mode == "reduce" and BACKEND == "nccl":
        # the collective by itself (the timed steps overlap it, so their 'reduce' segment
        # only covers its enqueue): events around reduce + wait on the caller's stream
        ra = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            w = dist.reduce(pipe.est, dst=0, op=dist.ReduceOp.SUM, async_op=True)
            w.wait()
            e1.record(stream)
            torch.cuda.synchronize()
            ra.append(e0.elapsed_time(e1))
        reduce_alone = round(float(np.median(ra)), 4)

    seg = np.array([[evs[k][i].elapsed_time(evs[k][i + 1]) for i in range(4)] for k in range(args.steps)])
    seg_ms = seg.mean(axis=0)  # l1, quantize, mean, reduce
    per_rank = gather_per_rank(dist, rank, rank_record(rank, local, seg_ms, probe, elapsed_local, reduce_alone))
    ms_per_step = elapsed * 1e3 / args.steps
    value = n_total * args.steps / elapsed / 1e6

    q_ms = float(seg_ms[1])
    # algorithmic bytes per K2 launch: read x (4d) + write q (4d); the int8
    # code stream (1d) is this design's own traffic and is reported apart, not as achieved
    alg_bytes = float(d * n) * (8 if args.pipeline in ("q", "codes", "codes4") else 4)
    impl_bytes = float(d * n) * {"q": 0.0, "codes4": 0.5}.get(args.pipeline, 1.0)
    achieved = alg_bytes / (q_ms * 1e-3) / 1e9
    traffic, traffic_src, step_traffic = load_traffic(args.traffic_json, d, n, args.pipeline)
    step_alg = float(d * n_total) * 8 / world      # quantize+dequantize bytes of one rank's clients
    step_achieved = step_alg / (ms_per_step * 1e-3) / 1e9
    # CPU baseline + parity sample on the timed steps' own output q (before any side line)
    base = parity = None
    if world == 1 and not args.no_cpu_baseline:
        base, parity = cpu_baseline(args, x, X_cpu, q, m, T)
    side = {}
    if args.side_pipelines and world == 1:
        for pl in ("q", "codes", "encode", "codes4"):
            if pl != args.pipeline and (pl != "codes4" or uqdme.codes4_fits(n, d, args.bits)):
                ms = time_pipeline(pl, max(3, args.steps // 2))
                side[pl] = {"ms_per_step": round(ms, 4), "value": round(n_total / ms / 1e3, 6),
                            "what": PIPELINE_WHAT[pl]}
        pipe.check_status()                       # status after the side pipelines
        side["biased"] = time_biased(uqdme, x, args.bits, T, max(3, args.steps // 2))
        side["eden"] = time_eden(uqdme, x, q, max(3, args.steps // 2))
        side["codec"] = time_codec(uqdme, pipe, max(3, args.steps // 2))
        side["quicfl"] = time_quicfl(uqdme, x, max(2, args.steps // 4))
        if int(torch.count_nonzero(ovf > 127)):
            raise RuntimeError("type-code overflow in the bench workload")

    result = None
    if rank == 0:
        result = {
            "metric": METRIC, "value": round(value, 6), "unit": "M-vectors/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": {"normal": "synthetic: i.i.d. N(0,1) f32 per client (torch CUDA generator)",
                     "laplace": "synthetic: i.i.d. Laplace(1,2) f32 per client (torch CUDA generator, inversion)",
                     "uniform": "synthetic: i.i.d. U(-1,1) f32 per client (torch CUDA generator)"}[args.dist]
                    + ", X ~ U[0,1) from a CPU generator",
            "config": {"workload": ("C2 (BASELINE.json configs[1]): 1024 clients/GPU x d=2^20, Gaussian, R=1, "
                                    if args.dist == "normal" else
                                    f"C3-style sweep (BASELINE.json configs[2]): {n} clients/GPU x d=2^20, {args.dist}, R=1, ")
                                   + "unbiased L1 type quantizer + client-ordered mean" + ((" + RCCL reduce" if BACKEND == "nccl" else " + host-staged gloo reduce (rehearsal)") if world > 1 else ""),
                       "dist": args.dist,
                       "clients_per_gpu": n, "d": d, "bits_per_dimension": args.bits, "m": m,
                       "torch_threads_l1_order": T, "parallelism": f"client-sharded x{world}",
                       "mean_mode": (args.mean_mode + (" (RCCL reduce of step k overlapped with step k+1)" if overlap else ""))
                                    if world > 1 else "single",
                       **({"backend": BACKEND} if world > 1 and BACKEND != "nccl" else {}), "pipeline": args.pipeline},
            "kernel_ms": {"l1": round(float(seg_ms[0]), 4), "quantize": round(q_ms, 4),
                          # the probe's median K2 time over all candidate output sets: what a
                          # caller that allocates fresh outputs (no probe) gets on average
                          "quantize_median_unprobed": probe["k2_ms_median_unprobed"] if probe else None,
                          "client_mean": round(float(seg_ms[2]), 4),
                          # overlapped RCCL reduce: the segment times its enqueue only;
                          # reduce_alone = the collective timed by itself after the steps
                          ("reduce_enqueue" if overlap else "reduce"): round(float(seg_ms[3]), 4),
                          "reduce_alone": reduce_alone},
            "per_rank": per_rank,
            "pipelines": side,
            "output_placement_probe": probe,
            "roofline": {"kernel": "quantize_stream_kernel (K2)", "bound": "hbm", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes, "impl_bytes_per_launch": impl_bytes,
                         "alg_bytes_rule": ("8*d per vector (read x, write q), SURVEY.md §8(d); the type codes "
                                            f"({'0.5*d as 4-bit fields' if args.pipeline == 'codes4' else '1*d as int8'})"
                                            " K2 also writes are implementation traffic"
                                            if args.pipeline != "encode" else "4*d per vector (read x); no q"),
                         "step": {"alg_bytes": step_alg, "ms": round(ms_per_step, 4),
                                  "achieved": round(step_achieved, 2),
                                  "frac": round(step_achieved / HBM_PEAK_GBS, 4),
                                  "traffic": step_traffic,
                                  "traffic_over_alg": (round(step_traffic / step_alg, 3) if step_traffic else None),
                                  "what": "whole step (L1 + quantize + mean [+ reduce]) priced at 8*d per vector; "
                                          "traffic = PMC HBM bytes of all the step's kernels per step"}},
        }
        if base is not None:
            result["cpu_baseline"], result["parity_sample"] = base, parity
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def time_biased(uqdme, x, bits, T, steps):
    """Side line: the biased type quantizer (AS:669-687, torch tie policy) on the same
    resident batch, one uq_type_biased_f32 call per step (into its own output buffer)."""
    n, d = x.shape
    q = torch.empty_like(x)
    m = uqdme.rate_to_m(bits, d)
    for _ in range(2):
        uqdme.biased_quantize(x, m=m, torch_threads=T, ties="torch", out=q)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        uqdme.biased_quantize(x, m=m, torch_threads=T, ties="torch", out=q)
    e1.record()
    torch.cuda.synchronize()
    uqdme.check_status()
    ms = e0.elapsed_time(e1) / steps
    return {"ms_per_step": round(ms, 4), "value": round(n / ms / 1e3, 6), "what": "Type_biased_quantize batch, no mean"}


def time_eden(uqdme, x, q, steps):
    """Side line: EDEN + RHT baseline (AS:792-811, 1 bit) on the same resident batch,
    one compress + decompress per step, rotation seeds as the reference draws them."""
    n, d = x.shape
    seeds = torch.randint(0, 100, (n,), generator=torch.Generator().manual_seed(5))
    for _ in range(2):
        out = uqdme.eden_quantize(x, 1, seeds=seeds)
    del out
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        uqdme.eden_quantize(x, 1, seeds=seeds)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    return {"ms_per_step": round(ms, 4), "value": round(n / ms / 1e3, 6), "what": "EDEN 1-bit batch (RHT, bins, scale, inverse RHT), no mean"}


def time_quicfl(uqdme, x, steps):
    """Side line: the QUIC-FL baseline (AS:429-535, 1 bit) on the same resident batch: the
    sender (RHT, norm, KQ1: h stream, SR rounding, table X / p, bernoulli(p_X)) and the receiver
    (KQ2 + inverse RHT) per step.  Sender tables: the synthetic ones the parity fixtures use
    (tests/golden/quicfl_tables.py; the published tables are not in the reference), with the
    reference's data.txt parameters; receiver tables: the reference's."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from quicfl_tables import DATA, sender_tables
    n, d = x.shape
    X, p = sender_tables(1)
    snd = uqdme.QuicFLSender(tables={1: (X, p, DATA[1])})
    rt = np.load(os.path.join(ROOT, "tests", "golden", "quicfl_recv_vectors.npz"))["recv1"]
    seeds, rots, pxs = list(range(n)), [123] * n, list(range(7, 7 + n))
    held = {}

    def timed(f):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / steps, 4)

    res = {"compress_ms": timed(lambda: held.update(
        m=uqdme.quicfl_compress(x, 1, seeds, rots, sender=snd, px_seeds=pxs)))}
    res["decompress_ms"] = timed(lambda: uqdme.quicfl_decompress_messages(held["m"], rt))
    ms = res["compress_ms"] + res["decompress_ms"]
    res.update({"ms_per_step": round(ms, 4), "value": round(n / ms / 1e3, 6),
                "what": "QUIC-FL 1-bit batch (sender + receiver), synthetic sender tables, no mean"})
    return res


def time_codec(uqdme, pipe, steps):
    """Side line: the UQR1 type-message codec (codes.py, uq_tc_*) on the timed steps' type
    codes: encode (int8 codes -> one rANS message per client) and decode, per batch."""
    import ctypes
    from uqdme_amd import _lib
    lib = _lib.load()
    n, d = pipe.n, pipe.d
    b, w = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(lib.uq_tc_bound(d, ctypes.byref(b)), "bound")
    _lib.check(lib.uq_tc_workspace_bytes(n, d, ctypes.byref(w)), "ws")
    data = torch.empty(n * b.value, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ws = torch.empty(w.value, dtype=torch.uint8, device="cuda")
    src = pipe.codes.contiguous()      # the pipeline's rows are pitched; the codec takes dense [n, d]
    codes = torch.empty_like(src)
    l1 = torch.empty_like(pipe.l1)
    km = torch.empty_like(pipe.kmax)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    enc = lambda: _lib.check(lib.uq_tc_encode(P(src), P(pipe.l1), n, d, pipe.m, 0, P(data), data.numel(),  # noqa: E731
                                              P(off), P(ws), ws.numel(), sp), "encode")
    dec = lambda: _lib.check(lib.uq_tc_decode(P(data), data.numel(), P(off), n, d, pipe.m, P(codes), P(l1), P(km),  # noqa: E731
                                              P(status), sp),
                             "decode")
    res = {}
    for name, f in (("encode", enc), ("decode", dec)):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_ms"] = round(e0.elapsed_time(e1) / steps, 4)
    total = int(off[n].item())
    ok = bool(torch.equal(codes, torch.where(src == -1, torch.zeros_like(src), src))
              and int(torch.count_nonzero(status).item()) == 0)
    res.update({"bits_per_dim": round(8.0 * total / (n * d), 4), "bytes_per_client": round(total / n, 1),
                "roundtrip_ok": ok, "what": "UQR1 rANS type messages (value mode) of the bench batch's codes, "
                                            "encode and decode per 1024-client batch"})
    return res


def host_threads() -> int:
    """Cores this process may use: its CPU affinity, capped by OMP_NUM_THREADS when the
    host sets it (the GPU box allots 16 per GPU although it shows many more)."""
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def cpu_baseline(args, x, X_cpu, q, m, T):
    """Time the C restatement of the reference path (oracle/, a checker) on host cores:
    the whole batch with clients spread over all allotted cores (OpenMP; primary entry),
    and a bounded single-thread sample.  The whole-batch output doubles as a bit-parity
    and NMSE check of the GPU's q from the timed steps."""
    from oracle import uq_oracle_c as C
    from oracle import uq_oracle as O
    n, d = x.shape
    xh = x.cpu().numpy()
    Xh = X_cpu.numpy()
    # single thread: a bounded sample spread over the batch
    budget = args.cpu_seconds
    t1 = 0.0
    done = 0
    for j in range(0, n, max(1, n // 64)):
        t0 = time.perf_counter()
        C.quantize_batch(xh[j:j + 1], m, Xh[j:j + 1], T)
        t1 += time.perf_counter() - t0
        done += 1
        if t1 >= budget:
            break
    # all allotted cores: the whole batch (clients are independent, AS:609-641)
    nth = host_threads()
    t0 = time.perf_counter()
    ref, _, used = C.quantize_batch_mt(xh, m, Xh, T, nth)
    t_mt = time.perf_counter() - t0
    qh = q.cpu().numpy()
    mism = int(np.count_nonzero(qh.view(np.uint32) != ref.view(np.uint32)))
    # NMSE on the batch (script formula ND:151-157), GPU vs CPU restatement
    emp = (xh.sum(axis=0, dtype=np.float32) / np.float32(n)).astype(np.float32)
    vns = float(sum(np.sum(np.square(xh[j:j + 64], dtype=np.float64)) for j in range(0, n, 64)))
    nmse_gpu = O.script_nmse(C.client_mean(qh, n), emp, vns, n)
    nmse_cpu = O.script_nmse(C.client_mean(ref, n), emp, vns, n)
    del xh, qh, ref
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ratio = None
    try:
        ratio = json.load(open(os.path.join(ROOT, "profiles", "r02_cpu_port_vs_reference.json")))
    except (OSError, ValueError):
        pass
    base = {"value": round(n / t_mt / 1e6, 9), "unit": "M-vectors/s", "cores": used, "kind": "port",
            "sample": f"all {n} benchmark clients (d=2^20, R=1), C restatement oracle/uq_oracle.c with clients "
                      f"over {used} OpenMP threads (allotted cores; {os.cpu_count()} logical CPUs visible), "
                      f"{t_mt:.2f} s on '{cpu_model}'",
            "ms_per_vector": round(t_mt * 1e3 / n, 4),
            "single_thread": {"value": round(done / t1 / 1e6, 9), "unit": "M-vectors/s", "cores": 1,
                              "ms_per_vector": round(t1 * 1e3 / done, 3),
                              "sample": f"{done} of the {n} clients, one thread, {t1:.1f} s"}}
    if ratio:
        base["port_vs_reference"] = {
            "host": ratio.get("host_cpu"), "logical_cpus": ratio.get("logical_cpus"),
            "source": "profiles/r02_cpu_port_vs_reference.json (tools/cpu_port_ratio.py: the reference's "
                      "Type_unbiased_quantize and this port on the same vectors, one host)",
            **{k: {kk: v[kk] for kk in ("reference_ms_per_vector", "port_ms_per_vector",
                                        "port_speedup_over_reference", "bit_mismatches")}
               for k, v in ratio.items() if k.startswith("threads_")}}
    par = {"clients_checked": n, "bit_mismatches": mism, "nmse_gpu": nmse_gpu, "nmse_cpu": nmse_cpu,
           "nmse_rel_diff": abs(nmse_gpu - nmse_cpu) / max(nmse_cpu, 1e-300)}
    return base, par


if __name__ == "__main__":
    main()
