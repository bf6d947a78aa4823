"""Phase timers of the torch-tie replay workgroups (rez_ties_kernel): a scratch build whose
TT_* hooks (uq_biased_torch_ties.h, no-ops in the product) accumulate wall-clock deltas of
workgroup thread 0 per phase.  Timing probe only; the product library is untouched.

    python tools/exp/tie_prof.py build          # here (CPU): tools/exp/_tieprof/libuq_dme.so
    python tools/exp/tie_prof.py run [--steps 3] # on the GPU box: per-call phase sums

Phases: 0 queue fill, 1 stop counts + lists (global levels), 2 J search, 3 swaps, 4 median
to first, 8 LDS copy in, 7 workgroup LDS levels, 9 one-wave LDS levels, 5 copy out, 10 insertion sort, 6 marking;
inside the one-wave levels: 11 level count (x 1), 15 median, 12 stops, 13 J search, 14 swaps."""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
OUT = os.path.join(ROOT, "tools", "exp", "_tieprof")
SO = os.path.join(OUT, "libuq_dme.so")
sys.path.insert(0, ROOT)

TIMERS = """#define TT_DECL() uint64_t _tt0 = 0; (void)_tt0
#define TT_T0() _tt0 = wall_clock64()
#define TT_ACC(k) do { if (threadIdx.x == 0) { const uint64_t _t = wall_clock64(); \\
    atomicAdd((unsigned long long*)&g_tie_prof[k], (unsigned long long)(_t - _tt0)); _tt0 = _t; } } while (0)
#define TT_CNT(k) do { if (threadIdx.x == 0) atomicAdd((unsigned long long*)&g_tie_prof[k], 100ull); } while (0)
__device__ unsigned long long g_tie_prof[16];
"""
FETCH = """
extern "C" int uq_exp_tie_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tie_prof), sizeof(unsigned long long) * 16) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tie_prof), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
"""


def build():
    from importlib import util
    spec = util.spec_from_file_location("build_ext", os.path.join(PKG, "build_ext.py"))
    be = util.module_from_spec(spec)
    spec.loader.exec_module(be)
    src = os.path.join(OUT, "pkg", "csrc")
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(src)
    os.symlink(os.path.join(ROOT, "include"), os.path.join(OUT, "include"))
    for f in os.listdir(os.path.join(PKG, "csrc")):
        shutil.copy(os.path.join(PKG, "csrc", f), src)
    h = os.path.join(src, "uq_biased_torch_ties.h")
    t = open(h).read()
    noop = ("#define TT_DECL() do {} while (0)\n#define TT_T0() do {} while (0)\n"
            "#define TT_ACC(k) do {} while (0)\n#define TT_CNT(k) do {} while (0)\n")
    assert noop in t
    open(h, "w").write(t.replace(noop, TIMERS))
    main = os.path.join(src, "uq_dme.hip")
    open(main, "a").write(FETCH)
    obj = os.path.join(OUT, "uq_mt_poly.o")
    subprocess.run(["g++", *be.HOST_FLAGS, "-c", "-o", obj, os.path.join(src, "uq_mt_poly.cpp")], check=True)
    subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-o", SO, main, "-x", "none", obj], check=True)
    print("built", SO)


def run(steps):
    import torch
    import uqdme
    from uqdme_amd import build_ext, _lib
    build_ext.SO = SO
    lib = _lib.load()
    lib.uq_exp_tie_prof.restype = ctypes.c_int
    lib.uq_exp_tie_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    n, d = 1024, 1 << 20
    x = torch.randn(n, d, generator=g, device=dev)
    out = torch.empty_like(x)
    m = uqdme.rate_to_m(1, d)
    buf = (ctypes.c_ulonglong * 16)()
    uqdme.biased_quantize(x, m=m, torch_threads=1, ties="torch", out=out)
    torch.cuda.synchronize()
    lib.uq_exp_tie_prof(buf, 1)
    for _ in range(steps):
        uqdme.biased_quantize(x, m=m, torch_threads=1, ties="torch", out=out)
    torch.cuda.synchronize()
    lib.uq_exp_tie_prof(buf, 1)
    _, info = uqdme.biased_quantize(x, m=m, torch_threads=1, ties="torch", out=out, return_info=True)
    amb = int(((info[:, 1] & 1) != 0).sum())
    # wall_clock64 runs at 100 MHz: ticks * 10 ns
    names = ["fill", "stops", "jsearch", "swaps", "median", "lds_copy_out", "mark", "lds_multiwave", "lds_copy_in",
             "wave_levels", "insertion_sort", "wave_level_count", "w_stops", "w_jsearch", "w_swaps", "w_median"]
    per = {nm: round(buf[k] * 0.01 / steps / max(amb, 1), 2) for k, nm in enumerate(names)}
    print(json.dumps({"tool": "tie_prof", "steps": steps, "replayed_clients": amb,
                      "us_per_client_per_call": per,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("UQDME_TIE")}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    build() if a.cmd == "build" else run(a.steps)
