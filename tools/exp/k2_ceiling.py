"""K2's ceilings in BOTH placement modes: the product kernel, its arithmetic-free copy
variant (-DUQ_ABL_COPY: same loads, LDS images and stores) and its memory-free variant
(-DUQ_ABL_NOIO: every access dropped), each timed on the fastest and on the slowest of six
output sets (placement probe of pipeline.py).  Round 1 measured the ceilings without
knowing the mode.  Results of ablated builds are wrong by construction (timing only).
    python tools/exp/k2_ceiling.py build    (container: patched builds into _build/abl_ceiling)
    python tools/exp/k2_ceiling.py run      (GPU box)"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
OUT = os.path.join(PKG, "_build", "abl_ceiling")
VARIANTS = {"copy": ["-DUQ_ABL_COPY"], "noio": ["-DUQ_ABL_NOIO"]}


def build():
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import build_ext as be
    from ablation_src import patched_csrc
    src = os.path.join(patched_csrc(), "uq_dme.hip")
    os.makedirs(OUT, exist_ok=True)
    for k, fl in VARIANTS.items():
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, *fl, "-o", os.path.join(OUT, f"{k}.so"), src], check=True)


def run():
    import torch
    sys.path.insert(0, ROOT)
    import uqdme
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    x = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    p = uqdme.DMEPipeline(n, d, m=m, torch_threads=1)
    p.l1_norms(x)
    sets = [(p.q, p.codes)] + [p._alloc_outputs() for _ in range(5)]
    libs = {"product": p.lib}
    for k in VARIANTS:
        L = ctypes.CDLL(os.path.join(OUT, f"{k}.so"))
        L.uq_type_unbiased_codes_f32.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 3 + \
            [ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        libs[k] = L
    sp = torch.cuda.current_stream().cuda_stream

    def t(L, q, c, reps=5):
        f = lambda: L.uq_type_unbiased_codes_f32(x.data_ptr(), 0 if q is None else q.data_ptr(),  # noqa: E731
                                                 0 if c is None else c.data_ptr(), p.kmax.data_ptr(), n, d, m,
                                                 X.data_ptr(), p.l1.data_ptr(), None, 1, p.ws.data_ptr(), p.ws_bytes, sp)
        for _ in range(2):
            if f() != 0:
                raise RuntimeError("launch failed")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    base = [t(p.lib, q, c) for q, c in sets]
    fast, slow = min(range(6), key=lambda i: base[i]), max(range(6), key=lambda i: base[i])
    print(json.dumps({"probe_q+codes_ms": base, "fast_set": fast, "slow_set": slow}), flush=True)
    for name, L in libs.items():
        for mode, i in (("fast", fast), ("slow", slow)):
            q, c = sets[i]
            print(json.dumps({"variant": name, "mode": mode, "q+codes_ms": t(L, q, c), "q_only_ms": t(L, q, None),
                              "codes_only_ms": t(L, None, c)}), flush=True)
    p.check_status()


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
