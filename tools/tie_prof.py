"""Phase timers of the tie-replay kernel (KB7): builds uq_dme.hip with -DUQ_TIE_PROF into
_build/abl/tieprof.so, runs one biased call on a resident batch and prints the
accumulated wall-clock time per phase (thread 0 of each workgroup; summed over clients).

    python tools/tie_prof.py build          (container)
    python tools/tie_prof.py run normal 64  (GPU box)"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
SO = os.path.join(PKG, "_build", "abl", "tieprof.so")
def ok(rc):
    """Raise on a non-zero C-ABI status (not an assert: calls must run under python -O)."""
    if rc != 0:
        raise RuntimeError(f"C-ABI call returned {rc}")


PHASES = ["fill", "sweeps", "search", "swaps", "pivot", "lds", "mark", "levels(count)"]


def build():
    sys.path.insert(0, PKG)
    import build_ext as be
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))
    from ablation_src import patched_csrc           # UQ_TIE_PROF lives in tools/exp/ablations.patch
    subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-DUQ_TIE_PROF", "-o", SO,
                    os.path.join(patched_csrc(), "uq_dme.hip")], check=True)


def run(dist, n):
    import torch
    d = 1 << 20
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(n, d, generator=g, device="cuda") if dist == "normal" else \
        torch.randint(-3, 4, (n, d), generator=g, device="cuda").float()
    out = torch.empty_like(x)
    info = torch.empty((n, 2), dtype=torch.int32, device="cuda")
    L = ctypes.CDLL(SO)
    b = ctypes.c_size_t()
    ok(L.uq_biased_workspace_bytes(ctypes.c_int64(n), ctypes.c_int64(d), 1, ctypes.byref(b)))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    prof = torch.zeros(8, dtype=torch.int64, device="cuda")
    L.uq_debug_set_tie_prof.argtypes = [ctypes.c_void_p]
    f = L.uq_type_biased_f32
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int64] * 3 + [ctypes.c_int32] * 2 + \
                 [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p]
    sp = torch.cuda.current_stream().cuda_stream
    call = lambda: f(x.data_ptr(), out.data_ptr(), n, d, 224426, 1, 0, None, info.data_ptr(), ws.data_ptr(),  # noqa
                     b.value, sp)
    ok(call())
    torch.cuda.synchronize()
    ok(L.uq_debug_set_tie_prof(ctypes.c_void_p(prof.data_ptr())))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ok(call())
    e1.record()
    torch.cuda.synchronize()
    amb = int(((info[:, 1] & 8) != 0).sum())
    p = prof.cpu().tolist()
    print(f"dist={dist} n={n} replayed={amb} call_ms={e0.elapsed_time(e1):.3f}")
    for k, v in zip(PHASES, p):
        per = v / max(amb, 1)
        print(f"  {k:14s} total {v / 100.0:10.1f} us   per client {per / 100.0 if k != 'levels(count)' else per:9.1f}")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run(sys.argv[2], int(sys.argv[3]))
