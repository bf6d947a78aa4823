"""Timing-only ablation of the EDEN norm kernel (KE2): EDEN compress on 1024 x 2^20 with the
norm's chain work removed (-DUQ_NORM_ABL_NOCHAIN) or its global loads removed
(-DUQ_NORM_ABL_NOLOAD).  Results of ablated builds are wrong by construction.
    python tools/exp/norm_abl.py build      (here)
    python tools/exp/norm_abl.py run        (GPU box)"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
OUT = os.path.join(PKG, "_build", "abl_norm")
VARIANTS = {"base": [], "nochain": ["-DUQ_NORM_ABL_NOCHAIN"], "noload": ["-DUQ_NORM_ABL_NOLOAD"],
            "neither": ["-DUQ_NORM_ABL_NOCHAIN", "-DUQ_NORM_ABL_NOLOAD"]}


def build():
    sys.path.insert(0, PKG)
    import build_ext as be
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ablation_src import patched_csrc           # the switches live in tools/exp/ablations.patch
    src = os.path.join(patched_csrc(), "uq_dme.hip")
    os.makedirs(OUT, exist_ok=True)
    for k, fl in VARIANTS.items():
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, *fl, "-o", os.path.join(OUT, f"{k}.so"), src], check=True)


def run():
    import torch
    n, d = 1024, 1 << 20
    x = torch.randn(n, d, device="cuda")
    bins = torch.empty((n, d), dtype=torch.uint8, device="cuda")
    scale = torch.empty(n, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    for k in VARIANTS:
        L = ctypes.CDLL(os.path.join(OUT, f"{k}.so"))
        b = ctypes.c_size_t()
        if (L.uq_eden_workspace_bytes(ctypes.c_int64(n), ctypes.c_int64(d), ctypes.byref(b))) != 0:
            raise RuntimeError('L.uq_eden_workspace_bytes(ctypes.c_int64(n), ctypes.c_int64(d), ctypes.byref(b))' + ' failed')
        ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
        signs = torch.ones(d, dtype=torch.int8, device="cuda")
        rows = torch.zeros(n, dtype=torch.int32, device="cuda")
        f = L.uq_eden_compress_f32
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        call = lambda: f(x.data_ptr(), n, d, 1, signs.data_ptr(), rows.data_ptr(), bins.data_ptr(), scale.data_ptr(),
                         ws.data_ptr(), b.value, sp)
        for _ in range(2):
            if (call()) != 0:
                raise RuntimeError('call()' + ' failed')
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            call()
        e1.record()
        torch.cuda.synchronize()
        print(f"{k:8s} compress {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
