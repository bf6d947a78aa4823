"""Timing-only ablation of the quantize kernel: builds variants with -D switches and
times each on the C2 batch.  Results of ablated builds are wrong by construction."""
import ctypes, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
SRC = os.path.join(PKG, "csrc", "uq_dme.hip")
OUT = os.path.join(PKG, "_build", "abl")
VARIANTS = {"base": [], "copy": ["-DUQ_ABL_COPY"],
            "k1default": ["-DUQ_K1_NO_NT"]}
def build():
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))
    import build_ext as be
    from ablation_src import patched_csrc           # the -D switches live in tools/exp/ablations.patch
    src = os.path.join(patched_csrc(), "uq_dme.hip")
    os.makedirs(OUT, exist_ok=True)
    for k, fl in VARIANTS.items():
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, *fl, "-o", os.path.join(OUT, f"{k}.so"), src], check=True)
    for extra in sys.argv[2:]:          # name=path/to/alternative.hip
        k, src = extra.split("=", 1)
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-I", os.path.join(PKG, "csrc"), "-o", os.path.join(OUT, f"{k}.so"), src], check=True)
def run():
    import torch
    n, d = int(os.environ.get("N", 1024)), 1 << 20
    x = torch.randn(n, d, device="cuda"); q = torch.empty_like(x)
    X = torch.rand(n, device="cuda"); l1 = x.abs().sum(1)
    names = sorted(f[:-3] for f in os.listdir(OUT) if f.endswith(".so"))
    for k in names:
        L = ctypes.CDLL(os.path.join(OUT, f"{k}.so"))
        b = ctypes.c_size_t(); L.uq_workspace_bytes(ctypes.c_int64(n), ctypes.c_int64(d), 1, ctypes.byref(b))
        ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
        f = L.uq_type_unbiased_f32
        f.argtypes = [ctypes.c_void_p]*2 + [ctypes.c_int64]*3 + [ctypes.c_void_p]*3 + [ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        sp = torch.cuda.current_stream().cuda_stream
        call = lambda: f(x.data_ptr(), q.data_ptr(), n, d, 224426, X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, sp)
        calls = {"q": (call, 8)}
        if hasattr(L, "uq_type_unbiased_codes_f32"):
            g = L.uq_type_unbiased_codes_f32
            g.argtypes = [ctypes.c_void_p]*4 + [ctypes.c_int64]*3 + [ctypes.c_void_p]*3 + [ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            codes = torch.empty((n, d), dtype=torch.int8, device="cuda"); km = torch.zeros(n, dtype=torch.int32, device="cuda")
            calls["q+codes"] = (lambda: g(x.data_ptr(), q.data_ptr(), codes.data_ptr(), km.data_ptr(), n, d, 224426, X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, sp), 9)
            calls["codes"] = (lambda: g(x.data_ptr(), None, codes.data_ptr(), km.data_ptr(), n, d, 224426, X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, sp), 5)
        h = L.uq_l1_torch_order_f32
        h.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_size_t, ctypes.c_void_p]
        l1o = torch.empty(n, device="cuda")
        calls["l1"] = (lambda: h(x.data_ptr(), n, d, 1, l1o.data_ptr(), ws.data_ptr(), b.value, sp), 4)
        if "q+codes" in calls:
            qc = calls["q+codes"][0]
            calls["l1,q+codes"] = (lambda: h(x.data_ptr(), n, d, 1, l1o.data_ptr(), ws.data_ptr(), b.value, sp) or qc(), 13)
        for cname, (fn, bpe) in calls.items():
            for _ in range(3):
                rc = fn()
                if rc != 0:
                    raise RuntimeError(f"{cname} returned {rc}")
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): fn()
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(f"{k:12s} {cname:8s} {ms:8.3f} ms  {bpe*d*n/ms/1e6:8.1f} GB/s", flush=True)
if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
