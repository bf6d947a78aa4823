"""Do row pitches on K2's OUTPUTS remove its two placement speeds?

K2 (q + codes, C2 batch) runs at ~1.67 ms or ~1.95 ms depending on where q and the codes
land in physical memory.  Every one of the 1024 concurrent workgroups writes
tile t of its row at the same offset inside its own 4 MiB q row (1 MiB codes row), so all
concurrent writes share their low address bits and the channel mix is left to the
physical frames.  The first run used a variant library
taking the row pitches from constant memory (`build`); the product now takes them
(uq_type_unbiased_codes_ld_f32), and `run` / `run2` time that:

    python tools/exp/k2_pitch.py run|run2     (GPU box: JSON lines, one per config/sweep)

Configs hold several fresh output sets each (all held at once, so each is on its own
pages) and time K2 on every set; a config that is fast on every set removes the lottery.
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
OUT = os.path.join(ROOT, "tools", "exp", "_pitch")
SO = os.path.join(OUT, "libpitch.so")

SUBS = [
    ("const __amdgpu_buffer_rsrc_t ro = make_rsrc(WQ ? out + vec * d : x, row_bytes);",
     "const __amdgpu_buffer_rsrc_t ro = make_rsrc(WQ ? out + vec * (g_ldo ? g_ldo : d) : x, row_bytes);"),
    ("const __amdgpu_buffer_rsrc_t rc = make_rsrc(WC ? (const void*)(codes + vec * d) : (const void*)x, row_bytes / 4u);",
     "const __amdgpu_buffer_rsrc_t rc = make_rsrc(WC ? (const void*)(codes + vec * (g_ldc ? g_ldc : d)) : (const void*)x, row_bytes / 4u);"),
    ("template <bool WQ, bool WC, bool CVEC>\n__global__ void __launch_bounds__(kQBlock, 4)\nquantize_stream_kernel(",
     "__constant__ int64_t g_ldo;\n__constant__ int64_t g_ldc;\ntemplate <bool WQ, bool WC, bool CVEC>\n"
     "__global__ void __launch_bounds__(kQBlock, 4)\nquantize_stream_kernel("),
]
SETTER = """
extern "C" int uq_exp_set_ld(int64_t ldo, int64_t ldc) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ldo), &ldo, sizeof(ldo)) != hipSuccess) return -2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ldc), &ldc, sizeof(ldc)) != hipSuccess) return -2;
    return 0;
}
"""


def build():
    sys.path.insert(0, PKG)
    import build_ext as be
    top = tempfile.mkdtemp(prefix="uq_pitch_")
    d = os.path.join(top, "pkg", "csrc")
    os.makedirs(d)
    os.symlink(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    for f in os.listdir(os.path.join(PKG, "csrc")):
        shutil.copy(os.path.join(PKG, "csrc", f), d)
    src = os.path.join(d, "uq_dme.hip")
    s = open(src).read()
    for a, b in SUBS:
        if s.count(a) != 1:
            raise SystemExit(f"pattern found {s.count(a)} times: {a[:60]}")
        s = s.replace(a, b)
    open(src, "w").write(s + SETTER)
    os.makedirs(OUT, exist_ok=True)
    subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-o", SO, src], check=True)
    print("built", SO)


# (name, extra q floats per row, extra code bytes per row, codes inside the q allocation)
CONFIGS = [
    ("dense", 0, 0, False),
    ("pad256B", 64, 256, False),
    ("pad4K", 1024, 4096, False),
    ("pad16K+256", 4096 + 64, 4096 + 256, False),
    ("combined", 0, 0, True),           # row = [q (4d B) | codes (d B)], pitch 5d B
    ("combined+4K", 1024, 0, True),
]
# round 2 of the experiment: small pads (q floats, code bytes)
CONFIGS2 = [
    ("dense", 0, 0, False),
    ("pad64B", 16, 64, False),
    ("pad128B", 32, 128, False),
    ("pad256B", 64, 256, False),
    ("pad512B", 128, 512, False),
    ("pad256B_q_only", 64, 0, False),
    ("pad256B_codes_only", 0, 256, False),
]


def run(trials=4, reps=3, configs=None):
    configs = configs or CONFIGS
    import torch
    sys.path.insert(0, ROOT)
    import uqdme  # noqa: F401  (registers the package alias)
    from uqdme_amd import _lib
    lib = _lib.load()                # the product library: uq_type_unbiased_codes_ld_f32 takes the pitches
    n, d = 1024, 1 << 20
    m = 224426
    torch.manual_seed(0)
    x = torch.empty((n, d), device="cuda").normal_()
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    assert lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b)) == 0
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    km = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st) == 0

    def alloc(cfg):
        _, eq, ec, comb = cfg
        if comb:
            ldq = d + d // 4 + eq                       # floats per row; codes after the q part
            buf = torch.empty((n, ldq), device="cuda")
            q = buf[:, :d]
            cbytes = buf.view(torch.int8)               # [n, 4*ldq]
            codes = cbytes[:, 4 * d:4 * d + d]
            return buf, q, codes, ldq, 4 * ldq
        ldq, ldc = d + eq, d + ec
        qb = torch.empty((n, ldq), device="cuda")
        cb = torch.empty((n, ldc), dtype=torch.int8, device="cuda")
        return (qb, cb), qb[:, :d], cb[:, :d], ldq, ldc

    def k2(q, codes, ldq, ldc):
        rc = lib.uq_type_unbiased_codes_ld_f32(x.data_ptr(), q.data_ptr(), ldq, codes.data_ptr(), ldc, km.data_ptr(),
                                               n, d, m, X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value,
                                               st)
        if rc != 0:
            raise RuntimeError(lib.uq_last_error())

    def timed(q, codes, ldq, ldc):
        for _ in range(2):
            k2(q, codes, ldq, ldc)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            k2(q, codes, ldq, ldc)
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    sets = []
    for t in range(trials):
        for cfg in configs:
            sets.append((cfg, t, alloc(cfg)))
    ref_q = ref_c = None
    for sweep in range(2):
        order = sets if sweep == 0 else list(reversed(sets))
        res = {}
        for cfg, t, (_keep, q, codes, ldq, ldc) in order:
            ms = timed(q, codes, ldq, ldc)
            res.setdefault(cfg[0], [None] * trials)[t] = ms
            if sweep == 0:
                if ref_q is None:
                    ref_q, ref_c = q[:8].clone(), codes[:8].clone()
                elif not (torch.equal(q[:8], ref_q) and torch.equal(codes[:8], ref_c)):
                    raise SystemExit(f"{cfg[0]}: outputs differ from the dense set")
        for name, _, _, _ in configs:
            print(json.dumps({"sweep": sweep, "config": name, "k2_ms": res[name]}), flush=True)
    print(json.dumps({"done": True, "sets": len(sets)}))


if __name__ == "__main__":
    if sys.argv[1] == "run2":
        run(trials=5, configs=CONFIGS2)
    else:
        {"build": build, "run": run}[sys.argv[1]]()
