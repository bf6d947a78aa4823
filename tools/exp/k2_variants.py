"""Build timing variants of the product K2 source by string substitution (the product
csrc/ keeps no experiment switches), into _build/abl/<name>.so; time them all in one
process with `python tools/ablate.py run` (same x / q / codes buffers for every variant)."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unbiased-quantization-distributed-mean-estimation_amd")
sys.path.insert(0, PKG)
import build_ext as be  # noqa: E402

OUT = os.path.join(PKG, "_build", "abl")
LOOP_ST = "        if (tile > tb) {\n            const uint32_t tp = (uint32_t)(tile - 1) * (uint32_t)kQTile;\n"
LOOP_LD = "        if (tile + 1 < te) load_tile_buf(pre_x, rx, (uint32_t)(tile + 1) * (uint32_t)(kQTile * 4), tid);\n"
VARIANTS = {
    "base": [],
    # raise the wave's issue priority while it issues the tile's stores and loads
    "prio_mem": [(LOOP_ST, "        __builtin_amdgcn_s_setprio(2);\n" + LOOP_ST),
                 (LOOP_LD, LOOP_LD + "        __builtin_amdgcn_s_setprio(0);\n")],
    # ... only while it issues the loads of the next tile
    # K1a: rows per unrolled group of the leaf loop (product: 4)
    "k1_unroll4": [("        for (int r = 0; r < step; ++r) {", "#pragma unroll 4\n        for (int r = 0; r < step; ++r) {")],
    "k1_unroll8": [("        for (int r = 0; r < step; ++r) {", "#pragma unroll 8\n        for (int r = 0; r < step; ++r) {")],
    "prio_ld": [(LOOP_LD, "        __builtin_amdgcn_s_setprio(2);\n" + LOOP_LD + "        __builtin_amdgcn_s_setprio(0);\n")],
}


def build(names):
    top = tempfile.mkdtemp(prefix="uq_k2v_")
    os.symlink(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    os.makedirs(OUT, exist_ok=True)
    for name in names:
        d = os.path.join(top, name, "pkg", "csrc")
        os.makedirs(d)
        os.symlink(os.path.join(ROOT, "include"), os.path.join(top, name, "include"))
        for f in os.listdir(os.path.join(PKG, "csrc")):
            shutil.copy(os.path.join(PKG, "csrc", f), d)
        src = os.path.join(d, "uq_dme.hip")
        s = open(src).read()
        key = "l1_partial_kernel(" if name.startswith("k1_") else "quantize_stream_kernel(const float* __restrict__ x"
        i = s.index(key)                                  # that kernel's body only
        j = s.index("__global__", i)
        body = s[i:j]
        for a, b in VARIANTS[name]:
            if body.count(a) != 1:
                raise SystemExit(f"{name}: pattern found {body.count(a)} times")
            body = body.replace(a, b)
        s = s[:i] + body + s[j:]
        open(src, "w").write(s)
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-o", os.path.join(OUT, f"{name}.so"), src], check=True)
        print("built", name, flush=True)


if __name__ == "__main__":
    build(sys.argv[1:] or list(VARIANTS))
