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
    # K3 (client mean from q): non-temporal loads / the next 8 rows loaded before the adds
    "k3_nt": [('            for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const float4*>(q + (j + u) * ld + col);', '            for (int u = 0; u < 8; ++u) {\n                typedef float m4 __attribute__((ext_vector_type(4)));\n                const m4 v = __builtin_nontemporal_load(reinterpret_cast<const m4*>(q + (j + u) * ld + col));\n                t[u] = make_float4(v.x, v.y, v.z, v.w);\n            }')],
    "k3_db": [('        int64_t j = 0;\n        for (; j + 8 <= n; j += 8) {\n            float4 t[8];\n#pragma unroll\n            for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const float4*>(q + (j + u) * ld + col);\n#pragma unroll\n            for (int u = 0; u < 8; ++u) {', '        int64_t j = 0;\n        float4 nx[8];\n        if (n >= 8) {\n#pragma unroll\n            for (int u = 0; u < 8; ++u) nx[u] = *reinterpret_cast<const float4*>(q + u * ld + col);\n        }\n        for (; j + 8 <= n; j += 8) {\n            float4 t[8];\n#pragma unroll\n            for (int u = 0; u < 8; ++u) t[u] = nx[u];\n            if (j + 16 <= n) {\n#pragma unroll\n                for (int u = 0; u < 8; ++u) nx[u] = *reinterpret_cast<const float4*>(q + (j + 8 + u) * ld + col);\n            }\n#pragma unroll\n            for (int u = 0; u < 8; ++u) {')],
    # EDEN norm loaders (KE2, both kernels): non-temporal loads of the rotated vectors
    "eden_norm_nt": [("uq_eden_kernels.h",
                      "nx[q] = *reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q));",
                      "nx[q] = ld_stream(reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q)));",
                      2)],
    # EDEN low pass (KE1 fwht_low4096_kernel): non-temporal loads of its input rows
    "eden_low_nt": [("uq_eden_kernels.h", "const float4 t = *reinterpret_cast<const float4*>(x + i0 + 4 * q);",
                     "const float4 t = ld_stream(reinterpret_cast<const float4*>(x + i0 + 4 * q));", 1),
                    ("uq_eden_kernels.h", "const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);",
                     "const float4 t = ld_stream(reinterpret_cast<const float4*>(p + 4 * q));", 2)],
    # K1a: the leaf loop loads a batch of rows before it adds them (all loads in flight)
    "k1_batch8": [('        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        for (int r = 0; r < step; ++r) {\n            float v[4];', '        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        int r = 0;\n        if (VEC4) {\n            typedef float kbx4 __attribute__((ext_vector_type(4)));\n            for (; r + 8 <= step; r += 8) {\n                kbx4 tv[8];\n#pragma unroll\n                for (int u = 0; u < 8; ++u)\n                    tv[u] = __builtin_nontemporal_load(reinterpret_cast<const kbx4*>(p + (int64_t)(r + u) * 32));\n#pragma unroll\n                for (int u = 0; u < 8; ++u) {\n                    const float w[4] = {tv[u].x, tv[u].y, tv[u].z, tv[u].w};\n                    op.apply4(w, a);\n                }\n            }\n        }\n        for (; r < step; ++r) {\n            float v[4];')],
    "k1_batch16": [('        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        for (int r = 0; r < step; ++r) {\n            float v[4];', '        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        int r = 0;\n        if (VEC4) {\n            typedef float kbx4 __attribute__((ext_vector_type(4)));\n            for (; r + 16 <= step; r += 16) {\n                kbx4 tv[16];\n#pragma unroll\n                for (int u = 0; u < 16; ++u)\n                    tv[u] = __builtin_nontemporal_load(reinterpret_cast<const kbx4*>(p + (int64_t)(r + u) * 32));\n#pragma unroll\n                for (int u = 0; u < 16; ++u) {\n                    const float w[4] = {tv[u].x, tv[u].y, tv[u].z, tv[u].w};\n                    op.apply4(w, a);\n                }\n            }\n        }\n        for (; r < step; ++r) {\n            float v[4];')],
    "k1_batch32": [('        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        for (int r = 0; r < step; ++r) {\n            float v[4];', '        float a[4] = {0.f, 0.f, 0.f, 0.f};\n        int r = 0;\n        if (VEC4) {\n            typedef float kbx4 __attribute__((ext_vector_type(4)));\n            for (; r + 32 <= step; r += 32) {\n                kbx4 tv[32];\n#pragma unroll\n                for (int u = 0; u < 32; ++u)\n                    tv[u] = __builtin_nontemporal_load(reinterpret_cast<const kbx4*>(p + (int64_t)(r + u) * 32));\n#pragma unroll\n                for (int u = 0; u < 32; ++u) {\n                    const float w[4] = {tv[u].x, tv[u].y, tv[u].z, tv[u].w};\n                    op.apply4(w, a);\n                }\n            }\n        }\n        for (; r < step; ++r) {\n            float v[4];')],
    # UQR1 code histogram (KC1): non-temporal loads of the codes
    "codec_hist_nt": [("uq_codec_kernels.h",
                       "const uint4 w0 = *reinterpret_cast<const uint4*>(row + i);\n            const uint4 w1 = *reinterpret_cast<const uint4*>(row + i + 256 * 16);",
                       "const uint4 w0 = ld_stream_u4(reinterpret_cast<const uint4*>(row + i));\n            const uint4 w1 = ld_stream_u4(reinterpret_cast<const uint4*>(row + i + 256 * 16));",
                       1),
                      ("uq_codec_kernels.h", "// Type-message codec",
                       "__device__ __forceinline__ uint4 ld_stream_u4(const uint4* p) {\n    typedef uint32_t u4v __attribute__((ext_vector_type(4)));\n    const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));\n    return make_uint4(v.x, v.y, v.z, v.w);\n}\n// Type-message codec", 1)],
    "prio_ld": [(LOOP_LD, "        __builtin_amdgcn_s_setprio(2);\n" + LOOP_LD + "        __builtin_amdgcn_s_setprio(0);\n")],
}

# the batched loads for the plain L1 (AbsOp) only: the k' ops keep the row loop
VARIANTS["k1_batch8_abs"] = [(VARIANTS["k1_batch8"][0][0],
                              VARIANTS["k1_batch8"][0][1].replace("if (VEC4) {",
                                                                  "if (VEC4 && std::is_same<Op, AbsOp>::value) {"))]


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
        header_subs = [v for v in VARIANTS[name] if len(v) == 4]      # (file, old, new, count)
        for fn, a, b, cnt in header_subs:
            hp = os.path.join(d, fn)
            h = open(hp).read()
            if h.count(a) != cnt:
                raise SystemExit(f"{name}: {fn} pattern found {h.count(a)} times")
            open(hp, "w").write(h.replace(a, b))
        s = open(src).read()
        key = ("l1_partial_kernel(" if name.startswith("k1_") else
               "client_mean_kernel(const float* __restrict__ q" if name.startswith("k3_") else
               "quantize_stream_kernel(const float* __restrict__ x")
        i = s.index(key)                                  # that kernel's body only
        j = s.index("__global__", i)
        body = s[i:j]
        for a, b in (v for v in VARIANTS[name] if len(v) == 2):
            if body.count(a) != 1:
                raise SystemExit(f"{name}: pattern found {body.count(a)} times")
            body = body.replace(a, b)
        s = s[:i] + body + s[j:]
        open(src, "w").write(s)
        subprocess.run([be.hipcc(), *be.HIPCC_FLAGS, "-o", os.path.join(OUT, f"{name}.so"), src], check=True)
        print("built", name, flush=True)


if __name__ == "__main__":
    build(sys.argv[1:] or list(VARIANTS))
