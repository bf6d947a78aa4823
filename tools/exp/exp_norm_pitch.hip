// Experiment: is EDEN's torch-order norm (KE2, eden_norm_kernel)
// bounded by HBM channel camping -- 1024 client rows 4 MiB apart, all loaders at the same
// offset?  Same kernel as csrc/uq_eden_kernels.h KE2 with a row pitch `ld` (floats) instead of
// D, timed on rows staggered by ld - D floats.  Timing only; the norms are checked equal
// across pitches by the driver script (tools/exp/norm_pitch.py).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/exp/libexp_norm_pitch.so tools/exp/exp_norm_pitch.hip
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int kWave = 64;
constexpr int kNormClients = 4;
constexpr int kNormChunk = 1024;
constexpr int kNormRow = kNormChunk / 8 + 4;
constexpr int kNormClientStride = 8 * kNormRow;
constexpr int kNormBuf = kNormClients * kNormClientStride;
constexpr int kNormThreads = 64 + 256;

__global__ void __launch_bounds__(kNormThreads)
norm_pitch_kernel(const float* __restrict__ v, int64_t n, int64_t D, int64_t ld, float* __restrict__ nrm) {
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nv = D - D % 8;
    const int64_t nchunks = (nv + kNormChunk - 1) / kNormChunk;
    const bool chain = tid < kWave;
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = !chain && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * ld;
    constexpr int kLQ = kNormChunk / 256;
    float4 nx[kLQ];
    auto load = [&](int64_t ch) {
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int64_t i = ch * kNormChunk + 4 * (lj + 64 * q);
            if (lvalid && i + 3 < nv) nx[q] = *reinterpret_cast<const float4*>(lp + i);
            else nx[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](float* sb) {
        if (chain) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int e = 4 * (lj + 64 * q);
            const int i = e >> 3, l = e & 7;
            float* base = sb + lk * kNormClientStride + i;
            base[(l + 0) * kNormRow] = nx[q].x;
            base[(l + 1) * kNormRow] = nx[q].y;
            base[(l + 2) * kNormRow] = nx[q].z;
            base[(l + 3) * kNormRow] = nx[q].w;
        }
    };
    const int ck = (tid >> 3) & (kNormClients - 1), cl = tid & 7;
    float acc = 0.f;
    if (nchunks > 0) {
        if (!chain) load(0);
        store(s[0]);
        if (!chain && nchunks > 1) load(1);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunks; ++ch) {
        if (chain) {
            const int cnt = (int)((nv - ch * kNormChunk < kNormChunk ? nv - ch * kNormChunk : kNormChunk) / 8);
            const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
            int i = 0;
            for (; i + 16 <= cnt; i += 16) {
                float4 t[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(row + i + 4 * u);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc = fmaf(t[u].x, t[u].x, acc);
                    acc = fmaf(t[u].y, t[u].y, acc);
                    acc = fmaf(t[u].z, t[u].z, acc);
                    acc = fmaf(t[u].w, t[u].w, acc);
                }
            }
            for (; i < cnt; ++i) acc = fmaf(row[i], row[i], acc);
        } else if (ch + 1 < nchunks) {
            store(s[(ch + 1) % 3]);
            if (ch + 2 < nchunks) load(ch + 2);
        }
        __syncthreads();
    }
    if (chain) {
        const int base = tid & ~7;
        float tot = __shfl(acc, base, kWave);
        for (int j = 1; j < 8; ++j) tot = tot + __shfl(acc, base + j, kWave);
        const int64_t vec = v0 + ck;
        if (tid < 8 * kNormClients && cl == 0 && vec < n) nrm[vec] = sqrtf(tot);
    }
}
}  // namespace

// pad_lds: extra dynamic LDS bytes per workgroup (81920+ leaves room for one workgroup per CU)
extern "C" int exp_norm_pitch(const float* v, int64_t n, int64_t D, int64_t ld, float* nrm, int pad_lds, void* stream) {
    if (D % 8 != 0 || ld < D) return -1;
    hipLaunchKernelGGL(norm_pitch_kernel, dim3((unsigned)((n + kNormClients - 1) / kNormClients)), dim3(kNormThreads),
                       (unsigned)pad_lds, (hipStream_t)stream, v, n, D, ld, nrm);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
