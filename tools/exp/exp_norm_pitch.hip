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
constexpr int kNormChunk = 1024;
constexpr int kNormRow = kNormChunk / 8 + 4;
constexpr int kNormClientStride = 8 * kNormRow;

// NC clients per workgroup: one chain wave (NC x 8 chains) + NC loader waves
template <int kNormClients>
__global__ void __launch_bounds__(64 + 64 * kNormClients)
norm_pitch_kernel(const float* __restrict__ v, int64_t n, int64_t D, int64_t ld, float* __restrict__ nrm) {
    constexpr int kNormBuf = kNormClients * kNormClientStride;
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

// 4 clients per workgroup, loads two chunks ahead (two register sets, loop unrolled by 2 so
// the set is static): the loads of chunk ch + 2 stay in flight across iteration ch + 1.
__global__ void __launch_bounds__(64 + 256)
norm_ahead2_kernel(const float* __restrict__ v, int64_t n, int64_t D, int64_t ld, float* __restrict__ nrm) {
    constexpr int kNormClients = 4;
    constexpr int kNormBuf = kNormClients * kNormClientStride;
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nv = D - D % 8;
    const int64_t nchunks = nv / kNormChunk;                 // whole chunks only (experiment)
    const bool chain = tid < kWave;
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = !chain && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * ld;
    constexpr int kLQ = kNormChunk / 256;
    float4 na[kLQ], nb[kLQ];
    auto load = [&](float4 (&nx)[kLQ], int64_t ch) {
        if (!lvalid || ch >= nchunks) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) nx[q] = *reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q));
    };
    auto store = [&](const float4 (&nx)[kLQ], float* sb) {
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
    auto chainstep = [&](int64_t ch) {
        const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
        for (int i = 0; i < kNormChunk / 8; i += 16) {
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
    };
    if (!chain) {
        load(na, 0);
        store(na, s[0]);
        load(na, 1);                    // chunk 1 -> na, chunk 2 -> nb
        load(nb, 2);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunks; ch += 2) {
        // iteration ch: chunk ch+1 (na) into LDS, chunk ch+3 -> na
        if (chain) chainstep(ch);
        else if (ch + 1 < nchunks) {
            store(na, s[(ch + 1) % 3]);
            load(na, ch + 3);
        }
        __syncthreads();
        if (ch + 1 >= nchunks) break;
        // iteration ch+1: chunk ch+2 (nb) into LDS, chunk ch+4 -> nb
        if (chain) chainstep(ch + 1);
        else if (ch + 2 < nchunks) {
            store(nb, s[(ch + 2) % 3]);
            load(nb, ch + 4);
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

// loads three chunks ahead: three register sets, loop unrolled by 3
__global__ void __launch_bounds__(64 + 256)
norm_ahead3_kernel(const float* __restrict__ v, int64_t n, int64_t D, int64_t ld, float* __restrict__ nrm) {
    constexpr int kNormClients = 4;
    constexpr int kNormBuf = kNormClients * kNormClientStride;
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nchunks = (D - D % 8) / kNormChunk;
    const bool chain = tid < kWave;
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = !chain && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * ld;
    constexpr int kLQ = kNormChunk / 256;
    float4 r0[kLQ], r1[kLQ], r2[kLQ];
    auto load = [&](float4 (&nx)[kLQ], int64_t ch) {
        if (!lvalid || ch >= nchunks) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) nx[q] = *reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q));
    };
    auto store = [&](const float4 (&nx)[kLQ], float* sb) {
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
    auto chainstep = [&](int64_t ch) {
        const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
        for (int i = 0; i < kNormChunk / 8; i += 16) {
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
    };
    if (!chain) {
        load(r0, 0);
        store(r0, s[0]);
        load(r1, 1);                    // chunk 1 -> r1, 2 -> r2, 3 -> r0
        load(r2, 2);
        load(r0, 3);
    }
    __syncthreads();
    // iteration c (c mod 3 = 0, 1, 2): chunk c + 1 sits in r1, r2, r0 respectively
    for (int64_t ch = 0; ch < nchunks; ch += 3) {
        if (chain) chainstep(ch);
        else if (ch + 1 < nchunks) { store(r1, s[(ch + 1) % 3]); load(r1, ch + 4); }
        __syncthreads();
        if (ch + 1 >= nchunks) break;
        if (chain) chainstep(ch + 1);
        else if (ch + 2 < nchunks) { store(r2, s[(ch + 2) % 3]); load(r2, ch + 5); }
        __syncthreads();
        if (ch + 2 >= nchunks) break;
        if (chain) chainstep(ch + 2);
        else if (ch + 3 < nchunks) { store(r0, s[(ch + 3) % 3]); load(r0, ch + 6); }
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

extern "C" int exp_norm_nc(const float* v, int64_t n, int64_t D, int64_t ld, float* nrm, int pad_lds, int nc, void* stream) {
    if (D % 8 != 0 || ld < D) return -1;
    const unsigned grid = (unsigned)((n + nc - 1) / nc);
    hipStream_t st = (hipStream_t)stream;
    if (nc == 4) hipLaunchKernelGGL(norm_pitch_kernel<4>, dim3(grid), dim3(64 + 256), (unsigned)pad_lds, st, v, n, D, ld, nrm);
    else if (nc == 2) hipLaunchKernelGGL(norm_pitch_kernel<2>, dim3(grid), dim3(64 + 128), (unsigned)pad_lds, st, v, n, D, ld, nrm);
    else if (nc == 1) hipLaunchKernelGGL(norm_pitch_kernel<1>, dim3(grid), dim3(64 + 64), (unsigned)pad_lds, st, v, n, D, ld, nrm);
    else if (nc == 444) hipLaunchKernelGGL(norm_ahead3_kernel, dim3((unsigned)((n + 3) / 4)), dim3(64 + 256), 0, st, v, n, D, ld, nrm);
    else if (nc == 44) hipLaunchKernelGGL(norm_ahead2_kernel, dim3((unsigned)((n + 3) / 4)), dim3(64 + 256), 0, st, v, n, D, ld, nrm);
    else return -3;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// pad_lds: extra dynamic LDS bytes per workgroup (81920+ leaves room for one workgroup per CU);
// nc: clients per workgroup (1, 2 or 4)
extern "C" int exp_norm_pitch(const float* v, int64_t n, int64_t D, int64_t ld, float* nrm, int pad_lds, void* stream) {
    return exp_norm_nc(v, n, D, ld, nrm, pad_lds, 4, stream);
}
