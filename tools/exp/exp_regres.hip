// Experiment (tools/, not shipped): data-flow bound of a fused K1+K2 whose client vector
// stays in VGPRs between the L1 pass and the output pass, so x is read from HBM ONCE.
// A client of d floats is spread over S workgroups of 1024 threads (E = d / (S*1024)
// floats per thread, held as E/4 float4 registers).  Per client: load the segment,
// |x| partial sum -> part[j*S + w], arrive counter, spin (bounded) until all S arrived,
// L1 = ordered sum of the S partials, optional chain (WG w waits for WG w-1's flag,
// the latency a serial exact-prefix hand-off would add), then write q (f32) and an
// int8 code per element.  Arithmetic is a stand-in (x * m / L1), not the quantizer.
//
// Persistent grid = slots * S workgroups with slots * S <= resident capacity, so every
// workgroup of a client is resident; spins are bounded and set err[0] on timeout.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kT = 1024;
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ld_acq(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int E>
__global__ void __launch_bounds__(kT, 1)
regres_kernel(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes, int64_t n,
              int64_t d, float fm, int S, int slots, float* part, uint32_t* cnt, uint32_t* chain, uint32_t* err,
              int mode) {
    constexpr int V = E / 4;
    __shared__ float s_red[kT / 64];
    __shared__ float s_l1;
    const int tid = threadIdx.x;
    const int w = blockIdx.x % S;
    const int slot = blockIdx.x / S;
    const int64_t seg = (int64_t)E * kT;               // floats per workgroup segment
    for (int64_t j = slot; j < n; j += slots) {
        const f4* xs = reinterpret_cast<const f4*>(x + j * d + w * seg);
        f4 v[V];
#pragma unroll
        for (int c = 0; c < V; ++c) v[c] = __builtin_nontemporal_load(xs + c * kT + tid);
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < V; ++c) acc += (fabsf(v[c].x) + fabsf(v[c].y)) + (fabsf(v[c].z) + fabsf(v[c].w));
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if ((tid & 63) == 0) s_red[tid >> 6] = acc;
        __syncthreads();
        if (tid == 0) {
            float p = 0.f;
            for (int i = 0; i < kT / 64; ++i) p += s_red[i];
            part[j * S + w] = p;
            __hip_atomic_fetch_add(cnt + j, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t spins = 0;
            while (ld_acq(cnt + j) < (uint32_t)S) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1u << 22)) { atomicOr(err, 1u); break; }
            }
            float l1 = 0.f;
            for (int i = 0; i < S; ++i) l1 += __hip_atomic_load(part + j * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (mode & 1) {                               // serial hand-off chain across the S workgroups
                spins = 0;
                while (ld_acq(chain + j) < (uint32_t)w) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 22)) { atomicOr(err, 2u); break; }
                }
                __hip_atomic_store(chain + j, (uint32_t)(w + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_l1 = l1;
        }
        __syncthreads();
        const float sc = fm / s_l1;
        f4* os = reinterpret_cast<f4*>(out + j * d + w * seg);
        uint32_t* cs = reinterpret_cast<uint32_t*>(codes + j * d + w * seg);
#pragma unroll
        for (int c = 0; c < V; ++c) {
            f4 o;
            o.x = v[c].x * sc; o.y = v[c].y * sc; o.z = v[c].z * sc; o.w = v[c].w * sc;
            __builtin_nontemporal_store(o, os + c * kT + tid);
            const uint32_t cw = ((uint32_t)(int8_t)o.x & 255u) | (((uint32_t)(int8_t)o.y & 255u) << 8) |
                                (((uint32_t)(int8_t)o.z & 255u) << 16) | ((uint32_t)(int8_t)o.w << 24);
            __builtin_nontemporal_store(cw, cs + c * kT + tid);
        }
    }
}

template <int E>
int launch(const float* x, float* out, int8_t* codes, int64_t n, int64_t d, float fm, int slots_req, void* ws,
           int mode, hipStream_t st, int* used) {
    const int S = (int)(d / ((int64_t)E * kT));
    if (S < 1 || (int64_t)S * E * kT != d) return -1;
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) return -2;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, regres_kernel<E>, kT, 0)) return -3;
    if (per < 1) return -4;
    int slots = ncu * per / S;
    if (slots_req > 0 && slots_req < slots) slots = slots_req;
    if (slots < 1) return -5;
    if (slots > n) slots = (int)n;
    float* part = (float*)ws;
    uint32_t* cnt = (uint32_t*)(part + n * S);
    uint32_t* chain = cnt + n;
    uint32_t* err = chain + n;
    if (hipMemsetAsync(cnt, 0, (2 * n + 1) * 4, st)) return -6;
    hipLaunchKernelGGL(regres_kernel<E>, dim3(slots * S), dim3(kT), 0, st, x, out, codes, n, d, fm, S, slots, part, cnt,
                       chain, err, mode);
    if (hipGetLastError()) return -7;
    *used = slots * 1000 + per;
    return 0;
}
}  // namespace

extern "C" int exp_regres(const float* x, float* out, int8_t* codes, int64_t n, int64_t d, float fm, int E, int slots,
                          void* ws, int mode, void* st, int* used) {
    hipStream_t s = (hipStream_t)st;
    switch (E) {
        case 32: return launch<32>(x, out, codes, n, d, fm, slots, ws, mode, s, used);
        case 64: return launch<64>(x, out, codes, n, d, fm, slots, ws, mode, s, used);
        case 96: return -1;
        case 128: return launch<128>(x, out, codes, n, d, fm, slots, ws, mode, s, used);
        default: return -1;
    }
}
