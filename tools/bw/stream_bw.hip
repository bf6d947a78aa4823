// Calibration of K2's memory structure: one workgroup streams one row of d floats in
// 4096-element tiles (16 B per lane per load), writing the row back (+ optionally 1 B per
// element of codes), with DEPTH tiles of loads in flight in registers.  Compared with the
// plain grid-stride float4 copy in copy_bw.hip.  Timing-only: the stored data is the input.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
template <int DEPTH, bool CODES, int AUX>
__global__ void __launch_bounds__(256) stream_k(const float* __restrict__ x, float* __restrict__ y,
                                                int8_t* __restrict__ c, int64_t d, int spin) {
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const auto rx = rsrc(x + row * d, (uint32_t)(d * 4));
    const auto ry = rsrc(y + row * d, (uint32_t)(d * 4));
    const auto rc = rsrc(c + row * d, (uint32_t)d);
    const int tiles = (int)(d / 4096);
    f32x4 buf[DEPTH][4];
#pragma unroll
    for (int p = 0; p < DEPTH; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            buf[p][j] = __builtin_amdgcn_raw_buffer_load_b128(rx, (uint32_t)(p * 16384 + (tid + j * 256) * 16), 0, AUX);
    for (int t = 0; t < tiles; t += DEPTH) {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p) {
            f32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = buf[p][j];
            // stand-in for the compute: spin cycles
            for (int s = 0; s < spin; ++s) __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_buffer_store_b128(v[j], ry, (uint32_t)((t + p) * 16384 + (tid + j * 256) * 16), 0, AUX);
            if (CODES) {
                const u32x4 w = {__float_as_uint(v[0].x), __float_as_uint(v[1].x), __float_as_uint(v[2].x), __float_as_uint(v[3].x)};
                __builtin_amdgcn_raw_buffer_store_b128(w, rc, (uint32_t)((t + p) * 4096 + tid * 16), 0, AUX);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                buf[p][j] = __builtin_amdgcn_raw_buffer_load_b128(rx, (uint32_t)((t + p + DEPTH) * 16384 + (tid + j * 256) * 16), 0, AUX);
        }
    }
}
extern "C" int bw_stream(const void* x, void* y, void* c, int64_t n, int64_t d, int depth, int codes, int nt, int spin,
                         void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define L(D, C, A) hipLaunchKernelGGL((stream_k<D, C, A>), dim3((unsigned)n), dim3(256), 0, st, (const float*)x, (float*)y, (int8_t*)c, d, spin)
#define LC(D, A) if (codes) L(D, true, A); else L(D, false, A);
#define LD(A) switch (depth) { case 1: LC(1, A); break; case 2: LC(2, A); break; case 3: LC(3, A); break; case 4: LC(4, A); break; default: return -2; }
    if (nt) { LD(2) } else { LD(0) }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
