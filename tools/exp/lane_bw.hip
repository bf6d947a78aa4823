// Access-pattern ceiling of K2's streams without compute: one 256-thread workgroup per
// client row (d floats), 4096-float tiles, the next tile's loads in registers, q (f32) and
// 16 codes per thread written per tile, buffer descriptors with the non-temporal policy.
//   PAT 0: coalesced lanes (float4 index tid + 256 j), as K2 loads/stores today
//   PAT 1: thread-contiguous (thread tid owns floats 16 tid .. 16 tid + 15 of the tile: the
//          row K2's passes work on), no LDS image
// Codes are thread-contiguous in both (16 B per thread, as K2 stores them).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/exp/lane_bw.hip -o tools/exp/liblane_bw.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void* p = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int PAT>
__device__ __forceinline__ uint32_t off(int tid, int j) {
    return PAT == 0 ? (uint32_t)(tid + j * 256) * 16u : (uint32_t)tid * 64u + (uint32_t)j * 16u;
}

template <int PAT>
__global__ void __launch_bounds__(256, 4) lane_copy(const float* __restrict__ x, float* __restrict__ q,
                                                    int8_t* __restrict__ c, int64_t d) {
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const uint32_t rb = (uint32_t)(d * 4);
    const auto rx = rsrc(x + row * d, rb), rq = rsrc(q + row * d, rb), rc = rsrc(c + row * d, rb / 4u);
    const int tiles = (int)(d / 4096);
    f32x4v v[4], w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rx, off<PAT>(tid, j), 0, 2);
    for (int t = 0; t < tiles; ++t) {
        const uint32_t tb = (uint32_t)t * 16384u;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = v[j];
        if (t + 1 < tiles) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rx, tb + 16384u + off<PAT>(tid, j), 0, 2);
        }
        uint32_t cw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cw[j] = __float_as_uint(w[j].x) ^ __float_as_uint(w[j].w);
            w[j] = w[j] * 0.5f;
            __builtin_amdgcn_raw_buffer_store_b128(w[j], rq, tb + off<PAT>(tid, j), 0, 2);
        }
        const u32x4v cv = {cw[0], cw[1], cw[2], cw[3]};
        __builtin_amdgcn_raw_buffer_store_b128(cv, rc, (uint32_t)t * 4096u + (uint32_t)tid * 16u, 0, 2);
    }
}

extern "C" int lane_bw(const float* x, float* q, int8_t* c, int64_t n, int64_t d, int pat, void* st) {
    if (d % 4096 != 0 || 4 * d >= (1ll << 31) || n <= 0) return -1;
    hipStream_t s = (hipStream_t)st;
    if (pat == 0)
        lane_copy<0><<<(unsigned)n, 256, 0, s>>>(x, q, c, d);
    else
        lane_copy<1><<<(unsigned)n, 256, 0, s>>>(x, q, c, d);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
