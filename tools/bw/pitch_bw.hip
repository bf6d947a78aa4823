// Calibration: does the row pitch of the [n][d] client buffers decide K2's memory speed?
// One workgroup streams one row (as K2): 4096-element tiles, 16 B per lane, DEPTH tiles of
// loads in flight, stores of tile t before the loads of tile t+DEPTH.  Rows start `pitch`
// floats apart in x and y (codes: pitch bytes apart).  MODE 0: read x + write y (+codes),
// MODE 1: read only (K1-like), MODE 2: write only.  Timing-only: the stored data is the input.
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
template <int DEPTH, bool CODES, int MODE>
__global__ void __launch_bounds__(256) pitch_k(const float* __restrict__ x, float* __restrict__ y,
                                               int8_t* __restrict__ c, int64_t d, int64_t pitch, int64_t cpitch,
                                               float* __restrict__ sink) {
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const auto rx = rsrc(x + row * pitch, (uint32_t)(d * 4));
    const auto ry = rsrc(y + row * pitch, (uint32_t)(d * 4));
    const auto rc = rsrc(c + row * cpitch, (uint32_t)d);
    const int tiles = (int)(d / 4096);
    f32x4 buf[DEPTH][4];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (MODE != 2) {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                buf[p][j] = __builtin_amdgcn_raw_buffer_load_b128(rx, (uint32_t)(p * 16384 + (tid + j * 256) * 16), 0, 2);
    } else {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p)
#pragma unroll
            for (int j = 0; j < 4; ++j) buf[p][j] = (f32x4){(float)tid, 1.f, 2.f, (float)p};
    }
    for (int t = 0; t < tiles; t += DEPTH) {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p) {
            f32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = buf[p][j];
            if (MODE == 1) {
#pragma unroll
                for (int j = 0; j < 4; ++j) acc += v[j];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    __builtin_amdgcn_raw_buffer_store_b128(v[j], ry, (uint32_t)((t + p) * 16384 + (tid + j * 256) * 16), 0, 2);
                if (CODES) {
                    const u32x4 w = {__float_as_uint(v[0].x), __float_as_uint(v[1].x), __float_as_uint(v[2].x),
                                     __float_as_uint(v[3].x)};
                    __builtin_amdgcn_raw_buffer_store_b128(w, rc, (uint32_t)((t + p) * 4096 + tid * 16), 0, 2);
                }
            }
            if (MODE != 2) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    buf[p][j] = __builtin_amdgcn_raw_buffer_load_b128(rx, (uint32_t)((t + p + DEPTH) * 16384 + (tid + j * 256) * 16),
                                                                      0, 2);
            }
        }
    }
    if (MODE == 1 && acc.x == 12345.678f) sink[row] = acc.y + acc.z + acc.w;
}
extern "C" int bw_pitch(const void* x, void* y, void* c, int64_t n, int64_t d, int64_t pitch, int64_t cpitch, int depth,
                        int codes, int mode, void* sink, void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define L(D, C, M) hipLaunchKernelGGL((pitch_k<D, C, M>), dim3((unsigned)n), dim3(256), 0, st, (const float*)x, (float*)y, \
                                      (int8_t*)c, d, pitch, cpitch, (float*)sink)
#define LM(D, C) if (mode == 0) L(D, C, 0); else if (mode == 1) L(D, C, 1); else L(D, C, 2);
#define LC(D) if (codes) { LM(D, true) } else { LM(D, false) }
    switch (depth) {
        case 1: LC(1); break;
        case 2: LC(2); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
