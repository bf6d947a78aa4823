// Access-pattern calibration for the EDEN high pass: each workgroup copies one tile of
// 2^RB rows x COLS contiguous floats, rows `stride` floats apart (the FWHT high pass reads
// 256 rows x 64 floats at a 4096-float stride).  No compute, loads all held in registers,
// non-temporal loads/stores.  Experiment, not shipped.
#include <hip/hip_runtime.h>
#include <cstdint>
template <int COLS, int RB, int NT>
__global__ void __launch_bounds__(NT) tile_copy(const float* __restrict__ a, float* __restrict__ b, int64_t D,
                                                int64_t stride) {
    constexpr int ROWS = 1 << RB;
    constexpr int LPR = COLS / 4 < 64 ? COLS / 4 : 64;          // lanes per row segment (float4 each)
    constexpr int VPL = COLS / 4 / LPR;                          // float4 per lane per row
    constexpr int RPP = NT / LPR;                                // rows per pass of the workgroup
    constexpr int PASSES = ROWS / RPP;
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int64_t vec = blockIdx.y;
    const int64_t col_groups = stride / COLS;
    const int64_t t = blockIdx.x;
    const int64_t hi = (t / col_groups) * stride * ROWS;
    const int64_t c0 = (t % col_groups) * COLS;
    const int tid = threadIdx.x;
    const int lane_c = tid % LPR, r0 = tid / LPR;
    const f4* src = reinterpret_cast<const f4*>(a + vec * D + hi + c0);
    f4* dst = reinterpret_cast<f4*>(b + vec * D + hi + c0);
    f4 v[PASSES][VPL];
#pragma unroll
    for (int p = 0; p < PASSES; ++p)
#pragma unroll
        for (int k = 0; k < VPL; ++k)
            v[p][k] = __builtin_nontemporal_load(src + ((int64_t)(r0 + p * RPP) * stride) / 4 + lane_c + k * LPR);
#pragma unroll
    for (int p = 0; p < PASSES; ++p)
#pragma unroll
        for (int k = 0; k < VPL; ++k)
            __builtin_nontemporal_store(v[p][k], dst + ((int64_t)(r0 + p * RPP) * stride) / 4 + lane_c + k * LPR);
}
// scalar-lane variant as the product high pass: lane = column, 4 B per lane, 64 columns
template <int RB>
__global__ void __launch_bounds__(512) tile_copy_dw(const float* __restrict__ a, float* __restrict__ b, int64_t D,
                                                    int64_t stride) {
    constexpr int ROWS = 1 << RB;
    const int64_t vec = blockIdx.y;
    const int64_t col_groups = stride / 64;
    const int64_t t = blockIdx.x;
    const int64_t hi = (t / col_groups) * stride * ROWS;
    const int64_t c0 = (t % col_groups) * 64;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const float* src = a + vec * D + hi + c0 + c;
    float* dst = b + vec * D + hi + c0 + c;
    constexpr int PER = ROWS / 8;
    float v[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) v[m] = __builtin_nontemporal_load(src + (int64_t)(PER * g + m) * stride);
#pragma unroll
    for (int m = 0; m < PER; ++m) __builtin_nontemporal_store(v[m], dst + (int64_t)(PER * g + m) * stride);
}
// 16384 floats per workgroup (32 per thread) whatever the segment width: rows = 16384 / cols
extern "C" int tile_bw(const float* a, float* b, int64_t n, int64_t D, int64_t stride, int cols, void* st) {
    if (D % 16384 || stride % 1024 || (int64_t)(16384 / (cols ? cols : 64)) * stride > D) return -3;
    dim3 grid((unsigned)(D / 16384), (unsigned)n);
    hipStream_t s = (hipStream_t)st;
    switch (cols) {
        case 0: hipLaunchKernelGGL((tile_copy_dw<8>), grid, dim3(512), 0, s, a, b, D, stride); break;
        case 64: hipLaunchKernelGGL((tile_copy<64, 8, 512>), grid, dim3(512), 0, s, a, b, D, stride); break;
        case 128: hipLaunchKernelGGL((tile_copy<128, 7, 512>), grid, dim3(512), 0, s, a, b, D, stride); break;
        case 256: hipLaunchKernelGGL((tile_copy<256, 6, 512>), grid, dim3(512), 0, s, a, b, D, stride); break;
        case 1024: hipLaunchKernelGGL((tile_copy<1024, 4, 512>), grid, dim3(512), 0, s, a, b, D, stride); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
