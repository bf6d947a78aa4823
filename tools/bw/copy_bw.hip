// Calibration: plain float4 streaming copy of n*d floats (grid-stride), default and nt policies.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(256) copy_k(const f32x4* __restrict__ a, f32x4* __restrict__ b, int64_t n4) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n4; i += stride) {
        if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
        else b[i] = a[i];
    }
}
extern "C" int bw_copy(const void* a, void* b, int64_t n4, int nt, int grid, void* stream) {
    if (nt) hipLaunchKernelGGL(copy_k<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f32x4*)a, (f32x4*)b, n4);
    else hipLaunchKernelGGL(copy_k<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f32x4*)a, (f32x4*)b, n4);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
