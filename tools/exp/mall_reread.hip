// Does a second read of the same buffer hit the MI355X Infinity Cache (MALL)?  Read-reduce
// kernel with default or non-temporal loads; the caller times a cold read and an immediate
// re-read over buffer sizes around the 256 MB MALL.  Experiment, not shipped.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(256) read_k(const f32x4* __restrict__ a, int64_t n4, float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (; i < n4; i += stride) acc += NT ? __builtin_nontemporal_load(a + i) : a[i];
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 1.2345f) out[0] = s;        // keeps the loads; never true for the test data
}
extern "C" int mall_read(const void* a, int64_t n4, int nt, int grid, float* out, void* stream) {
    if (nt) hipLaunchKernelGGL(read_k<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f32x4*)a, n4, out);
    else hipLaunchKernelGGL(read_k<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f32x4*)a, n4, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
