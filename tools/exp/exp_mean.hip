// Experiment: the q pipeline's client mean (K3 client_mean_kernel, ND:137-138) reads 4 GB
// at ~4.8 TB/s.  Variants of workgroup size and columns per thread, same adds in the same
// order (timing only; est compared across variants by tools/exp/mean_variants.py).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -fno-gpu-flush-denormals-to-zero -shared -fPIC -o tools/exp/libexp_mean.so tools/exp/exp_mean.hip
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
template <int TPB, int CPT>
__global__ void __launch_bounds__(TPB)
mean_kernel(const float* __restrict__ q, int64_t n, int64_t d, float n_div, float* __restrict__ est) {
    typedef float fv __attribute__((ext_vector_type(CPT)));
    const int64_t col = ((int64_t)blockIdx.x * TPB + threadIdx.x) * CPT;
    if (col >= d) return;
    float e[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) e[k] = 0.f;
    int64_t j = 0;
    for (; j + 8 <= n; j += 8) {
        fv t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const fv*>(q + (j + u) * d + col);
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int k = 0; k < CPT; ++k) e[k] += t[u][k] / n_div;
    }
    for (; j < n; ++j) {
        const fv t = *reinterpret_cast<const fv*>(q + j * d + col);
#pragma unroll
        for (int k = 0; k < CPT; ++k) e[k] += t[k] / n_div;
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k) est[col + k] = e[k];
}
}  // namespace

extern "C" int exp_mean(const float* q, int64_t n, int64_t d, float n_div, float* est, int variant, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    auto blocks = [&](int tpb, int cpt) { return dim3((unsigned)((d / cpt + tpb - 1) / tpb)); };
    switch (variant) {
        case 0: hipLaunchKernelGGL((mean_kernel<256, 4>), blocks(256, 4), dim3(256), 0, st, q, n, d, n_div, est); break;
        case 1: hipLaunchKernelGGL((mean_kernel<1024, 4>), blocks(1024, 4), dim3(1024), 0, st, q, n, d, n_div, est); break;
        case 2: hipLaunchKernelGGL((mean_kernel<256, 2>), blocks(256, 2), dim3(256), 0, st, q, n, d, n_div, est); break;
        case 3: hipLaunchKernelGGL((mean_kernel<64, 4>), blocks(64, 4), dim3(64), 0, st, q, n, d, n_div, est); break;
        case 4: hipLaunchKernelGGL((mean_kernel<128, 2>), blocks(128, 2), dim3(128), 0, st, q, n, d, n_div, est); break;
        default: return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
