// Experiment (tools/, not shipped): rate of one dependent f32 fma chain per lane (the
// torch-order norm's chains, KE2), with operands from registers (mode 0) or from LDS
// read 16 at a time as in eden_norm_kernel (mode 1), one wave per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) chain_kernel(float* out, int steps, int mode, float seed) {
    __shared__ __attribute__((aligned(16))) float s[8 * 132];
    const int lane = threadIdx.x;
    for (int i = lane; i < 8 * 132; i += 64) s[i] = seed + 1e-3f * i;
    __syncthreads();
    float acc = 0.f;
    if (mode == 0) {
        float t = seed + lane * 1e-3f;
        for (int i = 0; i < steps; i += 16) {
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = fmaf(t, t, acc);
            t += 1e-7f;
        }
    } else {
        const float* row = s + (lane & 7) * 132;
        for (int i = 0; i < steps; i += 16) {
            const int j = i & 127;
            float4 tt[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) tt[u] = *reinterpret_cast<const float4*>(row + j + 4 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = fmaf(tt[u].x, tt[u].x, acc);
                acc = fmaf(tt[u].y, tt[u].y, acc);
                acc = fmaf(tt[u].z, tt[u].z, acc);
                acc = fmaf(tt[u].w, tt[u].w, acc);
            }
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

extern "C" int chain_rate(float* out, int blocks, int steps, int mode, void* st) {
    hipLaunchKernelGGL(chain_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)st, out, steps, mode, 1.0f);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
