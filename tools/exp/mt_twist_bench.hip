// MT19937 block twist by one wave: the LDS in-place form of uq_quicfl_kernels.h (V0) against
// register forms (state word 64g + lane in VGPR g): V1 moves operands with ds_bpermute
// (__shfl), V2 takes the +1 neighbour with a DPP wave shift.  Each wave twists N blocks from its
// own seed and XORs the tempered words into a checksum (checked against a host MT19937).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mtb tools/exp/mt_twist_bench.hip && /tmp/mtb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kN = 624, kG = 10;

__host__ __device__ inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}
__host__ __device__ inline uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
}
__device__ inline void fence() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
}

__device__ void twist_lds(uint32_t* s, int lane) {
    uint32_t a[kG], b[kG], c[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const int i = 64 * g + lane;
        if (i < kN) { a[g] = s[i]; b[g] = s[i + 1 < kN ? i + 1 : 0]; }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) { const int i = 64 * g + lane; if (i < 227) c[g] = s[i + 397]; }
    fence();
#pragma unroll
    for (int g = 0; g < 4; ++g) { const int i = 64 * g + lane; if (i < 227) s[i] = mix(a[g], b[g], c[g]); }
    fence();
#pragma unroll
    for (int g = 3; g < 7; ++g) { const int i = 64 * g + lane; if (i >= 227) c[g] = s[i - 227]; }
#pragma unroll
    for (int g = 3; g < 7; ++g) { const int i = 64 * g + lane; if (i >= 227) s[i] = mix(a[g], b[g], c[g]); }
    fence();
#pragma unroll
    for (int g = 7; g < kG; ++g) {
        const int i = 64 * g + lane;
        if (i < kN) { c[g] = s[i - 227]; if (i == kN - 1) b[g] = s[0]; }
    }
#pragma unroll
    for (int g = 7; g < kG; ++g) { const int i = 64 * g + lane; if (i < kN) s[i] = mix(a[g], b[g], c[g]); }
    fence();
}

__device__ inline uint32_t perm(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v); }

template <bool DPP>
__device__ inline uint32_t next1(uint32_t v, int lane) {      // v of lane + 1 (lane 63: don't care)
    if (DPP) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);   // wave_shl:1
    return perm(v, (lane + 1) & 63);
}

// register twist: s[g] = word 64g + lane (g = 9: lanes < 48)
template <bool DPP>
__device__ void twist_reg(uint32_t (&s)[kG], int lane) {
    uint32_t N[kG];
    const int r13 = (lane + 13) & 63, r29 = (lane + 29) & 63;
    uint32_t bb[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const uint32_t nx = next1<DPP>(s[g], lane);
        const uint32_t first = g + 1 < kG ? (uint32_t)__builtin_amdgcn_readlane((int)s[g + 1], 0) : 0u;
        bb[g] = lane == 63 ? first : nx;
    }
#pragma unroll
    for (int g = 0; g < 3; ++g) {                                  // i < 192: c = old s[i + 397]
        const uint32_t t1 = perm(s[g + 6], r13), t2 = perm(s[g + 7], r13);
        N[g] = mix(s[g], bb[g], lane < 51 ? t1 : t2);
    }
    {                                                              // g = 3: lanes < 35 old s[9], else new N[0]
        const uint32_t t1 = perm(s[9], r13), t2 = perm(N[0], r29);
        N[3] = mix(s[3], bb[3], lane < 35 ? t1 : t2);
    }
#pragma unroll
    for (int g = 4; g < kG; ++g) {                                 // c = new word i - 227
        const uint32_t t1 = perm(N[g - 4], r29), t2 = perm(N[g - 3], r29);
        uint32_t b = bb[g];
        if (g == kG - 1) {
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)N[0], 0);
            b = lane == 47 ? n0 : b;
        }
        N[g] = mix(s[g], b, lane < 35 ? t1 : t2);
    }
#pragma unroll
    for (int g = 0; g < kG; ++g) s[g] = N[g];
}

template <int V>
__global__ void __launch_bounds__(64) bench_kernel(int nblk, uint32_t* out) {
    __shared__ uint32_t S[kN];
    const int lane = threadIdx.x;
    const uint32_t seed = 1000u + blockIdx.x;
    if (lane == 0) {
        S[0] = seed;
        for (int i = 1; i < kN; ++i) S[i] = 1812433253u * (S[i - 1] ^ (S[i - 1] >> 30)) + (uint32_t)i;
    }
    fence();
    uint32_t acc = 0;
    if (V == 0) {
        for (int k = 0; k < nblk; ++k) {
            twist_lds(S, lane);
#pragma unroll
            for (int g = 0; g < kG; ++g) { const int i = 64 * g + lane; if (i < kN) acc ^= temper(S[i]); }
        }
    } else {
        uint32_t s[kG];
#pragma unroll
        for (int g = 0; g < kG; ++g) { const int i = 64 * g + lane; s[g] = i < kN ? S[i] : 0u; }
        for (int k = 0; k < nblk; ++k) {
            twist_reg<V == 2>(s, lane);
#pragma unroll
            for (int g = 0; g < kG; ++g) { const int i = 64 * g + lane; if (i < kN) acc ^= temper(s[g]); }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o);
    if (lane == 0) out[blockIdx.x] = acc;
}

static uint32_t host_check(uint32_t seed, int nblk) {
    std::vector<uint32_t> s(kN);
    s[0] = seed;
    for (int i = 1; i < kN; ++i) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
    uint32_t acc = 0;
    for (int k = 0; k < nblk; ++k) {
        for (int i = 0; i < kN; ++i) s[i] = mix(s[i], s[(i + 1) % kN], s[(i + 397) % kN]);
        for (int i = 0; i < kN; ++i) acc ^= temper(s[i]);
    }
    return acc;
}

int main() {
    const int nblk = 2000;
    const int grids[] = {256, 1024, 4096};
    uint32_t* d_out;
    hipMalloc(&d_out, 4096 * 4);
    std::vector<uint32_t> h(4096);
    std::vector<uint32_t> want(4);
    for (int b = 0; b < 4; ++b) want[b] = host_check(1000u + b, nblk);
    printf("{\"tool\": \"mt_twist_bench\", \"blocks_per_wave\": %d, \"rows\": [", nblk);
    bool firstrow = true;
    for (int v = 0; v < 3; ++v) {
        for (int gi = 0; gi < 3; ++gi) {
            const int g = grids[gi];
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            auto launch = [&]() {
                if (v == 0) hipLaunchKernelGGL(bench_kernel<0>, dim3(g), dim3(64), 0, 0, nblk, d_out);
                if (v == 1) hipLaunchKernelGGL(bench_kernel<1>, dim3(g), dim3(64), 0, 0, nblk, d_out);
                if (v == 2) hipLaunchKernelGGL(bench_kernel<2>, dim3(g), dim3(64), 0, 0, nblk, d_out);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), d_out, g * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int b = 0; b < 4; ++b) bad += h[b] != want[b];
            printf("%s{\"variant\": %d, \"waves\": %d, \"ms\": %.4f, \"ns_per_twist_per_wave\": %.1f, \"bad\": %d}",
                   firstrow ? "" : ", ", v, g, ms, ms * 1e6 / nblk, bad);
            firstrow = false;
        }
    }
    printf("]}\n");
    return 0;
}
