// Experiment (tools/, not shipped): data-flow upper bound of a fused K1+K2 over client
// segments.  Same reads, compute and writes as a fused kernel would do, with NO
// cross-workgroup waits (the L1 and prefixes are wrong on purpose): if this is not
// clearly faster than K1 + K2, the fused design is not worth its spin waits.
#include "../../unbiased-quantization-distributed-mean-estimation_amd/csrc/uq_dme.hip"

namespace {
template <int S>
__global__ void __launch_bounds__(kQBlock, 4)
exp_fused_kernel(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes,
                 int32_t* __restrict__ overflow, int64_t n, int64_t d, int32_t tiles, float fm,
                 const float* __restrict__ Xs, uint32_t* __restrict__ ctrl, float* __restrict__ part,
                 uint64_t* __restrict__ agg, int phases) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ __attribute__((aligned(16))) float s_o[kQTile];
    __shared__ float s_tab[kTab];
    __shared__ double s_wave[kQBlock / kWave];
    __shared__ uint32_t s_ticket;
    __shared__ float s_red[kQBlock / kWave];
    const int tid = threadIdx.x;
    const int R = tiles / S;
    const uint32_t total = (uint32_t)(n * S);
    for (;;) {
        if (tid == 0) s_ticket = atomicAdd(ctrl, 1u);
        __syncthreads();
        const uint32_t k = s_ticket;
        __syncthreads();
        if (k >= total) break;
        const int64_t vec = k / S;
        const int32_t tb = (int32_t)(k % S) * R, te = tb + R;
        const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + vec * d, (uint32_t)(d * 4));
        const __amdgpu_buffer_rsrc_t ro = make_rsrc(out + vec * d, (uint32_t)(d * 4));
        const __amdgpu_buffer_rsrc_t rc = make_rsrc(codes + vec * d, (uint32_t)d);
        // phase A: |x| partial sums of the segment
        TileRegs pre;
        float acc = 0.f;
        if (phases & 1) {
            load_tile_buf(pre, rx, (uint32_t)tb * kQTile * 4u, tid);
            for (int32_t t = tb; t < te; ++t) {
                TileRegs cur = pre;
                if (t + 1 < te) load_tile_buf(pre, rx, (uint32_t)(t + 1) * kQTile * 4u, tid);
#pragma unroll
                for (int j = 0; j < kQItems / 4; ++j)
                    acc += fabsf(cur.v[j].x) + fabsf(cur.v[j].y) + fabsf(cur.v[j].z) + fabsf(cur.v[j].w);
            }
            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
            if ((tid & 63) == 0) s_red[tid >> 6] = acc;
            __syncthreads();
            if (tid == 0) part[k] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        }
        const float L = 1000.0f + (float)(vec & 7);   // stands in for the client's L1
        const DivPlan dp = div_plan(L);
        // phase B: tile aggregates of the segment (pass 1)
        if (phases & 2) {
            load_tile_buf(pre, rx, (uint32_t)tb * kQTile * 4u, tid);
            for (int32_t t = tb; t < te; ++t) {
                stage_tile<true>(pre, s_x, tid);
                __syncthreads();
                if (t + 1 < te) load_tile_buf(pre, rx, (uint32_t)(t + 1) * kQTile * 4u, tid);
                TileState st;
                TileVals tv;
                tile_pass1<true>(s_x, tv, s_wave, tid, kQTile, dp, fm, st);
                if (tid == 0) agg[vec * tiles + t] = (uint64_t)__double_as_longlong(st.total);
            }
        }
        // phase D: outputs of the segment (pass 1 + pass 2, q and codes)
        if (phases & 4) {
            build_table(s_tab, tid, L, fm);
            double P = 0.0;
            uint32_t cw[4] = {0, 0, 0, 0};
            float kmax = 0.f;
            load_tile_buf(pre, rx, (uint32_t)tb * kQTile * 4u, tid);
            for (int32_t t = tb; t < te; ++t) {
                stage_tile<true>(pre, s_x, tid);
                __syncthreads();
                if (t > tb) {
                    const uint32_t tp = (uint32_t)(t - 1) * (uint32_t)kQTile;
                    store_tile_buf(s_o, ro, tp * 4u, tid);
                    store_codes_buf<true>(rc, codes + vec * d, cw, tp, d, tid);
                }
                if (t + 1 < te) load_tile_buf(pre, rx, (uint32_t)(t + 1) * kQTile * 4u, tid);
                TileState st;
                TileVals tv;
                tile_pass1<true>(s_x, tv, s_wave, tid, kQTile, dp, fm, st);
                tile_pass2<true, true>(s_o, tv, s_tab, tid, P, L, fm, Xs[vec], st, cw, kmax);
                P = P + st.total;
            }
            __syncthreads();
            const uint32_t tp = (uint32_t)(te - 1) * (uint32_t)kQTile;
            store_tile_buf(s_o, ro, tp * 4u, tid);
            store_codes_buf<true>(rc, codes + vec * d, cw, tp, d, tid);
            publish_kmax(kmax, L, overflow, vec, tid);
        }
        __syncthreads();
    }
}
}  // namespace

extern "C" int exp_fused(const float* x, float* out, int8_t* codes, int32_t* overflow, int64_t n, int64_t d,
                         int64_t m, const float* X, void* ws, int segs, int grid, int phases, void* stream) {
    const int32_t tiles = (int32_t)(d / kQTile);
    char* wsb = (char*)ws;
    uint32_t* ctrl = (uint32_t*)wsb;
    float* part = (float*)(wsb + 256);
    uint64_t* agg = (uint64_t*)(wsb + 256 + (size_t)n * 64 * 4);
    hipStream_t st = (hipStream_t)stream;
    hipMemsetAsync(ctrl, 0, 4, st);
    if (segs == 32)
        hipLaunchKernelGGL(exp_fused_kernel<32>, dim3(grid), dim3(kQBlock), 0, st, x, out, codes, overflow, n, d, tiles,
                           (float)m, X, ctrl, part, agg, phases);
    else if (segs == 16)
        hipLaunchKernelGGL(exp_fused_kernel<16>, dim3(grid), dim3(kQBlock), 0, st, x, out, codes, overflow, n, d, tiles,
                           (float)m, X, ctrl, part, agg, phases);
    else
        hipLaunchKernelGGL(exp_fused_kernel<64>, dim3(grid), dim3(kQBlock), 0, st, x, out, codes, overflow, n, d, tiles,
                           (float)m, X, ctrl, part, agg, phases);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
