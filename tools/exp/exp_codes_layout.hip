// Experiment (tools/, not shipped): does the layout of K2's int8 code stream decide K2's
// two speeds (1.7 / 2.0 ms on the C2 batch)?  Row-major codes are a third
// per-client stream (1024 concurrent 4 KB/tile writes at 1 MiB pitch); tile-major codes
// ([tile][client][4096]) make all clients' codes of one tile one contiguous 4 MiB block,
// which the 1024 workgroups (all at about the same tile) fill together.
// Same kernel as the product's quantize_stream_kernel<true, true, true> except the code
// store address.  Built against the product source:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
//     -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero \
//     -o tools/exp/libexp_codes_layout.so tools/exp/exp_codes_layout.hip
#include "../../unbiased-quantization-distributed-mean-estimation_amd/csrc/uq_dme.hip"

namespace {
__global__ void __launch_bounds__(kQBlock, 4)
k2_tile_major_codes(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes,
                    int32_t* __restrict__ overflow, int64_t n, int64_t d, int32_t tiles, float fm,
                    const float* __restrict__ Xs, const float* __restrict__ l1) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ __attribute__((aligned(16))) float s_o[kQTile];
    __shared__ float s_tab[kTab];
    __shared__ ScanLds sl;
    const int tid = threadIdx.x;
    const int64_t vec = blockIdx.x;
    const float L = l1[vec];
    const DivPlan dp = div_plan(L);
    const float Xv = Xs[vec];
    const uint32_t row_bytes = (uint32_t)(d * 4);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + vec * d, row_bytes);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(out + vec * d, row_bytes);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(codes, (uint32_t)(n * d));      // whole buffer (< 4 GiB)
    TileRegs pre_x;
    load_tile_buf(pre_x, rx, 0u, tid);
    build_table(s_tab, tid, L, fm);
    double P = 0.0;
    uint32_t cw[4] = {0u, 0u, 0u, 0u};
    float kmax = 0.0f;
    auto store_codes_tm = [&](int32_t t) {
        const u32x4v v = {cw[0], cw[1], cw[2], cw[3]};
        const uint32_t off = ((uint32_t)t * (uint32_t)n + (uint32_t)vec) * (uint32_t)kQTile + (uint32_t)(tid * kQItems);
        __builtin_amdgcn_raw_buffer_store_b128(v, rc, off, 0, kAuxNT);
    };
    for (int32_t tile = 0; tile < tiles; ++tile) {
        stage_tile<true>(pre_x, s_x, tid);
        __syncthreads();
        if (tile > 0) {
            store_tile_buf(s_o, ro, (uint32_t)(tile - 1) * (uint32_t)kQTile * 4u, tid);
            store_codes_tm(tile - 1);
        }
        if (tile + 1 < tiles) load_tile_buf(pre_x, rx, (uint32_t)(tile + 1) * (uint32_t)(kQTile * 4), tid);
        TileState st;
        TileVals tv;
        P = uniform_d(P);
        const Binade B = binade_of(P);
        tile_pass1<true, true>(s_x, tv, sl, tid, kQTile, dp, fm, B, st);
        double pnext;
        const double base = resolve_exact(P, B, st, tv, s_x, sl, tid, pnext);
        tile_pass2<true, true>(s_o, tv, s_tab, tid, base, L, fm, Xv, cw, kmax);
        P = pnext;
    }
    __syncthreads();
    store_tile_buf(s_o, ro, (uint32_t)(tiles - 1) * (uint32_t)kQTile * 4u, tid);
    store_codes_tm(tiles - 1);
    publish_kmax(kmax, L, overflow, vec, tid);
}
}  // namespace

extern "C" int exp_k2_tile_major(const float* x, float* q, int8_t* codes, int32_t* kmax, int64_t n, int64_t d, int64_t m,
                                 const float* X, const float* l1, void* stream) {
    if (d % kQTile != 0 || n * d >= ((int64_t)1 << 32)) return -2;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(kmax, 0, n * sizeof(int32_t), st) != hipSuccess) return -1;
    hipLaunchKernelGGL(k2_tile_major_codes, dim3((unsigned)n), dim3(kQBlock), 0, st, x, q, codes, kmax, n, d,
                       (int32_t)(d / kQTile), (float)m, X, l1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
