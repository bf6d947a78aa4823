// uq_dme.hip — MI355X (gfx950) kernels + C-ABI for the unbiased L1-ball type quantizer.
//
// Reference path (paths relative to the reference root):
//   NMSE_Results/Codes/All_Schemes.py:609-641   Type_unbiased_quantize
//   NMSE_Results/Codes/Normal_dist.py:137-138    est += Q(v, R) / n   (client mean)
//
// Kernels (one HIP stage per group of reference torch ops):
//   K1a l1_partial_kernel   AS:624 |x|.sum(), torch CPU cascade: level-1 block sums
//   K1b l1_finalize_kernel  AS:624 the rest of the cascade tree, one wave per client
//   K2  quantize_kernel     AS:625-640 normalize -> floor/frac -> fp64 scan (cumsum)
//                           -> crossing test -> dequantize, decoupled look-back
//   K3  client_mean_kernel  ND:137-138 client-ordered f32 mean
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction: the
// reference computes m*p then floor then subtract as separate f32 ops), IEEE f32
// division and denormals kept (the reference runs on torch CPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../../include/uq_dme.h"

namespace {

constexpr int kWave = 64;
constexpr int kGrain = 32768;     // at::internal::GRAIN_SIZE (torch CPU intra-op split)
constexpr int kMaxThreads = 4096; // torch_threads supported by the L1 plan (per-thread buffer in LDS)

// ---- quantize tile geometry --------------------------------------------------------
constexpr int kQBlock = 256;               // threads per workgroup (4 waves)
constexpr int kQItems = 16;                // contiguous elements per thread
constexpr int kQTile = kQBlock * kQItems;  // 4096 elements per tile
// LDS tile image: 256 rows of 16 floats (thread t owns row t); float4 column c of row r
// lives at swz(r, c) (XOR swizzle, see there): bank-conflict-free without padding.
constexpr int64_t kStreamMinClients = 256; // >= this many clients: one workgroup per vector
constexpr int64_t kSegMinTiles = 1024;     // fewer clients but >= this many tiles: segmented stream
constexpr int64_t kMaxGridY = 65535;       // clients per launch of the per-tile kernels

// ---- workspace layout --------------------------------------------------------------
// [0,256)            control: u32 ticket, u32 abort (both reset by every call),
//                    u32 sticky error word (set on timeout; cleared by uq_check_status).
//                    A new workspace must be zero-filled once before first use.
// [256, ...)         u64 agg[n][tiles]           (small batches: tile sums A_t, then map m0)
// then               u64 incl[n][tiles]          (small batches: prefixes P'_t, then exact P_t)
// then               u64 map1[n][tiles]          (small batches: map m1)
// then               f32 l1part[n][groups][32]  (level-1 block sums)
// then               f32 l1[n]                  (computed norms)
constexpr size_t kCtrlBytes = 256;

// torch CPU `sum` of a contiguous f32 vector with T intra-op threads (ATen
// TensorIteratorBase::parallel_reduce -> two_pass_reduction, SumKernel cascade_sum):
//   d < GRAIN or T == 1: one cascade over the whole vector.
//   else: nt = min(T, ceil(d/GRAIN)) chunks of cs = ceil(d/nt) (ATen invoke_parallel); thread
//   t < nt sums chunk t into buffer[t] (buffer of T zeros), and the result is the SAME cascade
//   sum over the T-element buffer -- not a sequential add of the chunk sums (verified against
//   torch 2.10 for T = 1..39, 47, 63..65, 96, 128, 200, 256 at five sizes; T in {1,2,3,4,8}
//   happen to coincide with sequential order).
// Chunks are uniform except the last, so two geometries describe them all.
struct ChunkGeo {
    int64_t size;                    // chunk length
    int32_t lp;                      // log2(step) of its cascade
    int32_t ng1;                     // full level-1 groups in the chunk
};
struct L1Plan {
    int32_t nchunks;                 // nt
    int32_t nbuf;                    // T (length of the per-thread buffer), 1 in the one-chunk case
    int32_t total_groups;            // level-1 groups per vector, all chunks
    int64_t cs;                      // chunk stride (size of every chunk but the last)
    ChunkGeo full, last;             // chunks 0 .. nt-2, chunk nt-1
    __host__ __device__ int64_t off(int c) const { return (int64_t)c * cs; }
    __host__ __device__ const ChunkGeo& geo(int c) const { return c + 1 < nchunks ? full : last; }
    __host__ __device__ int32_t gbase(int c) const { return c * full.ng1; }
    __host__ __device__ int chunk_of_group(int32_t G) const {
        const int32_t nfull = (nchunks - 1) * full.ng1;
        return G < nfull ? G / full.ng1 : nchunks - 1;
    }
};

__host__ __device__ inline int ceil_log2_i64(int64_t x) {
    if (x <= 1) return 0;
    int r = 0;
    uint64_t v = (uint64_t)(x - 1);
    while (v) { ++r; v >>= 1; }
    return r;
}
__device__ inline int ceil_log2_dev(int64_t x) { return ceil_log2_i64(x); }

bool chunk_geo(int64_t s, ChunkGeo* g) {
    const int64_t rows = (s / 8) / 4;   // rows of 32 floats (8 lanes x 4 ILP)
    int lp = ceil_log2_i64(rows) / 4;
    if (lp < 4) lp = 4;
    if (lp > 8) return false;
    const int64_t step = (int64_t)1 << lp;
    const int64_t ng1 = (rows / step) / step;
    if (ng1 > (int64_t)1 << 28) return false;
    g->size = s;
    g->lp = lp;
    g->ng1 = (int32_t)ng1;
    return true;
}

bool make_plan(int64_t d, int32_t T, L1Plan* p) {
    std::memset(p, 0, sizeof(*p));
    if (T < 1) T = 1;
    if (T > kMaxThreads) return false;
    int64_t nt = 1, cs = d;
    if (!(d < kGrain || T == 1)) {
        nt = (d + kGrain - 1) / kGrain;
        if (nt > T) nt = T;
        cs = (d + nt - 1) / nt;
        nt = (d + cs - 1) / cs;        // chunks past d are empty (their buffer slots stay 0)
        p->nbuf = T;
    } else {
        p->nbuf = 1;
    }
    p->nchunks = (int32_t)nt;
    p->cs = cs;
    if (!chunk_geo(nt > 1 ? cs : d, &p->full)) return false;
    if (!chunk_geo(d - (nt - 1) * cs, &p->last)) return false;
    const int64_t g = (nt - 1) * (int64_t)p->full.ng1 + p->last.ng1;
    if (g > (int64_t)1 << 30) return false;
    p->total_groups = (int32_t)g;
    return true;
}

// v = x / den (AS:625) without the IEEE division sequence (~10 VALU per element).  den is
// one per client, so y = RN(1/den) is computed once (IEEE) and each quotient takes a
// product and two residual corrections (Markstein):
//     q0 = RN(x*y);  q1 = RN(q0 + RN(x - den*q0)*y)    (faithful)
//                    q2 = RN(q1 + RN(x - den*q1)*y)    (= RN(x/den): y correctly rounded,
//                                                       q1 faithful, no underflow)
// as packed fma pairs.  No underflow: den = L1 + 1e-12 >= 2^-39.9 always and den < 2^40 is
// required per client (else the IEEE division is used throughout), and elements with
// |q2| < 2^-59/den (covers every 0 < |x| < 2^-60) or q2 NaN (x = inf/NaN, overflow) are
// recomputed with the IEEE division.  x = +-0 gives q = +-0 in either sign, which is
// immaterial (only v < 0 and |v| are used).  tools/markstein_check.c checks this exact
// function against IEEE division over every finite f32 x for divisors across the range.
struct DivPlan {
    float den, y, thr;
    bool fast;
};
__device__ __forceinline__ DivPlan div_plan(float L) {
    DivPlan p;
    p.den = L + 1e-12f;                  // AS:625 (f32 add)
    p.fast = p.den < 0x1p40f;            // false for NaN / inf
    p.y = 1.0f / p.den;
    p.thr = 0x1p-59f / p.den;
    return p;
}
// z / nrm of EDEN's bins (AS:329): the Markstein sequence for a divisor in [2^-39, 2^40)
// (tools/markstein_check.c checks every f32 numerator for divisors over that range)
__device__ __forceinline__ DivPlan div_plan_norm(float nv) {
    DivPlan p;
    p.den = nv;
    p.fast = nv >= 0x1p-39f && nv < 0x1p40f;
    p.y = 1.0f / nv;
    p.thr = 0x1p-59f / nv;
    return p;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void div4(const float (&xs)[4], const DivPlan& dp, float (&vs)[4]) {
    if (dp.fast) {
        const f32x2 Y = {dp.y, dp.y}, B = {-dp.den, -dp.den};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x2 a = {xs[2 * h], xs[2 * h + 1]};
            f32x2 q = a * Y;
            f32x2 r = __builtin_elementwise_fma(B, q, a);
            q = __builtin_elementwise_fma(r, Y, q);
            r = __builtin_elementwise_fma(B, q, a);
            q = __builtin_elementwise_fma(r, Y, q);
            vs[2 * h] = q.x;
            vs[2 * h + 1] = q.y;
        }
        // one test per four: the smallest |q| (q is finite here: den >= |x| and finite)
        const float mn = fminf(fminf(fabsf(vs[0]), fabsf(vs[1])), fminf(fabsf(vs[2]), fabsf(vs[3])));
        if (__builtin_expect(!(mn >= dp.thr), 0)) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (!(fabsf(vs[c]) >= dp.thr) && xs[c] != 0.0f) vs[c] = xs[c] / dp.den;
        }
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) vs[c] = xs[c] / dp.den;
    }
}
// One quotient, the same operations as div4 (so the same bits).
__device__ __forceinline__ float div1(float x, const DivPlan& dp) {
    if (!dp.fast) return x / dp.den;
    float q = x * dp.y;
    float r = fmaf(-dp.den, q, x);
    q = fmaf(r, dp.y, q);
    r = fmaf(-dp.den, q, x);
    q = fmaf(r, dp.y, q);
    if (__builtin_expect(!(fabsf(q) >= dp.thr) && x != 0.0f, 0)) q = x / dp.den;
    return q;
}
// N quotients with div1's bits and no per-element branch: the Markstein steps on pairs
// (packed fma), one guard test over the lane's N elements and a wave-uniform branch into the
// IEEE division for the rare lane that needs it.  Elements whose bit is set in `skip` are
// left out of the guard (their quotient is discarded by the caller).
template <int N>
__device__ __forceinline__ void div_n(const float (&xs)[N], const DivPlan& dp, float (&vs)[N], uint32_t skip = 0u) {
    static_assert(N % 2 == 0, "pairs");
    if (dp.fast) {
        const f32x2 Y = {dp.y, dp.y}, B = {-dp.den, -dp.den};
#pragma unroll
        for (int h = 0; h < N / 2; ++h) {
            const f32x2 a = {xs[2 * h], xs[2 * h + 1]};
            f32x2 q = a * Y;
            f32x2 r = __builtin_elementwise_fma(B, q, a);
            q = __builtin_elementwise_fma(r, Y, q);
            r = __builtin_elementwise_fma(B, q, a);
            q = __builtin_elementwise_fma(r, Y, q);
            vs[2 * h] = q.x;
            vs[2 * h + 1] = q.y;
        }
        bool bad = false;
#pragma unroll
        for (int c = 0; c < N; ++c) bad |= !(fabsf(vs[c]) >= dp.thr) && xs[c] != 0.0f && !((skip >> c) & 1u);
        if (__builtin_expect(__ballot(bad) != 0ull, 0)) {
#pragma unroll
            for (int c = 0; c < N; ++c)
                if (!(fabsf(vs[c]) >= dp.thr) && xs[c] != 0.0f) vs[c] = xs[c] / dp.den;
        }
    } else {
#pragma unroll
        for (int c = 0; c < N; ++c) vs[c] = xs[c] / dp.den;
    }
}
// RN(k / m) for the dequantize step (m >= 1 is exact in f32 up to 2^24 and below 2^40
// always): the same Markstein sequence with den = m itself (no 1e-12 term).
__device__ __forceinline__ DivPlan div_plan_m(float fm) {
    DivPlan p;
    p.den = fm;
    p.fast = fm >= 1.0f && fm < 0x1p40f;
    p.y = 1.0f / fm;
    p.thr = 0x1p-59f / fm;
    return p;
}


// Element transforms summed by the K1 cascade.  The cascade itself (order of f32 adds)
// is the torch CPU `sum` order whatever is summed.
struct AbsOp {            // AS:624  input_vector.abs().sum()
    static constexpr bool kHist = false;   // no radix-digit histogram (see RezKHistOp)
    float den, fm;
    uint32_t *h, *zn;
    __device__ static AbsOp make(const float*, float, int64_t) { return AbsOp{0.f, 0.f, nullptr, nullptr}; }
    __device__ float operator()(float v) const { return fabsf(v); }
    __device__ void apply4(const float (&v)[4], float (&a)[4]) const {
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] += fabsf(v[c]);
    }
};
struct RezKOp {           // AS:648-649  k' = floor(m * p + 0.5), p = |x| / (L1 + 1e-12)
    DivPlan dp;
    float fm;
    uint32_t *h, *zn;
    __device__ static RezKOp make(const float* l1, float fm, int64_t vec) {
        return RezKOp{div_plan(l1[vec]), fm, nullptr, nullptr};
    }
    __device__ float operator()(float v) const { return floorf(fm * div1(fabsf(v), dp) + 0.5f); }
    // four elements per call (K1a): the quotients by div4 (one underflow test per four,
    // the same bits as div1), then the per-element op; a[c] += op(v[c]) in the same order
    __device__ void apply4(const float (&v)[4], float (&a)[4]) const {
        const float ab[4] = {fabsf(v[0]), fabsf(v[1]), fabsf(v[2]), fabsf(v[3])};
        float qs[4];
        div4(ab, dp, qs);
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] += floorf(fm * qs[c] + 0.5f);
    }
};
constexpr int kHistSlots = 4;                       // per biased client: key-digit passes 0-2, KB2's fine bins
constexpr int kFineSlot = 3;
// The fine bin of a selection value v: non-decreasing in v (so in the key), 2^11 bins linear
// in |v| (delta' lies in [-0.5, 0.5]): v > 0 -> 1024 + min(1023, floor(2048 |v|)), v < 0 ->
// 1023 - min(1023, floor(2048 |v|)), +-0 -> 1024, NaN -> 2047 (ATen's topk puts NaN first).
// For v != 0 and not NaN, fbin(-v) = 2047 - fbin(v): KB2 counts +delta' and KB4a mirrors the
// counts for Delta < 0, moving zeros (1023 -> 1024) and NaNs (0 -> 2047) back.
__device__ __forceinline__ uint32_t rez_fbin(float v) {
    if (v != v) return 2047u;
    const float a = fabsf(v) * 2048.0f;                   // exact (a power-of-two scale)
    const uint32_t q = a >= 1023.0f ? 1023u : (uint32_t)a;
    return v > 0.f ? 1024u + q : (v < 0.f ? 1023u - q : 1024u);
}

// RezKOp that also counts the fine bin (rez_fbin) of +delta' = k' - m p into h[2048] (KB4a's
// histogram), and delta' == 0 / NaN elements into zn[0] / zn[1] so that the histogram of
// -delta' can be mirrored from it.
// h / zn point to LDS in K1a (flushed per workgroup) and to global memory in K1b.
struct RezKHistOp {
    static constexpr bool kHist = true;
    DivPlan dp;
    float fm;
    uint32_t *h, *zn;
    __device__ static RezKHistOp make(const float* l1, float fm, int64_t vec) {
        return RezKHistOp{div_plan(l1[vec]), fm, nullptr, nullptr};
    }
    __device__ float count(float mp) const {
        const float kp = floorf(mp + 0.5f);
        const float dp = (kp - mp) + 0.0f;                 // the value rez_key_of(dp, true) encodes
        atomicAdd(&h[rez_fbin(dp)], 1u);
        if (dp == 0.0f) atomicAdd(&zn[0], 1u);
        else if (dp != dp) atomicAdd(&zn[1], 1u);
        return kp;
    }
    __device__ float operator()(float v) const { return count(fm * div1(fabsf(v), dp)); }
    __device__ void apply4(const float (&v)[4], float (&a)[4]) const {     // as RezKOp::apply4
        const float ab[4] = {fabsf(v[0]), fabsf(v[1]), fabsf(v[2]), fabsf(v[3])};
        float qs[4];
        div4(ab, dp, qs);
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] += count(fm * qs[c]);
    }
};

// =====================================================================================
// K1a: level-1 block sums of op(x) in torch cascade order.
// One workgroup = one level-1 group = step leaves x step rows x 32 streams.
// Thread (leaf b, quad q) sums rows [b*step, (b+1)*step) of streams 4q..4q+3
// sequentially (ATen level 0); then 32 threads add the step leaves in order (level 1).
// BIG: cascade steps 64-256 (one chunk of more than 2^28 elements, e.g. T = 1 beyond
// d = 2^28): 256 threads, each taking leaves b, b + 32, ...; 32 KB of leaf sums.
// =====================================================================================
// gpw level-1 groups per workgroup, one after the other (the histogram op: its 2048-bin LDS
// histogram is flushed -- one global atomic per nonzero bin, ~1700 per 8192 coordinates of
// Gaussian rows -- once per gpw groups instead of once per group).
template <bool VEC4, class Op, bool BIG = false>
__global__ void __launch_bounds__(256)
l1_partial_kernel(const float* __restrict__ x, int64_t d, L1Plan plan, float* __restrict__ part,
                  const float* __restrict__ l1, float fm, uint32_t* __restrict__ hist_g, uint32_t* __restrict__ zn_g,
                  int gpw = 1) {
    const int64_t vec = blockIdx.y;
    Op op = Op::make(l1, fm, vec);
    __shared__ uint32_t hs[Op::kHist ? 2048 + 2 : 1];
    if (Op::kHist) {
        for (int b = threadIdx.x; b < 2048 + 2; b += blockDim.x) hs[b] = 0u;
        __syncthreads();
        op.h = hs;
        op.zn = hs + 2048;
    }
    __shared__ float leaf[(BIG ? 256 : 32) * 32];   // [leaf][32]
    const int32_t G0 = (int32_t)blockIdx.x * gpw;
    const int32_t G1 = min((int32_t)plan.total_groups, G0 + gpw);
    for (int32_t G = G0; G < G1; ++G) {
    if (G > G0) __syncthreads();              // the previous group's leaf sums are read
    const int c = plan.chunk_of_group(G);
    const int32_t g = G - plan.gbase(c);
    const int lp = plan.geo(c).lp;
    const int step = 1 << lp;
    const int tid = threadIdx.x;
    const int nthreads = 8 * step;            // 8 quads x step leaves
    const float* base = x + vec * d + plan.off(c) + (int64_t)g * step * step * 32;
    for (int b = tid >> 3; BIG ? b < step : tid < nthreads; b += 32) {
        const int q = tid & 7;
        const float* p = base + ((int64_t)b * step) * 32 + 4 * q;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < step; ++r) {
            float v[4];
            if (VEC4) {
                typedef float k1x4 __attribute__((ext_vector_type(4)));
                const k1x4 tv = __builtin_nontemporal_load(reinterpret_cast<const k1x4*>(p + (int64_t)r * 32));
                v[0] = tv.x; v[1] = tv.y; v[2] = tv.z; v[3] = tv.w;
            } else {
                const float* pr = p + (int64_t)r * 32;
                v[0] = pr[0]; v[1] = pr[1]; v[2] = pr[2]; v[3] = pr[3];
            }
            op.apply4(v, a);                  // a[c] += op(v[c]), streams 4q..4q+3 in row order
        }
        float* l = leaf + b * 32 + 4 * q;
        l[0] = a[0]; l[1] = a[1]; l[2] = a[2]; l[3] = a[3];
        if (!BIG) break;
    }
    __syncthreads();
    if (tid < 32) {
        float acc = 0.f;
        for (int b = 0; b < step; ++b) acc += leaf[b * 32 + tid];
        part[(vec * plan.total_groups + G) * 32 + tid] = acc;
    }
    }
    if (Op::kHist) {
        const int tid = threadIdx.x;
        __syncthreads();                      // every group's LDS counts are in
        for (int b = tid; b < 2048; b += blockDim.x)
            if (hs[b]) atomicAdd(&hist_g[((size_t)vec * kHistSlots + kFineSlot) * 2048 + b], hs[b]);
        if (tid < 2 && hs[2048 + tid]) atomicAdd(&zn_g[vec * 2 + tid], hs[2048 + tid]);
    }
}

// Sequential sum of `nrows` rows of stream `a` starting at element `start`.
// Loads go out 16 at a time ahead of the (ordered) adds: one memory round trip per 16 rows.
template <class Op>
__device__ float seq_rows(const Op& op, const float* __restrict__ xv, int64_t start, int64_t nrows, int a) {
    float acc = 0.f;
    int64_t r = 0;
    for (; r + 16 <= nrows; r += 16) {
        float t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) t[u] = xv[start + (r + u) * 32 + a];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += op(t[u]);
    }
    for (; r < nrows; ++r) acc += op(xv[start + r * 32 + a]);
    return acc;
}

// =====================================================================================
// K1b: finish the cascade for each client (one wave per client).
// Lanes 0..31 own the 32 streams (8 lanes x 4 ILP): level-2/3 accumulation over the
// level-1 block sums, the open level-1 group and the tail rows (ATen multi_row_sum),
// then the ILP/lane/tail combination of ATen row_sum / vectorized_inner_sum, then the
// chunk results in chunk order (torch parallel_reduce).
// =====================================================================================
constexpr int kFinStage = 64;       // level-1 block sums staged in LDS per wave at a time (8 KB)
constexpr int kFinWaves = 8;        // chunks are finished by different waves, summed in order
// LDS written and read back by lanes of the same wave: a wave-level barrier suffices.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Column k of ATen multi_row_sum over R rows of width W (row stride W), f32 accumulate
// (the same level structure as the K1a/K1b cascade, walked by one lane).
__device__ float cascade_col(const float* a, int64_t R, int W, int k) {
    int lp = ceil_log2_dev(R) / 4;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int64_t i = 0;
    for (; i + step <= R;) {
        for (int64_t j = 0; j < step; ++j, ++i) a0 += a[i * W + k];
        a1 += a0; a0 = 0.f;
        if ((i & (mask << lp)) != 0) continue;
        a2 += a1; a1 = 0.f;
        if ((i & (mask << (2 * lp))) != 0) continue;
        a3 += a2; a2 = 0.f;
    }
    for (; i < R; ++i) a0 += a[i * W + k];
    return ((a0 + a1) + a2) + a3;
}
// torch cascade_sum of a[0..s) (ATen vectorized_inner_sum for s >= 8, scalar row_sum below),
// computed by the lanes of one wave; the result is valid in lane 0.  Used on the two-pass
// reduction's per-thread buffer (s = T <= kMaxThreads, so it is cheap).
__device__ float lds_torch_sum(const float* a, int s, int lane) {
    if (s < 8) {
        float p[4] = {0.f, 0.f, 0.f, 0.f};
        if (s >= 4)
            for (int k = 0; k < 4; ++k) p[k] = 0.f + a[k];
        for (int k = (s >= 4 ? 4 : 0); k < s; ++k) p[0] += a[k];
        return ((p[0] + p[1]) + p[2]) + p[3];
    }
    const int vs = s / 8, nilp = vs / 4;
    const float col = (lane < 32 && nilp) ? cascade_col(a, nilp, 32, lane) : 0.f;
    float p[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) p[j] = __shfl(col, j, kWave);
    float p0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) p0[l] = p[l];
    for (int v = nilp * 4; v < vs; ++v)
#pragma unroll
        for (int l = 0; l < 8; ++l) p0[l] += a[v * 8 + l];
#pragma unroll
    for (int k = 1; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < 8; ++l) p0[l] += p[k * 8 + l];
    float acc = 0.f;
    for (int k = vs * 8; k < s; ++k) acc += a[k];
#pragma unroll
    for (int l = 0; l < 8; ++l) acc += p0[l];
    return acc;
}

// WAVES = 1 when there is one torch chunk (T = 1 or d < 32768): the eight waves' staging
// buffers (64 KB of LDS) held two workgroups per CU for one working wave (37 us at
// 1024 x 2^20, T = 1).
// WIDE (one chunk, a few clients: WAVES = 8, host choice): the level-2 group sums
// B_h = sum of `step` level-1 block sums in order are independent of each other, so all eight
// waves form them at once (step loads in flight per thread) and only acc3 = sum of B_h in order
// stays serial: one client's chain of ng1 dependent adds through eight LDS stages took 65 us at
// d = 2^22 (half of the n = 1 call, profiles/r6d_c4_unbiased_kernel_stats.csv).  Same adds in
// the same order.
template <class Op, int WAVES = kFinWaves, bool WIDE = false>
__global__ void __launch_bounds__(64 * WAVES)
l1_finalize_kernel(const float* __restrict__ x, int64_t d, L1Plan plan,
                   const float* __restrict__ part, float* __restrict__ l1_out,
                   const float* __restrict__ l1, float fm, uint32_t* __restrict__ hist_g,
                   uint32_t* __restrict__ zn_g) {
    const int64_t vec = blockIdx.x;
    Op op = Op::make(l1, fm, vec);
    // the elements outside full level-1 groups (open leaves, tail rows) count into an LDS
    // histogram, flushed once: one global atomic per element on the few hot first-digit bins
    // took 74 us per call at d = 172 554 (six torch chunks of 130 such rows)
    __shared__ uint32_t hs[Op::kHist ? 2048 + 2 : 1];
    if (Op::kHist) {
        for (int b = threadIdx.x; b < 2048 + 2; b += blockDim.x) hs[b] = 0u;
        __syncthreads();
        op.h = hs;
        op.zn = hs + 2048;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float* xv = x + vec * d;
    __shared__ float fin_w[WAVES][32];
    __shared__ __attribute__((aligned(16))) float s_stage_w[WAVES][kFinStage * 32];
    __shared__ float s_tail_w[WAVES][64];
    // the per-thread buffer of the two-pass reduction: plan.nbuf floats of dynamic LDS (a
    // static kMaxThreads buffer would halve the workgroups per CU for every T)
    extern __shared__ float s_chunk[];
    float* fin = fin_w[wv];
    float* s_stage = s_stage_w[wv];
    float* s_tail = s_tail_w[wv];
    for (int t = plan.nchunks + (int)threadIdx.x; t < plan.nbuf; t += 64 * WAVES) s_chunk[t] = 0.0f;
    float wide_acc3 = 0.f;                            // WIDE: acc3 of chunk 0, lanes < 32 of wave 0
    if (WIDE) {
        const ChunkGeo& geo = plan.geo(0);
        const int64_t step = (int64_t)1 << geo.lp;
        const int64_t ng2 = geo.ng1 / step;
        const float* pc = part + (vec * plan.total_groups + plan.gbase(0)) * 32;
        float* sB = &s_stage_w[0][0];                 // WAVES * kFinStage groups x 32 streams
        constexpr int kG = WAVES * kFinStage;
        for (int64_t h0 = 0; h0 < ng2; h0 += kG) {
            const int nh = (int)std::min<int64_t>(kG, ng2 - h0);
            for (int t = threadIdx.x; t < nh * 32; t += 64 * WAVES) {
                const float* src = pc + ((h0 + t / 32) * step) * 32 + (t & 31);
                float b = 0.f;
                for (int64_t j0 = 0; j0 < step; j0 += 16) {
                    float v[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = src[(j0 + u) * 32];
#pragma unroll
                    for (int u = 0; u < 16; ++u) b += v[u];
                }
                sB[t] = b;
            }
            __syncthreads();
            if (wv == 0 && lane < 32)
                for (int h = 0; h < nh; ++h) wide_acc3 += sB[h * 32 + lane];
            __syncthreads();
        }
    }
    for (int c = wv; c < plan.nchunks; c += WAVES) {
        const int64_t off = plan.off(c);
        const ChunkGeo& geo = plan.geo(c);
        const int64_t s = geo.size;
        float chunk_sum;
        if (s < 8) {
            // ATen scalar row_sum (ILP 4, rows < step -> all rows land in acc0).  Lane 0
            // only: the op may count each element (RezKHistOp's histogram)
            float p[4] = {0.f, 0.f, 0.f, 0.f};
            if (lane == 0) {
                if (s >= 4)
                    for (int k = 0; k < 4; ++k) p[k] = 0.f + op(xv[off + k]);
                for (int64_t k = (s >= 4 ? 4 : 0); k < s; ++k) p[0] += op(xv[off + k]);
            }
            chunk_sum = ((p[0] + p[1]) + p[2]) + p[3];
        } else {
            const int64_t vs = s / 8, rows = vs / 4;
            const int lp = geo.lp;
            const int64_t step = (int64_t)1 << lp;
            const int64_t nleaf = rows / step;
            const int64_t ng1 = geo.ng1;
            const int64_t ng2 = ng1 / step;
            // level-2/3 over the ng1 block sums in order: groups [h*step, (h+1)*step) for
            // h < ng2 into b2 then acc3, the rest into acc2.  The block sums are staged
            // through LDS by the whole wave (coalesced, all loads in flight), so the
            // sequential adds read LDS instead of one dependent global load each.
            const float* pc = part + (vec * plan.total_groups + plan.gbase(c)) * 32;
            float acc3 = 0.f, acc2 = 0.f, b2 = 0.f;
            const int64_t n3 = ng2 * step;
            if (WIDE) {                               // B_h formed above; the rest after n3 in order
                acc3 = wide_acc3;
                if (lane < 32)
                    for (int64_t k = n3; k < ng1; ++k) acc2 += pc[k * 32 + lane];
            }
            for (int64_t k0 = WIDE ? ng1 : 0; k0 < ng1; k0 += kFinStage) {
                const int nk = (int)std::min<int64_t>(kFinStage, ng1 - k0);
                wave_sync();
                const float4* src = reinterpret_cast<const float4*>(pc + k0 * 32);
                float4* dst = reinterpret_cast<float4*>(s_stage);
                for (int i = lane; i < nk * 8; i += 64) dst[i] = src[i];
                wave_sync();
                if (lane < 32) {
                    for (int kk = 0; kk < nk; ++kk) {
                        const int64_t k = k0 + kk;
                        const float v = s_stage[kk * 32 + lane];
                        if (k < n3) {
                            b2 += v;
                            if (((k + 1) & (step - 1)) == 0) {         // step = 2^lp (no 64-bit modulo)
                                acc3 += b2;
                                b2 = 0.f;
                            }
                        } else {
                            acc2 += v;
                        }
                    }
                }
            }
            if (lane < 32) {
                float acc1 = 0.f;
                for (int64_t b = ng1 * step; b < nleaf; ++b)
                    acc1 += seq_rows(op, xv, off + b * step * 32, step, lane);
                float acc0 = seq_rows(op, xv, off + nleaf * step * 32, rows - nleaf * step, lane);
                fin[lane] = ((acc0 + acc1) + acc2) + acc3;
            }
            // the < 40 elements after the 32-stream rows, one load per lane, into LDS
            const int64_t t0 = rows * 32;
            const int nt = (int)(s - t0);
            if (lane < nt) s_tail[lane] = xv[off + t0 + lane];
            wave_sync();
            if (lane == 0) {
                float p0[8];
                for (int l = 0; l < 8; ++l) p0[l] = fin[l];
                for (int64_t v = rows * 4; v < vs; ++v)
                    for (int l = 0; l < 8; ++l) p0[l] += op(s_tail[v * 8 + l - t0]);
                for (int k = 1; k < 4; ++k)
                    for (int l = 0; l < 8; ++l) p0[l] += fin[k * 8 + l];
                float acc = 0.f;
                for (int64_t k = vs * 8; k < s; ++k) acc += op(s_tail[k - t0]);
                for (int l = 0; l < 8; ++l) acc += p0[l];
                fin[0] = acc;
            }
            wave_sync();
            chunk_sum = fin[0];
            wave_sync();
        }
        if (lane == 0) s_chunk[c] = 0.0f + chunk_sum;     // buffer[t] = 0 + (thread t's chunk)
    }
    __syncthreads();
    if (Op::kHist) {
        for (int b = threadIdx.x; b < 2048; b += blockDim.x)
            if (hs[b]) atomicAdd(&hist_g[((size_t)vec * kHistSlots + kFineSlot) * 2048 + b], hs[b]);
        if (threadIdx.x < 2 && hs[2048 + threadIdx.x]) atomicAdd(&zn_g[vec * 2 + threadIdx.x], hs[2048 + threadIdx.x]);
    }
    // second pass of the two-pass reduction: out = 0 + cascade sum of the T-element buffer
    if (wv == 0) {
        const float total = lds_torch_sum(s_chunk, plan.nbuf, lane);
        if (lane == 0) l1_out[vec] = 0.0f + total;
    }
}

// =====================================================================================
// K2: fused normalize / floor / fp64 scan / crossing / dequantize.
//
// Scan (AS:635): torch CPU cumsum of f32 accumulates SEQUENTIALLY in fp64 and rounds
// each prefix to f32.  K2 reproduces every fp64 prefix bit-for-bit, in parallel:
//
//   While the running sum S stays in one fp64 binade [2^E, 2^(E+1)) (spacing G =
//   2^(E-52)), the add S + f rounds to a multiple of G, and the result depends on S
//   only through S mod 2G (round-half-even looks at the parity of S/G).  So a thread
//   runs its 16 adds twice, from B0 = 2^E (parity 0) and B1 = 2^E + G (parity 1):
//   T_p = chain_p - B_p is its EXACT increment for a start of parity p.  All T are
//   multiples of G, so the block scan of T0 is exact in any order.  Threads with
//   T0 != T1 ("ties": an element with remainder exactly G/2) are resolved in order
//   from their exact start parity (the lowest mantissa bit of the start).  A tile is
//   "regular" when its exact start P >= 32 and P + total + 1 < 2^(E+1); otherwise
//   (tile 0, binade crossings: about log2(d) tiles per vector) each thread takes the
//   binade of its approximate start, threads near a binade edge add their 16 values
//   one by one, and one lane walks the threads in order.
//
// Forms: the stream kernel carries the exact P from tile to tile (one workgroup per
// client).  Batches of fewer clients fold per client: approximate tile sums ->
// approximate prefixes P' (binade of each tile) -> exact tile maps (T for a start of
// parity 0 / 1, ties resolved for both) -> exact serial fold (irregular tiles are
// recomputed from their exact start) -> outputs from the exact P.  Every form gives
// the sequential cumsum's bits, hence the same bits.
// =====================================================================================
// 64-bit DPP move (two 32-bit halves); lanes without a source (or outside ROWMASK) read 0.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, CTRL, ROWMASK, 0xF, true);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(u >> 32), CTRL, ROWMASK, 0xF, true);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// Inclusive wave scan by DPP (row_shr 1/2/4/8, then row_bcast 15/31): no LDS round trips.
// Only used on sums that are exact in any order (multiples of one G below 2^E).
__device__ __forceinline__ double wave_incl_scan(double v, int) {
    v = v + dpp_d<0x111, 0xF>(v);                  // row_shr:1
    v = v + dpp_d<0x112, 0xF>(v);                  // row_shr:2
    v = v + dpp_d<0x114, 0xF>(v);                  // row_shr:4
    v = v + dpp_d<0x118, 0xF>(v);                  // row_shr:8
    v = v + dpp_d<0x142, 0xA>(v);                  // row_bcast:15 -> rows 1, 3
    v = v + dpp_d<0x143, 0xC>(v);                  // row_bcast:31 -> rows 2, 3
    return v;
}
// value of the previous lane (0 in lane 0): wave_shr:1
__device__ __forceinline__ double wave_prev(double v) { return dpp_d<0x138, 0xF>(v); }

// Chain bases of the binade holding s: b0 = 2^E, b1 = 2^E + G (odd: lowest mantissa bit
// set), top = 2^(E+1).  Below 32 (and for NaN / huge s) the E = 5 bases: such tiles and
// threads are never "regular", the bases then only serve approximate sums.
struct Binade {
    double b0, b1, top;
};
__device__ __forceinline__ Binade binade_of(double s) {
    const uint64_t e = (s >= 32.0 && s < 0x1p1000) ? ((uint64_t)__double_as_longlong(s) >> 52) : (uint64_t)(1023 + 5);
    Binade b;
    b.b0 = __longlong_as_double((long long)(e << 52));
    b.b1 = __longlong_as_double((long long)((e << 52) | 1ull));
    b.top = __longlong_as_double((long long)((e + 1) << 52));
    return b;
}
// A block-uniform double moved to scalar registers (keeps B and P out of VGPRs).
__device__ __forceinline__ double uniform_d(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// parity of s/G for s in its own binade: the lowest mantissa bit
__device__ __forceinline__ bool lowbit(double s) { return ((uint32_t)__double_as_longlong(s) & 1u) != 0u; }
// relative margin between an approximate prefix and a binade edge (covers the distance
// between the sequential fp64 sum and any approximation of it for d < 2^31)
constexpr double kEdge = 0x1p-20;

// f(r) = ((r >> 2) ^ (r >> 1)) & 3 makes the 16-lane ds_read_b128 groups (banks mod 64)
// AND the 8-lane ds_write_b128 groups (banks mod 32) conflict-free for row accesses,
// staging writes and store reads alike.
__device__ __forceinline__ int swz(int r, int c) { return r * 16 + 4 * (c ^ (((r >> 2) ^ (r >> 1)) & 3)); }
__device__ __forceinline__ int swz_elem(int i) { return swz(i >> 4, (i >> 2) & 3) + (i & 3); }

struct TileRegs {
    float4 v[kQItems / 4];   // VEC4: float4 q = tid + j*256; scalar: element tid + 256*(4j+c)
};

// x is read once and q written once per call: non-temporal loads/stores (measured ~4%
// faster on the C2 batch than default-policy accesses).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
    const f32x4 t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
}

template <bool VEC4>
__device__ __forceinline__ void load_tile(TileRegs& r, const float* __restrict__ x, int64_t d, int32_t tiles,
                                          uint32_t ticket, int tid) {
    const int64_t vec = ticket / (uint32_t)tiles;
    const int64_t t0 = (int64_t)(ticket % (uint32_t)tiles) * kQTile;
    const int64_t rem = d - t0;
    const float* xt = x + vec * d + t0;
    if (VEC4 && rem >= kQTile) {
#pragma unroll
        for (int j = 0; j < kQItems / 4; ++j) r.v[j] = ld_stream(reinterpret_cast<const float4*>(xt) + tid + j * kQBlock);
    } else if (VEC4) {
#pragma unroll
        for (int j = 0; j < kQItems / 4; ++j) {
            const int64_t e = (int64_t)(tid + j * kQBlock) * 4;
            if (e + 3 < rem) {
                r.v[j] = reinterpret_cast<const float4*>(xt)[tid + j * kQBlock];
            } else {                              // ragged end of the row: never read past d
                r.v[j].x = e < rem ? xt[e] : 0.f;
                r.v[j].y = e + 1 < rem ? xt[e + 1] : 0.f;
                r.v[j].z = e + 2 < rem ? xt[e + 2] : 0.f;
                r.v[j].w = 0.f;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < kQItems / 4; ++j) {
            float t[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int64_t e = tid + (int64_t)kQBlock * (4 * j + c);
                t[c] = e < rem ? xt[e] : 0.0f;
            }
            r.v[j] = make_float4(t[0], t[1], t[2], t[3]);
        }
    }
}

template <bool VEC4>
__device__ __forceinline__ void stage_tile(const TileRegs& r, float* s_x, int tid) {
    if (VEC4) {
#pragma unroll
        for (int j = 0; j < kQItems / 4; ++j) {
            const int q = tid + j * kQBlock;        // float4 index = row*4 + column
            *reinterpret_cast<float4*>(&s_x[swz(q >> 2, q & 3)]) = r.v[j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kQItems / 4; ++j) {
            const float t[4] = {r.v[j].x, r.v[j].y, r.v[j].z, r.v[j].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) s_x[swz_elem(tid + kQBlock * (4 * j + c))] = t[c];
        }
    }
}

// Buffer descriptors for the stream kernel (guide T8/T20): built from wave-uniform values
// only (readfirstlane on the inputs), 32-bit per-lane byte offsets, hardware range check
// (out-of-range loads return 0, out-of-range stores are dropped: ragged last tiles need no
// branches).  aux = 2: non-temporal (x and q are touched once per call).
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void* p = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kAuxNT = 2;

__device__ __forceinline__ void load_tile_buf(TileRegs& r, __amdgpu_buffer_rsrc_t rx, uint32_t t0_bytes, int tid) {
#pragma unroll
    for (int j = 0; j < kQItems / 4; ++j) {
        const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(rx, t0_bytes + (uint32_t)(tid + j * kQBlock) * 16u, 0,
                                                               kAuxNT);
        r.v[j] = make_float4(v.x, v.y, v.z, v.w);
    }
}

__device__ __forceinline__ void store_tile_buf(const float* s_data, __amdgpu_buffer_rsrc_t ro, uint32_t t0_bytes,
                                               int tid) {
#pragma unroll
    for (int j = 0; j < kQTile / 4 / kQBlock; ++j) {
        const int q = tid + j * kQBlock;
        const float4 v = *reinterpret_cast<const float4*>(&s_data[swz(q >> 2, q & 3)]);
        const f32x4v w = {v.x, v.y, v.z, v.w};
        __builtin_amdgcn_raw_buffer_store_b128(w, ro, t0_bytes + (uint32_t)q * 16u, 0, kAuxNT);
    }
}

// Per-tile compute shared by both K2 kernels.  The tile (kQTile elements, zero-padded)
// is staged in LDS as 256 rows of 16 (+4 pad) floats; thread `tid` owns row `tid`.
//   pass 1: x -> v = x/den, p = |v|, mp = fm*p, fl = floor(mp), fr = mp - fl
//           (fl overwrites x in LDS, fr stays in registers, sign(v) as 2-bit codes),
//           thread sums in fp64, then a fixed-tree block exclusive scan.
//   pass 2: from base = P_t + exclusive prefix: c_i = f32(s += fr_i), crossing test,
//           out = ((L1*sign(v)) * (fl + r)) / m  -> LDS (overwrites fl).
// Output table (AS:640).  out = ((L1 * sign(v)) * (fl + r)) / f32(m) with k = fl + r a
// small non-negative integer, so per client the workgroup tabulates
//     tab[k] = RN( RN(L1 * k) / f32(m) )          k = 0 .. kTab-1   (IEEE division)
// and every element with k < kTab reads its |out| from LDS; (-L1)*k = -RN(L1*k) and
// (-a)/m = -(a/m) under round-to-nearest, so the sign is applied afterwards with
// copysign.  k >= kTab (high rates, large coordinates) and NaN take the arithmetic path.
constexpr int kTab = 256;

__device__ __forceinline__ void build_table(float* s_tab, int tid, float L, float fm) {
    for (int k = tid; k < kTab; k += kQBlock) s_tab[k] = (L * (float)k) / fm;
}

// sign(v) is folded into fl: fl_s = v < 0 ? -fl : fl (fl >= 0, so -0.0 marks a negative
// coordinate whose floor is 0).  torch.sign(v) == 0 (v = +-0 or NaN) needs no code of
// its own: v = +-0 gives fr = 0, hence r = 0 and out = (L1*0)*0/m = +0 = tab[0]; v = NaN
// makes fl NaN and out NaN either way (AS:640).
struct TileState {
    double texcl;        // exclusive prefix of t0 over the tile's threads (exact in a regular tile)
    double total;        // sum of t0 over the tile (same value in every thread)
    double t0, t1;       // this thread's increment from a start of parity 0 / 1 in the binade
};

// mp = m*p of this thread's kQItems elements stays in registers between the passes, with
// sign(v) folded in (v < 0 -> -mp; -0.0 marks a negative coordinate whose floor is 0); fl
// and fr are re-derived from it (floor / subtract: the same f32 ops, so the same bits) --
// one register per element instead of two.
struct TileVals {
    float mps[kQItems];
};
__device__ __forceinline__ float fr_of(float mps) {
    const float mp = fabsf(mps);
    return mp - floorf(mp);                     // AS:631
}

// LDS of the tile scan and the exact resolution (besides the scratch slots, see
// resolve_exact)
struct ScanLds {
    double wave[kQBlock / kWave];        // wave sums of t0
    uint64_t tmask[kQBlock / kWave];     // tie threads (pass 1); events (irregular tiles)
    uint64_t kmask[kQBlock / kWave];     // constant parity transfer (pass 1)
    uint64_t vmask[kQBlock / kWave];     // its value, else the flip bit (pass 1)
    uint64_t cmask[kQBlock / kWave];     // clean threads (irregular tiles)
    double rsum[kQBlock / kWave];        // irregular tiles: sum of the run ending the wave
    uint32_t rhead[kQBlock / kWave];     // irregular tiles: that run starts inside the wave
    double misc[2];
    double aux[kQBlock];                 // t1 - t0 of tie threads (pass 1); run sums (irregular)
};

// pass 1.  TIES: run the parity-1 chain too and publish, before the barrier, the tie mask,
// each thread's parity transfer in B's binade and t1 - t0 of tie threads; otherwise
// t1 = t0 (approximate tile sums).
template <bool FULL, bool TIES>
__device__ __forceinline__ void tile_pass1(const float* s_x, TileVals& tv, ScanLds& sl, int tid, int len,
                                           const DivPlan& dp, float fm, const Binade& B, TileState& st) {
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    const int i0 = tid * kQItems;
    double c0 = B.b0, c1 = B.b1;
#pragma unroll
    for (int k4 = 0; k4 < kQItems / 4; ++k4) {
        const float4 xv4 = *reinterpret_cast<const float4*>(&s_x[swz(tid, k4)]);
        const float xs[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
        float vs[4];
        div4(xs, dp, vs);                       // AS:625 x / den, correctly rounded
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float v = vs[c];
            const float p = fabsf(v);           // AS:626
            const float mp = fm * p;            // AS:629
            const float fl = floorf(mp);        // AS:630
            float fr = mp - fl;                 // AS:631
            float mps = v < 0.0f ? -mp : mp;
            if (!FULL && i0 + 4 * k4 + c >= len) fr = mps = 0.0f;
            tv.mps[4 * k4 + c] = mps;
            c0 += (double)fr;                   // AS:635, from a parity-0 start
            if (TIES) c1 += (double)fr;         // ... and from a parity-1 start
        }
    }
    st.t0 = c0 - B.b0;                          // exact (Sterbenz)
    st.t1 = TIES ? c1 - B.b1 : st.t0;
    const double incl_w = wave_incl_scan(st.t0, lane);
    const double wexcl = wave_prev(incl_w);
    if (lane == kWave - 1) sl.wave[wid] = incl_w;
    if (TIES) {
        // parity transfer (regular tiles): a start of parity 0 ends on parity e0 = par(t0),
        // one of parity 1 on e1 = 1 ^ par(t1); par(t) = lowest mantissa bit of t + 2^E
        const bool tie = st.t0 != st.t1;
        const bool e0 = lowbit(st.t0 + B.b0);
        const bool e1 = !lowbit(st.t1 + B.b0);
        const uint64_t tm = __ballot(tie);
        const uint64_t km = __ballot(e0 == e1);
        const uint64_t vm = __ballot(e0);
        if (lane == 0) {
            sl.tmask[wid] = tm;
            sl.kmask[wid] = km;
            sl.vmask[wid] = vm;
        }
        if (tie) sl.aux[tid] = st.t1 - st.t0;
    }
    __syncthreads();
    double wbase = 0.0, total = 0.0;
#pragma unroll
    for (int w = 0; w < kQBlock / kWave; ++w) {
        if (w < wid) wbase += sl.wave[w];
        total += sl.wave[w];
    }
    st.texcl = wbase + wexcl;
    st.total = uniform_d(total);
}

__device__ __forceinline__ double* slot_of(float* s_scr, int t) { return reinterpret_cast<double*>(s_scr + t * kQItems); }

// Cumulative tie correction of the last tie thread before `tid` (slot[3]), 0 if none.
__device__ __forceinline__ double tie_corr(float* s_scr, const ScanLds& sl, int tid) {
    const int lane = tid & (kWave - 1);
    int w = tid / kWave;
    uint64_t mk = sl.tmask[w] & ((1ull << lane) - 1ull);
    while (mk == 0ull && w > 0) mk = sl.tmask[--w];
    if (mk == 0ull) return 0.0;
    return slot_of(s_scr, w * kWave + 63 - __builtin_clzll(mk))[3];
}

__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
constexpr int kFastTies = 32;   // ties per regular tile resolved from the parity transfers

// Parity of the running sum at the start of each thread of a regular tile whose start
// has parity pP: the threads' parity transfers composed in order.  Each is a constant (a
// tie thread whose two chains end on the same parity) or an xor with a fixed bit, so a
// thread's start parity is the last constant before it xor the flips after that.  The
// masks and the four wave-start parities live in scalar registers (built once per tile).
struct ParityCtx {
    uint64_t km[kQBlock / kWave], vm[kQBlock / kWave];
    bool pw[kQBlock / kWave];
};
__device__ __forceinline__ void parity_ctx(const ScanLds& sl, bool pP, ParityCtx& c) {
    bool p = pP;
#pragma unroll
    for (int w = 0; w < kQBlock / kWave; ++w) {
        const uint64_t km = uniform_u64(sl.kmask[w]), vm = uniform_u64(sl.vmask[w]);
        c.km[w] = km;
        c.vm[w] = vm;
        c.pw[w] = p;
        if (km) {
            const int j = 63 - __builtin_clzll(km);
            p = (((vm >> j) & 1ull) != 0ull) != ((__builtin_popcountll(~km & vm & ~((2ull << j) - 1ull)) & 1) != 0);
        } else {
            p = p != ((__builtin_popcountll(vm) & 1) != 0);
        }
    }
}
// start parity of lane b of wave W (W a compile-time index after unrolling)
template <int W>
__device__ __forceinline__ bool parity_in(const ParityCtx& c, int b) {
    const uint64_t lim = (1ull << b) - 1ull;
    const uint64_t cc = c.km[W] & lim;
    const uint64_t x = ~c.km[W] & c.vm[W] & lim;
    if (cc) {
        const int j = 63 - __builtin_clzll(cc);
        return (((c.vm[W] >> j) & 1ull) != 0ull) != ((__builtin_popcountll(x & ~((2ull << j) - 1ull)) & 1) != 0);
    }
    return c.pw[W] != ((__builtin_popcountll(x) & 1) != 0);
}

// Sum of t1 - t0 over the tie threads of wave W whose start is odd: all of them (Dt) and
// those before thread `tid` (Db).
template <int W>
__device__ __forceinline__ void tie_sums(const ScanLds& sl, const ParityCtx& c, int tid, double& Db, double& Dt) {
    uint64_t mk = uniform_u64(sl.tmask[W]);
    while (mk) {
        const int b = __builtin_ctzll(mk);
        mk &= mk - 1ull;
        if (parity_in<W>(c, b)) {
            const double dd = sl.aux[W * kWave + b];
            Dt = Dt + dd;
            if (W * kWave + b < tid) Db = Db + dd;
        }
    }
}

// Irregular tile, up to the walk: each thread takes the binade of its approximate start
// Ps + texcl (Ps: the exact start, or P' when a map kernel records the tile), writes its
// scratch slot (t0, t1 of a clean thread, else its 16 fractions), the event / clean masks
// (tmask / cmask) and its inclusive run sum (aux).
// Events: threads whose increment is not a fixed multiple of their run's G -- not clean
// (added one by one from their exact start) or a clean tie (t0 != t1).  Between events,
// clean threads form runs inside one binade (consecutive clean threads cannot straddle an
// edge: each ends 1 below it); their t0 are multiples of that G and a run sums to less than
// 2^E, so a SEGMENTED scan of t0 (a run starts after each event) is exact in any order.
struct IrrThread {
    bool event;
    double v, x;         // own run value (0 for an event), inclusive run sum
};
__device__ void irregular_prep(double Ps, const TileState& st, const TileVals& tv, float* s_scr, ScanLds& sl, int tid,
                               IrrThread& it) {
    double* slot = slot_of(s_scr, tid);
    const int wid = tid / kWave;
    const int lane = tid & (kWave - 1);
    const double sa = Ps + st.texcl;
    const Binade bt = binade_of(sa);
    const bool clean = sa >= 32.0 && sa >= bt.b0 * (1.0 + kEdge) && (sa + st.t0) + 1.0 < bt.top;
    double t0c = 0.0, t1c = 0.0;
    if (clean) {
        double c0 = bt.b0, c1 = bt.b1;
#pragma unroll
        for (int k = 0; k < kQItems; ++k) {
            const double f = (double)fr_of(tv.mps[k]);
            c0 += f;
            c1 += f;
        }
        t0c = c0 - bt.b0;
        t1c = c1 - bt.b1;
        slot[0] = t0c;
        slot[1] = t1c;
    } else {
#pragma unroll
        for (int k4 = 0; k4 < kQItems / 4; ++k4)
            reinterpret_cast<float4*>(slot)[k4] = make_float4(fr_of(tv.mps[4 * k4]), fr_of(tv.mps[4 * k4 + 1]),
                                                              fr_of(tv.mps[4 * k4 + 2]), fr_of(tv.mps[4 * k4 + 3]));
    }
    const bool event = !clean || t0c != t1c;
    const double v = event ? 0.0 : t0c;
    it.event = event;
    it.v = v;
    const uint64_t em = __ballot(event);
    const uint64_t cm = __ballot(clean);
    bool f = tid == 0 || (lane > 0 && ((em >> (lane - 1)) & 1ull) != 0ull);   // run head, in-wave view
    double x = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {                       // segmented inclusive scan, wave level
        const double xu = __shfl_up(x, o, kWave);
        const int fu = __shfl_up((int)f, o, kWave);
        if (lane >= o) {
            if (!f) x = xu + x;
            f = f || fu != 0;
        }
    }
    if (lane == kWave - 1) {
        sl.rsum[wid] = x;                                      // sum of the run that ends the wave
        sl.rhead[wid] = f ? 1u : 0u;                           // that run starts inside the wave
    }
    if (lane == 0) {
        sl.tmask[wid] = em;
        sl.cmask[wid] = cm;
    }
    __syncthreads();
    if (!f) {                                                  // the run comes from earlier waves
        for (int w = wid - 1; w >= 0; --w) {
            if ((sl.tmask[w] >> (kWave - 1)) & 1ull) break;    // wave w ends with an event
            x = sl.rsum[w] + x;
            if (sl.rhead[w]) break;
        }
    }
    sl.aux[tid] = x;                                           // inclusive run sum
    it.x = x;
    __syncthreads();
}

// Exact thread base (prefix before this thread's first element) and exact P_{t+1}, from
// the exact tile start P.  s_scr: the tile's LDS image after pass 1 (thread t's row =
// floats [16t, 16t+16) is its scratch slot).  Ends with a barrier whenever it used the
// scratch, so the caller may rewrite the image right after.
__device__ double resolve_exact(double P, const Binade& B, const TileState& st, const TileVals& tv, float* s_scr,
                                ScanLds& sl, int tid, double& pnext) {
    double* slot = slot_of(s_scr, tid);
    if (P >= 32.0 && (P + st.total) + 1.0 < B.top) {            // regular (uniform)
        int nt = 0;
#pragma unroll
        for (int w = 0; w < kQBlock / kWave; ++w) nt += __builtin_popcountll(uniform_u64(sl.tmask[w]));
        if (nt == 0) {
            pnext = P + st.total;                                // exact: multiples of G in the binade
            return P + st.texcl;
        }
        if (nt <= kFastTies) {
            // a tie thread adds t1 - t0 when its start is odd: no barrier, no walk
            ParityCtx pc;
            parity_ctx(sl, lowbit(P), pc);
            double Db = 0.0, Dt = 0.0;
            tie_sums<0>(sl, pc, tid, Db, Dt);
            tie_sums<1>(sl, pc, tid, Db, Dt);
            tie_sums<2>(sl, pc, tid, Db, Dt);
            tie_sums<3>(sl, pc, tid, Db, Dt);
            pnext = (P + st.total) + Dt;
            return (P + st.texcl) + Db;
        }
        if (st.t0 != st.t1) {
            slot[0] = st.texcl;
            slot[1] = st.t0;
            slot[2] = st.t1;
        }
        __syncthreads();
        if (tid == 0) {
            double D = 0.0;
            for (int w = 0; w < kQBlock / kWave; ++w) {
                uint64_t mk = sl.tmask[w];
                while (mk) {
                    double* q = slot_of(s_scr, w * kWave + __builtin_ctzll(mk));
                    mk &= mk - 1ull;
                    const double t0 = q[1], t1 = q[2];
                    const double Sk = (P + q[0]) + D;            // exact start of the tie thread
                    D = D + ((lowbit(Sk) ? t1 : t0) - t0);
                    q[3] = D;
                }
            }
            sl.misc[0] = D;
        }
        __syncthreads();
        const double corr = tie_corr(s_scr, sl, tid);
        const double D = sl.misc[0];
        __syncthreads();
        pnext = (P + st.total) + D;
        return (P + st.texcl) + corr;
    }
    // irregular tile: the events walked by one lane from the exact start
    IrrThread it;
    irregular_prep(P, st, tv, s_scr, sl, tid, it);
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    if (tid == 0) {
        double S = P;                                          // exact value at the current run head
        for (int w = 0; w < kQBlock / kWave; ++w) {
            uint64_t mk = sl.tmask[w];
            while (mk) {
                const int b = __builtin_ctzll(mk);
                const int k = w * kWave + b;
                mk &= mk - 1ull;
                double* q = slot_of(s_scr, k);
                S = S + sl.aux[k];                             // exact start of event k (its own v is 0)
                sl.aux[k] = S;
                if ((sl.cmask[w] >> b) & 1ull) {
                    const double t0 = q[0], t1 = q[1];
                    S = S + (lowbit(S) ? t1 : t0);
                } else {
                    for (int k4 = 0; k4 < kQItems / 4; ++k4) {
                        const float4 f4 = reinterpret_cast<const float4*>(q)[k4];
                        S = (((S + (double)f4.x) + (double)f4.y) + (double)f4.z) + (double)f4.w;
                    }
                }
                q[6] = S;                                      // value at the head of the next run
            }
        }
        const bool last_event = (sl.tmask[kQBlock / kWave - 1] >> (kWave - 1)) & 1ull;
        sl.misc[0] = last_event ? S : S + sl.aux[kQBlock - 1];
    }
    __syncthreads();
    double base;
    if (it.event) {
        base = sl.aux[tid];
    } else {
        int w = wid;                                           // the last event before this thread
        uint64_t mk = sl.tmask[w] & ((1ull << lane) - 1ull);
        while (mk == 0ull && w > 0) mk = sl.tmask[--w];
        const double start = mk ? slot_of(s_scr, w * kWave + 63 - __builtin_clzll(mk))[6] : P;
        base = start + (it.x - it.v);                                // + exclusive run sum (exact)
    }
    pnext = sl.misc[0];
    __syncthreads();
    return base;
}

// Tile map from an APPROXIMATE start Pg (the per-client fold of the small-batch forms):
// if the exact start is certainly in Pg's binade and the tile stays in it, the tile's
// exact increment for a start of parity p is m[p] (ties resolved for both parities).
// Returns false for an irregular tile (resolved later from its exact start).
__device__ bool resolve_map(double Pg, const Binade& B, const TileState& st, float* s_scr, ScanLds& sl, int tid,
                            double& m0, double& m1) {
    if (!(Pg >= 32.0 && Pg >= B.b0 * (1.0 + kEdge) && (Pg + st.total) + 1.0 < B.top)) return false;   // uniform
    int nt = 0;
#pragma unroll
    for (int w = 0; w < kQBlock / kWave; ++w) nt += __builtin_popcountll(uniform_u64(sl.tmask[w]));
    if (nt == 0) {
        m0 = m1 = st.total;
        return true;
    }
    if (nt <= kFastTies) {
        ParityCtx p0, p1;
        parity_ctx(sl, false, p0);
        parity_ctx(sl, true, p1);
        double D0 = 0.0, D1 = 0.0, unused = 0.0;
        tie_sums<0>(sl, p0, 0, unused, D0);
        tie_sums<1>(sl, p0, 0, unused, D0);
        tie_sums<2>(sl, p0, 0, unused, D0);
        tie_sums<3>(sl, p0, 0, unused, D0);
        tie_sums<0>(sl, p1, 0, unused, D1);
        tie_sums<1>(sl, p1, 0, unused, D1);
        tie_sums<2>(sl, p1, 0, unused, D1);
        tie_sums<3>(sl, p1, 0, unused, D1);
        m0 = st.total + D0;
        m1 = st.total + D1;
        return true;
    }
    double* slot = slot_of(s_scr, tid);
    if (st.t0 != st.t1) {
        slot[0] = st.texcl;
        slot[1] = st.t0;
        slot[2] = st.t1;
    }
    __syncthreads();
    if (tid < 2) {
        // start parity p = tid: the parity at a tie thread is p xor parity((texcl + D)/G),
        // read off (texcl + D) + 2^E (exact: texcl + D < 2^E is a multiple of G)
        const bool p = tid != 0;
        double D = 0.0;
        for (int w = 0; w < kQBlock / kWave; ++w) {
            uint64_t mk = sl.tmask[w];
            while (mk) {
                const double* q = slot_of(s_scr, w * kWave + __builtin_ctzll(mk));
                mk &= mk - 1ull;
                const double t0 = q[1], t1 = q[2];
                const bool par = p != lowbit((q[0] + D) + B.b0);
                D = D + ((par ? t1 : t0) - t0);
            }
        }
        sl.misc[tid] = D;
    }
    __syncthreads();
    m0 = st.total + sl.misc[0];
    m1 = st.total + sl.misc[1];
    __syncthreads();
    return true;
}

// Wire code of one coordinate (type codes, see uq_dme.h): k = fl + r ->
// code = k for sign(v) >= 0 and ~k = -k-1 for sign(v) < 0 (keeps the reference's -0.0
// outputs).  kmax (float) tracks the largest k; a client whose kmax > 127 is flagged as
// overflow (its codes are meaningless).  fl is finite whenever L1 is finite, and a
// non-finite L1 flags the client separately (publish_kmax).
__device__ __forceinline__ uint32_t code_of(float mps, float kf) {
    const int mask = (int)__float_as_uint(mps) >> 31;       // 0 or -1: sign(v) < 0
    return (uint32_t)(((int)kf ^ mask) & 0xFF);
}

// pass 2; WQ: outputs into the LDS image s_o, WC: this thread's 16 codes into cw (NIB: as
// 4-bit codes, element e of the thread in bits 4e..4e+3 of cw[0..1]).
template <bool WQ, bool WC, bool NIB = false>
__device__ __forceinline__ void tile_pass2(float* s_o, const TileVals& tv, const float* s_tab, int tid, double base,
                                           float L, float fm, float Xv, uint32_t (&cw)[4], float& kmax) {
    double s = base;                           // exact prefix before this thread's first element
    float fprev = floorf((float)s - Xv);       // floor(c_{i-1} - X) of this thread's first element
    // k = fl + r can only be NaN when L1 is not finite: such a client takes the arithmetic
    // path for every element; otherwise a running max of k bounds the table reads
    const bool arith = !(fabsf(L) <= 3.40282347e38f);
#pragma unroll
    for (int k4 = 0; k4 < kQItems / 4; ++k4) {
        float o[4], kfs[4];
        float m4 = 0.0f;
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float mps = tv.mps[4 * k4 + c];
            const float mp = fabsf(mps);
            const float fla = floorf(mp);                      // AS:630
            s += (double)(mp - fla);                           // AS:631, AS:635 fp64 running sum
            const float fcur = floorf((float)s - Xv);          // AS:636 floor(c_i - X)
            const float r = (fcur - fprev == 1.0f) ? 1.0f : 0.0f;   // AS:636-637
            fprev = fcur;
            const float kf = fla + r;                          // fl + r
            kfs[c] = kf;
            m4 = fmaxf(m4, kf);
            // AS:640 via the table, sign(v) from mps; k >= kTab is recomputed below (rare)
            if (WQ) o[c] = copysignf(s_tab[(int)kf & (kTab - 1)], mps);
            if (WC) w |= NIB ? (code_of(mps, kf) & 0xFu) << (4 * c)       // padding elements: mps = 0, r = 0
                             : code_of(mps, kf) << (8 * c);
        }
        if (WC) kmax = fmaxf(kmax, m4);
        if (WQ && __builtin_expect(!(m4 < (float)kTab) || arith, 0)) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (!(kfs[c] < (float)kTab) || arith)
                    o[c] = (copysignf(L, tv.mps[4 * k4 + c]) * kfs[c]) / fm;   // ((L1*sign)*(fl+r))/m
        }
        if (WQ) *reinterpret_cast<float4*>(&s_o[swz(tid, k4)]) = make_float4(o[0], o[1], o[2], o[3]);
        if (WC && !NIB) cw[k4] = w;
        if (WC && NIB) cw[k4 >> 1] = (k4 & 1) ? (cw[k4 >> 1] | (w << 16)) : w;
    }
}

template <bool CVEC>
__device__ __forceinline__ void store_codes(int8_t* __restrict__ ct, const uint32_t (&cw)[4], int len, int tid) {
    const int i0 = tid * kQItems;
    if (CVEC && i0 + kQItems <= len) {
        const u32x4v v = {cw[0], cw[1], cw[2], cw[3]};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(ct + i0));
    } else {
        for (int k = 0; k < kQItems && i0 + k < len; ++k) ct[i0 + k] = (int8_t)((cw[k >> 2] >> (8 * (k & 3))) & 0xFF);
    }
}

// codes of tile t0 (element offset) of one row: one 16-byte buffer store per thread
// (beyond d: dropped by the range check), or bytewise when d % 16 != 0.
template <bool CVEC, bool NIB = false>
__device__ __forceinline__ void store_codes_buf(__amdgpu_buffer_rsrc_t rc, int8_t* __restrict__ crow,
                                                const uint32_t (&cw)[4], uint32_t t0, int64_t d, int tid) {
    if (NIB) {                                   // 4-bit codes: 8 bytes per thread (d % 32 == 0)
        typedef uint32_t u32x2n __attribute__((ext_vector_type(2)));
        const u32x2n v = {cw[0], cw[1]};
        __builtin_amdgcn_raw_buffer_store_b64(v, rc, (t0 + (uint32_t)(tid * kQItems)) / 2u, 0, kAuxNT);
    } else if (CVEC) {
        const u32x4v v = {cw[0], cw[1], cw[2], cw[3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rc, t0 + (uint32_t)(tid * kQItems), 0, kAuxNT);
    } else {
        const int64_t rem = d - (int64_t)t0;
        store_codes<false>(crow + t0, cw, (int)(rem < kQTile ? rem : kQTile), tid);
    }
}

__device__ __forceinline__ void publish_kmax(float kmaxf, float L, int32_t* kmaxv, int64_t vec, int tid) {
    int kmax = (kmaxf <= 127.0f && isfinite(L)) ? (int)kmaxf : 128;     // 128 = overflow / not codable
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o, kWave));
    if ((tid & (kWave - 1)) == 0) atomicMax(&kmaxv[vec], kmax);
}
// The whole client in this workgroup (the stream form with nseg == 1): the block's max is
// the client's, stored plainly -- kmax needs no zero-fill before the launch (one memset per
// call less: ~5 us of the bench step).  s_red: kQBlock / kWave ints of LDS.
__device__ __forceinline__ void store_kmax_block(float kmaxf, float L, int32_t* kmaxv, int64_t vec, int tid,
                                                 int* s_red) {
    int kmax = (kmaxf <= 127.0f && isfinite(L)) ? (int)kmaxf : 128;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o, kWave));
    if ((tid & (kWave - 1)) == 0) s_red[tid / kWave] = kmax;
    __syncthreads();
    if (tid == 0) {
        int m = s_red[0];
#pragma unroll
        for (int w = 1; w < kQBlock / kWave; ++w) m = max(m, s_red[w]);
        kmaxv[vec] = m;
    }
}

template <bool VEC4>
__device__ __forceinline__ void store_tile(const float* s_data, float* __restrict__ ot, int len, int tid) {
    if (VEC4 && len == kQTile) {
#pragma unroll
        for (int j = 0; j < kQTile / 4 / kQBlock; ++j) {
            const int q = tid + j * kQBlock;
            st_stream(reinterpret_cast<float4*>(ot) + q, *reinterpret_cast<const float4*>(&s_data[swz(q >> 2, q & 3)]));
        }
    } else {
        for (int i = tid; i < len; i += kQBlock) ot[i] = s_data[swz_elem(i)];
    }
}

// K2-stream: one workgroup streams one whole client vector, tiles in order, the next
// tile prefetched into registers; the exact prefix P is carried in the workgroup.  No
// inter-workgroup communication at all.  Used when there are enough clients to fill
// the GPU (batched DME, the bench workload).  Requires d % 4 == 0 and 4*d < 2^31
// (buffer addressing); the host uses the per-tile form otherwise.
//
// Order of the vector-memory operations per iteration t: stores of tile t-1 (q from the
// LDS image s_o, codes from registers), THEN the loads of tile t+1.  vmcnt counts stores
// too and retires in issue order, so with the loads last the wait before staging tile
// t+1 never waits on a store acknowledgement, and stores and loads both overlap the
// whole compute of tile t.
//
// Segments: workgroup b takes client b / nseg, tiles [s*seg_tiles, (s+1)*seg_tiles) with
// s = b % nseg, starting from the exact P = pre[first tile] (the per-client fold of the
// small-batch form) -- or from P = 0 over the whole vector when nseg == 1 (pre == nullptr).
// The tile loop of one workgroup (tiles [tb, te) of client `vec` from the exact start P).
template <bool WQ, bool WC, bool CVEC, bool NIB = false>
__device__ __forceinline__ void stream_tiles(const float* __restrict__ x, float* __restrict__ out,
                                             int8_t* __restrict__ codes, int32_t* __restrict__ overflow, int64_t d,
                                             int32_t tb, int32_t te, float fm, float Xv, float L, int32_t nseg,
                                             double P, int64_t ldo, int64_t ldc, int64_t vec, float* s_x, float* s_o,
                                             float* s_tab, ScanLds& sl) {
    const int tid = threadIdx.x;
    const DivPlan dp = div_plan(L);
    const uint32_t row_bytes = (uint32_t)(d * 4);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + vec * d, row_bytes);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(WQ ? out + vec * ldo : x, row_bytes);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(WC ? (const void*)(codes + vec * ldc) : (const void*)x,
                                                row_bytes / (NIB ? 8u : 4u));
    TileRegs pre_x;
    load_tile_buf(pre_x, rx, (uint32_t)tb * (uint32_t)(kQTile * 4), tid);
    build_table(s_tab, tid, L, fm);
    uint32_t cw[4] = {0u, 0u, 0u, 0u};
    float kmax = 0.0f;
    for (int32_t tile = tb; tile < te; ++tile) {
        stage_tile<true>(pre_x, s_x, tid);
        __syncthreads();                           // s_x(t) staged; s_o(t-1) complete
        if (tile > tb) {
            const uint32_t tp = (uint32_t)(tile - 1) * (uint32_t)kQTile;
            if (WQ) store_tile_buf(s_o, ro, tp * 4u, tid);      // beyond d: dropped by the range check
            if (WC) store_codes_buf<CVEC, NIB>(rc, codes + vec * ldc, cw, tp, d, tid);
        }
        if (tile + 1 < te) load_tile_buf(pre_x, rx, (uint32_t)(tile + 1) * (uint32_t)(kQTile * 4), tid);
        const int64_t t0 = (int64_t)tile * kQTile;
        const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
        TileState st;
        TileVals tv;
        P = uniform_d(P);
        const Binade B = binade_of(P);
        // pass 1's barrier also orders the s_o reads above before pass 2's s_o writes
        if (len == kQTile)
            tile_pass1<true, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
        else
            tile_pass1<false, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
        double pnext;
        const double base = resolve_exact(P, B, st, tv, s_x, sl, tid, pnext);
        tile_pass2<WQ, WC, NIB>(s_o, tv, s_tab, tid, base, L, fm, Xv, cw, kmax);
        P = pnext;
    }
    __syncthreads();
    const uint32_t tp = (uint32_t)(te - 1) * (uint32_t)kQTile;
    if (WQ) store_tile_buf(s_o, ro, tp * 4u, tid);
    if (WC) {
        store_codes_buf<CVEC, NIB>(rc, codes + vec * ldc, cw, tp, d, tid);
        if (nseg == 1)
            store_kmax_block(kmax, L, overflow, vec, tid, reinterpret_cast<int*>(sl.wave));
        else
            publish_kmax(kmax, L, overflow, vec, tid);
    }
}

template <bool WQ, bool WC, bool CVEC, bool NIB = false>
__global__ void __launch_bounds__(kQBlock, 4)
quantize_stream_kernel(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes,
                       int32_t* __restrict__ overflow, int64_t d, int32_t tiles, float fm,
                       const float* __restrict__ Xs, float Xval, const float* __restrict__ l1, int32_t seg_tiles,
                       int32_t nseg, const uint64_t* __restrict__ pre, int64_t ldo, int64_t ldc) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];     // input image of tile t (then scratch)
    __shared__ __attribute__((aligned(16))) float s_o[kQTile];     // output image of tile t-1 / t
    __shared__ float s_tab[kTab];
    __shared__ ScanLds sl;
    const int64_t vec = blockIdx.x / (uint32_t)nseg;
    const int32_t tb = (int32_t)(blockIdx.x % (uint32_t)nseg) * seg_tiles;
    const int32_t te = min(tiles, tb + seg_tiles);
    const float Xv = Xs ? Xs[vec] : Xval;            // one vector per call: X passed by value
    const double P = pre ? __longlong_as_double((long long)pre[vec * tiles + tb]) : 0.0;
    stream_tiles<WQ, WC, CVEC, NIB>(x, out, codes, overflow, d, tb, te, fm, Xv, l1[vec], nseg, P, ldo, ldc, vec, s_x,
                                    s_o, s_tab, sl);
}

// torch CPU `f(x).sum()` of one vector shorter than GRAIN (one cascade, the same for every
// torch thread count; K1a + K1b's arithmetic with step 16) by one 256-thread workgroup, into
// every thread: f = abs for L1 (AS:624), k' for the biased quantizer's m' (AS:648-649).
// scr: >= 64 * 32 + 64 floats of LDS.
constexpr int64_t kSmallL1Max = kGrain - 1;
template <class F>
__device__ float block_torch_sum(const float* __restrict__ xv, int64_t s, float* scr, F f) {
    const int tid = threadIdx.x;
    float* leaf = scr;                               // [64 leaves][32 streams]
    float* col = scr + 64 * 32;                      // [32] stream results, then [0] the sum
    if (s < 8) {                                     // ATen scalar row_sum
        if (tid == 0) {
            float p[4] = {0.f, 0.f, 0.f, 0.f};
            if (s >= 4)
                for (int k = 0; k < 4; ++k) p[k] = 0.f + f(xv[k]);
            for (int64_t k = (s >= 4 ? 4 : 0); k < s; ++k) p[0] += f(xv[k]);
            col[0] = 0.0f + (((p[0] + p[1]) + p[2]) + p[3]);
        }
        __syncthreads();
        const float r = col[0];
        __syncthreads();
        return r;
    }
    const int64_t vs = s / 8, rows = vs / 4;         // rows of 32 floats (8 lanes x 4 ILP)
    const int nleaf = (int)(rows / 16);              // cascade step 16: rows < 1024
    for (int b = tid >> 3; b < nleaf; b += kQBlock / 8) {     // level 0: leaf b, streams 4q..4q+3
        const int q = tid & 7;
        const float* p = xv + (int64_t)b * 16 * 32 + 4 * q;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] += f(p[r * 32 + c]);
#pragma unroll
        for (int c = 0; c < 4; ++c) leaf[b * 32 + 4 * q + c] = a[c];
    }
    __syncthreads();
    if (tid < 32) {                                  // levels 1-2 (a3 never fills below 4096 rows), open rows
        float a1 = 0.f, a2 = 0.f, a0 = 0.f;
        for (int b = 0; b < nleaf; ++b) {
            a1 += leaf[b * 32 + tid];
            if (((b + 1) & 15) == 0) {
                a2 += a1;
                a1 = 0.f;
            }
        }
        for (int64_t r = (int64_t)nleaf * 16; r < rows; ++r) a0 += f(xv[r * 32 + tid]);
        col[tid] = ((a0 + a1) + a2) + 0.f;
    }
    __syncthreads();
    if (tid == 0) {                                  // ILP vectors, leftover 8-vectors, tail (ATen order)
        float p0[8];
        for (int l = 0; l < 8; ++l) p0[l] = col[l];
        for (int64_t v = rows * 4; v < vs; ++v)
            for (int l = 0; l < 8; ++l) p0[l] += f(xv[v * 8 + l]);
        for (int k = 1; k < 4; ++k)
            for (int l = 0; l < 8; ++l) p0[l] += col[k * 8 + l];
        float acc = 0.f;
        for (int64_t k = vs * 8; k < s; ++k) acc += f(xv[k]);
        for (int l = 0; l < 8; ++l) acc += p0[l];
        col[0] = 0.0f + acc;                         // the two-pass reduction's 0 + chunk
    }
    __syncthreads();
    const float r = col[0];
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_torch_l1(const float* __restrict__ xv, int64_t s, float* scr) {
    return block_torch_sum(xv, s, scr, [](float v) { return fabsf(v); });
}

// The whole AS:609-641 for vectors shorter than GRAIN in ONE launch (the reference's own
// harness sizes: d = 1024 in C1, 2048 in Normal_dist.py:40): one workgroup per client computes
// L1 in torch order (or takes l1in), then streams its tiles exactly as quantize_stream_kernel.
template <bool WQ, bool WC, bool CVEC>
__global__ void __launch_bounds__(kQBlock, 4)
quantize_small_kernel(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes,
                      int32_t* __restrict__ overflow, int64_t d, int32_t tiles, float fm,
                      const float* __restrict__ Xs, float Xval, const float* __restrict__ l1in,
                      float* __restrict__ l1out, int64_t ldo, int64_t ldc) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ __attribute__((aligned(16))) float s_o[kQTile];
    __shared__ float s_tab[kTab];
    __shared__ ScanLds sl;
    const int64_t vec = blockIdx.x;
    const float L = l1in ? l1in[vec] : block_torch_l1(x + vec * d, d, s_x);     // AS:624
    if (l1out && threadIdx.x == 0) l1out[vec] = L;
    const float Xv = Xs ? Xs[vec] : Xval;
    stream_tiles<WQ, WC, CVEC>(x, out, codes, overflow, d, 0, tiles, fm, Xv, L, 1, 0.0, ldo, ldc, vec, s_x, s_o, s_tab,
                               sl);
}

// ---- small-batch forms (fewer clients than fill the GPU one workgroup per client) ----
// (irregular-tile records, see TileRec below)
constexpr int kRecEvents = 48;          // events per record
constexpr int kRecPerClient = 32;       // records per client
constexpr int kRecClients = 256;        // clients per launch chunk with records
//   approximate tile sums A_t (agg_stream_kernel over segments, or tile_agg_kernel)
//   tile_map_kernel      per tile: P'_t = the sums before it (approximate prefix), then in
//                        the binade of P'_t the exact map (m0, m1), or an irregular tile's
//                        event record
//   exact_fold_kernel    per client, serial: P_0 = 0, P_{t+1} = P_t + m[parity(P_t)];
//                        irregular tiles recomputed from their exact P_t
//   outputs              quantize_stream_kernel over segments / tile_out_kernel from P_t
// Maps and prefixes are stored as raw fp64 bits in u64 arrays.

// Approximate tile sums over a segment, streamed with the stream kernel's prefetch.
__global__ void __launch_bounds__(kQBlock, 4)
agg_stream_kernel(const float* __restrict__ x, int64_t d, int32_t tiles, float fm, const float* __restrict__ l1,
                  int32_t seg_tiles, int32_t nseg, uint64_t* __restrict__ agg, uint32_t* __restrict__ reccnt) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ ScanLds sl;
    const int tid = threadIdx.x;
    const int64_t vec = blockIdx.x / (uint32_t)nseg;
    const int32_t tb = (int32_t)(blockIdx.x % (uint32_t)nseg) * seg_tiles;
    const int32_t te = min(tiles, tb + seg_tiles);
    if (tb == 0 && tid == 0 && vec < kRecClients) reccnt[vec] = 0u;   // tile_map_kernel's record counter
    const DivPlan dp = div_plan(l1[vec]);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + vec * d, (uint32_t)(d * 4));
    const Binade B = binade_of(0.0);
    TileRegs pre_x;
    load_tile_buf(pre_x, rx, (uint32_t)tb * (uint32_t)(kQTile * 4), tid);
    for (int32_t tile = tb; tile < te; ++tile) {
        stage_tile<true>(pre_x, s_x, tid);
        __syncthreads();
        if (tile + 1 < te) load_tile_buf(pre_x, rx, (uint32_t)(tile + 1) * (uint32_t)(kQTile * 4), tid);
        const int64_t t0 = (int64_t)tile * kQTile;
        const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
        TileState st;
        TileVals tv;
        if (len == kQTile)
            tile_pass1<true, false>(s_x, tv, sl, tid, len, dp, fm, B, st);
        else
            tile_pass1<false, false>(s_x, tv, sl, tid, len, dp, fm, B, st);
        if (tid == 0) agg[vec * tiles + tile] = (uint64_t)__double_as_longlong(st.total);
    }
}

// Approximate tile sums, one workgroup per tile (any row alignment).
template <bool VEC4>
__global__ void __launch_bounds__(kQBlock)
tile_agg_kernel(const float* __restrict__ x, int64_t d, int32_t tiles, float fm, const float* __restrict__ l1,
                uint64_t* __restrict__ agg, uint32_t* __restrict__ reccnt) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ ScanLds sl;
    const int tid = threadIdx.x;
    const int32_t tile = blockIdx.x;
    const int64_t vec = blockIdx.y;
    if (tile == 0 && tid == 0 && vec < kRecClients) reccnt[vec] = 0u;   // tile_map_kernel's record counter
    TileRegs r;
    load_tile<VEC4>(r, x, d, tiles, (uint32_t)(vec * tiles + tile), tid);
    stage_tile<VEC4>(r, s_x, tid);
    __syncthreads();
    const int64_t t0 = (int64_t)tile * kQTile;
    const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
    const DivPlan dp = div_plan(l1[vec]);
    const Binade B = binade_of(0.0);
    TileState st;
    TileVals tv;
    if (len == kQTile)
        tile_pass1<true, false>(s_x, tv, sl, tid, len, dp, fm, B, st);
    else
        tile_pass1<false, false>(s_x, tv, sl, tid, len, dp, fm, B, st);
    if (tid == 0) agg[vec * tiles + tile] = (uint64_t)__double_as_longlong(st.total);
}

// Irregular tiles of the small-batch forms are recorded by the map kernel as their event
// list (classified from P', valid for the exact start by the kEdge margin): per event the
// run sum before it, then a clean tie's (t0, t1) or an edge thread's 16 fractions, and the
// run sum after the last event.  The fold walks a record in LDS instead of loading and
// resolving the tile.  Tiles with more events, or beyond a client's record budget, or of
// clients past kRecClients, are resolved from the data as before.
struct EvEntry {
    double run;                         // run sum between the previous event and this one
    double t0, t1;                      // clean tie
    uint32_t tie;                       // 1: clean tie, 0: edge thread (fr)
    uint32_t pad;
    float fr[kQItems];
};
struct TileRec {
    uint32_t count;
    uint32_t pad;
    double last_run;                    // run sum after the last event
    EvEntry ev[kRecEvents];
};

// Exact tile maps in the binade E of P'_t, in units of G = 2^(E-52): map0[t] = m0/G | (E+1023)
// << 53 and map1[t] = m1/G (both < 2^52); an irregular tile has map0 = kIrrMap and map1 = its
// record number + 1 (0: no record).
// The approximate tile sums of each client -> their exclusive prefix P'_t, in place (one
// workgroup per client, fp64; any order would do: P' only picks each tile's binade).  Each
// tile_map workgroup used to sum its predecessors itself: O(tiles^2) loads per client, 4 MB per
// client at d = 2^22 (the map pass 420 us for 101 clients of 2^22, profiles/r6d_*).
__global__ void __launch_bounds__(kQBlock)
tile_prefix_kernel(uint64_t* __restrict__ agg, int32_t tiles) {
    __shared__ double s_w[kQBlock / kWave];
    constexpr int K = 8;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    uint64_t* a = agg + (int64_t)blockIdx.x * tiles;
    double carry = 0.0;
    for (int32_t b0 = 0; b0 < tiles; b0 += kQBlock * K) {
        const int32_t j0 = b0 + tid * K;
        double v[K], s = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k] = j0 + k < tiles ? __longlong_as_double((long long)a[j0 + k]) : 0.0;
            s += v[k];
        }
        double inc = s;                                  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const double t = __shfl_up(inc, o, kWave);
            if (lane >= o) inc += t;
        }
        if (lane == kWave - 1) s_w[wid] = inc;
        __syncthreads();
        double e = carry + inc - s, tot = 0.0;
#pragma unroll
        for (int w = 0; w < kQBlock / kWave; ++w) {
            if (w < wid) e += s_w[w];
            tot += s_w[w];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (j0 + k < tiles) a[j0 + k] = (uint64_t)__double_as_longlong(e);
            e += v[k];
        }
        carry += tot;
        __syncthreads();
    }
}

constexpr uint64_t kIrrMap = ~0ull;
template <bool VEC4>
__global__ void __launch_bounds__(kQBlock)
tile_map_kernel(const float* __restrict__ x, int64_t d, int32_t tiles, float fm, const float* __restrict__ l1,
                const uint64_t* __restrict__ agg, uint64_t* __restrict__ map0, uint64_t* __restrict__ map1,
                TileRec* __restrict__ recs, uint32_t* __restrict__ reccnt, int32_t prefixed) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ ScanLds sl;
    const int tid = threadIdx.x;
    const int32_t tile = blockIdx.x;
    const int64_t vec = blockIdx.y;
    const int64_t idx = vec * tiles + tile;
    TileRegs r;
    load_tile<VEC4>(r, x, d, tiles, (uint32_t)idx, tid);
    // P'_t = the approximate tile sums before t, in any order (it only picks the binade): from
    // tile_prefix_kernel (prefixed), or summed here (a single client: the extra launch costs
    // more than 1024 tiles' predecessors from L2, 0.155 -> 0.171 ms per call at 2^22)
    double Pg;
    if (prefixed) {
        Pg = uniform_d(__longlong_as_double((long long)agg[idx]));
    } else {
        double acc = 0.0;
        for (int32_t j = tid; j < tile; j += kQBlock) acc += __longlong_as_double((long long)agg[vec * tiles + j]);
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
        if ((tid & (kWave - 1)) == 0) sl.wave[tid / kWave] = acc;
        __syncthreads();
        Pg = uniform_d(((sl.wave[0] + sl.wave[1]) + sl.wave[2]) + sl.wave[3]);
    }
    const Binade B = binade_of(Pg);
    stage_tile<VEC4>(r, s_x, tid);
    __syncthreads();
    const int64_t t0 = (int64_t)tile * kQTile;
    const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
    const DivPlan dp = div_plan(l1[vec]);
    TileState st;
    TileVals tv;
    if (len == kQTile)
        tile_pass1<true, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
    else
        tile_pass1<false, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
    double m0 = 0.0, m1 = 0.0;
    if (resolve_map(Pg, B, st, s_x, sl, tid, m0, m1)) {
        if (tid == 0) {                                        // in units of G, with the binade
            const uint64_t eb = (uint64_t)__double_as_longlong(B.b0) >> 52;
            const int sh = 52 - ((int)eb - 1023);
            map0[idx] = (uint64_t)ldexp(m0, sh) | (eb << 53);
            map1[idx] = (uint64_t)ldexp(m1, sh);
        }
        return;
    }
    // irregular: record the events (classified from P')
    IrrThread it;
    irregular_prep(Pg, st, tv, s_x, sl, tid, it);
    int ne = 0;
#pragma unroll
    for (int w = 0; w < kQBlock / kWave; ++w) ne += __builtin_popcountll(uniform_u64(sl.tmask[w]));
    if (tid == 0) {
        uint32_t rn = 0;
        if (ne <= kRecEvents && vec < kRecClients) {
            const uint32_t slotno = atomicAdd(&reccnt[vec], 1u);
            rn = slotno < (uint32_t)kRecPerClient ? slotno + 1u : 0u;
        }
        sl.misc[0] = (double)rn;
    }
    __syncthreads();
    const uint32_t rno = (uint32_t)sl.misc[0];
    if (tid == 0) {
        map0[idx] = kIrrMap;
        map1[idx] = rno;
    }
    if (rno == 0u) return;
    TileRec* rec = recs + (vec * kRecPerClient + (rno - 1u));
    if (it.event) {
        const int lane = tid & (kWave - 1), wid = tid / kWave;
        int e = __builtin_popcountll(sl.tmask[wid] & ((1ull << lane) - 1ull));
        for (int w = 0; w < wid; ++w) e += __builtin_popcountll(sl.tmask[w]);
        EvEntry& ev = rec->ev[e];
        const double* q = slot_of(s_x, tid);
        ev.run = it.x;                                         // inclusive run sum; own v is 0
        const bool tie = (sl.cmask[wid] >> lane) & 1ull;
        ev.tie = tie ? 1u : 0u;
        if (tie) {
            ev.t0 = q[0];
            ev.t1 = q[1];
        } else {
#pragma unroll
            for (int k = 0; k < kQItems; ++k) ev.fr[k] = reinterpret_cast<const float*>(q)[k];
        }
    }
    if (tid == kQBlock - 1) {
        rec->count = (uint32_t)ne;
        rec->last_run = it.event ? 0.0 : it.x;
    }
}

constexpr int kFoldEvents = 256;   // record events prefetched into LDS (24 KB)
constexpr int kFoldMaps = 1024;    // tile maps prefetched into LDS (16 KB): d <= 2^22 in one go

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int o) {
    const uint32_t lo = __shfl_up((uint32_t)v, o, kWave), hi = __shfl_up((uint32_t)(v >> 32), o, kWave);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// One workgroup per client: the exact serial fold over its tile maps; irregular tiles are
// walked from their event records, or loaded and resolved from their exact start.
// pre[t] = exact P_t.  A run of regular maps is walked in integer units of its binade's G
// (P stays in the binade): a parity select and a 64-bit add per tile on uniform values,
// maps read 8 ahead.
template <bool VEC4>
__global__ void __launch_bounds__(kQBlock)
exact_fold_kernel(const float* __restrict__ x, int64_t d, int32_t tiles, float fm, const float* __restrict__ l1,
                  const uint64_t* __restrict__ map0, const uint64_t* __restrict__ map1, uint64_t* __restrict__ pre,
                  const TileRec* __restrict__ recs, const uint32_t* __restrict__ reccnt) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];
    __shared__ ScanLds sl;
    __shared__ EvEntry s_ev[kFoldEvents];                  // the client's records, prefetched
    __shared__ uint32_t s_roff[kRecPerClient], s_rcnt[kRecPerClient];
    __shared__ double s_rlast[kRecPerClient];
    __shared__ uint64_t s_m0[kFoldMaps], s_m1[kFoldMaps];
    const int tid = threadIdx.x;
    const int64_t vec = blockIdx.x;
    const int64_t base = vec * tiles;
    const DivPlan dp = div_plan(l1[vec]);
    // every map in LDS when they fit: a run restarted after an irregular tile then reads its
    // next 64 maps from LDS instead of waiting a global round trip (the fold at n = 1 is the
    // serial floor of the per-call drop-in)
    const bool mcache = tiles <= kFoldMaps;
    if (mcache)
        for (int i = tid; i < tiles; i += kQBlock) {
            s_m0[i] = map0[base + i];
            s_m1[i] = map1[base + i];
        }
    auto M0 = [&](int32_t t) -> uint64_t { return mcache ? s_m0[t] : map0[base + t]; };
    auto M1 = [&](int32_t t) -> uint64_t { return mcache ? s_m1[t] : map1[base + t]; };
    // prefetch every record of this client that fits (two dependent round trips in all)
    const int nrec = vec < kRecClients ? (int)min(reccnt[vec], (uint32_t)kRecPerClient) : 0;
    if (tid < nrec) {
        s_rcnt[tid] = recs[vec * kRecPerClient + tid].count;
        s_rlast[tid] = recs[vec * kRecPerClient + tid].last_run;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t off = 0;
        for (int r = 0; r < nrec; ++r) {
            const bool fits = off + s_rcnt[r] <= (uint32_t)kFoldEvents;
            s_roff[r] = fits ? off : ~0u;
            if (fits) off += s_rcnt[r];
        }
    }
    __syncthreads();
    for (int r = 0; r < nrec; ++r) {
        if (s_roff[r] == ~0u) continue;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(recs[vec * kRecPerClient + r].ev);
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_ev + s_roff[r]);
        const int nw = (int)(s_rcnt[r] * (sizeof(EvEntry) / 4));
        for (int i = tid; i < nw; i += kQBlock) dst[i] = src[i];
    }
    __syncthreads();
    constexpr uint64_t kMant = (1ull << 52) - 1ull;
    uint64_t Pb = 0;                                           // bits of the exact P (P_0 = 0)
    int32_t tile = 0;
    while (tile < tiles) {
        // a run of regular maps, 64 tiles at a time: lane l holds the map of tile blk + l
        // (the next 64 are loaded meanwhile).  A map in units of G is P -> P + d[P & 1];
        // two maps compose to the same form, (F then g).d[p] = F.d[p] + g.d[p ^ (F.d[p] & 1)],
        // so a wave scan gives every tile's exact start at once.  The run ends at the first
        // irregular map or map of another binade (P stays in its binade along a run).
        const int lane = tid & (kWave - 1);
        bool go = true;
        int32_t blk = tile;
        uint64_t am = M0(min(blk + lane, tiles - 1)), bm = M1(min(blk + lane, tiles - 1));
        while (go) {
            const int32_t nb = blk + kWave;
            const uint64_t an = M0(min(nb + lane, tiles - 1)), bn = M1(min(nb + lane, tiles - 1));
            const uint64_t E0 = Pb >> 52;
            const bool valid = blk + lane < tiles && am != kIrrMap && (am >> 53) == E0;
            const uint64_t inv = __ballot(!valid);
            const int f = inv ? (int)__builtin_ctzll(inv) : kWave;        // tiles in the run here
            uint64_t d0 = lane < f ? (am & ((1ull << 53) - 1ull)) : 0ull, d1 = lane < f ? bm : 0ull;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {               // inclusive scan of the maps
                const uint64_t f0 = shfl_up64(d0, o), f1 = shfl_up64(d1, o);
                if (lane >= o) {
                    const uint64_t n0 = f0 + ((f0 & 1ull) ? d1 : d0);
                    const uint64_t n1 = f1 + ((f1 & 1ull) ? d0 : d1);
                    d0 = n0;
                    d1 = n1;
                }
            }
            const uint64_t Pi0 = (Pb & kMant) | (1ull << 52);   // P / G
            const bool odd = (Pi0 & 1ull) != 0ull;
            uint64_t e0 = shfl_up64(d0, 1), e1 = shfl_up64(d1, 1);
            if (lane == 0) e0 = e1 = 0ull;
            const uint64_t st = Pi0 + (odd ? e1 : e0);            // exact start of tile blk + lane
            if (tid < f) pre[base + blk + tid] = (st & kMant) | (E0 << 52);   // wave 0, coalesced
            if (f > 0) {
                const uint64_t inc = odd ? readlane64(d1, f - 1) : readlane64(d0, f - 1);
                Pb = ((Pi0 + inc) & kMant) | (E0 << 52);
            }
            tile += f;
            go = f == kWave;
            blk = nb;
            am = an;
            bm = bn;
        }
        if (tile >= tiles) break;
        // an irregular tile (or a map whose binade P is not in: resolved from the data)
        double P = __longlong_as_double((long long)Pb);
        const int64_t idx = base + tile;
        if (tid == 0) pre[idx] = Pb;
        const uint32_t rid = M0(tile) == kIrrMap ? (uint32_t)M1(tile) : 0u;
        if (rid != 0u && s_roff[rid - 1u] != ~0u) {            // recorded and prefetched: walk it
            if (tid == 0) {
                const EvEntry* ev0 = s_ev + s_roff[rid - 1u];
                double S = P;
                for (uint32_t e = 0; e < s_rcnt[rid - 1u]; ++e) {
                    const EvEntry& ev = ev0[e];
                    S = S + ev.run;                            // exact start of the event
                    if (ev.tie) {
                        S = S + (lowbit(S) ? ev.t1 : ev.t0);
                    } else {
                        for (int k = 0; k < kQItems; ++k) S = S + (double)ev.fr[k];
                    }
                }
                sl.misc[0] = S + s_rlast[rid - 1u];
            }
            __syncthreads();
            P = sl.misc[0];
            __syncthreads();
        } else if (rid != 0u) {                                // recorded: copy it, walk it
            const TileRec* rec = recs + (vec * kRecPerClient + (rid - 1u));
            uint32_t* dst = reinterpret_cast<uint32_t*>(s_x);
            const uint32_t* src = reinterpret_cast<const uint32_t*>(rec);
            for (int i = tid; i < (int)(sizeof(TileRec) / 4); i += kQBlock) dst[i] = src[i];
            __syncthreads();
            if (tid == 0) {
                const TileRec* lr = reinterpret_cast<const TileRec*>(s_x);
                double S = P;
                for (uint32_t e = 0; e < lr->count; ++e) {
                    const EvEntry& ev = lr->ev[e];
                    S = S + ev.run;
                    if (ev.tie) {
                        S = S + (lowbit(S) ? ev.t1 : ev.t0);
                    } else {
                        for (int k = 0; k < kQItems; ++k) S = S + (double)ev.fr[k];
                    }
                }
                sl.misc[0] = S + lr->last_run;
            }
            __syncthreads();
            P = sl.misc[0];
            __syncthreads();
        } else {                                               // from the data
            TileRegs r;
            load_tile<VEC4>(r, x, d, tiles, (uint32_t)idx, tid);
            stage_tile<VEC4>(r, s_x, tid);
            __syncthreads();
            const int64_t t0 = (int64_t)tile * kQTile;
            const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
            const Binade B = binade_of(P);
            TileState st;
            TileVals tv;
            if (len == kQTile)
                tile_pass1<true, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
            else
                tile_pass1<false, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
            double pnext;
            (void)resolve_exact(P, B, st, tv, s_x, sl, tid, pnext);
            __syncthreads();                                   // s_x / sl reused by the next irregular tile
            P = pnext;
        }
        Pb = (uint64_t)__double_as_longlong(P);
        ++tile;
    }
}

// Outputs, one workgroup per tile, from the exact tile prefix pre[t] (any row alignment).
template <bool VEC4, bool WQ, bool WC, bool CVEC>
__global__ void __launch_bounds__(kQBlock)
tile_out_kernel(const float* __restrict__ x, float* __restrict__ out, int8_t* __restrict__ codes,
                int32_t* __restrict__ overflow, int64_t d, int32_t tiles, float fm, const float* __restrict__ Xs,
                float Xval, const float* __restrict__ l1, const uint64_t* __restrict__ pre, int64_t ldo, int64_t ldc) {
    __shared__ __attribute__((aligned(16))) float s_x[kQTile];     // input image, scratch, then output image
    __shared__ float s_tab[kTab];
    __shared__ ScanLds sl;
    const int tid = threadIdx.x;
    const int32_t tile = blockIdx.x;
    const int64_t vec = blockIdx.y;
    TileRegs r;
    load_tile<VEC4>(r, x, d, tiles, (uint32_t)(vec * tiles + tile), tid);
    const float L = l1[vec];
    build_table(s_tab, tid, L, fm);                 // read after pass 1's barrier
    stage_tile<VEC4>(r, s_x, tid);
    __syncthreads();
    const int64_t t0 = (int64_t)tile * kQTile;
    const int len = (int)((d - t0) < kQTile ? (d - t0) : kQTile);
    const DivPlan dp = div_plan(L);
    const double P = __longlong_as_double((long long)pre[vec * tiles + tile]);
    const Binade B = binade_of(P);
    TileState st;
    TileVals tv;
    if (len == kQTile)
        tile_pass1<true, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
    else
        tile_pass1<false, true>(s_x, tv, sl, tid, len, dp, fm, B, st);
    double pnext;
    const double base = resolve_exact(P, B, st, tv, s_x, sl, tid, pnext);   // barrier-terminated if it used s_x
    uint32_t cw[4];
    float kmax = 0.0f;
    tile_pass2<WQ, WC>(s_x, tv, s_tab, tid, base, L, fm, Xs ? Xs[vec] : Xval, cw, kmax);   // each thread rewrites its own row
    if (WC) {
        store_codes<CVEC>(codes + vec * ldc + t0, cw, len, tid);
        publish_kmax(kmax, L, overflow, vec, tid);
    }
    __syncthreads();
    if (WQ) store_tile<VEC4>(s_x, out + vec * ldo + t0, len, tid);
}

// =====================================================================================
// K3: est[i] (+)= q[j][i] / n_div, j = 0..n-1 in order (ND:137-138).
// Each thread owns 4 consecutive columns; loads for 8 clients are issued ahead.  1024-thread
// workgroups (16 KB of a client row each): 0.85-0.88 -> 0.75-0.78 ms at 1024 x 2^20 against
// 256 (tools/exp/exp_mean.hip, profiles/r03s_exp_mean_variants.jsonl); non-temporal loads (q
// is read once): 0.740-0.754 -> 0.673-0.684 ms (profiles/r05k_exp_mean_q_variants.jsonl).
// =====================================================================================
constexpr int kMeanThreads = 1024;
template <bool VEC4>
__global__ void __launch_bounds__(kMeanThreads)
client_mean_kernel(const float* __restrict__ q, int64_t n, int64_t d, int64_t ld, float n_div, int accumulate,
                   float* __restrict__ est) {
    const int64_t col = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (col >= d) return;
    if (VEC4) {
        float4 e = accumulate ? *reinterpret_cast<const float4*>(est + col) : make_float4(0.f, 0.f, 0.f, 0.f);
        int64_t j = 0;
        for (; j + 8 <= n; j += 8) {
            float4 t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = ld_stream(reinterpret_cast<const float4*>(q + (j + u) * ld + col));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                e.x += t[u].x / n_div; e.y += t[u].y / n_div;
                e.z += t[u].z / n_div; e.w += t[u].w / n_div;
            }
        }
        for (; j < n; ++j) {
            const float4 t = *reinterpret_cast<const float4*>(q + j * ld + col);
            e.x += t.x / n_div; e.y += t.y / n_div; e.z += t.z / n_div; e.w += t.w / n_div;
        }
        *reinterpret_cast<float4*>(est + col) = e;
    } else {
        const int cnt = (int)((d - col) < 4 ? (d - col) : 4);
        for (int k = 0; k < cnt; ++k) {
            float e = accumulate ? est[col + k] : 0.f;
            for (int64_t j = 0; j < n; ++j) e += q[j * ld + col + k] / n_div;
            est[col + k] = e;
        }
    }
}

// =====================================================================================
// Type codes (the wire format, see uq_dme.h): decode and decode+mean.
// For one client, |q| = tab[k] = RN(RN(L1*k)/f32(m)) and q carries the code's sign, so
// decoding rebuilds q bit-for-bit (including -0.0).  For the mean, (-a)/n = -(a/n), so
// a per-client table tabn[k] = RN(tab[k]/n_div) gives q/n_div exactly.
// =====================================================================================
constexpr int kDecChunk = 4096;   // elements per decode workgroup (256 threads x 16)
constexpr int kMeanClients = 32;  // clients whose tables are staged in LDS at a time

__device__ __forceinline__ float decode_one(int8_t c, const float* tab) {
    const int ci = (int)c;
    const int k = ci ^ (ci >> 31);                 // ci < 0 ? -ci-1 : ci
    return __uint_as_float(__float_as_uint(tab[k]) ^ ((uint32_t)ci & 0x80000000u));
}

template <bool VEC>
__global__ void __launch_bounds__(256)
codes_decode_kernel(const int8_t* __restrict__ codes, const float* __restrict__ l1, int64_t d, float fm,
                    float* __restrict__ out) {
    __shared__ float tab[128];
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const float L = l1[vec];
    if (tid < 128) tab[tid] = (L * (float)tid) / fm;
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kDecChunk + (int64_t)tid * 16;
    const int8_t* cr = codes + vec * d;
    float* orow = out + vec * d;
    if (VEC && i0 + 16 <= d) {
        const uint4 w = *reinterpret_cast<const uint4*>(cr + i0);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            float o[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) o[c] = decode_one((int8_t)((ws[k4] >> (8 * c)) & 0xFF), tab);
            *reinterpret_cast<float4*>(orow + i0 + 4 * k4) = make_float4(o[0], o[1], o[2], o[3]);
        }
    } else {
        for (int64_t i = i0; i < i0 + 16 && i < d; ++i) orow[i] = decode_one(cr[i], tab);
    }
}

// est[i] (+)= q_j[i] / n_div for clients j in order, q decoded from codes.  Each thread
// owns kMeanCpt consecutive columns (one 8-byte code load per client).  Client tables
// tabn[j][k] = RN(RN(RN(L1_j*k)/m)/n_div) for k <= kmax_j are staged kMeanClients at a
// time (kmax_j from the encoder keeps them tiny: ~8 entries at R = 1); each wave builds
// whole clients' tables from wave-uniform SCALAR loads of L1_j and kmax_j, so the table
// build never waits on the vector-memory counter.  Code loads go in batches of
// kMeanUnroll clients, double-buffered: batch b+1 (crossing group boundaries) is in
// flight while batch b is summed.
constexpr int kMeanCpt = 8;
constexpr int kCodesMeanThreads = 512;          // per workgroup: the tables serve 4 K columns
constexpr int kMeanUnroll = 16;
static_assert(kMeanClients == 2 * kMeanUnroll, "two code batches per table group");
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void mean_load_batch(uint2 (&w)[kMeanUnroll], const int8_t* cp, int64_t ldc) {
#pragma unroll
    for (int u = 0; u < kMeanUnroll; ++u) {
        const u32x2v t = __builtin_nontemporal_load(reinterpret_cast<const u32x2v*>(cp + (int64_t)u * ldc));
        w[u] = make_uint2(t.x, t.y);
    }
}

__device__ __forceinline__ void mean_add_batch(float (&e)[kMeanCpt], const uint2 (&w)[kMeanUnroll],
                                               const float (*tabn)[256], int jj) {
#pragma unroll
    for (int u = 0; u < kMeanUnroll; ++u) {
        const float* tb = tabn[jj + u];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] += tb[(w[u].x >> (8 * k)) & 0xFF];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[4 + k] += tb[(w[u].y >> (8 * k)) & 0xFF];
    }
}

// Tables of clients j0 .. j0+nb-1 into tabn (callers bracket it with barriers).
__device__ __forceinline__ void mean_build_tables(float (*tabn)[256], const float* __restrict__ l1,
                                                  const int32_t* __restrict__ kmaxv, int64_t j0, int nb, int wid,
                                                  int lane, float fm, float n_div) {
    for (int jj = wid; jj < nb; jj += kCodesMeanThreads / kWave) {
        const float L = l1[j0 + jj];                // wave-uniform: scalar loads
        const int km = min(127, max(0, kmaxv[j0 + jj]));
        for (int k = lane; k <= km; k += kWave) {
            const float v = ((L * (float)k) / fm) / n_div;
            tabn[jj][k] = v;                        // code k
            tabn[jj][255 - k] = -v;                 // code ~k = -k-1 -> byte 255-k; (-a)/n = -(a/n)
        }
    }
}

// ragged / unaligned columns: bytewise, clients j0 .. j0+nb-1 in order
__device__ __forceinline__ void mean_add_bytes(float (&e)[kMeanCpt], const int8_t* __restrict__ codes, int64_t ldc,
                                               const float (*tabn)[256], int64_t j0, int nb, int64_t i0, int64_t d) {
    for (int jj = 0; jj < nb; ++jj)
        for (int k = 0; k < kMeanCpt; ++k)
            if (i0 + k < d) e[k] += tabn[jj][(uint8_t)codes[(j0 + jj) * ldc + i0 + k]];
}

// Overflowed clients (kmax > 127: a count saturated its int8 code) among j0 .. j0+nb-1.
__device__ __forceinline__ uint32_t mean_ovf_mask(const int32_t* __restrict__ kmaxv, int64_t j0, int nb) {
    uint32_t mk = 0;
    for (int jj = 0; jj < nb; ++jj) mk |= (kmaxv[j0 + jj] > 127 ? 1u : 0u) << jj;
    return mk;
}

// Clients j0 .. j0+nb-1 in order when some client overflowed: an overflowed client adds
// q[j][i] / n_div read from the dequantized batch (what K2 wrote correctly beside the
// saturated codes; the same bits as its table entry would have had), the others their
// table entries.  Any column alignment.
__device__ __forceinline__ void mean_add_mixed(float (&e)[kMeanCpt], const int8_t* __restrict__ codes, int64_t ldc,
                                            const float* __restrict__ q, int64_t ldq, const float (*tabn)[256],
                                            uint32_t ovf, int64_t j0, int nb, int64_t i0, int64_t d, float n_div) {
    for (int jj = 0; jj < nb; ++jj) {
        const int64_t j = j0 + jj;
        if ((ovf >> jj) & 1u) {
            for (int k = 0; k < kMeanCpt; ++k)
                if (i0 + k < d) e[k] += q[j * ldq + i0 + k] / n_div;
        } else {
            for (int k = 0; k < kMeanCpt; ++k)
                if (i0 + k < d) e[k] += tabn[jj][(uint8_t)codes[j * ldc + i0 + k]];
        }
    }
}

// ALL: every thread's kMeanCpt columns lie inside d (d a multiple of kCodesMeanThreads *
// kMeanCpt), so no
// per-thread `full` test anywhere (a per-thread guard around the adds cost the loads'
// overlap in other kernels here).
template <bool VEC, bool ALL = false>
__global__ void __launch_bounds__(kCodesMeanThreads)
codes_mean_kernel(const int8_t* __restrict__ codes, int64_t ldc, const float* __restrict__ l1,
                  const int32_t* __restrict__ kmaxv, int64_t n, int64_t d, float fm, float n_div, int accumulate,
                  float* __restrict__ est, const float* __restrict__ q, int64_t ldq) {
    __shared__ float tabn[kMeanClients][256];     // indexed by the raw code byte, sign included
    __shared__ uint32_t s_ovf;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wid = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int64_t i0 = ((int64_t)blockIdx.x * kCodesMeanThreads + tid) * kMeanCpt;
    const bool full = ALL || (VEC && i0 + kMeanCpt <= d);
    float e[kMeanCpt];
#pragma unroll
    for (int k = 0; k < kMeanCpt; ++k) e[k] = (accumulate && i0 + k < d) ? est[i0 + k] : 0.0f;
    // With q: does any client overflow its codes?  (n kmax words per workgroup, L2-served.)
    // Then the whole launch takes the mixed loop below, which reads those clients from q;
    // the common case keeps the straight-line loop untouched (no per-group test in it).
    bool any = false;
    if (q) {
        if (tid == 0) s_ovf = 0u;
        __syncthreads();
        bool a = false;
        for (int64_t j = tid; j < n; j += kCodesMeanThreads) a = a || kmaxv[j] > 127;
        if (a) s_ovf = 1u;
        __syncthreads();
        any = s_ovf != 0u;
    }
    const int64_t groups = n / kMeanClients;
    if (any) {
        for (int64_t j0 = 0; j0 < n; j0 += kMeanClients) {
            const int nb = (int)min((int64_t)kMeanClients, n - j0);
            const uint32_t ovf = mean_ovf_mask(kmaxv, j0, nb);
            __syncthreads();
            mean_build_tables(tabn, l1, kmaxv, j0, nb, wid, lane, fm, n_div);
            __syncthreads();
            mean_add_mixed(e, codes, ldc, q, ldq, tabn, ovf, j0, nb, i0, d, n_div);
        }
    } else {
    // full groups of kMeanClients: straight-line, unconditional loads (the prefetch of the
    // group after the last one is clamped to a valid row and never used), so the waits
    // before each batch cover that batch only
    const int8_t* cbase = codes + (full ? i0 : 0);
    uint2 wa[kMeanUnroll], wb[kMeanUnroll];
    if (VEC && groups > 0) mean_load_batch(wa, cbase, ldc);
    for (int64_t g = 0; g < groups; ++g) {
        const int64_t j0 = g * kMeanClients;
        __syncthreads();                            // previous group's tables no longer read
        mean_build_tables(tabn, l1, kmaxv, j0, kMeanClients, wid, lane, fm, n_div);
        __syncthreads();
        if (VEC) {
            mean_load_batch(wb, cbase + (j0 + kMeanUnroll) * ldc, ldc);
            if (full) mean_add_batch(e, wa, tabn, 0);
            const int64_t jn = (j0 + kMeanClients + kMeanUnroll <= n) ? j0 + kMeanClients : n - kMeanUnroll;
            mean_load_batch(wa, cbase + jn * ldc, ldc);
            if (full) mean_add_batch(e, wb, tabn, kMeanUnroll);
        }
        if (!full) mean_add_bytes(e, codes, ldc, tabn, j0, kMeanClients, i0, d);
    }
    const int64_t jr = groups * kMeanClients;
    const int nr = (int)(n - jr);
    if (nr > 0) {                                   // the last n % kMeanClients clients
        __syncthreads();
        mean_build_tables(tabn, l1, kmaxv, jr, nr, wid, lane, fm, n_div);
        __syncthreads();
        if (full) {
            for (int jj = 0; jj < nr; ++jj) {
                const uint2 w = *reinterpret_cast<const uint2*>(codes + (jr + jj) * ldc + i0);
#pragma unroll
                for (int k = 0; k < 4; ++k) e[k] += tabn[jj][(w.x >> (8 * k)) & 0xFF];
#pragma unroll
                for (int k = 0; k < 4; ++k) e[4 + k] += tabn[jj][(w.y >> (8 * k)) & 0xFF];
            }
        } else {
            mean_add_bytes(e, codes, ldc, tabn, jr, nr, i0, d);
        }
    }
    }
    if (full) {
        *reinterpret_cast<float4*>(est + i0) = make_float4(e[0], e[1], e[2], e[3]);
        *reinterpret_cast<float4*>(est + i0 + 4) = make_float4(e[4], e[5], e[6], e[7]);
    } else {
        for (int k = 0; k < kMeanCpt; ++k)
            if (i0 + k < d) est[i0 + k] = e[k];
    }
}

// ---- 4-bit type codes (the bench pipeline "codes4") ------------------------------------
// uq_type_unbiased_nibbles_ld_f32 writes the type codes of K2 as 4-bit fields (element 2i in
// the low nibble of byte i): the byte code's low nibble, i.e. k for sign >= 0 and 15 - k for
// ~k, exact while k <= kNibMax.  At R <= 2 the counts stay below that for all but extreme
// tails (k <= 2 at R = 1 for |x| < 11 sigma), and a client with kmax > kNibMax is read from q.
// Half the code bytes of K2's write and K3's read: K2 1.69 -> 1.66 ms, K3 0.187 -> 0.148 ms on
// the C2 batch (timing probe tools/exp/variants.py, profiles/r5ai_nibble_codes_probe.jsonl).
constexpr int kNibMax = 7;
constexpr int64_t kNibAlign = kCodesMeanThreads * kMeanCpt;   // d % 4096 == 0: whole mean threads

__device__ __forceinline__ void nib_load_batch(uint32_t (&w)[kMeanUnroll], const uint8_t* cp, int64_t ldn) {
#pragma unroll
    for (int u = 0; u < kMeanUnroll; ++u) w[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(cp + (int64_t)u * ldn));
}

__device__ __forceinline__ void nib_add_batch(float (&e)[kMeanCpt], const uint32_t (&w)[kMeanUnroll],
                                              const float (*tab)[16], int jj) {
#pragma unroll
    for (int u = 0; u < kMeanUnroll; ++u) {
        const float* tb = tab[jj + u];
#pragma unroll
        for (int k = 0; k < kMeanCpt; ++k) e[k] += tb[(w[u] >> (4 * k)) & 0xFu];
    }
}

// tab[jj][c]: nibble c of client j0 + jj = RN(RN(RN(L1*k)/m)/n_div) with k = c (c <= 7) and
// its negation at c = 15 - k (the byte table's values, so est keeps K3c's bits).  All nb
// clients of a chunk at once, entries spread over the workgroup: one round of l1 / kmax loads
// per chunk (per 32-client group, those loads' latency and two barriers were most of K3n).
constexpr int kNibChunk = 1024;                 // clients whose tables sit in LDS at a time (64 KB)
__device__ __forceinline__ void nib_build_tables(float (*tab)[16], const float* __restrict__ l1,
                                                 const int32_t* __restrict__ kmaxv, int64_t j0, int nb, float fm,
                                                 float n_div) {
    for (int e = threadIdx.x; e < nb * 8; e += kCodesMeanThreads) {
        const int jj = e >> 3, k = e & 7;
        const float L = l1[j0 + jj];
        const int km = min(kNibMax, max(0, kmaxv[j0 + jj]));
        if (k <= km) {
            const float v = ((L * (float)k) / fm) / n_div;
            tab[jj][k] = v;
            tab[jj][15 - k] = -v;
        }
    }
}

// K3n: est[i] (+)= q_j[i] / n_div, clients in order, from the 4-bit codes (4 bytes per client
// per thread's 8 columns): the tables of up to kNibChunk clients built once, then the code
// loads in double-buffered batches of kMeanUnroll clients with no barrier between them.
// d % 4096 == 0 (every thread's columns inside d).  Any client with kmax > kNibMax sends the
// launch down the mixed loop: those clients add q[j][i] / n_div (q is required).
__global__ void __launch_bounds__(kCodesMeanThreads)
nibbles_mean_kernel(const uint8_t* __restrict__ nib, int64_t ldn, const float* __restrict__ l1,
                    const int32_t* __restrict__ kmaxv, int64_t n, int64_t d, float fm, float n_div, int accumulate,
                    float* __restrict__ est, const float* __restrict__ q, int64_t ldq) {
    __shared__ float tab[kNibChunk][16];
    __shared__ uint32_t s_ovf;
    const int tid = threadIdx.x;
    const int64_t i0 = ((int64_t)blockIdx.x * kCodesMeanThreads + tid) * kMeanCpt;
    float e[kMeanCpt];
    if (accumulate) {
        const float4 a = *reinterpret_cast<const float4*>(est + i0), b = *reinterpret_cast<const float4*>(est + i0 + 4);
        e[0] = a.x; e[1] = a.y; e[2] = a.z; e[3] = a.w; e[4] = b.x; e[5] = b.y; e[6] = b.z; e[7] = b.w;
    } else {
#pragma unroll
        for (int k = 0; k < kMeanCpt; ++k) e[k] = 0.0f;
    }
    if (tid == 0) s_ovf = 0u;
    __syncthreads();
    bool a = false;
    for (int64_t j = tid; j < n; j += kCodesMeanThreads) a = a || kmaxv[j] > kNibMax;
    if (a) s_ovf = 1u;
    __syncthreads();
    const bool any = s_ovf != 0u;
    const uint8_t* cbase = nib + i0 / 2;
    for (int64_t c0 = 0; c0 < n; c0 += kNibChunk) {
        const int nc = (int)min((int64_t)kNibChunk, n - c0);
        __syncthreads();                               // the previous chunk's tables no longer read
        nib_build_tables(tab, l1, kmaxv, c0, nc, fm, n_div);
        __syncthreads();
        const int full = any ? 0 : nc / kMeanClients * kMeanClients;
        if (full > 0) {
            uint32_t wa[kMeanUnroll], wb[kMeanUnroll];
            const uint8_t* cb = cbase + c0 * ldn;
            nib_load_batch(wa, cb, ldn);
            for (int g = 0; g < full; g += kMeanClients) {
                nib_load_batch(wb, cb + (int64_t)(g + kMeanUnroll) * ldn, ldn);
                nib_add_batch(e, wa, tab, g);
                // the next group's first batch (clamped to a row inside the chunk when none)
                const int gn = (g + kMeanClients + kMeanUnroll <= nc) ? g + kMeanClients : nc - kMeanUnroll;
                nib_load_batch(wa, cb + (int64_t)gn * ldn, ldn);
                nib_add_batch(e, wb, tab, g + kMeanUnroll);
            }
        }
        for (int jj = full; jj < nc; ++jj) {           // mixed / the chunk's last clients
            const int64_t j = c0 + jj;
            if (kmaxv[j] > kNibMax) {
                const float4 a4 = *reinterpret_cast<const float4*>(q + j * ldq + i0);
                const float4 b4 = *reinterpret_cast<const float4*>(q + j * ldq + i0 + 4);
                const float qq[kMeanCpt] = {a4.x, a4.y, a4.z, a4.w, b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int k = 0; k < kMeanCpt; ++k) e[k] += qq[k] / n_div;
            } else {
                const uint32_t w = *reinterpret_cast<const uint32_t*>(cbase + j * ldn);
#pragma unroll
                for (int k = 0; k < kMeanCpt; ++k) e[k] += tab[jj][(w >> (4 * k)) & 0xFu];
            }
        }
    }
    *reinterpret_cast<float4*>(est + i0) = make_float4(e[0], e[1], e[2], e[3]);
    *reinterpret_cast<float4*>(est + i0 + 4) = make_float4(e[4], e[5], e[6], e[7]);
}

#include "uq_biased_kernels.h"
#include "uq_biased_torch_ties.h"
#include "uq_eden_kernels.h"
#include "uq_quicfl_kernels.h"
#include "uq_codec_kernels.h"

// ---- host-side helpers ---------------------------------------------------------------
thread_local std::string g_err;
// test hook (uq_test_force_replay_failure): every torch-tie replay takes its failure path
std::atomic<int> g_force_replay_failure{0};

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(UQ_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return UQ_OK;
}

struct WsLayout {
    size_t agg_off, incl_off, map1_off, rec_off, cnt_off, part_off, l1_off, total;
    int32_t tiles;
};

WsLayout layout(int64_t n, int64_t d, const L1Plan& plan) {
    WsLayout w{};
    const int64_t tiles = (d + kQTile - 1) / kQTile;
    w.tiles = (int32_t)tiles;
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    w.agg_off = kCtrlBytes;
    w.incl_off = up(w.agg_off + (size_t)n * tiles * sizeof(uint64_t));
    w.map1_off = up(w.incl_off + (size_t)n * tiles * sizeof(uint64_t));
    const size_t rec_clients = (size_t)std::min<int64_t>(n, kRecClients);
    w.rec_off = up(w.map1_off + (size_t)n * tiles * sizeof(uint64_t));
    w.cnt_off = up(w.rec_off + rec_clients * kRecPerClient * sizeof(TileRec));
    w.part_off = up(w.cnt_off + rec_clients * sizeof(uint32_t));
    w.l1_off = up(w.part_off + (size_t)n * plan.total_groups * 32 * sizeof(float));
    w.total = up(w.l1_off + (size_t)n * sizeof(float));
    return w;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// KB2 (the k' sum with the fine-bin histogram): at most this many level-1 groups per
// workgroup, fewer while that would leave fewer than ~4096 workgroups (a few-client call keeps
// one group each).  1024 x 2^20: KB2 1.16 -> 0.97 ms at 4 (torch-tie batch 5.43 -> 5.21 ms,
// lowest-index 4.23 -> 3.97 ms on one box; 8: 5.21 / 3.96), profiles/r5n_biased_gpw.jsonl.
// Env UQDME_HIST_GPW overrides the cap (measurements).
static const int kHistGroupsPerWG = [] {
    const char* e = std::getenv("UQDME_HIST_GPW");
    const int v = e ? std::atoi(e) : 8;
    return v >= 1 && v <= 64 ? v : 8;
}();

template <class Op>
int launch_cascade(const float* x, int64_t n, int64_t d, const L1Plan& plan, float* part, float* sum_out,
                   const float* l1, float fm, hipStream_t st, uint32_t* hist = nullptr, uint32_t* zn = nullptr) {
    if (plan.total_groups > 0) {
        bool vec4 = aligned16(x) && (d % 4 == 0 || n == 1);
        vec4 = vec4 && (plan.nchunks == 1 || plan.cs % 4 == 0);
        int maxstep = std::max(16, 1 << plan.last.lp);
        if (plan.nchunks > 1) maxstep = std::max(maxstep, 1 << plan.full.lp);
        const int gpw = Op::kHist ? (int)std::max<int64_t>(1, std::min<int64_t>(kHistGroupsPerWG,
                                                                                (int64_t)plan.total_groups * n / 4096))
                                  : 1;
        dim3 grid((unsigned)((plan.total_groups + gpw - 1) / gpw), (unsigned)n);
        if (maxstep > 32) {              // steps 64..256 (chunk_geo stops at 256)
            if (vec4)
                hipLaunchKernelGGL((l1_partial_kernel<true, Op, true>), grid, dim3(256), 0, st, x, d, plan, part, l1, fm,
                                   hist, zn, gpw);
            else
                hipLaunchKernelGGL((l1_partial_kernel<false, Op, true>), grid, dim3(256), 0, st, x, d, plan, part, l1, fm,
                                   hist, zn, gpw);
        } else {
            dim3 block(8 * maxstep);
            if (vec4)
                hipLaunchKernelGGL((l1_partial_kernel<true, Op>), grid, block, 0, st, x, d, plan, part, l1, fm, hist, zn,
                                   gpw);
            else
                hipLaunchKernelGGL((l1_partial_kernel<false, Op>), grid, block, 0, st, x, d, plan, part, l1, fm, hist, zn,
                                   gpw);
        }
        int rc = hip_check(hipGetLastError(), "l1_partial_kernel launch");
        if (rc) return rc;
    }
    if (plan.nchunks == 1 && n <= 128 && plan.last.size >= 8 && plan.last.ng1 >= 64 && !std::getenv("UQDME_K1B_NARROW")) {
        hipLaunchKernelGGL((l1_finalize_kernel<Op, kFinWaves, true>), dim3((unsigned)n), dim3(64 * kFinWaves),
                           (size_t)plan.nbuf * sizeof(float), st, x, d, plan, part, sum_out, l1, fm, hist, zn);
        return hip_check(hipGetLastError(), "l1_finalize_kernel (wide) launch");
    }
    if (plan.nchunks == 1) {
        hipLaunchKernelGGL((l1_finalize_kernel<Op, 1>), dim3((unsigned)n), dim3(64), (size_t)plan.nbuf * sizeof(float), st,
                           x, d, plan, part, sum_out, l1, fm, hist, zn);
        return hip_check(hipGetLastError(), "l1_finalize_kernel launch");
    }
    hipLaunchKernelGGL(l1_finalize_kernel<Op>, dim3((unsigned)n), dim3(64 * kFinWaves), (size_t)plan.nbuf * sizeof(float), st,
                       x, d, plan, part, sum_out, l1, fm, hist, zn);
    return hip_check(hipGetLastError(), "l1_finalize_kernel launch");
}

int launch_l1(const float* x, int64_t n, int64_t d, const L1Plan& plan, float* part, float* l1_out,
              hipStream_t st) {
    return launch_cascade<AbsOp>(x, n, d, plan, part, l1_out, nullptr, 0.f, st);
}

// Resident stream-kernel workgroups on this device: 4 per CU (launch bounds).
int stream_slots(int* out) {
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    static thread_local int cache_dev = -1, cache_slots = 0;
    if (cache_dev != dev) {
        int cus = 0;
        rc = hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "CU count");
        if (rc) return rc;
        cache_slots = 4 * std::max(1, cus);
        cache_dev = dev;
    }
    *out = cache_slots;
    return UQ_OK;
}

int check_common(const void* x, int64_t n, int64_t d, int32_t T, void* ws, size_t ws_bytes,
                 L1Plan* plan, WsLayout* w) {
    if (n < 0 || d < 0) return fail(UQ_E_INVALID, "n and d must be >= 0");
    if (n > (int64_t)1 << 31 || d > (int64_t)1 << 40) return fail(UQ_E_INVALID, "n or d too large");
    if (T < 1) return fail(UQ_E_INVALID, "torch_threads must be >= 1");
    if (!make_plan(d, T, plan)) return fail(UQ_E_INVALID, "torch_threads > 4096 (or d too large) unsupported by the L1 plan");
    *w = layout(n, d, *plan);
    if ((int64_t)w->tiles * n > 0xFFFFFFFFll) return fail(UQ_E_INVALID, "batch too large for one call");
    if (n > 0 && d > 0) {
        if (!x) return fail(UQ_E_INVALID, "null input pointer");
        if (!ws) return fail(UQ_E_INVALID, "null workspace");
        if (ws_bytes < w->total) return fail(UQ_E_WORKSPACE, "workspace too small");
    }
    return UQ_OK;
}

// Biased-quantizer workspace: [ctrl 256][K1 parts][l1 n][m' n][state n x 32B]
// [hist n x 3 x 2048 u32][zero/NaN counts n x 2][candidate counts n][candidates n x cap u32]
// [tie counts n x tiles u32][tie bits n x ceil(d/32) u32]
// [KB7 slots: keys + indices S x 2d u32][KB7 positions S x 2d u32], S = min(n, kTieSlots)
struct BiasedLayout {
    size_t part_off, l1_off, msum_off, st_off, hist_off, zn_off, cn_off, fl_off, cand_off, tcnt_off, bits_off,
        pairs_off, pos_off, list_off, tls_off, tcnt2_off, alist_off, total;
    int32_t tiles;
    int32_t slots;
    uint32_t cap;      // candidate region per client in u32 (KB6f lists cap / 2 (index, key) pairs)
    uint32_t capf;     // listed pairs per client at most: a larger fine bucket takes the full-row passes
};

BiasedLayout biased_layout(int64_t n, int64_t d, const L1Plan& plan) {
    BiasedLayout w{};
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    w.tiles = (int32_t)((d + kSelTile - 1) / kSelTile);
    w.part_off = kCtrlBytes;
    w.l1_off = up(w.part_off + (size_t)n * plan.total_groups * 32 * sizeof(float));
    w.msum_off = up(w.l1_off + (size_t)n * sizeof(float));
    w.st_off = up(w.msum_off + (size_t)n * sizeof(float));
    w.hist_off = up(w.st_off + (size_t)n * sizeof(RezState));
    w.cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(d, 1), std::max<int64_t>(4096, d / 8));
    w.capf = w.cap / 2;
    w.zn_off = up(w.hist_off + (size_t)n * kHistSlots * kRadixBins * sizeof(uint32_t));
    w.cn_off = w.zn_off + (size_t)n * 2 * sizeof(uint32_t);           // zn and cand_n adjacent
    w.fl_off = w.cn_off + (size_t)n * sizeof(uint32_t);               // the full clients' list (zeroed count)
    w.cand_off = up(w.fl_off + (size_t)(n + 1) * sizeof(uint32_t));
    w.tcnt_off = up(w.cand_off + (size_t)n * w.cap * sizeof(uint32_t));
    w.bits_off = up(w.tcnt_off + (size_t)n * w.tiles * sizeof(uint32_t));
    w.slots = (int32_t)std::min<int64_t>(n, kTieSlots);
    w.pairs_off = up(w.bits_off + (size_t)n * ((d + 31) / 32) * sizeof(uint32_t));
    w.pos_off = up(w.pairs_off + (size_t)w.slots * 2 * ((d + 3) & ~(int64_t)3) * sizeof(uint32_t) + 16);
    w.list_off = up(w.pos_off + (size_t)w.slots * 2 * d * sizeof(uint32_t));
    w.tls_off = up(w.list_off + (size_t)(n + 1) * sizeof(uint32_t));    // KB7's client list
    w.tcnt2_off = up(w.tls_off + (size_t)w.slots * sizeof(TieLevelState));
    w.alist_off = up(w.tcnt2_off + (size_t)w.slots * kTieSegs * 2 * sizeof(uint32_t));
    w.total = up(w.alist_off + (size_t)(kTieSlots + 1) * sizeof(uint32_t));    // KB7a's active slots
    return w;
}

// ---- EDEN host helpers ------------------------------------------------------------------
bool eden_tables(int nbits, EdenTables* t) {
    // AS:302-315: centroids (-c reversed, c) as f32; boundaries = midpoints of neighbours
    std::memset(t, 0, sizeof(*t));
    double pos[2];
    int np = 0;
    if (nbits == 1) { pos[0] = 0.7978845608028654; np = 1; }
    else if (nbits == 2) { pos[0] = 0.4527800398860679; pos[1] = 1.5104176087114887; np = 2; }
    else return false;
    double c[4];
    for (int i = 0; i < np; ++i) { c[i] = -pos[np - 1 - i]; c[np + i] = pos[i]; }
    for (int i = 0; i < 2 * np; ++i) t->c[i] = (float)c[i];
    // the reference forms the midpoints from the f32 tensor elements, in double, then
    // stores them as f32 (torch.Tensor of Python floats)
    for (int i = 0; i + 1 < 2 * np; ++i) t->b[i] = (float)(((double)t->c[i] + (double)t->c[i + 1]) / 2.0);
    t->nb = 2 * np - 1;
    return true;
}

int ilog2_pow2(int64_t D) {
    int p = 0;
    while (((int64_t)1 << p) < D) ++p;
    return p;
}

// torch.norm of few clients: the segmented chains (KE2a-KE2d) instead of KE2's sequential
// ones.  KE2 keeps batches above kSegNormMaxN: it hides its chains behind the reads there,
// while KE2s reads the vectors twice.
constexpr int64_t kSegNormMaxN = 256;
// ... and the dot's (KE4s): its one-wave-per-client form runs 6-19 VALU per step, so the
// segmented form pays for its second read only with few clients.  KE4's time is one client's
// chain whatever n (2.67 ms at D = 2^22: 44 % of a 101-client EDEN call, profiles/r6z_*), KE4s
// costs ~15 us per client of 2^22 (~4 per client of 2^20): they cross near 170 clients.
constexpr int64_t kDotSegMaxN = 128;
// biased quantizer: batches of at most this many clients run the candidate digits (KB4d) over
// many workgroups per client (one workgroup per client walks up to d/8 keys twice)
constexpr int64_t kCandMultiMaxN = 16;

bool segnorm_applies(int64_t n, int64_t D) {
    return n >= 1 && n <= kSegNormMaxN && D >= kSegMinD && (D & (D - 1)) == 0;
}

struct SegNormLayout {
    size_t segsum, g, e, kind, cnt, tseg, tab, thr, acc, total;      // offsets from the region start
};
SegNormLayout segnorm_layout(int64_t n, int64_t D) {
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t nk = (size_t)n * 8 * (size_t)(D / kSegBlock);
    SegNormLayout L{};
    L.segsum = 0;
    L.g = up(nk * sizeof(double));
    L.e = up(L.g + nk * sizeof(float));
    L.kind = up(L.e + nk * sizeof(float));
    L.cnt = up(L.kind + nk * sizeof(int32_t));
    L.tseg = up(L.cnt + (size_t)n * sizeof(int32_t));
    const size_t cap = (size_t)seg_tab_cap(D);
    L.tab = up(L.tseg + (size_t)n * cap * sizeof(int32_t));
    L.thr = up(L.tab + (size_t)n * cap * kSegTab * sizeof(float));   // KE4s: thresholds [n][4]
    L.acc = up(L.thr + (size_t)n * 4 * sizeof(float));                 //       chain ends [n][64]
    L.total = up(L.acc + (size_t)n * 64 * sizeof(float));
    return L;
}

int launch_segnorm(const float* v, int64_t n, int64_t D, char* region, float* nrm, hipStream_t st) {
    const SegNormLayout L = segnorm_layout(n, D);
    double* segsum = (double*)(region + L.segsum);
    float* g = (float*)(region + L.g);
    float* e = (float*)(region + L.e);
    int32_t* kind = (int32_t*)(region + L.kind);
    int32_t* cnt = (int32_t*)(region + L.cnt);
    int32_t* tseg = (int32_t*)(region + L.tseg);
    float* tab = (float*)(region + L.tab);
    const int64_t K = D / kSegBlock;
    const dim3 grid((unsigned)(K / kSegPerWG), (unsigned)n);
    hipLaunchKernelGGL(eden_segsum_kernel, grid, dim3(256), 0, st, v, D, segsum);
    hipLaunchKernelGGL(eden_segscan_kernel, dim3(8u, (unsigned)n), dim3(256), 0, st, segsum, K, g, cnt);
    const int cap = seg_tab_cap(D);
    hipLaunchKernelGGL(eden_segchain_kernel, grid, dim3(256), 0, st, v, D, g, e, kind, cnt, tseg, cap);
    hipLaunchKernelGGL(eden_segtab_kernel, dim3((unsigned)cap, (unsigned)n), dim3(256), 0, st, v, D, g, cnt, tseg, tab, cap);
    hipLaunchKernelGGL(eden_segwalk_kernel, dim3((unsigned)n), dim3(512), 0, st, v, D, g, e, kind, tab, nrm, cap);
    return hip_check(hipGetLastError(), "eden segmented norm launch");
}

// KE4s (few clients): the bins and the dot's 64 chains in segments, in the segmented norm's
// region (the norm is done with it); the same bits as eden_dotbins_kernel
int launch_eden_dotseg(const float* v, int64_t n, int64_t D, float sqrtD, const float* nrm, const EdenTables& tab,
                       uint8_t* bins, float* scale, char* region, hipStream_t st) {
    const SegNormLayout L = segnorm_layout(n, D);
    double* segsum = (double*)(region + L.segsum);
    float* g = (float*)(region + L.g);
    float* e = (float*)(region + L.e);
    int32_t* kind = (int32_t*)(region + L.kind);
    int32_t* cnt = (int32_t*)(region + L.cnt);
    int32_t* tseg = (int32_t*)(region + L.tseg);
    float* tabv = (float*)(region + L.tab);
    float* thr4 = (float*)(region + L.thr);
    float* acc64 = (float*)(region + L.acc);
    const int64_t K = D / kEdenTile;
    const int cap = seg_tab_cap(D);
    hipLaunchKernelGGL(eden_thresh_kernel, dim3((unsigned)n), dim3(64), 0, st, nrm, tab, thr4);
    hipLaunchKernelGGL(eden_dseg_sum_kernel, dim3((unsigned)K, (unsigned)n), dim3(256), 0, st, v, D, sqrtD, nrm, thr4, tab,
                       bins, segsum);
    hipLaunchKernelGGL(eden_segscan_l_kernel<64>, dim3(64u, (unsigned)n), dim3(256), 0, st, segsum, K, g, cnt);
    hipLaunchKernelGGL(eden_dseg_chain_kernel, dim3((unsigned)(K / kDSegTiles), (unsigned)n), dim3(256), 0, st, v, D, sqrtD,
                       nrm, thr4, tab, g, e, kind, cnt, tseg, cap);
    hipLaunchKernelGGL(eden_dseg_tab_kernel, dim3((unsigned)cap, (unsigned)n), dim3(256), 0, st, v, D, sqrtD, nrm, thr4, tab,
                       g, cnt, tseg, tabv, cap);
    hipLaunchKernelGGL(eden_dseg_walk_kernel, dim3(8u, (unsigned)n), dim3(512), 0, st, v, D, sqrtD, nrm, thr4, tab, g, e,
                       kind, tabv, acc64, cap);
    hipLaunchKernelGGL(eden_dseg_final_kernel, dim3((unsigned)n), dim3(64), 0, st, acc64, nrm, scale);
    return hip_check(hipGetLastError(), "eden segmented dot launch");
}

// AS:329-335: the bins and the scale's dot in MKL sdot's order (KE4), scale = f32(nrm * nrm) / dot
int launch_eden_dotbins(const float* v, int64_t n, int64_t D, float sqrtD, const float* nrm, const EdenTables& tab,
                        uint8_t* bins, float* scale, hipStream_t st, const int32_t* redo = nullptr) {
    const dim3 grid((unsigned)((n + kDotWaves - 1) / kDotWaves)), block(64 * kDotWaves);
    if (tab.nb == 1)
        hipLaunchKernelGGL(eden_dotbins_kernel<1>, grid, block, 0, st, v, D, sqrtD, nrm, tab, bins, scale, n, redo);
    else
        hipLaunchKernelGGL(eden_dotbins_kernel<3>, grid, block, 0, st, v, D, sqrtD, nrm, tab, bins, scale, n, redo);
    return hip_check(hipGetLastError(), "eden_dotbins_kernel launch");
}

int launch_chainnorm(const float* v, int64_t n, int64_t D, float* nrm, hipStream_t st) {
    const dim3 grid((unsigned)((n + kNormClients - 1) / kNormClients));
    if (D % kNormChunk == 0)
        hipLaunchKernelGGL(eden_norm_whole_kernel, grid, dim3(kNormThreads), 0, st, v, n, D, nrm);
    else
        hipLaunchKernelGGL(eden_norm_kernel, grid, dim3(kNormThreads), 0, st, v, n, D, nrm);
    return hip_check(hipGetLastError(), "eden_norm_kernel launch");
}

struct EdenLayout {
    size_t vec_off, nrm_off, bins_off, scale_off, redo_off, seg_off, total;
    int64_t D;
    int32_t tiles;
    bool seg;                 // the segmented norm (its region at seg_off)
};

EdenLayout eden_layout(int64_t n, int64_t dim) {
    EdenLayout w{};
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    w.D = dim <= 1 ? 1 : ((int64_t)1 << ilog2_pow2(dim));
    w.tiles = (int32_t)((w.D + kEdenTile - 1) / kEdenTile);
    w.vec_off = kCtrlBytes;
    w.nrm_off = up(w.vec_off + (size_t)n * w.D * sizeof(float));
    w.bins_off = up(w.nrm_off + (size_t)n * sizeof(float));
    w.scale_off = up(w.bins_off + (size_t)n * w.D);
    w.redo_off = up(w.scale_off + (size_t)n * sizeof(float));
    w.seg_off = up(w.redo_off + (size_t)n * sizeof(int32_t));
    w.seg = segnorm_applies(n, w.D);
    w.total = w.seg_off + (w.seg ? segnorm_layout(n, w.D).total : 0);
    return w;
}

// One FWHT pass: the register-radix kernels for the 4096-element low pass and the
// 256 x 64 high pass, the generic LDS kernel otherwise (same stages, same bits).
template <int M, bool L, bool R>
void fwht_dispatch(dim3 grid, const FwhtArgs& b, int lo, int k, hipStream_t st) {
    if (lo == 0 && k == kFwhtLow16Bits && !L)
        hipLaunchKernelGGL((fwht_low16k_kernel<M>), dim3((unsigned)(b.D >> kFwhtLow16Bits), grid.y), dim3(1024), 0, st, b);
    else if (lo == 0 && k == kFwhtLowBits && (M != 2 || (b.D % 16) == 0))
        hipLaunchKernelGGL((fwht_low4096_kernel<M, L, R>), grid, dim3(256), 0, st, b);
    else if (lo > 0 && k == kFwhtHighBits && M == 0 && ((int64_t)1 << lo) % kHighCols == 0)
        hipLaunchKernelGGL((fwht_high256_kernel<L, R>), dim3(grid.x * kFwhtCols / kHighCols, grid.y), dim3(kHighT), 0, st,
                           b, lo);
    else if (lo > 0 && k <= 6 && M == 0 && (int64_t)grid.y * ((b.D >> k) / 256) >= 1024) {
        // (a thread per column: with fewer than 1024 workgroups, e.g. one client of 2^18,
        // the generic kernel's 2^k x 32 tiles spread the pass over more of the GPU)
        const dim3 g2((unsigned)(((b.D >> k) + 255) / 256), grid.y);
        switch (k) {
            case 1: hipLaunchKernelGGL((fwht_small_kernel<1, L, R>), g2, dim3(256), 0, st, b, lo); break;
            case 2: hipLaunchKernelGGL((fwht_small_kernel<2, L, R>), g2, dim3(256), 0, st, b, lo); break;
            case 3: hipLaunchKernelGGL((fwht_small_kernel<3, L, R>), g2, dim3(256), 0, st, b, lo); break;
            case 4: hipLaunchKernelGGL((fwht_small_kernel<4, L, R>), g2, dim3(256), 0, st, b, lo); break;
            case 5: hipLaunchKernelGGL((fwht_small_kernel<5, L, R>), g2, dim3(256), 0, st, b, lo); break;
            default: hipLaunchKernelGGL((fwht_small_kernel<6, L, R>), g2, dim3(256), 0, st, b, lo); break;
        }
    } else
        hipLaunchKernelGGL((fwht_pass_kernel<M, L, R>), grid, dim3(kFwhtT), 0, st, b, lo, k);
}

// Runs the FWHT passes of one transform.  MODE of the first pass: 1 sender, 2 receiver.
// Receiver: passes in place in `buf`, the last into `out`.  Sender: passes alternate
// between `buf` and `out` (out == buf: in place; the forward RHT passes its output so
// that a two-pass transform needs no copy); *result = the buffer holding the result.
// lo0 > 0 (receiver): the passes below bit lo0 are done already, into `buf`.
int launch_fwht(FwhtArgs a, int64_t n, bool receiver, float* buf, float* out, hipStream_t st,
                float** result = nullptr, int lo0 = 0) {
    const int p = ilog2_pow2(a.D);
    // D = 2^22 (config C4): a 14-bit first pass, then 8 (one pass fewer than 12 + 8 + 2)
    int lo = lo0, k = std::min(p - lo0, lo0 ? kFwhtHighBits : (p == kFwhtLow16Bits + kFwhtHighBits ? kFwhtLow16Bits
                                                                                                    : kFwhtLowBits));
    bool first = lo0 == 0;
    float* cur = buf;                              // sender: the buffer the next pass writes
    for (;;) {
        const bool last = lo + k >= p;
        const int cols = lo == 0 ? 1 : kFwhtCols;
        const int64_t tiles = a.D / (((int64_t)1 << k) * cols);
        FwhtArgs b = a;
        if (receiver) {
            b.out = last ? out : buf;
            if (!first) b.in = buf;
        } else {
            b.out = cur;
            if (!first) b.in = cur == buf ? out : buf;
            if (result) *result = cur;
            cur = cur == buf ? out : buf;
        }
        const dim3 grid((unsigned)tiles, (unsigned)n);
        if (first && !receiver) {
            if (last) fwht_dispatch<1, true, false>(grid, b, lo, k, st);
            else fwht_dispatch<1, false, false>(grid, b, lo, k, st);
        } else if (first && receiver) {
            if (last) fwht_dispatch<2, true, true>(grid, b, lo, k, st);
            else fwht_dispatch<2, false, false>(grid, b, lo, k, st);
        } else if (last && receiver) {
            fwht_dispatch<0, true, true>(grid, b, lo, k, st);
        } else if (last) {
            fwht_dispatch<0, true, false>(grid, b, lo, k, st);
        } else {
            fwht_dispatch<0, false, false>(grid, b, lo, k, st);
        }
        int rc = hip_check(hipGetLastError(), "fwht_pass_kernel launch");
        if (rc) return rc;
        if (last) break;
        first = false;
        lo += k;
        k = std::min(p - lo, kFwhtHighBits);
    }
    return UQ_OK;
}

int eden_check(int64_t n, int64_t dim, int32_t nbits, const int8_t* signs, EdenTables* tab) {
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 clients per call");
    if (dim > ((int64_t)1 << 28)) return fail(UQ_E_INVALID, "dim must be <= 2^28");
    if (!eden_tables(nbits, tab)) return fail(UQ_E_INVALID, "EDEN nbits must be 1 or 2 (the reference's tables)");
    if (n > 0 && dim > 0 && !signs) return fail(UQ_E_INVALID, "null signs");
    return UQ_OK;
}

// A second stream per device and thread (plus fork / join events) for work that can run
// beside the caller's stream inside one call; joined back before the call returns.
struct SideStream {
    hipStream_t s;
    hipEvent_t fork, join, mid;         // mid: KB7a's bandwidth-heavy first levels done
    uint32_t* count;            // pinned host word (UQ_TIES_HOST_CHECK reads the tie list's length)
    void* states;               // pinned host RezStates (the small-vector path's flags), kSmallCheckMaxN
};
constexpr int64_t kSmallCheckMaxN = 64;    // clients per host-checked small-vector biased call

int side_stream(SideStream** out) {
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    static thread_local SideStream cache[64];
    static thread_local bool made[64] = {};
    if (dev < 0 || dev >= 64) return fail(UQ_E_INVALID, "device index out of range");
    if (!made[dev]) {
        // the side stream carries short dependent chains (KB7) beside a bandwidth-bound kernel on
        // the caller's stream: give it the highest priority so its workgroups dispatch first
        int least = 0, greatest = 0;
        rc = hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priority range");
        if (rc) return rc;
        rc = hip_check(hipStreamCreateWithPriority(&cache[dev].s, hipStreamNonBlocking, greatest), "create side stream");
        if (rc) return rc;
        rc = hip_check(hipEventCreateWithFlags(&cache[dev].fork, hipEventDisableTiming), "create event");
        if (rc) return rc;
        rc = hip_check(hipEventCreateWithFlags(&cache[dev].join, hipEventDisableTiming), "create event");
        if (rc) return rc;
        rc = hip_check(hipEventCreateWithFlags(&cache[dev].mid, hipEventDisableTiming), "create event");
        if (rc) return rc;
        rc = hip_check(hipHostMalloc((void**)&cache[dev].count, sizeof(uint32_t), hipHostMallocDefault), "pinned word");
        if (rc) return rc;
        rc = hip_check(hipHostMalloc(&cache[dev].states, kSmallCheckMaxN * 32, hipHostMallocDefault), "pinned states");
        if (rc) return rc;
        made[dev] = true;
    }
    *out = &cache[dev];
    return UQ_OK;
}

// KB7 on stream `st`.  Without KB7a (d <= kTieLevelMin) one launch replays every listed
// client.  With KB7a, the replay's LDS tails run here in small workgroups (part 1) and
// *tls_out is set: the caller then runs launch_torch_ties_rest (part 2: heap-path clients
// and list entries beyond the slots) once the output kernel on its own stream is done.
// KB7's client list and cleared tie bits (before launch_torch_ties and the tie counts).
// KB7 replays through KB7a's multi-workgroup levels (else one rez_ties_kernel launch)
inline bool kb7a_path(int64_t n, int64_t d) {
    return !(d <= kTieLevelMin || (n < kTieLevelMinClients && d < kTieLevelBigD));
}

// clear_bits: without KB7a (whose level-0 kt_count clears the listed clients' rows) every row here.
int torch_ties_prepare(int64_t n, int64_t d, RezState* state, uint32_t* bits, char* wsb, const BiasedLayout& w,
                       hipStream_t st, bool clear_bits) {
    if (clear_bits) {
        const int rc = hip_check(hipMemsetAsync(bits, 0, (size_t)n * ((d + 31) / 32) * sizeof(uint32_t), st),
                                 "memset tie bits");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(rez_tie_list_kernel, dim3(1), dim3(1024), 0, st, state, n, (uint32_t*)(wsb + w.list_off));
    return hip_check(hipGetLastError(), "rez_tie_list_kernel launch");
}

// Captured KB7a level chains, per thread (streams and workspaces are per thread in practice):
// keyed by (device, every pointer the chain's kernels take, d, slots, levels).  *exec =
// nullptr when capture is unavailable (then the caller launches the chain directly).
struct LevelPtrs {
    const void *qbuf, *list, *tls, *cnt, *pos, *alist;
    bool operator==(const LevelPtrs& o) const {
        return qbuf == o.qbuf && list == o.list && tls == o.tls && cnt == o.cnt && pos == o.pos && alist == o.alist;
    }
};
template <class F>
int level_graph(const LevelPtrs& wsb, int64_t d, unsigned S, int levels, hipStream_t st, F&& launch,
                hipGraphExec_t* exec) {
    struct Entry {
        int dev;
        LevelPtrs wsb;
        int64_t d;
        unsigned S;
        int levels;                     // lv0 * 256 + lv1: the captured range of levels
        hipGraphExec_t exec;
    };
    static thread_local Entry cache[8] = {};
    static thread_local int next = 0;
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    for (const Entry& e : cache)
        if (e.exec && e.dev == dev && e.wsb == wsb && e.d == d && e.S == S && e.levels == levels) {
            *exec = e.exec;
            return UQ_OK;
        }
    *exec = nullptr;
    if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return UQ_OK;                                   // not capturable here: launch directly
    }
    const int lrc = launch(st);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(st, &g);
    if (lrc) {
        if (g) (void)hipGraphDestroy(g);
        return lrc;
    }
    if ((rc = hip_check(ec, "end KB7a capture"))) return rc;
    hipGraphExec_t ex = nullptr;
    rc = hip_check(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0), "instantiate KB7a graph");
    (void)hipGraphDestroy(g);
    if (rc) return rc;
    Entry& slot = cache[next];
    next = (next + 1) % 8;
    if (slot.exec) (void)hipGraphExecDestroy(slot.exec);
    slot = Entry{dev, wsb, d, S, levels, ex};
    *exec = ex;
    return UQ_OK;
}

// mid (may be empty): called once KB7a's first kTieHeavyLevels levels are enqueued on `st`
// (with KB7a; before anything else otherwise) -- the fork records an event there and lets KB6
// part 1 wait for it, so the bandwidth-heavy first levels (the listed clients' full rows)
// do not share HBM with KB6 and KB6 runs beside the later, latency-bound levels instead.
int launch_torch_ties(const float* x, int64_t n, int64_t d, const float* l1, float fm, RezState* state,
                      uint32_t* bits, char* wsb, const BiasedLayout& w, hipStream_t st, const TieLevelState** tls_out,
                      const std::function<int()>& mid) {
    *tls_out = nullptr;
    int rc = UQ_OK;
    uint32_t* list = (uint32_t*)(wsb + w.list_off);
    uint32_t* qbuf = (uint32_t*)(wsb + w.pairs_off);
    uint32_t* pos = (uint32_t*)(wsb + w.pos_off);
    // KB7a pays ~85 short launches whether or not any client is listed (the host does not
    // know): worth it for batches, where ~3 % of Gaussian clients are ambiguous at R = 1 and
    // several replays would share one workgroup each, and for vectors of 2^21 and more, whose
    // one-workgroup replay takes milliseconds; a few-client call at smaller d (the per-vector
    // drop-ins) replays in one kernel when it has to
    if (!kb7a_path(n, d)) {
        if (mid && (rc = mid())) return rc;
        hipLaunchKernelGGL(rez_ties_kernel<kTieThreads>, dim3((unsigned)w.slots), dim3(kTieThreads), 0, st, x, d, l1, fm,
                           state, bits, qbuf, pos, list, (uint32_t*)wsb, (const TieLevelState*)nullptr, 0,
                           (uint32_t*)(wsb + w.tcnt_off), w.tiles, g_force_replay_failure.load());
        return hip_check(hipGetLastError(), "rez_ties_kernel launch");
    }
    // KB7a: introselect's levels over (segments x slots) workgroups, level by level, down to
    // ranges that fit the LDS tail
    TieLevelState* tls = (TieLevelState*)(wsb + w.tls_off);
    uint32_t* cnt = (uint32_t*)(wsb + w.tcnt2_off);
    const unsigned S = (unsigned)w.slots;
    // a level keeps the side of the cut that holds nth, half the range on average; an idle
    // level costs four ~6 us launches, and a range still longer continues in part 1's
    // workgroup (UQDME_TIE_STOP / UQDME_TIE_MARGIN: experiments only)
    static const int64_t tie_stop = [] {
        const char* e = std::getenv("UQDME_TIE_STOP");
        const long long v = e ? std::atoll(e) : 0;
        return v >= kTieLevelMin ? (int64_t)v : kTieLevelStop;
    }();
    static const int tie_margin = [] {
        const char* e = std::getenv("UQDME_TIE_MARGIN");
        const int v = e ? std::atoi(e) : -1;
        return v >= 0 && v <= 8 ? v : kTieLevelMargin;
    }();
    int levels = tie_margin;
    for (int64_t r = d; r > tie_stop; r = (r + 1) / 2) ++levels;
    levels = std::max(levels, 1);
    uint32_t* alist = (uint32_t*)(wsb + w.alist_off);
    // the per-level launches take (active slot, segment) items, one per wave: S slots need at
    // most S * kTieSegs / 4 workgroups (a one-client call launched 2048, 1984 of them idle)
    const unsigned lgrid = (unsigned)std::min<int64_t>(kTieGrid, (int64_t)S * kTieSegs / 4);
    // level 0's pivot and counts with the queue fill from x (x, l1 and the states are
    // per-call arguments: launched directly, not captured)
    hipLaunchKernelGGL(kt_count_kernel, dim3(lgrid), dim3(256), 0, st, x, d, l1, fm, (const RezState*)state, qbuf, list,
                       tls, cnt, alist, bits, (int)S, tie_stop, 1);
    if ((rc = hip_check(hipGetLastError(), "kt_count_kernel launch"))) return rc;
    static const int heavy = [] {
        const char* e = std::getenv("UQDME_TIE_HEAVY");
        const int v = e ? std::atoi(e) : -1;
        return v >= 0 && v <= 16 ? v : kTieHeavyLevels;
    }();
    const int lsplit = std::min(heavy, levels);
    int lv0 = 0, lv1 = levels;                  // the range levels_on enqueues
    auto levels_on = [&](hipStream_t ls) {
        for (int lv = lv0; lv < lv1; ++lv) {
            if (lv > 0)
                hipLaunchKernelGGL(kt_count_kernel, dim3(lgrid), dim3(256), 0, ls, (const float*)nullptr, d,
                                   (const float*)nullptr, fm, (const RezState*)nullptr, qbuf, list, tls, cnt, alist,
                                   (uint32_t*)nullptr, (int)S, tie_stop, 0);
            hipLaunchKernelGGL(kt_list_kernel, dim3(lgrid), dim3(256), 0, ls, d, qbuf, pos, tls, cnt, alist);
            hipLaunchKernelGGL(kt_jcut_kernel, dim3(S), dim3(kJcutThreads), 0, ls, d, qbuf, pos, tls, cnt, alist);
            hipLaunchKernelGGL(kt_swap_kernel, dim3(lgrid), dim3(256), 0, ls, d, qbuf, pos, tls, alist);
        }
        return hip_check(hipGetLastError(), "KB7a level launch");
    };
    // The rest of the level chain (4 dependent launches per level, whether or not a client is
    // listed) is replayed as a captured HIP graph: its arguments are workspace pointers, d, S
    // and the stop only, so one capture serves every call on the same workspace (per-call
    // host cost was ~65 launches, more than the chain's GPU time for a few-client call).
    auto run_levels = [&](int a, int b) {
        if (a >= b) return (int)UQ_OK;
        lv0 = a;
        lv1 = b;
        hipGraphExec_t exec = nullptr;
        int grc = level_graph(LevelPtrs{qbuf, list, tls, cnt, pos, alist}, d, S, a * 256 + b, st, levels_on, &exec);
        if (grc) return grc;
        if (exec) return hip_check(hipGraphLaunch(exec, st), "KB7a level graph launch");
        return levels_on(st);
    };
    if ((rc = run_levels(0, lsplit))) return rc;
    if (mid && (rc = mid())) return rc;
    if ((rc = run_levels(lsplit, levels))) return rc;
    hipLaunchKernelGGL(kt_mark_kernel, dim3(kTieMarkSegs, S), dim3(256), 0, st, d, qbuf, list, state, tls, bits);
    if ((rc = hip_check(hipGetLastError(), "kt_mark_kernel launch"))) return rc;
    hipLaunchKernelGGL(rez_ties_kernel<kTieThreads>, dim3(S), dim3(kTieThreads), 0, st, x, d, l1, fm, state, bits,
                       qbuf, pos, list, (uint32_t*)wsb, (const TieLevelState*)tls, 1, (uint32_t*)(wsb + w.tcnt_off),
                       w.tiles, g_force_replay_failure.load());
    *tls_out = tls;
    return hip_check(hipGetLastError(), "rez_ties_kernel launch");
}

int launch_torch_ties_rest(const float* x, int64_t d, const float* l1, float fm, RezState* state, uint32_t* bits,
                           char* wsb, const BiasedLayout& w, const TieLevelState* tls, hipStream_t st) {
    hipLaunchKernelGGL(rez_ties_kernel<kTieThreads>, dim3((unsigned)w.slots), dim3(kTieThreads), 0, st, x, d, l1, fm,
                       state, bits, (uint32_t*)(wsb + w.pairs_off), (uint32_t*)(wsb + w.pos_off),
                       (const uint32_t*)(wsb + w.list_off), (uint32_t*)wsb, tls, 2, (uint32_t*)(wsb + w.tcnt_off),
                       w.tiles, g_force_replay_failure.load());
    return hip_check(hipGetLastError(), "rez_ties_kernel launch");
}

}  // namespace

extern "C" {

int uq_version(void) { return 102; }

#ifndef UQ_BUILD_ID
#define UQ_BUILD_ID "unknown"
#endif
const char* uq_build_id(void) { return UQ_BUILD_ID; }

int uq_test_force_replay_failure(int on) { return g_force_replay_failure.exchange(on ? 1 : 0); }

// test hooks of the QUIC-FL kernels (never set by the library itself): bit 0 makes every run
// of the few-message team kernels skip its waits and report UQ_QFL_TIMEOUT; bit 1 sends every
// call to the one-wave-per-message kernels (so a test can compare both forms on one message)
std::atomic<int> g_quicfl_hooks{0};
int uq_test_set_quicfl_hooks(int flags) { return g_quicfl_hooks.exchange(flags & 7); }

const char* uq_last_error(void) { return g_err.c_str(); }

int uq_rate_to_m(double bits, int64_t d, int64_t* m_out) {
    // AS:614-620
    static const double keys[20] = {0.5, 1, 1.5, 2, 2.5, 3, 3.5, 4, 4.5, 5,
                                    5.5, 6, 6.5, 7, 7.5, 8, 8.5, 9, 9.5, 10};
    static const double vals[20] = {0.08282, 0.21403, 0.39443, 0.63752, 0.96656, 1.41725, 2.04187,
                                    2.91504, 4.14217, 5.87195, 8.31416, 11.76507, 16.64332, 23.54075,
                                    33.29414, 47.0868, 66.59204, 94.17625, 133.18596, 188.35383};
    if (!m_out) return fail(UQ_E_INVALID, "null m_out");
    if (d < 0) return fail(UQ_E_INVALID, "d must be >= 0");
    for (int i = 0; i < 20; ++i)
        if (bits == keys[i]) {
            *m_out = (int64_t)(vals[i] * (double)d);   // AS:623 int(l * d), truncation
            return UQ_OK;
        }
    return fail(UQ_E_INVALID, "bits_per_dimension not in the rate table (reference raises KeyError)");
}

int uq_workspace_bytes(int64_t n, int64_t d, int32_t T, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    L1Plan plan;
    if (n < 0 || d < 0 || T < 1) return fail(UQ_E_INVALID, "bad n/d/torch_threads");
    if (!make_plan(d, T, &plan)) return fail(UQ_E_INVALID, "cannot build L1 plan");
    *bytes_out = layout(n, d, plan).total;
    return UQ_OK;
}

int uq_l1_torch_order_f32(const float* x, int64_t n, int64_t d, int32_t T, float* l1_out, void* ws,
                          size_t ws_bytes, void* stream) {
    L1Plan plan;
    WsLayout w;
    int rc = check_common(x, n, d, T, ws, ws_bytes, &plan, &w);
    if (rc) return rc;
    if (n == 0) return UQ_OK;
    if (!l1_out) return fail(UQ_E_INVALID, "null l1_out");
    hipStream_t st = (hipStream_t)stream;
    if (d == 0) return hip_check(hipMemsetAsync(l1_out, 0, n * sizeof(float), st), "memset l1");
    float* part = (float*)((char*)ws + w.part_off);
    return launch_l1(x, n, d, plan, part, l1_out, st);
}

}  // extern "C"

namespace {
// AS:609-641 for a batch.  X: per-client draws (device), or nullptr with n == 1 and the one
// draw passed by value in Xval (the per-call drop-in: no host-to-device copy of X).
// Row j of q at out + j*ldo, of the codes at codes + j*ldc (ldo, ldc >= d: row pitches let the
// caller stagger the rows' physical placement, see DMEPipeline).
// nib: codes as 4-bit fields (uq_type_unbiased_nibbles_ld_f32; the caller checked the stream
// form's conditions and ldc is then the row pitch in bytes of the packed rows).
int unbiased_codes_impl(const float* x, float* out, int64_t ldo, int8_t* codes, int64_t ldc, int32_t* overflow,
                        int64_t n, int64_t d, int64_t m, const float* X, float Xval, const float* l1, float* l1_out,
                        int32_t T, void* ws, size_t ws_bytes, void* stream, bool nib = false) {
    L1Plan plan;
    WsLayout w;
    int rc = check_common(x, n, d, T, ws, ws_bytes, &plan, &w);
    if (rc) return rc;
    if (m < 0) return fail(UQ_E_INVALID, "m must be >= 0");
    if ((out && ldo < d) || (codes && ldc < (nib ? d / 2 : d))) return fail(UQ_E_INVALID, "row pitches must be >= d");
    if (n == 0 || d == 0) return UQ_OK;
    if (!X && n != 1) return fail(UQ_E_INVALID, "null X");
    if (!out && !codes) return fail(UQ_E_INVALID, "nothing to write: out and codes are both NULL");
    if (codes && !overflow) return fail(UQ_E_INVALID, "codes need a kmax[n] array");
    hipStream_t st = (hipStream_t)stream;
    char* wsb = (char*)ws;
    float* l1buf = (float*)(wsb + w.l1_off);
    const float* l1use = l1;
    const bool vec4s = aligned16(x) && (!out || aligned16(out)) && ((d % 4 == 0 && ldo % 4 == 0) || n == 1);
    if (!nib && d <= kSmallL1Max && vec4s && n <= 0x7FFFFFFF) {
        // shorter than GRAIN: L1 (one torch cascade for any thread count) and the exact scan
        // in one workgroup per client, one launch
        const float fm = (float)m;
        const bool cv = !codes || (aligned16(codes) && d % 16 == 0 && (ldc % 16 == 0 || n == 1));
        const int sl = (out ? 4 : 0) | (codes ? 2 : 0) | (cv ? 1 : 0);
#define UQ_SMALL(Q, C, CV)                                                                                      \
    case ((Q) * 4 + (C) * 2 + (CV)):                                                                          \
        hipLaunchKernelGGL((quantize_small_kernel<Q, C, CV>), dim3((unsigned)n), dim3(kQBlock), 0, st, x, out, codes, \
                           overflow, d, w.tiles, fm, X, Xval, l1, l1_out, ldo, ldc);                            \
        break;
        switch (sl) {
            UQ_SMALL(1, 0, 1) UQ_SMALL(1, 1, 1) UQ_SMALL(1, 1, 0) UQ_SMALL(0, 1, 1) UQ_SMALL(0, 1, 0)
            default: return fail(UQ_E_INVALID, "internal: bad kernel selector");
        }
#undef UQ_SMALL
        return hip_check(hipGetLastError(), "quantize_small_kernel launch");      // (l1_out written there)
    }
    if (!l1use) {
        rc = launch_l1(x, n, d, plan, (float*)(wsb + w.part_off), l1buf, st);
        if (rc) return rc;
        l1use = l1buf;
    }
    if (l1_out && l1_out != l1use) {
        rc = hip_check(hipMemcpyAsync(l1_out, l1use, n * sizeof(float), hipMemcpyDeviceToDevice, st), "copy l1");
        if (rc) return rc;
    }
    // rows are 16-byte aligned when d % 4 == 0, or when there is only one row
    const bool vec4 = aligned16(x) && (!out || aligned16(out)) && ((d % 4 == 0 && ldo % 4 == 0) || n == 1);
    const bool stream_form = n >= kStreamMinClients && vec4 && d <= ((int64_t)1 << 29);
    if (codes && !stream_form) {          // the stream form stores each client's kmax itself
        rc = hip_check(hipMemsetAsync(overflow, 0, n * sizeof(int32_t), st), "memset kmax");
        if (rc) return rc;
    }
    const float fm = (float)m;   // torch casts the Python int to f32 for `m * p` and `/ m`
    const bool cvec = !codes || (aligned16(codes) && d % 16 == 0 && (ldc % 16 == 0 || n == 1));
    const int wq = out ? 1 : 0, wc = codes ? 1 : 0;
    const int sel = (vec4 ? 8 : 0) | (wq ? 4 : 0) | (wc ? 2 : 0) | (cvec ? 1 : 0);
    if (nib) {
        if (!stream_form || !out || !codes) return fail(UQ_E_INVALID, "internal: 4-bit codes outside the stream form");
        hipLaunchKernelGGL((quantize_stream_kernel<true, true, true, true>), dim3((unsigned)n), dim3(kQBlock), 0, st, x,
                           out, codes, overflow, d, w.tiles, fm, X, Xval, l1use, w.tiles, 1, nullptr, ldo, ldc);
        return hip_check(hipGetLastError(), "quantize_stream_kernel (4-bit codes) launch");
    }
    if (stream_form) {
        // enough clients to fill the GPU: one workgroup per client vector
#define UQ_STREAM(Q, C, CV)                                                                                 \
    case ((Q) * 4 + (C) * 2 + (CV)):                                                                      \
        hipLaunchKernelGGL((quantize_stream_kernel<Q, C, CV>), dim3((unsigned)n), dim3(kQBlock), 0, st, x, out, \
                           codes, overflow, d, w.tiles, fm, X, Xval, l1use, w.tiles, 1, nullptr, ldo, ldc); \
        break;
        switch (sel & 7) {
            UQ_STREAM(1, 0, 1) UQ_STREAM(1, 1, 1) UQ_STREAM(1, 1, 0) UQ_STREAM(0, 1, 1) UQ_STREAM(0, 1, 0)
            default: return fail(UQ_E_INVALID, "internal: bad kernel selector");
        }
#undef UQ_STREAM
        return hip_check(hipGetLastError(), "quantize_stream_kernel launch");
    }
    // Small batches: approximate sums -> approximate prefixes -> exact maps -> exact fold
    // -> outputs (see "small-batch forms").  Clients go in chunks of at most kMaxGridY.
    for (int64_t j0 = 0; j0 < n; j0 += kMaxGridY) {
        const int64_t nj = std::min<int64_t>(kMaxGridY, n - j0);
        const float* xj = x + j0 * d;
        float* outj = out ? out + j0 * ldo : nullptr;
        int8_t* codesj = codes ? codes + j0 * ldc : nullptr;
        int32_t* ovj = codes ? overflow + j0 : nullptr;
        const float* Xj = X ? X + j0 : nullptr;
        const float* l1j = l1use + j0;
        uint64_t* agg = (uint64_t*)(wsb + w.agg_off) + j0 * w.tiles;
        uint64_t* pre = (uint64_t*)(wsb + w.incl_off) + j0 * w.tiles;
        uint64_t* map1 = (uint64_t*)(wsb + w.map1_off) + j0 * w.tiles;
        TileRec* recs = (TileRec*)(wsb + w.rec_off);
        uint32_t* reccnt = (uint32_t*)(wsb + w.cnt_off);      // zeroed by the tile-sum kernels
        const int64_t total_tiles = nj * (int64_t)w.tiles;
        const bool seg = vec4 && d <= ((int64_t)1 << 29) && total_tiles >= kSegMinTiles;
        const dim3 tgrid((unsigned)w.tiles, (unsigned)nj);
        int32_t R = 1, nseg = 1;
        if (seg) {
            // segmented stream: runs of R tiles per workgroup, ~4 resident workgroups per CU
            int slots = 0;
            rc = stream_slots(&slots);
            if (rc) return rc;
            // at most `slots` workgroups in all, so that they run as one wave: ceil(total / slots)
            // tiles each made nj * ceil(tiles / R) > slots workgroups for most nj (101 x 2^22:
            // 1111 of 1024 slots, the last 87 workgroups a second round of R tiles)
            const int64_t segs = std::max<int64_t>(1, slots / nj);
            R = (int32_t)((w.tiles + segs - 1) / segs);
            nseg = (w.tiles + R - 1) / R;
            hipLaunchKernelGGL(agg_stream_kernel, dim3((unsigned)(nj * nseg)), dim3(kQBlock), 0, st, xj, d, w.tiles, fm,
                               l1j, R, nseg, agg, reccnt);
        } else if (vec4) {
            hipLaunchKernelGGL(tile_agg_kernel<true>, tgrid, dim3(kQBlock), 0, st, xj, d, w.tiles, fm, l1j, agg, reccnt);
        } else {
            hipLaunchKernelGGL(tile_agg_kernel<false>, tgrid, dim3(kQBlock), 0, st, xj, d, w.tiles, fm, l1j, agg, reccnt);
        }
        rc = hip_check(hipGetLastError(), "tile sums launch");
        if (rc) return rc;
        const int32_t prefixed = nj >= 4 ? 1 : 0;
        if (prefixed) {
            hipLaunchKernelGGL(tile_prefix_kernel, dim3((unsigned)nj), dim3(kQBlock), 0, st, agg, w.tiles);
            rc = hip_check(hipGetLastError(), "tile_prefix_kernel launch");
            if (rc) return rc;
        }
        if (vec4) {
            hipLaunchKernelGGL(tile_map_kernel<true>, tgrid, dim3(kQBlock), 0, st, xj, d, w.tiles, fm, l1j, agg, pre, map1, recs,
                               reccnt, prefixed);
            rc = hip_check(hipGetLastError(), "tile_map_kernel launch");
            if (rc) return rc;
            hipLaunchKernelGGL(exact_fold_kernel<true>, dim3((unsigned)nj), dim3(kQBlock), 0, st, xj, d, w.tiles, fm, l1j,
                               pre, map1, agg, recs, reccnt);
        } else {
            hipLaunchKernelGGL(tile_map_kernel<false>, tgrid, dim3(kQBlock), 0, st, xj, d, w.tiles, fm, l1j, agg, pre, map1, recs,
                               reccnt, prefixed);
            rc = hip_check(hipGetLastError(), "tile_map_kernel launch");
            if (rc) return rc;
            hipLaunchKernelGGL(exact_fold_kernel<false>, dim3((unsigned)nj), dim3(kQBlock), 0, st, xj, d, w.tiles, fm,
                               l1j, pre, map1, agg, recs, reccnt);
        }
        rc = hip_check(hipGetLastError(), "exact_fold_kernel launch");
        if (rc) return rc;
        pre = agg;                                             // the fold's exact prefixes
        if (seg) {
#define UQ_SEG(Q, C, CV)                                                                                    \
    case ((Q) * 4 + (C) * 2 + (CV)):                                                                      \
        hipLaunchKernelGGL((quantize_stream_kernel<Q, C, CV>), dim3((unsigned)(nj * nseg)), dim3(kQBlock), 0, st, xj, \
                           outj, codesj, ovj, d, w.tiles, fm, Xj, Xval, l1j, R, nseg, pre, ldo, ldc);      \
        break;
            switch (sel & 7) {
                UQ_SEG(1, 0, 1) UQ_SEG(1, 1, 1) UQ_SEG(1, 1, 0) UQ_SEG(0, 1, 1) UQ_SEG(0, 1, 0)
                default: return fail(UQ_E_INVALID, "internal: bad kernel selector");
            }
#undef UQ_SEG
            rc = hip_check(hipGetLastError(), "quantize_stream_kernel (segments) launch");
            if (rc) return rc;
            continue;
        }
#define UQ_PHASED(V, Q, C, CV)                                                                                \
    case ((V) * 8 + (Q) * 4 + (C) * 2 + (CV)):                                                              \
        hipLaunchKernelGGL((tile_out_kernel<V, Q, C, CV>), tgrid, dim3(kQBlock), 0, st, xj, outj, codesj, ovj, d, \
                           w.tiles, fm, Xj, Xval, l1j, pre, ldo, ldc);                                        \
        break;
        switch (sel) {
            UQ_PHASED(1, 1, 0, 1) UQ_PHASED(1, 1, 1, 1) UQ_PHASED(1, 1, 1, 0) UQ_PHASED(1, 0, 1, 1)
            UQ_PHASED(1, 0, 1, 0) UQ_PHASED(0, 1, 0, 1) UQ_PHASED(0, 1, 1, 1) UQ_PHASED(0, 1, 1, 0)
            UQ_PHASED(0, 0, 1, 1) UQ_PHASED(0, 0, 1, 0)
            default: return fail(UQ_E_INVALID, "internal: bad kernel selector");
        }
#undef UQ_PHASED
        rc = hip_check(hipGetLastError(), "tile_out_kernel launch");
        if (rc) return rc;
    }
    return UQ_OK;
}

}  // namespace

extern "C" {

int uq_type_unbiased_codes_ld_f32(const float* x, float* out, int64_t ldq, int8_t* codes, int64_t ldc,
                                  int32_t* overflow, int64_t n, int64_t d, int64_t m, const float* X, const float* l1,
                                  float* l1_out, int32_t T, void* ws, size_t ws_bytes, void* stream) {
    if (n > 0 && d > 0 && !X) return fail(UQ_E_INVALID, "null X");
    return unbiased_codes_impl(x, out, ldq, codes, ldc, overflow, n, d, m, X, 0.0f, l1, l1_out, T, ws, ws_bytes,
                               stream);
}

int uq_type_unbiased_nibbles_ld_f32(const float* x, float* out, int64_t ldq, uint8_t* nib, int64_t ldn,
                                    int32_t* kmax, int64_t n, int64_t d, int64_t m, const float* X, const float* l1,
                                    float* l1_out, int32_t T, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || d < 0) return fail(UQ_E_INVALID, "n and d must be >= 0");
    if (n == 0 || d == 0) return UQ_OK;
    if (!x || !out || !nib || !kmax || !X) return fail(UQ_E_INVALID, "null pointer (x, out, codes, kmax and X are required)");
    if (n < kStreamMinClients || d % kNibAlign != 0 || d > ((int64_t)1 << 29))
        return fail(UQ_E_INVALID, "4-bit codes need n >= 256 and d a multiple of 4096 (<= 2^29)");
    if (ldq < d || ldq % 4 != 0 || ldn < d / 2 || ldn % 16 != 0 || !aligned16(x) || !aligned16(out) || !aligned16(nib))
        return fail(UQ_E_INVALID, "4-bit codes need 16-byte aligned rows: ldq >= d, ldq % 4 == 0, ldn >= d/2, ldn % 16 == 0");
    return unbiased_codes_impl(x, out, ldq, (int8_t*)nib, ldn, kmax, n, d, m, X, 0.0f, l1, l1_out, T, ws, ws_bytes,
                               stream, true);
}

int uq_nibbles_q_mean_ld_f32(const uint8_t* nib, int64_t ldn, const float* q, int64_t ldq, const float* l1,
                             const int32_t* kmax, int64_t n, int64_t d, int64_t m, float n_div, int32_t accumulate,
                             float* est, void* stream) {
    if (n < 0 || d < 0 || m < 0) return fail(UQ_E_INVALID, "n, d and m must be >= 0");
    if (d == 0) return UQ_OK;
    if (!est || (n > 0 && (!nib || !l1 || !kmax || !q))) return fail(UQ_E_INVALID, "null pointer (q is required)");
    if (d % kNibAlign != 0 || ldq < d || ldq % 4 != 0 || ldn < d / 2 || ldn % 4 != 0 || !aligned16(est) ||
        (n > 0 && (!aligned16(q) || ((uintptr_t)nib & 3u))))
        return fail(UQ_E_INVALID, "4-bit code mean: d % 4096 == 0, ldq >= d (multiple of 4), ldn >= d/2 (multiple of 4), "
                                  "16-byte aligned est and q");
    const int64_t blocks = d / (kCodesMeanThreads * kMeanCpt);
    if (blocks > 0x7FFFFFFF) return fail(UQ_E_INVALID, "d too large");
    hipLaunchKernelGGL(nibbles_mean_kernel, dim3((unsigned)blocks), dim3(kCodesMeanThreads), 0, (hipStream_t)stream, nib,
                       ldn, l1, kmax, n, d, (float)m, n_div, accumulate, est, q, ldq);
    return hip_check(hipGetLastError(), "nibbles_mean_kernel launch");
}

int uq_type_unbiased_codes_f32(const float* x, float* out, int8_t* codes, int32_t* overflow, int64_t n, int64_t d,
                               int64_t m, const float* X, const float* l1, float* l1_out, int32_t T, void* ws,
                               size_t ws_bytes, void* stream) {
    return uq_type_unbiased_codes_ld_f32(x, out, d, codes, d, overflow, n, d, m, X, l1, l1_out, T, ws, ws_bytes,
                                         stream);
}

int uq_type_unbiased_vec_f32(const float* x, float* out, int64_t d, int64_t m, float X, int32_t T, void* ws,
                             size_t ws_bytes, void* stream) {
    if (d > 0 && !out) return fail(UQ_E_INVALID, "null out");
    return unbiased_codes_impl(x, out, d, nullptr, d, nullptr, 1, d, m, nullptr, X, nullptr, nullptr, T, ws, ws_bytes,
                               stream);
}

int uq_type_unbiased_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m, const float* X,
                         const float* l1, float* l1_out, int32_t T, void* ws, size_t ws_bytes,
                         void* stream) {
    if (n > 0 && d > 0 && !out) return fail(UQ_E_INVALID, "null out");
    return uq_type_unbiased_codes_f32(x, out, nullptr, nullptr, n, d, m, X, l1, l1_out, T, ws, ws_bytes, stream);
}

int uq_codes_decode_f32(const int8_t* codes, const float* l1, int64_t n, int64_t d, int64_t m, float* out,
                        void* stream) {
    if (n < 0 || d < 0 || m < 0) return fail(UQ_E_INVALID, "n, d and m must be >= 0");
    if (n == 0 || d == 0) return UQ_OK;
    if (!codes || !l1 || !out) return fail(UQ_E_INVALID, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    const int64_t chunks = (d + kDecChunk - 1) / kDecChunk;
    if (chunks > 0x7FFFFFFF) return fail(UQ_E_INVALID, "d too large");
    const bool vec = aligned16(codes) && aligned16(out) && d % 16 == 0;
    dim3 grid((unsigned)chunks, (unsigned)n);
    if (vec)
        hipLaunchKernelGGL(codes_decode_kernel<true>, grid, dim3(256), 0, st, codes, l1, d, (float)m, out);
    else
        hipLaunchKernelGGL(codes_decode_kernel<false>, grid, dim3(256), 0, st, codes, l1, d, (float)m, out);
    return hip_check(hipGetLastError(), "codes_decode_kernel launch");
}

int uq_codes_q_mean_ld_f32(const int8_t* codes, int64_t ldc, const float* q, int64_t ldq, const float* l1,
                           const int32_t* kmax, int64_t n, int64_t d, int64_t m, float n_div, int32_t accumulate,
                           float* est, void* stream) {
    if (n < 0 || d < 0 || m < 0) return fail(UQ_E_INVALID, "n, d and m must be >= 0");
    if (d == 0) return UQ_OK;
    if (!est || (n > 0 && (!codes || !l1 || !kmax))) return fail(UQ_E_INVALID, "null pointer");
    if (q && ldq < d) return fail(UQ_E_INVALID, "ldq must be >= d");
    if (ldc < d) return fail(UQ_E_INVALID, "ldc must be >= d");
    hipStream_t st = (hipStream_t)stream;
    const bool vec = (n == 0 || aligned16(codes)) && aligned16(est) && d % 16 == 0 && ldc % 16 == 0;
    const int64_t blocks = (d + kCodesMeanThreads * kMeanCpt - 1) / (kCodesMeanThreads * kMeanCpt);
    if (blocks > 0x7FFFFFFF) return fail(UQ_E_INVALID, "d too large");
    const dim3 tb(kCodesMeanThreads);
    if (vec && d % (kCodesMeanThreads * kMeanCpt) == 0)
        hipLaunchKernelGGL((codes_mean_kernel<true, true>), dim3((unsigned)blocks), tb, 0, st, codes, ldc, l1, kmax, n,
                           d, (float)m, n_div, accumulate, est, q, ldq);
    else if (vec)
        hipLaunchKernelGGL(codes_mean_kernel<true>, dim3((unsigned)blocks), tb, 0, st, codes, ldc, l1, kmax, n, d,
                           (float)m, n_div, accumulate, est, q, ldq);
    else
        hipLaunchKernelGGL(codes_mean_kernel<false>, dim3((unsigned)blocks), tb, 0, st, codes, ldc, l1, kmax, n, d,
                           (float)m, n_div, accumulate, est, q, ldq);
    return hip_check(hipGetLastError(), "codes_mean_kernel launch");
}

int uq_codes_q_mean_f32(const int8_t* codes, const float* q, int64_t ldq, const float* l1, const int32_t* kmax,
                        int64_t n, int64_t d, int64_t m, float n_div, int32_t accumulate, float* est, void* stream) {
    return uq_codes_q_mean_ld_f32(codes, d, q, ldq, l1, kmax, n, d, m, n_div, accumulate, est, stream);
}

int uq_codes_mean_f32(const int8_t* codes, const float* l1, const int32_t* kmax, int64_t n, int64_t d, int64_t m,
                      float n_div, int32_t accumulate, float* est, void* stream) {
    return uq_codes_q_mean_f32(codes, nullptr, d, l1, kmax, n, d, m, n_div, accumulate, est, stream);
}

int uq_client_mean_f32(const float* q, int64_t n, int64_t d, int64_t ld, float n_div, int32_t accumulate,
                       float* est, void* stream) {
    if (n < 0 || d < 0) return fail(UQ_E_INVALID, "n and d must be >= 0");
    if (ld < d) return fail(UQ_E_INVALID, "ld must be >= d");
    if (d == 0) return UQ_OK;
    if (!est || (n > 0 && !q)) return fail(UQ_E_INVALID, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    const bool vec4 = (n == 0 || aligned16(q)) && aligned16(est) && (d % 4 == 0) && (ld % 4 == 0);
    const int64_t threads = (d + 3) / 4;
    dim3 grid((unsigned)((threads + kMeanThreads - 1) / kMeanThreads));
    if (vec4)
        hipLaunchKernelGGL(client_mean_kernel<true>, grid, dim3(kMeanThreads), 0, st, q, n, d, ld, n_div, accumulate, est);
    else
        hipLaunchKernelGGL(client_mean_kernel<false>, grid, dim3(kMeanThreads), 0, st, q, n, d, ld, n_div, accumulate, est);
    return hip_check(hipGetLastError(), "client_mean_kernel launch");
}

int uq_type_unbiased_mean_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m, const float* X,
                              const float* l1, int32_t T, float n_div, int32_t accumulate, float* est,
                              void* ws, size_t ws_bytes, void* stream) {
    if (!out) return fail(UQ_E_INVALID, "out must be non-NULL in this version");
    int rc = uq_type_unbiased_f32(x, out, n, d, m, X, l1, nullptr, T, ws, ws_bytes, stream);
    if (rc) return rc;
    return uq_client_mean_f32(out, n, d, d, n_div, accumulate, est, stream);
}

int uq_check_status(void* ws, void* stream) {
    if (!ws) return fail(UQ_E_INVALID, "null workspace");
    hipStream_t st = (hipStream_t)stream;
    uint32_t status = 0;
    int rc = hip_check(hipMemcpyAsync(&status, (char*)ws + 8, 4, hipMemcpyDeviceToHost, st), "read status");
    if (rc) return rc;
    rc = hip_check(hipStreamSynchronize(st), "sync");
    if (rc) return rc;
    if (status) {
        (void)hipMemsetAsync((char*)ws + 8, 0, 4, st);
        (void)hipStreamSynchronize(st);
        if (status == 2) return fail(UQ_E_TIMEOUT, "torch tie replay inconsistent (internal error)");
        return fail(UQ_E_TIMEOUT, "inter-workgroup wait timed out");
    }
    return UQ_OK;
}


// ---- type-message codec "UQR1" (uq_codec_kernels.h) -----------------------------------
namespace {
struct TcLayout {
    size_t hist, tabs, cwords, states, sizes, scratch, total;
};
TcLayout tc_layout(int64_t n, int64_t d) {
    const int64_t nch = tc_nchunks(d);
    const int64_t csz = (int64_t)tc_lanes(d) * kTcSteps;
    TcLayout L;
    size_t o = 0;
    auto take = [&](size_t b) { const size_t r = o; o += (b + 255) & ~(size_t)255; return r; };
    L.hist = take((size_t)n * 256 * 4);
    L.tabs = take((size_t)n * sizeof(TcTable));
    L.cwords = take((size_t)(n * nch) * 4);
    L.states = take((size_t)(n * nch) * 64 * 4);
    L.sizes = take((size_t)n * 8);
    L.scratch = take((size_t)(n * nch * csz) * 2);
    L.total = o;
    return L;
}
}  // namespace

int uq_tc_bound(int64_t d, size_t* bytes_out) {
    if (d < 0 || d > ((int64_t)1 << 31) || !bytes_out) return fail(UQ_E_INVALID, "bad d / null bytes_out");
    *bytes_out = (size_t)tc_bound(d);
    return UQ_OK;
}

int uq_tc_workspace_bytes(int64_t n, int64_t d, size_t* bytes_out) {
    if (n < 0 || d < 0 || d > ((int64_t)1 << 31) || !bytes_out) return fail(UQ_E_INVALID, "bad n / d / null bytes_out");
    *bytes_out = tc_layout(n, d).total;
    return UQ_OK;
}

int uq_tc_encode(const int8_t* codes, const float* l1, int64_t n, int64_t d, int64_t m, int32_t flags, uint8_t* msgs,
                 size_t msgs_bytes, uint64_t* offsets, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || d < 0 || d > ((int64_t)1 << 31) || m < 0) return fail(UQ_E_INVALID, "bad n / d / m");
    if (flags & ~1) return fail(UQ_E_INVALID, "unknown codec flags");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) return offsets ? hip_check(hipMemsetAsync(offsets, 0, 8, st), "offsets") : fail(UQ_E_INVALID, "null offsets");
    if (!l1 || !msgs || !offsets || !ws || (d > 0 && !codes)) return fail(UQ_E_INVALID, "null pointer");
    if (msgs_bytes < (size_t)n * tc_bound(d)) return fail(UQ_E_INVALID, "message buffer below n * uq_tc_bound(d)");
    const TcLayout L = tc_layout(n, d);
    if (ws_bytes < L.total) return fail(UQ_E_WORKSPACE, "workspace too small (uq_tc_workspace_bytes)");
    char* w = (char*)ws;
    uint32_t* hist = (uint32_t*)(w + L.hist);
    TcTable* tabs = (TcTable*)(w + L.tabs);
    uint32_t* cwords = (uint32_t*)(w + L.cwords);
    uint32_t* states = (uint32_t*)(w + L.states);
    uint64_t* sizes = (uint64_t*)(w + L.sizes);
    uint16_t* scratch = (uint16_t*)(w + L.scratch);
    const int64_t nch = tc_nchunks(d);
    const int exact = flags & 1;
    int rc = hip_check(hipMemsetAsync(hist, 0, (size_t)n * 256 * 4, st), "memset hist");
    if (rc) return rc;
    for (int64_t j0 = 0; j0 < n; j0 += kMaxGridY) {
        const int64_t nj = std::min<int64_t>(kMaxGridY, n - j0);
        if (d > 0) {
            hipLaunchKernelGGL(tc_hist_kernel, dim3((unsigned)((d + kTcHistSeg - 1) / kTcHistSeg), (unsigned)nj), dim3(256), 0,
                               st, codes + j0 * d, d, hist + j0 * 256);
            if ((rc = hip_check(hipGetLastError(), "tc_hist_kernel launch"))) return rc;
        }
        hipLaunchKernelGGL(tc_table_kernel, dim3((unsigned)nj), dim3(64), 0, st, hist + j0 * 256, d, exact, tabs + j0);
        if ((rc = hip_check(hipGetLastError(), "tc_table_kernel launch"))) return rc;
        if (nch > 0) {
            hipLaunchKernelGGL(tc_encode_kernel, dim3((unsigned)((nch + kTcEncWaves - 1) / kTcEncWaves), (unsigned)nj),
                               dim3(64 * kTcEncWaves), 0, st, codes + j0 * d, d, exact,
                               tabs + j0, scratch + j0 * nch * ((int64_t)tc_lanes(d) * kTcSteps), cwords + j0 * nch,
                               states + j0 * nch * tc_lanes(d));
            if ((rc = hip_check(hipGetLastError(), "tc_encode_kernel launch"))) return rc;
        }
        hipLaunchKernelGGL(tc_layout_kernel, dim3((unsigned)nj), dim3(64), 0, st, d, tabs + j0, cwords + j0 * nch, sizes + j0);
        if ((rc = hip_check(hipGetLastError(), "tc_layout_kernel launch"))) return rc;
    }
    hipLaunchKernelGGL(tc_scan_kernel, dim3(1), dim3(1024), 0, st, sizes, n, offsets);
    if ((rc = hip_check(hipGetLastError(), "tc_scan_kernel launch"))) return rc;
    if (nch == 0) {
        // d == 0: header-only messages, written by one "chunk" each
        for (int64_t j0 = 0; j0 < n; j0 += kMaxGridY) {
            const int64_t nj = std::min<int64_t>(kMaxGridY, n - j0);
            hipLaunchKernelGGL(tc_pack_kernel, dim3(1, (unsigned)nj), dim3(256), 0, st, d, m, exact, l1 + j0, tabs + j0,
                               scratch, cwords, states, offsets + j0, msgs);
            if ((rc = hip_check(hipGetLastError(), "tc_pack_kernel launch"))) return rc;
        }
        return UQ_OK;
    }
    for (int64_t j0 = 0; j0 < n; j0 += kMaxGridY) {
        const int64_t nj = std::min<int64_t>(kMaxGridY, n - j0);
        hipLaunchKernelGGL(tc_pack_kernel, dim3((unsigned)nch, (unsigned)nj), dim3(256), 0, st, d, m, exact, l1 + j0,
                           tabs + j0, scratch + j0 * nch * ((int64_t)tc_lanes(d) * kTcSteps), cwords + j0 * nch,
                           states + j0 * nch * tc_lanes(d), offsets + j0, msgs);
        if ((rc = hip_check(hipGetLastError(), "tc_pack_kernel launch"))) return rc;
    }
    return UQ_OK;
}

int uq_tc_decode(const uint8_t* msgs, size_t msgs_bytes, const uint64_t* offsets, int64_t n, int64_t d, int64_t m,
                 int8_t* codes, float* l1, int32_t* kmax, int32_t* status, void* stream) {
    if (n < 0 || d < 0 || d > ((int64_t)1 << 31)) return fail(UQ_E_INVALID, "bad n / d");
    if (n == 0) return UQ_OK;
    if (!msgs || !offsets || !l1 || !kmax || !status || (d > 0 && !codes)) return fail(UQ_E_INVALID, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    int rc = hip_check(hipMemsetAsync(status, 0, (size_t)n * 4, st), "memset status");
    if (rc) return rc;
    const int64_t nch = std::max<int64_t>(1, tc_nchunks(d));
    for (int64_t j0 = 0; j0 < n; j0 += kMaxGridY) {
        const int64_t nj = std::min<int64_t>(kMaxGridY, n - j0);
        hipLaunchKernelGGL(tc_decode_kernel, dim3((unsigned)((nch + kTcDecWaves - 1) / kTcDecWaves), (unsigned)nj),
                           dim3(64 * kTcDecWaves), 0, st, msgs, (uint64_t)msgs_bytes, offsets + j0, d, m,
                           codes ? codes + j0 * d : codes, l1 + j0, kmax + j0, status + j0);
        if ((rc = hip_check(hipGetLastError(), "tc_decode_kernel launch"))) return rc;
    }
    return UQ_OK;
}

int uq_biased_workspace_bytes(int64_t n, int64_t d, int32_t T, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    L1Plan plan;
    if (n < 0 || d < 0 || T < 1) return fail(UQ_E_INVALID, "bad n/d/torch_threads");
    if (!make_plan(d, T, &plan)) return fail(UQ_E_INVALID, "cannot build L1 plan");
    *bytes_out = biased_layout(n, d, plan).total;
    return UQ_OK;
}

int uq_type_biased_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m, int32_t T,
                       int32_t tie_policy, float* l1_out, int32_t* info, void* ws, size_t ws_bytes,
                       void* stream) {
    if (n < 0 || d < 0) return fail(UQ_E_INVALID, "n and d must be >= 0");
    if (m < 0) return fail(UQ_E_INVALID, "m must be >= 0");
    if (d >= ((int64_t)1 << 31)) return fail(UQ_E_INVALID, "d must be < 2^31");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 clients per call");
    if (T < 1) return fail(UQ_E_INVALID, "torch_threads must be >= 1");
    const bool host_check = (tie_policy & UQ_TIES_HOST_CHECK) != 0;
    tie_policy &= ~UQ_TIES_HOST_CHECK;
    if (tie_policy != UQ_TIES_LOWEST_INDEX && tie_policy != UQ_TIES_TORCH)
        return fail(UQ_E_INVALID, "unknown tie_policy");
    L1Plan plan;
    if (!make_plan(d, T, &plan)) return fail(UQ_E_INVALID, "cannot build L1 plan for this d/torch_threads");
    const BiasedLayout w = biased_layout(n, d, plan);
    if (n == 0) return UQ_OK;
    hipStream_t st = (hipStream_t)stream;
    if (d == 0) {
        int rc = UQ_OK;
        if (l1_out) rc = hip_check(hipMemsetAsync(l1_out, 0, n * sizeof(float), st), "memset l1");
        if (!rc && info) rc = hip_check(hipMemsetAsync(info, 0, n * 2 * sizeof(int32_t), st), "memset info");
        return rc;
    }
    if (!x || !out) return fail(UQ_E_INVALID, "null x or out");
    if (!ws) return fail(UQ_E_INVALID, "null workspace");
    if (ws_bytes < w.total) return fail(UQ_E_WORKSPACE, "workspace too small");
    char* wsb = (char*)ws;
    float* part = (float*)(wsb + w.part_off);
    float* l1buf = (float*)(wsb + w.l1_off);
    float* msum = (float*)(wsb + w.msum_off);
    RezState* state = (RezState*)(wsb + w.st_off);
    auto finish = [&]() {                     // l1_out and the info pairs
        int frc = UQ_OK;
        if (l1_out) frc = hip_check(hipMemcpyAsync(l1_out, l1buf, n * sizeof(float), hipMemcpyDeviceToDevice, st), "copy l1");
        if (!frc && info)
            frc = hip_check(hipMemcpy2DAsync(info, 2 * sizeof(int32_t), state, sizeof(RezState), 2 * sizeof(int32_t), n,
                                             hipMemcpyDeviceToDevice, st), "copy info");
        return frc;
    };
    // vectors shorter than GRAIN: one launch (KB-small) with the lowest-index rule; with torch
    // ties only under UQ_TIES_HOST_CHECK, which reads the clients' flags back and runs the
    // multi-kernel path below when a threshold tie needs torch's choice
    if (d <= kSmallBiasedMax &&
        (tie_policy == UQ_TIES_LOWEST_INDEX || (host_check && n <= kSmallCheckMaxN))) {
        static std::atomic<uint64_t> attr_set{0};             // per device (bit = device index < 64)
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 && !((attr_set.load() >> dev) & 1u)) {
            (void)hipFuncSetAttribute((const void*)biased_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(kSmallBiasedMax * sizeof(uint32_t)));
            attr_set.fetch_or(1ull << dev);
        }
        hipLaunchKernelGGL(biased_small_kernel, dim3((unsigned)n), dim3(256), (size_t)d * sizeof(uint32_t), st, x, out, d,
                           (float)m, (const float*)nullptr, l1buf, state);
        int rc = hip_check(hipGetLastError(), "biased_small_kernel launch");
        if (rc) return rc;
        if (tie_policy == UQ_TIES_LOWEST_INDEX) return finish();
        SideStream* sb = nullptr;
        if ((rc = side_stream(&sb))) return rc;
        rc = hip_check(hipMemcpyAsync(sb->states, state, (size_t)n * sizeof(RezState), hipMemcpyDeviceToHost, st),
                       "copy states");
        if (rc) return rc;
        if ((rc = hip_check(hipStreamSynchronize(st), "sync"))) return rc;
        bool tie = false;
        for (int64_t i = 0; i < n; ++i) tie |= (((const RezState*)sb->states)[i].flags & kRezAmbiguous) != 0;
        if (!tie) return finish();
    }
    uint32_t* hist = (uint32_t*)(wsb + w.hist_off);
    uint32_t* tcnt = (uint32_t*)(wsb + w.tcnt_off);
    uint32_t* bits = (uint32_t*)(wsb + w.bits_off);
    const float fm = (float)m;
    int rc = launch_l1(x, n, d, plan, part, l1buf, st);                                   // AS:680
    if (rc) return rc;
    uint32_t* zn = (uint32_t*)(wsb + w.zn_off);
    uint32_t* cand_n = (uint32_t*)(wsb + w.cn_off);
    uint32_t* cand = (uint32_t*)(wsb + w.cand_off);
    rc = hip_check(hipMemsetAsync(hist, 0, w.cand_off - w.hist_off, st), "memset hist/zn/cand_n");
    if (rc) return rc;
    // AS:648-649 m' = sum k' in torch order, with the first radix digit's histogram (KB2 + KB4 pass 0)
    rc = launch_cascade<RezKHistOp>(x, n, d, plan, part, msum, l1buf, fm, st, hist, zn);
    if (rc) return rc;
    hipLaunchKernelGGL(rez_setup_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, msum, fm, d, n, state);
    rc = hip_check(hipGetLastError(), "rez_setup_kernel launch");
    if (rc) return rc;
    const bool vec4 = aligned16(x) && aligned16(out) && d % 4 == 0;
    const dim3 fgrid((unsigned)((d + kSelTile - 1) / kSelTile), (unsigned)n);
    uint2* fcand = (uint2*)cand;
    // KB4a: the threshold's fine bin; a small bucket makes the client "fine", a large one "full"
    // full clients are listed by KB4a (flist[0] = count, in the zeroed range): the key-digit
    // passes below stride over the list, not over n x spans workgroups that mostly exit
    uint32_t* flist = (uint32_t*)(wsb + w.fl_off);
    hipLaunchKernelGGL((rez_select_kernel<0, true>), dim3((unsigned)n), dim3(256), 0, st, state, hist, zn, w.capf, flist);
    const unsigned fy = (unsigned)std::min<int64_t>(n, kListedGridY);
    const dim3 hlgrid((unsigned)((d + kHistSpan - 1) / kHistSpan), fy);
    // full clients (tie-heavy rows): the key digits by three full-row histogram passes
#define UQ_RADIX(P)                                                                                          \
    if (vec4)                                                                                                \
        hipLaunchKernelGGL((rez_hist_kernel<P, true>), hlgrid, dim3(256), 0, st, x, d, l1buf, fm, state, hist, flist); \
    else                                                                                                     \
        hipLaunchKernelGGL((rez_hist_kernel<P, false>), hlgrid, dim3(256), 0, st, x, d, l1buf, fm, state, hist, flist); \
    hipLaunchKernelGGL((rez_select_kernel<P, false>), dim3((unsigned)std::min<int64_t>(n, kTieSlots)), dim3(256), 0, st, \
                       state, hist, zn, w.capf, flist);
    UQ_RADIX(0) UQ_RADIX(1) UQ_RADIX(2)
#undef UQ_RADIX
    // fine clients: KB6f writes every output and lists the bucket, KB4d finds the threshold
    // key among the listed keys, KB6p patches the selected listed coordinates (tie-free clients)
    if (vec4)
        hipLaunchKernelGGL(rez_output_fine_kernel<true>, fgrid, dim3(256), 0, st, x, out, d, l1buf, fm, state, fcand,
                           cand_n, w.capf);
    else
        hipLaunchKernelGGL(rez_output_fine_kernel<false>, fgrid, dim3(256), 0, st, x, out, d, l1buf, fm, state, fcand,
                           cand_n, w.capf);
    const unsigned cspans = (unsigned)((w.capf + kCandSpan - 1) / kCandSpan);
    if (n <= kCandMultiMaxN && cspans > 1) {         // few clients: the passes over many workgroups
#define UQ_CAND(P)                                                                                           \
        hipLaunchKernelGGL(rez_cand_hist_kernel<P>, dim3(cspans, (unsigned)n), dim3(256), 0, st, state, fcand, cand_n, \
                           w.capf, hist);                                                                    \
        hipLaunchKernelGGL(rez_cand_pick_kernel<P>, dim3((unsigned)n), dim3(256), 0, st, state, hist);
        UQ_CAND(0) UQ_CAND(1) UQ_CAND(2)
#undef UQ_CAND
    } else {
        hipLaunchKernelGGL(rez_cand_select_kernel, dim3((unsigned)n), dim3(256), 0, st, state, fcand, cand_n, w.capf);
    }
    rc = hip_check(hipGetLastError(), "radix select launch");
    if (rc) return rc;
    // KB6p: the tie-free fine clients' selected bin coordinates (independent of KB7: with the
    // torch-tie fork it runs on the caller's stream beside the replay chain, off its path)
    auto fine_patch = [&](hipStream_t ps) {
        hipLaunchKernelGGL(rez_fine_patch_kernel, dim3(kPatchBlocks, (unsigned)n), dim3(256), 0, ps, x, out, d, l1buf,
                           fm, state, fcand, cand_n, w.capf);
        return hip_check(hipGetLastError(), "rez_fine_patch_kernel launch");
    };
    const bool fork_ties = tie_policy == UQ_TIES_TORCH && !(host_check && kb7a_path(n, d));
    if (!fork_ties && (rc = fine_patch(st))) return rc;
    // KB6 for the clients of a list (list-strided grid): part 0 / 1 over KB4a's list (the full
    // clients and those without a selection -- every client KB6f did not write), part 3 over
    // the ambiguous ones (their fine clients)
    // ol == nullptr: the n x tiles grid (part 1 beside the torch-tie chain: the list-strided
    // form was 0.01-0.02 ms slower there, profiles/r5aw_*; the lowest-index batch gains 0.075 ms
    // from it, its launches being on the critical path)
    const dim3 lgrid((unsigned)w.tiles, (unsigned)std::min<int64_t>(n, kListedGridY));
    auto output = [&](hipStream_t os, int part, const uint32_t* ol) {
        const dim3 ogrid((unsigned)w.tiles, (unsigned)(ol ? std::min<int64_t>(n, kListedGridY) : n));
        if (vec4)
            hipLaunchKernelGGL(rez_output_kernel<true>, ogrid, dim3(256), 0, os, x, out, d, l1buf, fm, state, tcnt,
                               w.tiles, bits, part, ol);
        else
            hipLaunchKernelGGL(rez_output_kernel<false>, ogrid, dim3(256), 0, os, x, out, d, l1buf, fm, state, tcnt,
                               w.tiles, bits, part, ol);
        return hip_check(hipGetLastError(), "rez_output_kernel launch");
    };
    // after KB7: its listed clients only (a list-strided grid, not n x tiles workgroups that
    // mostly exit): full rows for index-order ranks and full clients, KB6t's patch of the
    // listed threshold bin for the replayed fine clients
    auto output_listed = [&](hipStream_t os) {
        const uint32_t* list = (const uint32_t*)(wsb + w.list_off);
        if (vec4)
            hipLaunchKernelGGL(rez_output_kernel<true>, lgrid, dim3(256), 0, os, x, out, d, l1buf, fm, state, tcnt,
                               w.tiles, bits, 2, list);
        else
            hipLaunchKernelGGL(rez_output_kernel<false>, lgrid, dim3(256), 0, os, x, out, d, l1buf, fm, state, tcnt,
                               w.tiles, bits, 2, list);
        int orc = hip_check(hipGetLastError(), "rez_output_kernel launch");
        if (orc) return orc;
        hipLaunchKernelGGL(rez_tie_patch_kernel, dim3(kPatchBlocks, (unsigned)std::min<int64_t>(n, kListedGridY)),
                           dim3(256), 0, os, x, out, d, l1buf, fm, state, fcand, cand_n, w.capf, bits, list);
        return hip_check(hipGetLastError(), "rez_tie_patch_kernel launch");
    };
    auto tiecount = [&](hipStream_t ts, const uint32_t* list) {
        // index-order tie ranks of the listed (ambiguous) clients
        if (vec4)
            hipLaunchKernelGGL(rez_tiecount_kernel<true>, lgrid, dim3(256), 0, ts, x, d, l1buf, fm, state, tcnt, w.tiles,
                               list);
        else
            hipLaunchKernelGGL(rez_tiecount_kernel<false>, lgrid, dim3(256), 0, ts, x, d, l1buf, fm, state, tcnt, w.tiles,
                               list);
        return hip_check(hipGetLastError(), "rez_tiecount_kernel launch");
    };
    // (the check pays only where the replay would be KB7a's level chain; a one-kernel replay
    // costs less than the synchronisation)
    const bool kb7a = kb7a_path(n, d);
    if (tie_policy == UQ_TIES_TORCH && host_check && kb7a) {
        // UQ_TIES_HOST_CHECK (synchronous few-client callers): one stream; after the tie list
        // is built, wait for it and skip the replay chain -- KB7a's ~65 level launches --
        // when no client is listed; then every client's output in one launch
        // (no tie counts: every ambiguous client is listed and replayed; a failed replay
        // counts its own tiles)
        rc = torch_ties_prepare(n, d, state, bits, wsb, w, st, false);
        if (rc) return rc;
        SideStream* sb = nullptr;
        rc = side_stream(&sb);                            // (its pinned word)
        if (rc) return rc;
        rc = hip_check(hipMemcpyAsync(sb->count, wsb + w.list_off, sizeof(uint32_t), hipMemcpyDeviceToHost, st),
                       "copy tie list length");
        if (rc) return rc;
        rc = hip_check(hipStreamSynchronize(st), "sync");
        if (rc) return rc;
        if (*sb->count != 0u) {
            const TieLevelState* tls = nullptr;
            rc = launch_torch_ties(x, n, d, l1buf, fm, state, bits, wsb, w, st, &tls, nullptr);
            if (rc) return rc;
            if (tls && (rc = launch_torch_ties_rest(x, d, l1buf, fm, state, bits, wsb, w, tls, st))) return rc;
            if ((rc = output_listed(st))) return rc;
        }
        rc = output(st, 1, nullptr);
        if (rc) return rc;
    } else if (tie_policy == UQ_TIES_TORCH) {
        // fork: KB7 (few workgroups, latency-bound) on the side stream while KB6 writes the
        // clients without a threshold tie on the caller's stream; join, then the rest
        SideStream* sb = nullptr;
        rc = side_stream(&sb);
        if (rc) return rc;
        // the tie list (and, without KB7a, cleared tie bits) before the fork: both streams read it
        rc = torch_ties_prepare(n, d, state, bits, wsb, w, st, !kb7a);
        if (rc) return rc;
        rc = hip_check(hipEventRecord(sb->fork, st), "record fork");
        if (rc) return rc;
        rc = hip_check(hipStreamWaitEvent(sb->s, sb->fork, 0), "wait fork");
        if (rc) return rc;
        // KB6 for the clients without a tie waits for KB7a's first (bandwidth-heavy) levels
        // and then runs beside the later, latency-bound ones (the chain is the critical path).
        // No tie counts: every ambiguous client is listed and replayed (a failed replay counts
        // its own tiles; the launch was 66 us of early-exit workgroups beside the chain)
        const TieLevelState* tls = nullptr;
        rc = launch_torch_ties(x, n, d, l1buf, fm, state, bits, wsb, w, sb->s, &tls, [&]() {
            int mrc = hip_check(hipEventRecord(sb->mid, sb->s), "record mid");
            if (!mrc) mrc = hip_check(hipStreamWaitEvent(st, sb->mid, 0), "wait mid");
            if (!mrc) mrc = output(st, 1, nullptr);
            if (!mrc) mrc = fine_patch(st);
            return mrc;
        });
        if (rc) return rc;
        rc = hip_check(hipEventRecord(sb->join, sb->s), "record join");
        if (rc) return rc;
        rc = hip_check(hipStreamWaitEvent(st, sb->join, 0), "wait join");
        if (rc) return rc;
        if (tls) {                       // replays KB7a did not take (full 1024-thread replays)
            rc = launch_torch_ties_rest(x, d, l1buf, fm, state, bits, wsb, w, tls, st);
            if (rc) return rc;
        }
        rc = output_listed(st);
        if (rc) return rc;
    } else {
        // the lowest-index rule: the ambiguous clients' list (rez_tie_list_kernel), their tie
        // counts, then KB6 over the full / no-selection clients and over the ambiguous fine ones
        rc = torch_ties_prepare(n, d, state, bits, wsb, w, st, false);
        if (rc) return rc;
        const uint32_t* amb = (const uint32_t*)(wsb + w.list_off);
        if ((rc = tiecount(st, amb))) return rc;
        if ((rc = output(st, 0, flist))) return rc;
        if ((rc = output(st, 3, amb))) return rc;
    }
    return finish();
}

// ---- EDEN + RHT ------------------------------------------------------------------------
int uq_rht_signs(const int32_t* seeds, int64_t rows, int64_t D, int8_t* signs, void* stream) {
    if (rows < 0 || D < 0) return fail(UQ_E_INVALID, "rows and D must be >= 0");
    if (rows == 0 || D == 0) return UQ_OK;
    if (rows > 65535) return fail(UQ_E_INVALID, "at most 65535 rows per call");
    if (!seeds || !signs) return fail(UQ_E_INVALID, "null pointer");
    hipLaunchKernelGGL(rht_signs_kernel, dim3((unsigned)rows), dim3(640), 0, (hipStream_t)stream, seeds, D, signs);
    return hip_check(hipGetLastError(), "rht_signs_kernel launch");
}

// The jump path (KQ0s + KQ0j + KQ1j + KQ1f, uq_quicfl_kernels.h) for few messages: R runs of L
// rounds per message, R from a cost model of the phases (measured round-5 constants): the
// streams (~20 us), the jumps (~tJ of the whole GPU per jump) and a round of passes A + B on one
// wave (~tR; a run wave per SIMD).  The one-wave kernel when the model gives the jumps no gain.
struct QflJumpPlan {
    bool use = false;
    int32_t R = 0;
    int64_t L = 0, qL = 0;
};

// Up to 1024 run waves a wave per SIMD; up to 2048 two (quicfl_send_runs_kernel<., true>), a
// round then costing ~1.3 tR (round 6, profiles/r6k_* .. r6x_*: 512 x 2^20 compress 12.0 -> 7.6
// ms, 1024 x 2^20 14.4 -> 12.9 with R = 2 once the runs' pass A moved to the side stream and the
// counting pass went; 256 x 2^22 round trip 24.2 -> 17.5).
constexpr int64_t kQfJumpMaxN = 1024;
constexpr int64_t kQfRunWaves1 = 1024, kQfRunWaves2 = 2048;
static QflJumpPlan qfl_jump_plan(int64_t n, int64_t D) {
    QflJumpPlan p;
    const int64_t nch = (D + kMtN - 1) / kMtN;
    if (n < 1 || n > kQfJumpMaxN || nch < 8 || D > ((int64_t)1 << 28)) return p;
    const double tS = 20.0, tJ = 0.12, tR = 7.5, f2 = 1.3;
    double best = 1e300;
    for (int64_t R = 1; R <= 1024 && R <= nch; ++R) {
        const int64_t L = (nch + R - 1) / R, Ru = (nch + L - 1) / L;
        if (Ru != R || n * R > kQfRunWaves2) continue;
        const double t = tS + (double)(n * (3 * R - 2)) * tJ + (double)L * tR * (n * R > kQfRunWaves1 ? f2 : 1.0);
        if (t < best) {
            best = t;
            p.R = (int32_t)R;
            p.L = L;
        }
    }
    // against: up to 128 messages the team kernel as round 5 measured it; 129-256 the team kernel
    // at ~2.85 us per round, the model ~1.4x optimistic (r6l: 256 x 2^20 team 5.5 / jump 5.9 ms,
    // 2^21 11.3 / 10.3, 2^22 round trip 24.3 / 18.7); above, a wave per message
    if (n <= 128 || n > kQfTeamMaxN)
        p.use = best < 0.8 * (double)((n + 1023) / 1024) * (double)nch * tR;
    else
        p.use = best < 2.0 * (double)nch;
    p.qL = ((int64_t)kMtN + D) / kMtN;               // block of the first pass-B local word (qfl_ctx)
    return p;
}

// The receiver's jump path: one stream, one jump per run; a round (one wave: the h word, the
// table gather, X, the mask and the exact value) ~tR, ~1.3 tR at two waves per SIMD (more than
// 1024 run waves; 512 x 2^20 decompress 5.60 -> 3.53 ms, 1024 x 2^20 7.4 -> 6.4, profiles/r6r_*,
// r6w_*, r6x_*).  Taken when it beats the team kernel (~1 us per round of the h scout's twists
// and the runs behind it).
static QflJumpPlan qfl_recv_jump_plan(int64_t n, int64_t D) {
    QflJumpPlan p;
    const int64_t nch = (D + kMtN - 1) / kMtN;
    if (n < 1 || n > kQfJumpMaxN || nch < 8 || D > ((int64_t)1 << 28)) return p;
    const double tS = 20.0, tJ = 0.12, tR = 3.0;
    double best = 1e300;
    for (int64_t R = 1; R <= 1024 && R <= nch; ++R) {
        const int64_t L = (nch + R - 1) / R, Ru = (nch + L - 1) / L;
        if (Ru != R || n * R > kQfRunWaves2) continue;                 // (its kernels fit 2 waves per SIMD)
        const double t = tS + (double)(n * (R - 1)) * tJ + (double)L * tR * (n * R > kQfRunWaves1 ? 1.3 : 1.0);
        if (t < best) {
            best = t;
            p.R = (int32_t)R;
            p.L = L;
        }
    }
    // against the team kernel (~1 us per round) up to 256 messages, a wave per message (~tR per
    // round, one wave per SIMD) above
    p.use = best < 0.8 * (double)nch * (n <= kQfTeamMaxN ? 1.0 : tR);
    return p;
}

extern "C" int uq_mtpoly_progression(int64_t b0, int64_t step, int32_t count, uint32_t* out);   // uq_mt_poly.cpp

// t^(624 b) mod phi for the plan's run starts, on the device, cached per (device, qL, L, R):
// rows [0, R) = polyA (row r: b = r L - 1; row 0 unused), rows [R, 2R) = polyB (b = qL + r L - 1)
static int qfl_jump_polys(const QflJumpPlan& p, bool a_only, const uint32_t** out) {
    static std::mutex mu;
    static std::map<std::tuple<int, int64_t, int64_t, int32_t>, uint32_t*> cache;
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(dev, a_only ? (int64_t)-1 : p.qL, p.L, p.R);   // (A rows only: no qL)
    auto it = cache.find(key);
    if (it != cache.end()) {
        *out = it->second;
        return UQ_OK;
    }
    std::vector<uint32_t> h((size_t)2 * p.R * kMtN, 0u);
    if ((p.R > 1 && uq_mtpoly_progression(p.L - 1, p.L, p.R - 1, h.data() + kMtN)) ||
        (!a_only && uq_mtpoly_progression(p.qL - 1, p.L, p.R, h.data() + (size_t)p.R * kMtN)))
        return fail(UQ_E_INVALID, "MT19937 jump polynomials unavailable");
    // Entries live for the life of the process: a pointer handed out above may still be waiting
    // to be launched on another thread's stream, so nothing here is ever freed.  The key space is
    // one entry per (device, layout) in use -- 2 R * 624 words each, a few KB to ~1 MB.
    uint32_t* d = nullptr;
    rc = hip_check(hipMalloc(&d, h.size() * sizeof(uint32_t)), "hipMalloc jump polynomials");
    if (rc) return rc;
    rc = hip_check(hipMemcpy(d, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "copy jump polynomials");
    if (rc) {
        (void)hipFree(d);
        return rc;
    }
    cache.emplace(key, d);
    *out = d;
    return UQ_OK;
}

static int quicfl_recv_jump(const QflRecvArgs& r, int32_t x_kind, const QflJumpPlan& jp, char* wsb, hipStream_t st);

int uq_quicfl_receive_f32(const void* X, int32_t x_kind, int64_t n, int64_t D, const float* recv_table,
                          int32_t table_rows, int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask,
                          const float* exact_vals, int32_t exact_layout, const int32_t* exact_count, const float* scale,
                          float* out, int32_t* info, void* stream) {
    return uq_quicfl_receive_ws_f32(X, x_kind, n, D, recv_table, table_rows, h_len, prng_seeds, exact_mask, exact_vals,
                                    exact_layout, exact_count, scale, out, info, nullptr, 0, stream);
}

int uq_quicfl_receive_workspace_bytes(int64_t n, int64_t D, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    if (n < 0 || D < 0) return fail(UQ_E_INVALID, "n and D must be >= 0");
    const QflJumpPlan p = qfl_recv_jump_plan(n, D);
    *bytes_out = p.use ? ((size_t)n * kMjX + (size_t)n * p.R * (kMjParts * kMtN + 2)) * sizeof(uint32_t) : 0;
    return UQ_OK;
}

int uq_quicfl_receive_ws_f32(const void* X, int32_t x_kind, int64_t n, int64_t D, const float* recv_table,
                             int32_t table_rows, int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask,
                             const float* exact_vals, int32_t exact_layout, const int32_t* exact_count,
                             const float* scale, float* out, int32_t* info, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || D < 0) return fail(UQ_E_INVALID, "n and D must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 clients per call");
    if (D > ((int64_t)1 << 28)) return fail(UQ_E_INVALID, "at most 2^28 coordinates per message");
    if (x_kind < 0 || x_kind > 2) return fail(UQ_E_INVALID, "x_kind must be 0 (int64), 1 (uint8) or 2 (int32)");
    if (exact_layout != 0 && exact_layout != 1) return fail(UQ_E_INVALID, "exact_layout must be 0 (dense) or 1 (compact)");
    if (n == 0 || D == 0) return UQ_OK;
    if (!X || !recv_table || !prng_seeds || !scale || !out) return fail(UQ_E_INVALID, "null pointer");
    if ((exact_mask == nullptr) != (exact_vals == nullptr)) return fail(UQ_E_INVALID, "exact_mask and exact_vals go together");
    if (h_len < 1 || table_rows < 1 || (int64_t)h_len * table_rows > kQflTab)
        return fail(UQ_E_INVALID, "receiver table must hold 1..1024 entries");
    hipStream_t st = (hipStream_t)stream;
    QflRecvArgs r{};
    r.X = X;
    r.n = n;
    r.D = D;
    r.table = recv_table;
    r.tab_n = table_rows * h_len;
    r.h_len = h_len;
    r.prng_seeds = prng_seeds;
    r.exact_mask = exact_mask;
    r.exact_vals = exact_vals;
    r.compact = exact_layout;
    r.exact_count = exact_count;
    r.scale = scale;
    r.out = out;
    r.info = info;
    const int hooks = g_quicfl_hooks.load();
    r.force_timeout = hooks & 1;
    // few messages: every run at once from jumped blocks of the h stream (given a workspace), or
    // a workgroup per message (the h stream's scout + 7 runs); batches: a wave each
    const QflJumpPlan jp = qfl_recv_jump_plan(n, D);
    size_t need = 0;
    (void)uq_quicfl_receive_workspace_bytes(n, D, &need);
    if (!(hooks & 7) && jp.use && ws && ws_bytes >= need) return quicfl_recv_jump(r, x_kind, jp, (char*)ws, st);
    if (!(hooks & 2) && n <= kQfTeamMaxN && D >= (int64_t)kMtN * kQrRuns && D <= kQfTeamMaxD) {
        const dim3 grid((unsigned)n), block(64 * kQfTeamWaves);
        if (x_kind == 0) hipLaunchKernelGGL(quicfl_recv_team_kernel<0>, grid, block, 0, st, r);
        else if (x_kind == 1) hipLaunchKernelGGL(quicfl_recv_team_kernel<1>, grid, block, 0, st, r);
        else hipLaunchKernelGGL(quicfl_recv_team_kernel<2>, grid, block, 0, st, r);
        return hip_check(hipGetLastError(), "quicfl_recv_team_kernel launch");
    }
    const dim3 grid((unsigned)((n + kQfWavesPerWG - 1) / kQfWavesPerWG)), block(64 * kQfWavesPerWG);
    if (x_kind == 0) hipLaunchKernelGGL(quicfl_recv_wave_kernel<0>, grid, block, 0, st, r);
    else if (x_kind == 1) hipLaunchKernelGGL(quicfl_recv_wave_kernel<1>, grid, block, 0, st, r);
    else hipLaunchKernelGGL(quicfl_recv_wave_kernel<2>, grid, block, 0, st, r);
    return hip_check(hipGetLastError(), "quicfl_recv_wave_kernel launch");
}

// KQ0s + KQ0j (the h stream, one block per run) + KQ2c + KQ2j + KQ2f
static int quicfl_recv_jump(const QflRecvArgs& r, int32_t x_kind, const QflJumpPlan& jp, char* wsb, hipStream_t st) {
    const int64_t n = r.n;
    const uint32_t* polys = nullptr;
    int rc = qfl_jump_polys(jp, true, &polys);
    if (rc) return rc;
    uint32_t* xs = (uint32_t*)wsb;
    uint32_t* parts = xs + (size_t)n * kMjX;
    QflJumpArgs ja{};
    ja.prng_seeds = r.prng_seeds;
    ja.polyA = polys;
    ja.polyB = polys;                                    // (unused: one kind)
    ja.xs = xs;
    ja.parts = parts;
    ja.R = jp.R;
    ja.n = n;
    ja.nstreams = 1;
    ja.kinds = 1;
    hipLaunchKernelGGL(quicfl_stream_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, ja);
    if ((rc = hip_check(hipGetLastError(), "quicfl_stream_kernel launch"))) return rc;
    hipLaunchKernelGGL(quicfl_jump_kernel, dim3((unsigned)(n * jp.R * kMjParts)), dim3(256), 0, st, ja);
    if ((rc = hip_check(hipGetLastError(), "quicfl_jump_kernel launch"))) return rc;
    QflRunArgs ra{};
    ra.parts = parts;
    ra.runinfo = (int32_t*)(parts + (size_t)n * jp.R * kMjParts * kMtN);
    ra.R = jp.R;
    ra.L = jp.L;
    const dim3 rgrid((unsigned)((n * jp.R + kQfWavesPerWG - 1) / kQfWavesPerWG)), blk(64 * kQfWavesPerWG);
    hipLaunchKernelGGL(quicfl_recv_count_kernel, rgrid, blk, 0, st, r, ra);
    if ((rc = hip_check(hipGetLastError(), "quicfl_recv_count_kernel launch"))) return rc;
    if (x_kind == 0) hipLaunchKernelGGL(quicfl_recv_runs_kernel<0>, rgrid, blk, 0, st, r, ra);
    else if (x_kind == 1) hipLaunchKernelGGL(quicfl_recv_runs_kernel<1>, rgrid, blk, 0, st, r, ra);
    else hipLaunchKernelGGL(quicfl_recv_runs_kernel<2>, rgrid, blk, 0, st, r, ra);
    if ((rc = hip_check(hipGetLastError(), "quicfl_recv_runs_kernel launch"))) return rc;
    hipLaunchKernelGGL(quicfl_recv_fin_kernel, dim3((unsigned)((n + kQfWavesPerWG - 1) / kQfWavesPerWG)), blk, 0, st, r,
                       ra);
    return hip_check(hipGetLastError(), "quicfl_recv_fin_kernel launch");
}

int uq_quicfl_prepare_f32(const int32_t* X, int64_t n, int64_t D, const float* recv_table, int32_t table_rows,
                          int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask, const float* exact_vals,
                          const float* scale, float* out, void* stream) {
    return uq_quicfl_receive_f32(X, 2, n, D, recv_table, table_rows, h_len, prng_seeds, exact_mask, exact_vals, 0, nullptr,
                                 scale, out, nullptr, stream);
}

int uq_rht_f32(const float* x, float* out, int64_t n, int64_t dim, int32_t inverse, const int8_t* signs,
               const int32_t* sign_row, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 clients per call");
    if (n == 0 || dim == 0) return UQ_OK;
    if (!x || !out || !signs) return fail(UQ_E_INVALID, "null pointer");
    const EdenLayout w = eden_layout(n, dim);
    if (inverse && dim != w.D) return fail(UQ_E_INVALID, "inverse RHT input length must be a power of two");
    // the transform uses the vector region only (no norm: the segmented-norm tables past
    // seg_off are not needed here)
    if (!ws || ws_bytes < w.seg_off) return fail(UQ_E_WORKSPACE, "workspace too small");
    FwhtArgs a{};
    a.in = x;
    a.signs = signs;
    a.sign_row = sign_row;
    a.scale = nullptr;
    a.D = w.D;
    a.dim = inverse ? w.D : dim;
    a.sqrtD = (float)std::sqrt((double)w.D);
    hipStream_t st = (hipStream_t)stream;
    float* buf = (float*)((char*)ws + w.vec_off);
    if (!inverse) {                                           // AS:123-141: pad, * diag, H
        float* res = nullptr;
        int rc = launch_fwht(a, n, false, buf, out, st, &res);
        if (rc || res == out) return rc;
        return hip_check(hipMemcpyAsync(out, buf, (size_t)n * w.D * sizeof(float), hipMemcpyDeviceToDevice, st),
                         "copy rht");
    }
    // AS:146-153: H, then * diag (the receiver's last pass with no scale)
    const int p = ilog2_pow2(w.D);
    int lo = 0, k = std::min(p, kFwhtLowBits);
    bool first = true;
    for (;;) {
        const bool last = lo + k >= p;
        const int cols = lo == 0 ? 1 : kFwhtCols;
        const int64_t tiles = w.D / (((int64_t)1 << k) * cols);
        FwhtArgs b = a;
        b.in = first ? (const void*)x : (const void*)buf;
        b.out = last ? out : buf;
        const dim3 grid((unsigned)tiles, (unsigned)n);
        if (last) fwht_dispatch<0, true, true>(grid, b, lo, k, st);
        else fwht_dispatch<0, false, false>(grid, b, lo, k, st);
        int rc = hip_check(hipGetLastError(), "fwht_pass_kernel launch");
        if (rc) return rc;
        if (last) break;
        first = false;
        lo += k;
        k = std::min(p - lo, kFwhtHighBits);
    }
    return UQ_OK;
}

int uq_eden_workspace_bytes(int64_t n, int64_t dim, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    *bytes_out = eden_layout(n, dim).total;
    return UQ_OK;
}

// The sender up to the norms: RHT (AS:123-141) and torch.norm (AS:329); *rot = the rotated
// vectors (one of the workspace's two vector buffers).
int eden_front(const float* x, int64_t n, int64_t dim, const EdenTables& tab, const int8_t* signs,
               const int32_t* sign_row, const EdenLayout& w, char* wsb, FwhtArgs& a, float** rot, hipStream_t st,
               const uint32_t* sbits = nullptr) {
    float* nrm = (float*)(wsb + w.nrm_off);
    a = FwhtArgs{};
    a.in = x;
    a.signs = signs;
    a.sign_row = sign_row;
    a.sbits = sbits;
    a.D = w.D;
    a.dim = dim;
    a.sqrtD = (float)std::sqrt((double)w.D);                 // np.sqrt(d) -> f32 operand
    a.tab = tab;
    float* vec = (float*)(wsb + w.vec_off);
    int rc = launch_fwht(a, n, false, vec, vec, st, rot);
    if (rc) return rc;
    if (w.seg) return launch_segnorm(*rot, n, w.D, wsb + w.seg_off, nrm, st);       // AS:329 torch.norm
    return launch_chainnorm(*rot, n, w.D, nrm, st);
}

int uq_eden_norm_workspace_bytes(int64_t n, int64_t D, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    if (n < 0 || D < 0) return fail(UQ_E_INVALID, "n and D must be >= 0");
    *bytes_out = segnorm_applies(n, D) ? segnorm_layout(n, D).total : 0;
    return UQ_OK;
}

int uq_eden_norm_f32(const float* v, int64_t n, int64_t D, int32_t mode, float* nrm, void* ws, size_t ws_bytes,
                     void* stream) {
    if (n < 0 || D < 0) return fail(UQ_E_INVALID, "n and D must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 clients per call");
    if (mode < 0 || mode > 2) return fail(UQ_E_INVALID, "mode must be 0 (auto), 1 (chains) or 2 (segmented)");
    if (n == 0) return UQ_OK;
    if (!v || !nrm) return fail(UQ_E_INVALID, "null pointer");
    const bool seg = mode == 2 || (mode == 0 && segnorm_applies(n, D));
    if (seg && !segnorm_applies(n, D))
        return fail(UQ_E_INVALID, "segmented norm: 1 <= n <= 256 and D a power of two >= 16384");
    if (D == 0) return hip_check(hipMemsetAsync(nrm, 0, (size_t)n * sizeof(float), (hipStream_t)stream), "norm fill");
    if (!seg) return launch_chainnorm(v, n, D, nrm, (hipStream_t)stream);
    if (!ws || ws_bytes < segnorm_layout(n, D).total) return fail(UQ_E_WORKSPACE, "workspace too small");
    return launch_segnorm(v, n, D, (char*)ws, nrm, (hipStream_t)stream);
}

int uq_eden_compress_f32(const float* x, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                         const int32_t* sign_row, uint8_t* bins, float* scale, void* ws, size_t ws_bytes,
                         void* stream) {
    return uq_eden_compress_f32_sb(x, n, dim, nbits, signs, sign_row, nullptr, bins, scale, ws, ws_bytes, stream);
}

int uq_rht_sign_bits(const int8_t* signs, int64_t rows, int64_t D, uint32_t* bits, void* stream) {
    if (rows < 0 || D < 0) return fail(UQ_E_INVALID, "rows and D must be >= 0");
    if (rows == 0 || D == 0) return UQ_OK;
    if (!signs || !bits) return fail(UQ_E_INVALID, "null pointer");
    const int64_t words = rows * ((D + 31) / 32);
    hipLaunchKernelGGL(rht_sign_bits_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       signs, rows, D, bits);
    return hip_check(hipGetLastError(), "rht_sign_bits_kernel launch");
}

int uq_eden_compress_f32_sb(const float* x, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                            const int32_t* sign_row, const uint32_t* sign_bits, uint8_t* bins, float* scale, void* ws,
                            size_t ws_bytes, void* stream) {
    EdenTables tab;
    int rc = eden_check(n, dim, nbits, signs, &tab);
    if (rc) return rc;
    if (n == 0 || dim == 0) return UQ_OK;
    if (!x || !bins || !scale) return fail(UQ_E_INVALID, "null pointer");
    const EdenLayout w = eden_layout(n, dim);
    if (!ws || ws_bytes < w.total) return fail(UQ_E_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* wsb = (char*)ws;
    float* nrm = (float*)(wsb + w.nrm_off);
    if (!w.seg && tab.nb == 1 && w.D % kNormChunk == 0) {
        // 1 bit, many clients: the norm, the bins and the dot in one read (KE2+4), then KE4 for
        // the clients it flags (a norm that is not positive and finite, an underflowing quotient)
        FwhtArgs a{};
        a.in = x;
        a.signs = signs;
        a.sign_row = sign_row;
        a.sbits = sign_bits;
        a.D = w.D;
        a.dim = dim;
        a.sqrtD = (float)std::sqrt((double)w.D);
        float* vec = (float*)(wsb + w.vec_off);
        float* rot = nullptr;
        rc = launch_fwht(a, n, false, vec, vec, st, &rot);                          // AS:123-141
        if (rc) return rc;
        int32_t* redo = (int32_t*)(wsb + w.redo_off);
        hipLaunchKernelGGL(eden_normdot1_kernel, dim3((unsigned)((n + kNormClients - 1) / kNormClients)),
                           dim3(kNDThreads), 0, st, rot, n, w.D, a.sqrtD, tab, nrm, bins, scale, redo);
        rc = hip_check(hipGetLastError(), "eden_normdot1_kernel launch");           // AS:329-335
        if (rc) return rc;
        return launch_eden_dotbins(rot, n, w.D, a.sqrtD, nrm, tab, bins, scale, st, redo);
    }
    FwhtArgs a;
    float* vec = nullptr;
    rc = eden_front(x, n, dim, tab, signs, sign_row, w, wsb, a, &vec, st, sign_bits);
    if (rc) return rc;
    if (w.seg && n <= kDotSegMaxN)                                                   // AS:329-335
        return launch_eden_dotseg(vec, n, w.D, a.sqrtD, nrm, tab, bins, scale, wsb + w.seg_off, st);
    return launch_eden_dotbins(vec, n, w.D, a.sqrtD, nrm, tab, bins, scale, st);
}

int uq_eden_decompress_f32(const uint8_t* bins, const float* scale, int64_t n, int64_t dim, int32_t nbits,
                           const int8_t* signs, const int32_t* sign_row, float* out, void* ws, size_t ws_bytes,
                           void* stream) {
    return uq_eden_decompress_f32_sb(bins, scale, n, dim, nbits, signs, sign_row, nullptr, out, ws, ws_bytes, stream);
}

int uq_eden_decompress_f32_sb(const uint8_t* bins, const float* scale, int64_t n, int64_t dim, int32_t nbits,
                              const int8_t* signs, const int32_t* sign_row, const uint32_t* sign_bits, float* out,
                              void* ws, size_t ws_bytes, void* stream) {
    EdenTables tab;
    int rc = eden_check(n, dim, nbits, signs, &tab);
    if (rc) return rc;
    if (n == 0 || dim == 0) return UQ_OK;
    if (!bins || !scale || !out) return fail(UQ_E_INVALID, "null pointer");
    const EdenLayout w = eden_layout(n, dim);
    if (!ws || ws_bytes < w.total) return fail(UQ_E_WORKSPACE, "workspace too small");
    FwhtArgs a{};
    a.in = bins;
    a.signs = signs;
    a.sign_row = sign_row;
    a.sbits = sign_bits;
    a.scale = scale;
    a.D = w.D;
    a.dim = dim;
    a.sqrtD = (float)std::sqrt((double)w.D);
    a.tab = tab;
    return launch_fwht(a, n, true, (float*)((char*)ws + w.vec_off), out, (hipStream_t)stream);   // AS:378-413
}

int uq_eden_f32(const float* x, float* out, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                const int32_t* sign_row, float* scale_out, void* ws, size_t ws_bytes, void* stream) {
    return uq_eden_f32_sb(x, out, n, dim, nbits, signs, sign_row, nullptr, scale_out, ws, ws_bytes, stream);
}

int uq_eden_f32_sb(const float* x, float* out, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                   const int32_t* sign_row, const uint32_t* sign_bits, float* scale_out, void* ws, size_t ws_bytes,
                   void* stream) {
    // compress (RHT, norm, bins + the MKL-order dot) then decompress: the receiver's first
    // pass reads the 1-byte bins KE4 wrote instead of the 4-byte rotated vector
    const EdenLayout w = eden_layout(n < 0 ? 0 : n, dim < 0 ? 0 : dim);
    uint8_t* bins = (uint8_t*)((char*)ws + w.bins_off);
    float* scale = scale_out ? scale_out : (float*)((char*)ws + w.scale_off);
    int rc = uq_eden_compress_f32_sb(x, n, dim, nbits, signs, sign_row, sign_bits, bins, scale, ws, ws_bytes, stream);
    if (rc) return rc;
    return uq_eden_decompress_f32_sb(bins, scale, n, dim, nbits, signs, sign_row, sign_bits, out, ws, ws_bytes, stream);
}

// ---- QUIC-FL sender ----------------------------------------------------------------------
// Workspace: the EDEN layout (rotated vectors, norms, segmented-norm region) + h [n][D] u8 +
// the jump path's blocks [n][R][3][624] u32 and run records [n][R][2] i32.
static size_t quicfl_h_off(int64_t n, int64_t dim) {
    return (eden_layout(n, dim).total + 255) & ~(size_t)255;
}
static size_t quicfl_jump_off(int64_t n, int64_t dim) {
    return (quicfl_h_off(n, dim) + (size_t)n * (size_t)eden_layout(n, dim).D + 255) & ~(size_t)255;
}
// jump region: streams [n][2][kMjX], parts [n][R][3][kMjParts][624], run records [n][R][2]
// (without the jump path: the local blocks after KQ1a, [n][624])
static size_t quicfl_ws_total(int64_t n, int64_t dim) {
    const QflJumpPlan p = qfl_jump_plan(n, eden_layout(n, dim).D);
    const size_t jb = p.use ? ((size_t)n * 2 * kMjX + (size_t)n * p.R * (3 * kMjParts * kMtN + 2)) * sizeof(uint32_t)
                            : (size_t)n * kMtN * sizeof(uint32_t);
    return quicfl_jump_off(n, dim) + jb;
}

int uq_quicfl_workspace_bytes(int64_t n, int64_t dim, size_t* bytes_out) {
    if (!bytes_out) return fail(UQ_E_INVALID, "null bytes_out");
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    *bytes_out = quicfl_ws_total(n, dim);
    return UQ_OK;
}

// The jump path's first two phases (KQ0s + KQ0j) depend only on the generators, so they are
// issued first, on the side stream, and run beside the RHT and the norm on the caller's stream
// (~80 us of small kernels for one 2^20 message); the runs wait for them.
struct QflJumpLaunch {
    bool use = false;
    bool passa = false;             // KQ1a runs on the side stream instead (the one-wave form)
    bool passa_runs = false;        // KQ1ar ran every run's pass A on the side stream (the jump path)
    QflJumpPlan jp;
    uint32_t* parts = nullptr;
    uint32_t* lstate = nullptr;     // KQ1a's local blocks
    SideStream* sb = nullptr;
};
// Which sender form a call takes (launch_quicfl_send): 0 the jump path, 1 the team kernel
// (KQ1t), 2 the one-wave kernel (KQ1).
static int qfl_send_form(int64_t n, int64_t D, bool jump_use) {
    const int hooks = g_quicfl_hooks.load();
    if (jump_use) return 0;
    const QflJumpPlan jp = qfl_jump_plan(n, D);
    if (!(hooks & 2) && ((hooks & 5) || !jp.use) && n <= kQfTeamMaxN && D >= (int64_t)kMtN * kQfRuns &&
        D <= kQfTeamMaxD)
        return 1;
    return 2;
}
static int quicfl_jump_fork(int64_t n, int64_t D, int64_t dim, const int32_t* prng_seeds, const uint32_t* px_state,
                            const int32_t* px_seeds, int32_t h_len, char* wsb, hipStream_t st, QflJumpLaunch* jl) {
    *jl = QflJumpLaunch{};
    const int hooks = g_quicfl_hooks.load();
    const QflJumpPlan jp = qfl_jump_plan(n, D);
    if ((hooks & 7) || !jp.use) {
        if (qfl_send_form(n, D, false) != 2) return UQ_OK;
        // the one-wave form: its pass A (h from the message seeds) beside the RHT and the norm
        SideStream* sb = nullptr;
        int rc = side_stream(&sb);
        if (rc) return rc;
        if ((rc = hip_check(hipEventRecord(sb->fork, st), "record fork"))) return rc;
        if ((rc = hip_check(hipStreamWaitEvent(sb->s, sb->fork, 0), "wait fork"))) return rc;
        QflSendArgs qa{};
        qa.prng_seeds = prng_seeds;
        qa.hbuf = (uint8_t*)(wsb + quicfl_h_off(n, dim));
        qa.h_len = h_len;
        qa.D = D;
        qa.n = n;
        uint32_t* ls = (uint32_t*)(wsb + quicfl_jump_off(n, dim));
        hipLaunchKernelGGL(quicfl_pass_a_kernel, dim3((unsigned)((n + kQfWavesPerWG - 1) / kQfWavesPerWG)),
                           dim3(64 * kQfWavesPerWG), 0, sb->s, qa, ls);
        rc = hip_check(hipGetLastError(), "quicfl_pass_a_kernel launch");
        const int rj = hip_check(hipEventRecord(sb->join, sb->s), "record join");
        if (!rj) {
            jl->passa = true;                   // the guard and the wave launch wait on the join
            jl->lstate = ls;
            jl->sb = sb;
        } else if (hipEventRecord(sb->join, sb->s) == hipSuccess) {
            (void)hipStreamWaitEvent(st, sb->join, 0);
        }
        return rc ? rc : rj;
    }
    const uint32_t* polys = nullptr;
    int rc = qfl_jump_polys(jp, false, &polys);
    if (rc) return rc;
    SideStream* sb = nullptr;
    if ((rc = side_stream(&sb))) return rc;
    if ((rc = hip_check(hipEventRecord(sb->fork, st), "record fork"))) return rc;
    if ((rc = hip_check(hipStreamWaitEvent(sb->s, sb->fork, 0), "wait fork"))) return rc;
    auto join_on_error = [&](int err) {      // whatever reached the side stream finishes before st moves on
        if (hipEventRecord(sb->join, sb->s) == hipSuccess) (void)hipStreamWaitEvent(st, sb->join, 0);
        return err;
    };
    uint32_t* xs = (uint32_t*)(wsb + quicfl_jump_off(n, dim));
    uint32_t* parts = xs + (size_t)n * 2 * kMjX;
    QflJumpArgs ja{};
    ja.prng_seeds = prng_seeds;
    ja.px_state = px_state;
    ja.px_seeds = px_seeds;
    ja.polyA = polys;
    ja.polyB = polys + (size_t)jp.R * kMtN;
    ja.xs = xs;
    ja.parts = parts;
    ja.R = jp.R;
    ja.n = n;
    ja.nstreams = 2;
    ja.kinds = 3;
    hipLaunchKernelGGL(quicfl_stream_kernel, dim3((unsigned)((2 * n + 3) / 4)), dim3(256), 0, sb->s, ja);
    if ((rc = hip_check(hipGetLastError(), "quicfl_stream_kernel launch"))) return join_on_error(rc);
    hipLaunchKernelGGL(quicfl_jump_kernel, dim3((unsigned)(n * jp.R * 3 * kMjParts)), dim3(256), 0, sb->s, ja);
    if ((rc = hip_check(hipGetLastError(), "quicfl_jump_kernel launch"))) return join_on_error(rc);
    {   // KQ1ar: the runs' pass A (h) beside the RHT and the norm
        QflSendArgs qa{};
        qa.prng_seeds = prng_seeds;
        qa.hbuf = (uint8_t*)(wsb + quicfl_h_off(n, dim));
        qa.h_len = h_len;
        qa.D = D;
        qa.n = n;
        QflRunArgs ra{};
        ra.parts = parts;
        ra.R = jp.R;
        ra.L = jp.L;
        hipLaunchKernelGGL(quicfl_pass_a_runs_kernel, dim3((unsigned)((n * jp.R + kQfWavesPerWG - 1) / kQfWavesPerWG)),
                           dim3(64 * kQfWavesPerWG), 0, sb->s, qa, ra);
        if ((rc = hip_check(hipGetLastError(), "quicfl_pass_a_runs_kernel launch"))) return join_on_error(rc);
    }
    if ((rc = hip_check(hipEventRecord(sb->join, sb->s), "record join"))) return join_on_error(rc);
    jl->use = true;
    jl->passa_runs = true;
    jl->jp = jp;
    jl->parts = parts;
    jl->sb = sb;
    return UQ_OK;
}

static int launch_quicfl_send(QflSendArgs& q, int32_t x_kind, const QflJumpLaunch& jl, hipStream_t st);

// Once the fork has happened, the caller's stream waits on the side stream's join on every exit
// path: KQ0s / KQ0j write into the caller's workspace, which may be freed or reused after an
// early error return.  (Waiting twice on the join is harmless.)
struct QflJoinGuard {
    const QflJumpLaunch& jl;
    hipStream_t st;
    ~QflJoinGuard() {
        if (jl.use || jl.passa) (void)hipStreamWaitEvent(st, jl.sb->join, 0);
    }
};

int uq_quicfl_compress_f32(const float* x, int64_t n, int64_t dim, const int8_t* signs, const int32_t* sign_row,
                           const float* table_xp, const uint32_t* table_packed, int64_t table_numel, int32_t h_len,
                           float delta, const int32_t* prng_seeds, const uint32_t* px_state, const int32_t* px_seeds,
                           uint32_t* px_state_out, void* X, int32_t x_kind, uint8_t* exact_mask, float* exact_vals,
                           int32_t* exact_count, float* scale, int32_t* info, void* ws, size_t ws_bytes,
                           void* stream) {
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 messages per call");
    if (dim > ((int64_t)1 << 28)) return fail(UQ_E_INVALID, "dim must be <= 2^28");
    if (h_len < 1 || h_len > 256) return fail(UQ_E_INVALID, "h_len must be 1..256");
    if (table_numel < h_len || table_numel % h_len) return fail(UQ_E_INVALID, "table_numel must be a multiple of h_len");
    if (table_numel >= ((int64_t)1 << 24)) return fail(UQ_E_INVALID, "table_numel must be below 2^24");
    if (x_kind != 0 && x_kind != 1) return fail(UQ_E_INVALID, "x_kind must be 0 (int64) or 1 (uint8)");
    if (n == 0 || dim == 0) return UQ_OK;
    if (!x || !signs || !table_xp || !prng_seeds || !X || !exact_mask || !exact_vals || !exact_count || !scale || !info)
        return fail(UQ_E_INVALID, "null pointer");
    if (!px_state && !px_seeds) return fail(UQ_E_INVALID, "px_state or px_seeds is required");
    const EdenLayout w = eden_layout(n, dim);
    const size_t hoff = quicfl_h_off(n, dim);
    if (!ws || ws_bytes < quicfl_ws_total(n, dim)) return fail(UQ_E_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* wsb = (char*)ws;
    QflJumpLaunch jl;
    int rc = quicfl_jump_fork(n, w.D, dim, prng_seeds, px_state, px_seeds, h_len, wsb, st, &jl);
    if (rc) return rc;
    const QflJoinGuard join_guard{jl, st};
    FwhtArgs a;
    float* rot = nullptr;
    rc = eden_front(x, n, dim, EdenTables{}, signs, sign_row, w, wsb, a, &rot, st);     // AS:460-470
    if (rc) return rc;
    QflSendArgs q{};
    q.rot = rot;
    q.nrm = (const float*)(wsb + w.nrm_off);
    q.tab = (const float2*)table_xp;
    q.tabp = table_packed;
    q.numel = table_numel;
    q.half = ((table_numel / h_len) - 1) * h_len / 2;                                        // AS:443
    q.h_len = h_len;
    q.delta = delta;
    q.sqrtD = (float)std::sqrt((double)w.D);                                                  // np.sqrt(D) -> f32
    q.prng_seeds = prng_seeds;
    q.px_state = px_state;
    q.px_seeds = px_seeds;
    q.px_state_out = px_state_out;
    q.hbuf = (uint8_t*)(wsb + hoff);
    q.X = X;
    q.x_kind = x_kind;
    q.mask = exact_mask;
    q.ev = exact_vals;
    q.ecount = exact_count;
    q.scale = scale;
    q.info = info;
    q.D = w.D;
    q.n = n;
    return launch_quicfl_send(q, x_kind, jl, st);
}

// By batch size and the plan's cost model: the jump path (KQ0s + KQ0j + KQ1j + KQ1f: every run
// of every message at once from jumped stream blocks) when it beats a wave per message, else up
// to 256 the team kernel KQ1t (scouts + runs in one workgroup per message), batches a wave per
// message (KQ1).  Test hooks: bit 1 the
// one-wave kernel, bit 2 (or bit 0, whose timeouts only the team's runs can report) KQ1t.
static int launch_quicfl_send(QflSendArgs& q, int32_t x_kind, const QflJumpLaunch& jl, hipStream_t st) {
    const int hooks = g_quicfl_hooks.load();
    q.force_timeout = hooks & 1;
    const int64_t n = q.n;
    const QflJumpPlan jp = qfl_jump_plan(n, q.D);
    if (jl.use) {
        int rc = hip_check(hipStreamWaitEvent(st, jl.sb->join, 0), "wait join");   // KQ0s + KQ0j done
        if (rc) return rc;
        QflRunArgs ra{};
        ra.parts = jl.parts;
        ra.runinfo = (int32_t*)(jl.parts + (size_t)n * jl.jp.R * 3 * kMjParts * kMtN);
        ra.R = jl.jp.R;
        ra.L = jl.jp.L;
        ra.passa_done = jl.passa_runs ? 1 : 0;
        const dim3 rgrid((unsigned)((n * jl.jp.R + kQfWavesPerWG - 1) / kQfWavesPerWG)), blk(64 * kQfWavesPerWG);
        const bool w2 = n * jl.jp.R > kQfRunWaves1;
#define UQ_QRUNS(XK)                                                                                        \
    if (w2) hipLaunchKernelGGL((quicfl_send_runs_kernel<XK, true>), rgrid, blk, 0, st, q, ra);               \
    else hipLaunchKernelGGL((quicfl_send_runs_kernel<XK, false>), rgrid, blk, 0, st, q, ra);
        if (x_kind == 2) { UQ_QRUNS(2) } else if (x_kind == 0) { UQ_QRUNS(0) } else { UQ_QRUNS(1) }
#undef UQ_QRUNS
        rc = hip_check(hipGetLastError(), "quicfl_send_runs_kernel launch");
        if (rc) return rc;
        hipLaunchKernelGGL(quicfl_send_fin_kernel, dim3((unsigned)((n + kQfWavesPerWG - 1) / kQfWavesPerWG)), blk, 0, st,
                           q, ra);
        return hip_check(hipGetLastError(), "quicfl_send_fin_kernel launch");
    }
    if (!(hooks & 2) && ((hooks & 5) || !jp.use) && n <= kQfTeamMaxN && q.D >= (int64_t)kMtN * kQfRuns &&
        q.D <= kQfTeamMaxD) {
        if (x_kind == 2)
            hipLaunchKernelGGL(quicfl_send_team_kernel<2>, dim3((unsigned)n), dim3(64 * kQfTeamWaves), 0, st, q);
        else if (x_kind == 0)
            hipLaunchKernelGGL(quicfl_send_team_kernel<0>, dim3((unsigned)n), dim3(64 * kQfTeamWaves), 0, st, q);
        else
            hipLaunchKernelGGL(quicfl_send_team_kernel<1>, dim3((unsigned)n), dim3(64 * kQfTeamWaves), 0, st, q);
        return hip_check(hipGetLastError(), "quicfl_send_team_kernel launch");
    }
    const dim3 grid((unsigned)((n + kQfWavesPerWG - 1) / kQfWavesPerWG));
    if (jl.passa) {                                  // KQ1a (pass A) ran on the side stream
        const int rc = hip_check(hipStreamWaitEvent(st, jl.sb->join, 0), "wait join");
        if (rc) return rc;
        q.lstate = jl.lstate;
    }
    if (x_kind == 2)
        hipLaunchKernelGGL(quicfl_send_wave_kernel<2>, grid, dim3(64 * kQfWavesPerWG), 0, st, q);
    else if (x_kind == 0)
        hipLaunchKernelGGL(quicfl_send_wave_kernel<0>, grid, dim3(64 * kQfWavesPerWG), 0, st, q);
    else
        hipLaunchKernelGGL(quicfl_send_wave_kernel<1>, grid, dim3(64 * kQfWavesPerWG), 0, st, q);
    return hip_check(hipGetLastError(), "quicfl_send_wave_kernel launch");
}

// QUICFL_quantize (AS:814-832) for a batch: the sender as uq_quicfl_compress_f32 with the
// receiver fused into its stage 2 (no second h stream, no message in HBM), then the receiver's
// inverse RHT into out [n][dim].
int uq_quicfl_quantize_f32(const float* x, int64_t n, int64_t dim, const int8_t* signs, const int32_t* sign_row,
                           const float* table_xp, const uint32_t* table_packed, int64_t table_numel, int32_t h_len,
                           float delta, const float* recv_table, int32_t recv_numel, const int32_t* prng_seeds,
                           const uint32_t* px_state, const int32_t* px_seeds, uint32_t* px_state_out, float* out,
                           float* scale, int32_t* info, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || dim < 0) return fail(UQ_E_INVALID, "n and dim must be >= 0");
    if (n > 65535) return fail(UQ_E_INVALID, "at most 65535 messages per call");
    if (dim > ((int64_t)1 << 28)) return fail(UQ_E_INVALID, "dim must be <= 2^28");
    if (h_len < 1 || h_len > 256) return fail(UQ_E_INVALID, "h_len must be 1..256");
    if (table_numel < h_len || table_numel % h_len) return fail(UQ_E_INVALID, "table_numel must be a multiple of h_len");
    if (table_numel >= ((int64_t)1 << 24)) return fail(UQ_E_INVALID, "table_numel must be below 2^24");
    if (recv_numel < 1 || recv_numel > kQflRecvTab) return fail(UQ_E_INVALID, "receiver table must hold 1..1024 entries");
    if (n == 0 || dim == 0) return UQ_OK;
    if (!x || !signs || !table_xp || !recv_table || !prng_seeds || !out || !info)
        return fail(UQ_E_INVALID, "null pointer");
    if (!px_state && !px_seeds) return fail(UQ_E_INVALID, "px_state or px_seeds is required");
    const EdenLayout w = eden_layout(n, dim);
    const size_t hoff = quicfl_h_off(n, dim);
    if (!ws || ws_bytes < quicfl_ws_total(n, dim)) return fail(UQ_E_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* wsb = (char*)ws;
    QflJumpLaunch jl;
    int rc = quicfl_jump_fork(n, w.D, dim, prng_seeds, px_state, px_seeds, h_len, wsb, st, &jl);
    if (rc) return rc;
    const QflJoinGuard join_guard{jl, st};
    FwhtArgs a;
    float* rot = nullptr;
    rc = eden_front(x, n, dim, EdenTables{}, signs, sign_row, w, wsb, a, &rot, st);     // AS:460-470
    if (rc) return rc;
    QflSendArgs q{};
    q.rot = rot;
    q.nrm = (const float*)(wsb + w.nrm_off);
    q.tab = (const float2*)table_xp;
    q.tabp = table_packed;
    q.numel = table_numel;
    q.half = ((table_numel / h_len) - 1) * h_len / 2;                                        // AS:443
    q.h_len = h_len;
    q.delta = delta;
    q.sqrtD = (float)std::sqrt((double)w.D);
    q.prng_seeds = prng_seeds;
    q.px_state = px_state;
    q.px_seeds = px_seeds;
    q.px_state_out = px_state_out;
    q.hbuf = (uint8_t*)(wsb + hoff);
    q.scale = scale;
    q.info = info;
    q.D = w.D;
    q.n = n;
    q.rtab = recv_table;
    q.rtab_n = recv_numel;
    q.pre = rot;                       // in place: a coordinate's rot is loaded a round before its value is stored
    rc = launch_quicfl_send(q, 2, jl, st);              // (2: the fused instances)                 AS:455-503, 526-532
    if (rc) return rc;
    // AS:533-535: the receiver's inverse RHT (H, then * diag), [:dim]; D = 2^22 as 14 + 8 bits
    const int p = ilog2_pow2(w.D);
    int lo = 0, k = p == kFwhtLow16Bits + kFwhtHighBits ? kFwhtLow16Bits : std::min(p, kFwhtLowBits);
    for (;;) {
        const bool last = lo + k >= p;
        const int cols = lo == 0 ? 1 : kFwhtCols;
        const int64_t tiles = w.D / (((int64_t)1 << k) * cols);
        FwhtArgs b{};
        b.in = rot;
        b.out = last ? out : rot;
        b.signs = signs;
        b.sign_row = sign_row;
        b.scale = nullptr;
        b.D = w.D;
        b.dim = dim;
        b.sqrtD = q.sqrtD;
        const dim3 grid((unsigned)tiles, (unsigned)n);
        if (last) fwht_dispatch<0, true, true>(grid, b, lo, k, st);
        else fwht_dispatch<0, false, false>(grid, b, lo, k, st);
        rc = hip_check(hipGetLastError(), "fwht_pass_kernel launch");
        if (rc || last) return rc;
        lo += k;
        k = std::min(p - lo, kFwhtHighBits);
    }
}

// xxHash64 (the public XXH64 algorithm), for AS:457's prng seed
static inline uint64_t xxh_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t xxh_read64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
static inline uint32_t xxh_read32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

uint64_t uq_xxh64(const void* data, size_t len, uint64_t seed) {
    const uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                   P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
    auto round = [&](uint64_t acc, uint64_t lane) { return xxh_rotl(acc + lane * P2, 31) * P1; };
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        while (p + 32 <= end) {
            v1 = round(v1, xxh_read64(p));
            v2 = round(v2, xxh_read64(p + 8));
            v3 = round(v3, xxh_read64(p + 16));
            v4 = round(v4, xxh_read64(p + 24));
            p += 32;
        }
        h = xxh_rotl(v1, 1) + xxh_rotl(v2, 7) + xxh_rotl(v3, 12) + xxh_rotl(v4, 18);
        for (uint64_t v : {v1, v2, v3, v4}) h = (h ^ round(0, v)) * P1 + P4;
    } else {
        h = seed + P5;
    }
    h += (uint64_t)len;
    for (; p + 8 <= end; p += 8) h = xxh_rotl(h ^ round(0, xxh_read64(p)), 27) * P1 + P4;
    if (p + 4 <= end) {
        h = xxh_rotl(h ^ ((uint64_t)xxh_read32(p) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; ++p) h = xxh_rotl(h ^ ((uint64_t)*p * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

}  // extern "C"
