// Experiment (tools/, not shipped): the XCD-resident single-read form of K1 + K2
//  as a data-flow SKELETON, to decide whether the
// real kernel is worth building.  It is an optimistic bound: every HBM byte, LDS image,
// barrier and the bulk of the per-element arithmetic of the real form are here, but the
// exact-scan machinery that only some tiles need (tie walks, irregular tiles, records) is
// not, and the L1 is a plain sum instead of torch's cascade.
//
// Persistent grid: 256 workgroups x 1024 threads (one per CU, 128 KB of LDS each).  A
// workgroup reads its XCD from HW_REG_XCC_ID and takes a slot in its XCD's team (32 CUs).
// Team t quantizes clients t, t+8, ...: slot s holds elements [s*32768, (s+1)*32768) of the
// client (8 tiles of 4096) -- the client's 4 MiB is read from HBM ONCE, into LDS.  The next
// client's slice is prefetched into 32 VGPRs per thread while the current one is processed.
// Per client (3 team barriers, counters in global memory, payloads via sc1 atomics):
//   stage slice -> LDS image | |x| partial -> barrier 1 -> L1 from the 32 partials
//   pass 1 (x/den Markstein, floor, frac, fp64 chain per row; mp kept in registers)
//     -> 8 approximate tile sums -> barrier 2 -> approximate prefixes P'_t (wave scan of 256)
//   map pass (two fp64 chains per row in P'_t's binade, tie ballots, block scan)
//     -> 8 maps -> barrier 3 -> fold: one wave composes the 256 maps (wave scans)
//   pass 2 (sequential fp64 prefix per row, crossing test, output table, code) -> LDS
//     -> coalesced non-temporal stores of q and the int8 codes.
// mode bit 0: skip the barrier waits (pure data flow: wrong numbers, timing bound).
// Spins are bounded: a timeout sets err[0] and the workgroup continues (no hang).
#include "../../unbiased-quantization-distributed-mean-estimation_amd/csrc/uq_dme.hip"

namespace xcd {
// W workgroups per CU (1 or 2): 1024/W threads, a team of 32*W workgroups per XCD, a slice
// of 32768/W elements (8/W tiles) each; W = 2 keeps two clients in flight per CU.
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_rlx64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// team barrier: payload stores (sc1) acknowledged, then one counter add; wait for target
__device__ void team_barrier(uint32_t* cnt, uint32_t target, uint32_t* err, bool wait) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");     // s_waitcnt: payload acked
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wait && ld_rlx(err) == 0u) {                             // after a timeout: stop waiting
            uint32_t spins = 0;
            while (ld_rlx(cnt) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) { atomicOr(err, 1u); break; }
            }
        }
    }
    __syncthreads();
}

template <int W>
struct Lds {
    static constexpr int kT = 1024 / W, kSlice = 32768 / W, kTilesPer = 8 / W;
    float img[kSlice];                    // 8 tiles x 4096, swizzled rows (x, then q)
    float tab[kTab];
    double wsum[kT / kWave];              // per-wave sums
    double tsum[kTilesPer];               // tile sums / maps of this slice
    double pre[kTilesPer];                // tile starts
    double misc[4];
    uint64_t tmask[kT / kWave];
};

template <int W>
__global__ void __launch_bounds__(1024 / W, 4)     // 4 waves per SIMD: W workgroups per CU
xcd_kernel(const float* __restrict__ x, float* __restrict__ q, int8_t* __restrict__ codes, int64_t n, int64_t d,
           float fm, const float* __restrict__ Xs, float* __restrict__ l1out, uint32_t* ctrl, float* part,
           uint64_t* tiles_buf, uint64_t* maps_buf, uint32_t* err, int mode) {
    constexpr int kT = 1024 / W, kTeam = 32 * W, kSlice = 32768 / W, kTilesPer = 8 / W, kHalf = kT / 256;
    __shared__ Lds<W> s;
    __shared__ uint32_t s_slot, s_team;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const bool wait = !(mode & 1);
    // ---- team registration: slot within this XCD's team ----------------------------
    if (tid == 0) {
        const uint32_t t = xcc_id();
        s_team = t;
        s_slot = __hip_atomic_fetch_add(&ctrl[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint32_t team = s_team, slot = s_slot;
    if (slot >= (uint32_t)kTeam) {                       // placement not 32 per XCD: give up
        if (tid == 0) atomicOr(err, 4u);
        return;
    }
    uint32_t* bar = ctrl + 16 + team * 16;               // (team counters: 64 B apart)               // this team's barrier counter
    const int64_t nclient = (n - team + 7) / 8;          // clients team, team+8, ...
    const int64_t off = (int64_t)slot * kSlice;
    f4v pf[8];
    auto prefetch = [&](int64_t c) {
        const f4v* src = reinterpret_cast<const f4v*>(x + c * d + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = __builtin_nontemporal_load(src + tid + j * kT);
    };
    if (nclient > 0) prefetch(team);
    uint32_t phase = 0;
    for (int64_t ci = 0; ci < nclient; ++ci) {
        const int64_t c = team + ci * 8;
        // ---- stage: float4 f = tid + j*1024 -> element 4f: tile e/4096, row, column --
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + j * kT;
            const int t = f >> 10, r = (f >> 2) & 255, c4 = f & 3;
            *reinterpret_cast<f4v*>(&s.img[t * kQTile + swz(r, c4)]) = pf[j];
        }
        if (ci + 1 < nclient) prefetch(c + 8);           // next client's slice in flight
        __syncthreads();
        // this thread's rows: row t of tile (tid>>8) and of tile 4 + (tid>>8)
        const int rr = tid & 255, t0 = tid >> 8, t1 = kHalf + (tid >> 8);
        // ---- |x| partial -> barrier 1 -> L1 -----------------------------------------
        float a = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int tb = (h ? t1 : t0) * kQTile;
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const f4v v = *reinterpret_cast<const f4v*>(&s.img[tb + swz(rr, k4)]);
                a += (fabsf(v.x) + fabsf(v.y)) + (fabsf(v.z) + fabsf(v.w));
            }
        }
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) s.wsum[wid] = a;
        __syncthreads();
        if (tid == 0) {
            float p = 0.f;
            for (int w = 0; w < kT / kWave; ++w) p += (float)s.wsum[w];
            __hip_atomic_store(part + c * kTeam + slot, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        phase += kTeam;
        team_barrier(bar, phase, err, wait);
        if (tid < kWave) {
            float v = lane < kTeam ? __hip_atomic_load(part + c * kTeam + lane, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) : 0.f;
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) s.misc[0] = v;
        }
        __syncthreads();
        const float L = (float)s.misc[0];
        if (slot == 0 && tid == 0) l1out[c] = L;
        const DivPlan dp = div_plan(L);
        for (int k = tid; k < kTab; k += kT) s.tab[k] = (L * (float)k) / fm;
        // ---- pass 1: mp (sign folded) over the x row in LDS, approximate row sums --------
        double rs[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int tb = (h ? t1 : t0) * kQTile;
            double c0 = 0.0;
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const f4v v4 = *reinterpret_cast<const f4v*>(&s.img[tb + swz(rr, k4)]);
                const float xs[4] = {v4.x, v4.y, v4.z, v4.w};
                float vs[4];
                div4(xs, dp, vs);
                float ms[4];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const float mp = fm * fabsf(vs[cc]);
                    ms[cc] = vs[cc] < 0.f ? -mp : mp;
                    c0 += (double)(mp - floorf(mp));
                }
                *reinterpret_cast<f4v*>(&s.img[tb + swz(rr, k4)]) = f4v{ms[0], ms[1], ms[2], ms[3]};
            }
            rs[h] = c0;
        }
        // tile sums: a tile = 4 waves (256 rows); waves 0-3 hold tiles 0-3 (h=0) and 4-7 (h=1)
        double w0 = rs[0], w1 = rs[1];
        for (int o = 32; o > 0; o >>= 1) { w0 += __shfl_xor(w0, o, 64); w1 += __shfl_xor(w1, o, 64); }
        __syncthreads();
        if (lane == 0) { s.wsum[wid] = w0; s.misc[0] = 0.0; }
        if (lane == 1) s.tmask[wid] = (uint64_t)__double_as_longlong(w1);
        __syncthreads();
        if (tid < kTilesPer) {
            const int tt = tid % kHalf;
            double v = 0.0;
            for (int w = 4 * tt; w < 4 * tt + 4; ++w)
                v += tid < kHalf ? s.wsum[w] : __longlong_as_double((long long)s.tmask[w]);
            st_rlx64(tiles_buf + (c * kTeam + slot) * kTilesPer + tid, (uint64_t)__double_as_longlong(v));
        }
        phase += kTeam;
        team_barrier(bar, phase, err, wait);
        // ---- approximate prefixes of my tiles: wave scan over the 256 tile sums -------
        if (tid < kWave) {
            double v[4];
            double run = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v[i] = __longlong_as_double((long long)ld_rlx64(tiles_buf + c * kTeam * kTilesPer + lane * 4 + i));
            }
            double sv = (v[0] + v[1]) + (v[2] + v[3]);
            double inc = wave_incl_scan(sv, lane);
            run = inc - sv;                               // exclusive start of lane's 4 tiles
            for (int i = 0; i < 4; ++i) {
                const int gt = lane * 4 + i;              // global tile index
                if (gt >= (int)slot * kTilesPer && gt < ((int)slot + 1) * kTilesPer) s.pre[gt - slot * kTilesPer] = run;
                run += v[i];
            }
        }
        __syncthreads();
        // ---- map pass: two chains per row in the binade of P'_t -----------------------
        double m0[2], m1[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const Binade B = binade_of(s.pre[h ? t1 : t0]);
            double c0 = B.b0, c1 = B.b1;
            const int tb = (h ? t1 : t0) * kQTile;
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const f4v m4 = *reinterpret_cast<const f4v*>(&s.img[tb + swz(rr, k4)]);
                const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const float mp = fabsf(mv[cc]);
                    const double f = (double)(mp - floorf(mp));
                    c0 += f;
                    c1 += f;
                }
            }
            m0[h] = c0 - B.b0;
            m1[h] = c1 - B.b1;
        }
        const uint64_t tm0 = __ballot(m0[0] != m1[0]), tm1 = __ballot(m0[1] != m1[1]);
        const double i0 = wave_incl_scan(m0[0], lane), i1 = wave_incl_scan(m0[1], lane);
        const double x0 = i0 - m0[0], x1 = i1 - m0[1];      // in-wave exclusive row prefixes
        __syncthreads();
        if (lane == kWave - 1) { s.wsum[wid] = i0; s.tmask[wid] = (uint64_t)__double_as_longlong(i1); }
        if (lane == 0) s.misc[1] = (double)(tm0 | tm1);
        __syncthreads();
        if (tid < kTilesPer) {
            const int tt = tid % kHalf;
            double v = 0.0;
            for (int w = 4 * tt; w < 4 * tt + 4; ++w)
                v += tid < kHalf ? s.wsum[w] : __longlong_as_double((long long)s.tmask[w]);
            st_rlx64(maps_buf + (c * kTeam + slot) * kTilesPer + tid, (uint64_t)__double_as_longlong(v));
        }
        phase += kTeam;
        team_barrier(bar, phase, err, wait);
        // ---- fold: one wave composes the 256 maps (as exact_fold_kernel's wave scan) ---
        if (tid < kWave) {
            uint64_t P = 0;
            uint64_t mvs[4];                                  // all 256 maps: one round trip
#pragma unroll
            for (int i = 0; i < 4; ++i) mvs[i] = ld_rlx64(maps_buf + c * kTeam * kTilesPer + i * kWave + lane);
#pragma unroll
            for (int blk = 0; blk < kTeam * kTilesPer; blk += kWave) {
                const uint64_t mv = mvs[blk / kWave];
                uint64_t dd0 = mv & ((1ull << 40) - 1ull), dd1 = dd0 + (mv & 1ull);
#pragma unroll
                for (int o = 1; o < kWave; o <<= 1) {
                    const uint64_t f0 = shfl_up64(dd0, o), f1 = shfl_up64(dd1, o);
                    if (lane >= o) {
                        const uint64_t n0 = f0 + ((f0 & 1ull) ? dd1 : dd0);
                        const uint64_t n1 = f1 + ((f1 & 1ull) ? dd0 : dd1);
                        dd0 = n0;
                        dd1 = n1;
                    }
                }
                const uint64_t st = P + ((P & 1ull) ? shfl_up64(dd1, 1) : shfl_up64(dd0, 1));
                const int gt = blk + lane;
                if (gt >= (int)slot * kTilesPer && gt < ((int)slot + 1) * kTilesPer)
                    s.pre[gt - slot * kTilesPer] = s.pre[gt - slot * kTilesPer] + (double)(st & 1023ull) * 0x1p-60;
                P += (P & 1ull) ? readlane64(dd1, kWave - 1) : readlane64(dd0, kWave - 1);
            }
        }
        __syncthreads();
        // ---- pass 2: exact-prefix stand-in from the fold, crossing test, outputs --------
        const float Xv = Xs[c];
        float kmax = 0.f;
        int8_t* cd8 = codes + c * d + off;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int tt = h ? t1 : t0;
            double sacc = s.pre[tt] + (h ? x1 : x0);
            float fprev = floorf((float)sacc - Xv);
            uint32_t cw[4];
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const f4v m4 = *reinterpret_cast<const f4v*>(&s.img[tt * kQTile + swz(rr, k4)]);
                const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
                float o[4];
                uint32_t w = 0u;
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const float mp = fabsf(mv[cc]);
                    const float fla = floorf(mp);
                    sacc += (double)(mp - fla);
                    const float fcur = floorf((float)sacc - Xv);
                    const float r = (fcur - fprev == 1.0f) ? 1.0f : 0.0f;
                    fprev = fcur;
                    const float kf = fla + r;
                    kmax = fmaxf(kmax, kf);
                    o[cc] = copysignf(s.tab[(int)kf & (kTab - 1)], mv[cc]);
                    w |= code_of(mv[cc], kf) << (8 * cc);
                }
                cw[k4] = w;
                *reinterpret_cast<f4v*>(&s.img[tt * kQTile + swz(rr, k4)]) = f4v{o[0], o[1], o[2], o[3]};
            }
            const u32x4v v = {cw[0], cw[1], cw[2], cw[3]};           // this row's 16 codes
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(cd8 + tt * kQTile + rr * kQItems));
        }
        __syncthreads();
        // ---- stores: q coalesced from the LDS image, codes 16 B per row ---------------
        f4v* qd = reinterpret_cast<f4v*>(q + c * d + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + j * kT;
            const int t = f >> 10, r = (f >> 2) & 255, c4 = f & 3;
            __builtin_nontemporal_store(*reinterpret_cast<const f4v*>(&s.img[t * kQTile + swz(r, c4)]), qd + f);
        }
        __syncthreads();                                   // image free for the next stage
        (void)kmax;
    }
}
}  // namespace xcd

extern "C" int exp_xcd(const float* x, float* q, int8_t* codes, int64_t n, int64_t d, float fm, const float* X,
                       float* l1out, void* ws, int mode, void* stream) {
    if (d != 32768 * 32) return -1;
    const int W = (mode & 2) ? 2 : 1;
    char* w = (char*)ws;
    uint32_t* ctrl = (uint32_t*)w;                               // [0,16) team slots, then 8 x 16 counters
    uint32_t* err = ctrl + 16 * 9;
    float* part = (float*)(w + 4096);
    uint64_t* tiles = (uint64_t*)(w + 4096 + ((n * 64 * 4 + 255) & ~255));
    uint64_t* maps = tiles + n * 256;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(ctrl, 0, 16 * 10 * 4, st) != hipSuccess) return -2;
    if (W == 1)
        hipLaunchKernelGGL(xcd::xcd_kernel<1>, dim3(256), dim3(1024), 0, st, x, q, codes, n, d, fm, X, l1out, ctrl,
                           part, tiles, maps, err, mode);
    else
        hipLaunchKernelGGL(xcd::xcd_kernel<2>, dim3(512), dim3(512), 0, st, x, q, codes, n, d, fm, X, l1out, ctrl,
                           part, tiles, maps, err, mode);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
