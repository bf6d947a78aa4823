// uq_quicfl_kernels.h — QUIC-FL sender and receiver streams.  Included by
// uq_dme.hip inside its anonymous namespace, after uq_eden_kernels.h (the RHT and the norm are
// EDEN's).
//
// Reference (AS = NMSE_Results/Codes/All_Schemes.py), QuicFLSender.compress AS:455-503:
//   AS:457      prng_seed = xxh64(str(seed)) % 2^16; local generator seeded with it
//   AS:460-470  RHT (EDEN's KE1 passes), h = randint(0, h_len, (D,), local) = word % h_len,
//               scale = sqrt(D) / norm  ->  Tensor.__rtruediv__: f32(1 / norm) * f32(sqrt(D))
//   AS:472-481  v = rot * scale; exact = v > f32(T) | v < -f32(T), T = norm.ppf(1 - 2^-9);
//               q = v / f32(delta) (IEEE), q[exact] = 0
//   AS:483-484  p = q - floor(q); floor(q) + bernoulli(p, local): the local stream continues
//               after the D randint words, one word per element, 1 iff low24(w) * 2^-24 < p
//   AS:486-490  idx = ((iq * h_len) + h) + half in f32, .long(); X = table_X[idx] +
//               bernoulli(table_p[idx]) from the GLOBAL generator (one word per element), .long()
// QuicFLReceiver.decompress AS:526-532 (before its inverse RHT): h from the same local stream,
//   v = recv_table[X * h_len + h], exact overrides, v / scale.
//
// Both are serial in their MT19937 streams (ATen's mt19937: 624-word blocks, each twisted
// from the previous), so the unit of parallelism is the message: ONE WAVE per message (or, for
// a few messages, a team of waves: KQ1t), no workgroup barriers.  A wave keeps a block in
// registers (word 64 g + lane in VGPR g) and twists it with lane moves (mt_twist_reg).  A
// 624-element round takes the words of its elements from the current block and the next one:
// pass A and the receiver read word e of the round's own block (no lane move); pass B's words
// start at an offset, read from a two-block LDS ring.
//   KQ1 quicfl_send_wave_kernel     pass A: h = word % h_len (u8 scratch); pass B: the local
//       stream (words D..2D-1) and the global stream side by side, each lane 10 elements of
//       the round; the (X, p) table gather of round c is issued before round c-1 is finished
//       (its X, exact flag and value stored then), so the gather latency overlaps a round of
//       twisting.  Exact values are compacted in index order by wave ballots.
//   KQ2 quicfl_recv_wave_kernel     the receiver's h stream and table lookup (LDS table).
//   The global generator starts from ATen's state (left, next, 624 words): the first left - 1
//   words are state[next ..], then twisted blocks; the state after the D draws is written back
//   for the host to restore into torch's generator.

constexpr int kMtN = 624;              // MT19937 state words
constexpr int kMtGroups = 10;          // 64-word groups per block (the last one 48 words)
constexpr int kQfWavesPerWG = 4;       // messages per workgroup (one wave each)
constexpr float kQflExactT = 2.8856349124267573f;   // f32(norm.ppf(1 - 2^-9)) (AS:475-478)
constexpr int kQfStateWords = 2 + kMtN;             // (left, next, words) per generator state
constexpr int kQflRecvTab = 1024;                    // receiver table entries (LDS), as kQflTab below

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}

// new word = c ^ twist(a, b) (ATen mt19937::next_state)
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
}

// torch's uniform in bernoulli: (w & 0xFFFFFF) * 2^-24 (computed in double, then compared with
// the f32 p): both sides are exact f32 values, so the f32 comparison is the same test
__device__ __forceinline__ float u24(uint32_t w) { return (float)(w & 0xFFFFFFu) * 0x1p-24f; }

__device__ __forceinline__ void mt_seed(uint32_t* mt, uint32_t seed) {     // init_genrand, one lane
    mt[0] = seed;
    for (int i = 1; i < kMtN; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

// A block in registers: word 64 g + lane in s[g] (g = 9: lanes < 48).  One wave twists it into
// the next block (ATen's next_state): word i takes s[i], s[i + 1] (old) and s[(i + 397) % 624],
// which is old for i < 227 and new (227 words back) otherwise.  Operands move between lanes by
// a DPP wave shift (the +1 neighbour) and ds_bpermute (the +13 / +29 lane rotations of the c
// operand); the groups' dependencies (group g >= 4 needs new groups g-4 and g-3) leave four
// levels.  tools/exp/mt_twist_bench.hip: 0.59 us per twist (+ temper) against 1.39 us for the
// LDS in-place form with its wave fences, bit-identical to a host MT19937.
__device__ __forceinline__ uint32_t mt_perm(uint32_t v, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
__device__ __forceinline__ void mt_twist_reg(uint32_t (&s)[kMtGroups], int lane) {
    const int r13 = (lane + 13) & 63, r29 = (lane + 29) & 63;
    uint32_t b[kMtGroups], N[kMtGroups];
#pragma unroll
    for (int g = 0; g < kMtGroups; ++g) {                       // b = old word i + 1
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s[g], 0x130, 0xF, 0xF, false);  // wave_shl:1
        const uint32_t first = g + 1 < kMtGroups ? (uint32_t)__builtin_amdgcn_readlane((int)s[g + 1], 0) : 0u;
        b[g] = lane == 63 ? first : nx;
    }
#pragma unroll
    for (int g = 0; g < 3; ++g) {                               // i < 192: c = old word i + 397
        const uint32_t t1 = mt_perm(s[g + 6], r13), t2 = mt_perm(s[g + 7], r13);
        N[g] = mt_mix(s[g], b[g], lane < 51 ? t1 : t2);
    }
    {                                                           // i = 192..255: old s[9] below 227, new N[0] above
        const uint32_t t1 = mt_perm(s[9], r13), t2 = mt_perm(N[0], r29);
        N[3] = mt_mix(s[3], b[3], lane < 35 ? t1 : t2);
    }
#pragma unroll
    for (int g = 4; g < kMtGroups; ++g) {                       // c = new word i - 227
        const uint32_t t1 = mt_perm(N[g - 4], r29), t2 = mt_perm(N[g - 3], r29);
        uint32_t bb = b[g];
        if (g == kMtGroups - 1) {                               // word 623 twists with the new word 0
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)N[0], 0);
            bb = lane == 47 ? n0 : bb;
        }
        N[g] = mt_mix(s[g], bb, lane < 35 ? t1 : t2);
    }
#pragma unroll
    for (int g = 0; g < kMtGroups; ++g) s[g] = N[g];
}
__device__ __forceinline__ void mt_load(uint32_t (&s)[kMtGroups], const uint32_t* src, int lane) {
#pragma unroll
    for (int g = 0; g < kMtGroups; ++g) {
        const int i = 64 * g + lane;
        s[g] = src[i < kMtN ? i : 0];
    }
}
__device__ __forceinline__ void mt_store(const uint32_t (&s)[kMtGroups], uint32_t* dst, int lane) {
#pragma unroll
    for (int g = 0; g < kMtGroups; ++g) {
        const int i = 64 * g + lane;
        if (i < kMtN) dst[i] = s[g];
    }
}

struct QflSendArgs {
    const float* rot;           // [n][D] rotated vectors (the RHT's output)
    const float* nrm;           // [n] torch.norm of each
    const float2* tab;          // [numel] (table_X, table_p) pairs
    const uint32_t* tabp;       // or [numel] packed (X << 25) | ceil(p * 2^24): X in 0..127, p in [0, 1]
    int64_t numel;
    int64_t half;               // AS:443 half_table_size
    int32_t h_len;
    float delta;                // f32(data['delta'])
    float sqrtD;                // f32(np.sqrt(D))
    const int32_t* prng_seeds;  // [n] local generator seeds (AS:457)
    const uint32_t* px_state;   // [n][2 + 624] global generator state per message, or null
    const int32_t* px_seeds;    // [n] seeds of fresh generators (when px_state is null)
    uint32_t* px_state_out;     // [n][2 + 624] state after the D draws, or null
    uint8_t* hbuf;              // [n][D] scratch: h
    void* X;                    // [n][D] int64 (x_kind 0) or uint8 (x_kind 1)
    int32_t x_kind;
    uint8_t* mask;              // [n][D] exact_indeces
    float* ev;                  // [n][D] exact values, compacted per message (first ecount[j])
    int32_t* ecount;            // [n]
    float* scale;               // [n]
    int32_t* info;              // [n] UQ_QFL_* flags
    int64_t D;
    int64_t n;
    int32_t force_timeout;      // test hook (uq_test_set_quicfl_hooks): team runs skip their waits
    // fused receiver (the drop-in, AS:814-832): when `pre` is set, stage 2 writes the receiver's
    // values before its inverse RHT, pre[i] = (exact ? v : rtab[X * h_len + h]) / scale
    // (AS:526-532), instead of X / mask / exact values: h is the sender's own (the receiver
    // regenerates the same randint words from the same seed, AS:465 / AS:528)
    const float* rtab;          // receiver table (rtab_n <= 1024 floats)
    int32_t rtab_n;
    float* pre;                 // [n][D] (may alias rot: each coordinate is read before it is written)
    // [n][624] the local stream's block after pass A, when KQ1a (quicfl_pass_a_kernel) ran pass A
    // on the side stream beside the RHT and the norm; null: KQ1 runs pass A itself
    const uint32_t* lstate;
};

// Round state carried from stage 1 (words, flags, gather issued) to stage 2 (X, stores).
struct QflRound {
    uint32_t t[kMtGroups][2];   // gathered (table_X, table_p) bits
    uint32_t wg[kMtGroups];     // tempered global words
    float v[kMtGroups];
    uint32_t ex;                // bit k: element k of this lane is exact
    uint32_t act;               // bit k: element k of this lane exists
    uint32_t hp[3];             // h of element k in byte k % 4 of hp[k / 4] (fused receiver)
};

__device__ __forceinline__ uint32_t qf_off(bool ok, uint32_t off) { return ok ? off : 0xFFFFFFFFu; }  // dropped

// Per-message constants of the sender's passes (wave-uniform).
struct QflCtx {
    int64_t row, D;
    int64_t qL, qG;             // block of the first pass-B word of round 0 (local, global)
    int rL, rG;                 // its slot
    __amdgpu_buffer_rsrc_t rr, rh, rm, rX, rt, rP;
    bool packed;
    float sc, fh, fhalf, fnumel;
    DivPlan dp, dps;            // / delta (AS:480), / scale (the fused receiver, AS:532)
    int32_t rtab_n;
    bool fused;
    int32_t numel;
    uint32_t h_len;
    bool hpow2;
};

template <int XK>
__device__ __forceinline__ QflCtx qfl_ctx(const QflSendArgs& a, int64_t j, int32_t gleft, int32_t gnext) {
    QflCtx c;
    c.D = a.D;
    c.row = j * a.D;
    const uint32_t Du = (uint32_t)a.D;
    const int64_t vL = (int64_t)kMtN + a.D;                         // pass-B local words D + i
    c.qL = vL / kMtN;
    c.rL = (int)(vL % kMtN);
    const int64_t vG = gleft > 1 ? (int64_t)gnext : (int64_t)kMtN;  // the first left - 1 words are state[next ..]
    c.qG = vG / kMtN;
    c.rG = (int)(vG % kMtN);
    c.rr = make_rsrc(a.rot + c.row, Du * 4u);
    c.rh = make_rsrc(a.hbuf + c.row, Du);
    c.rm = make_rsrc(a.mask + c.row, Du);
    // XK 2: the fused receiver (QUICFL_quantize, a.pre set): no X / mask / exact values written,
    // and the compiler drops those paths (and their scalar state) from the instance
    c.rX = make_rsrc(XK == 0 ? (void*)((int64_t*)a.X + c.row) : (void*)((uint8_t*)a.X + c.row), XK == 0 ? Du * 8u : Du);
    c.packed = a.tabp != nullptr;
    c.rt = c.packed ? make_rsrc(a.tabp, (uint32_t)a.numel * 4u) : make_rsrc(a.tab, (uint32_t)a.numel * 8u);
    c.sc = (1.0f / a.nrm[j]) * a.sqrtD;                             // AS:466/470 (IEEE 1/x, then f32 mul)
    c.dp = div_plan_norm(a.delta);                                  // q = v / delta: reciprocal + Markstein (exact)
    c.dps = div_plan_norm(c.sc);
    c.fused = XK == 2;
    c.rP = make_rsrc(XK == 2 ? (void*)(a.pre + c.row) : (void*)a.rot, XK == 2 ? Du * 4u : 0u);
    c.rtab_n = a.rtab_n;
    c.fh = (float)a.h_len;
    c.fhalf = (float)a.half;
    c.fnumel = (float)a.numel;                                      // exact: numel < 2^24 (host check)
    c.numel = (int32_t)a.numel;
    c.h_len = (uint32_t)a.h_len;
    c.hpow2 = (c.h_len & (c.h_len - 1)) == 0;
    return c;
}

// Pass A over rounds [c0, c1): s holds block c0 of the local stream on entry (block c + 1 holds
// the words of round c), block c1 on exit.  h = randint(0, h_len, (D,), local) (AS:465/469):
// element e of a round is word e of its block, i.e. register group e / 64 of its own lane.
__device__ __forceinline__ void qfl_pass_a(const QflCtx& c, uint32_t (&s)[kMtGroups], int64_t c0, int64_t c1,
                                           int lane) {
    for (int64_t r = c0; r < c1; ++r) {
        mt_twist_reg(s, lane);
        const uint32_t i0 = (uint32_t)(r * kMtN);
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const int e = 64 * k + lane;
            const uint32_t w = mt_temper(s[k]);
            const uint32_t h = c.hpow2 ? (w & (c.h_len - 1u)) : (w % c.h_len);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)h, c.rh, qf_off(e < kMtN, i0 + (uint32_t)e), 0, 0);
        }
    }
}

// A stream read at an offset (pass B's words start at slot rL / rG of a block): the block in
// registers (`have` twists) and a two-block LDS ring W holding blocks have - 1 and have at
// (block & 1) * 624, so a round's 624 words are one ring read each, wherever they start.
__device__ __forceinline__ void qfl_window_to(uint32_t (&s)[kMtGroups], uint32_t* W, int64_t& have, int64_t need,
                                              int lane) {
    while (have < need) {
        mt_twist_reg(s, lane);
        ++have;
        mt_store(s, W + (have & 1) * kMtN, lane);
    }
}

// Pass B over rounds [c0, c1) (AS:472-490): sL / sG hold local block haveL <= qL + c0 and
// global block haveG <= qG + c0, each also stored in its ring (WL, WG) on entry.  Exact values
// go to ev[row + ev_base + count] in index order; returns the count, ORs UQ_QFL_* into flags.
// Every per-element global access goes through a buffer descriptor (out-of-range loads return
// 0, stores are dropped): no per-element branch, and a lane's ten loads of a round are in flight
// together.
template <int XK, bool LEAN = false>
__device__ __forceinline__ int64_t qfl_pass_b(const QflCtx& c, float* __restrict__ ev, uint32_t (&sL)[kMtGroups],
                                              uint32_t* WL, int64_t& haveL, uint32_t (&sG)[kMtGroups], uint32_t* WG,
                                              int64_t& haveG, int64_t c0, int64_t c1, int64_t ev_base, int32_t& flags,
                                              const float* rtab, int lane) {
    const int64_t D = c.D;
    const float thr = kQflExactT;
    int64_t etot = 0;
    // Two register sets for a round's inputs and for its pending stage 2, used alternately by
    // the loop unrolled by two: a set whose loads are in flight is never copied, so the next
    // round's loads and this round's gathers stay in flight across the round (with one set,
    // the end-of-round copies waited for every load).
    struct In {
        float r[kMtGroups];
        uint32_t h[kMtGroups];
    };
    In I0, I1;
    QflRound R0, R1;
    auto load_in = [&](uint32_t i0, In& o) {
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const uint32_t e = i0 + 64u * k + lane;
            o.r[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.rr, e * 4u, 0, kAuxNT));
            o.h[k] = __builtin_amdgcn_raw_buffer_load_b8(c.rh, e, 0, 0);
        }
    };
    load_in((uint32_t)(c0 * kMtN), I0);

    auto finish = [&](const QflRound& r, uint32_t i0) {          // stage 2 of a round (AS:489-490, 494-495)
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const uint32_t i = i0 + 64u * k + lane;
            const bool active = (r.act >> k) & 1u;
            const bool ex = (r.ex >> k) & 1u;
            float tx, bx;
            if (c.packed) {          // bernoulli(p): low24(w) * 2^-24 < p  <=>  low24(w) < ceil(p * 2^24)
                tx = (float)(r.t[k][0] >> 25);
                bx = ((r.wg[k] & 0xFFFFFFu) < (r.t[k][0] & 0x1FFFFFFu)) ? 1.f : 0.f;
            } else {
                tx = __uint_as_float(r.t[k][0]);
                const float tp = __uint_as_float(r.t[k][1]);
                flags |= (active && !(tp >= 0.f && tp <= 1.f)) ? UQ_QFL_BAD_PX : 0;
                bx = (u24(r.wg[k]) < tp) ? 1.f : 0.f;
            }
            const float xf = tx + bx;                                // AS:489
            if (c.fused) {                                           // the receiver, AS:526-532
                const bool ok = xf > -9.2e18f && xf < 9.2e18f;
                flags |= (active && !ok) ? UQ_QFL_X_RANGE : 0;
                const int64_t xv = ok ? (int64_t)xf : 0;             // AS:490 .long()
                const uint32_t h = (r.hp[k >> 2] >> (8 * (k & 3))) & 0xFFu;
                const int64_t it = (int64_t)((uint64_t)xv * (uint64_t)c.h_len + h);   // AS:530 (int64)
                const bool inr = it >= -(int64_t)c.rtab_n && it < (int64_t)c.rtab_n;
                flags |= (active && !inr) ? UQ_QFL_RECV_INDEX : 0;
                const int32_t idx = inr ? (int32_t)(it < 0 ? it + c.rtab_n : it) : 0;   // take wraps negatives
                const float val = ex ? r.v[k] : (inr ? rtab[idx] : 0.f);                 // AS:531
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(div1(val, c.dps)), c.rP,
                                                      qf_off(active, i * 4u), 0, 0);   // AS:532 / scale
                continue;
            }
            if (XK == 0) {
                const bool ok = xf > -9.2e18f && xf < 9.2e18f;
                flags |= (active && !ok) ? UQ_QFL_X_RANGE : 0;
                const int64_t xv = ok ? (int64_t)xf : 0;             // AS:490 .long()
                typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
                const u32x2v w = {(uint32_t)xv, (uint32_t)((uint64_t)xv >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(w, c.rX, qf_off(active, i * 8u), 0, kAuxNT);
            } else {
                const bool ok = xf > -1.0f && xf < 256.0f;
                flags |= (active && !ok) ? UQ_QFL_X_RANGE : 0;
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(ok ? (int32_t)xf : 0), c.rX, qf_off(active, i), 0, 0);
            }
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(ex ? 1 : 0), c.rm, qf_off(active, i), 0, 0);
            const uint64_t bal = __ballot(active && ex);            // index order: group k, then lane
            if (active && ex) ev[c.row + ev_base + etot + __popcll(bal & ((1ull << lane) - 1ull))] = r.v[k];
            etot += __popcll(bal);
        }
    };

    // stage 1 of round rd from `cur` into `cr` (its gathers issued)
    auto stage1 = [&](int64_t rd, const In& cur, QflRound& cr) {
        const uint32_t i0 = (uint32_t)(rd * kMtN);
        const int lastE = (int)((D - 1 - (int64_t)i0) < (kMtN - 1) ? (D - 1 - (int64_t)i0) : (kMtN - 1));
        // the words of this round: slots rX .. rX + lastE of block qX + rd and, past 623, of
        // block qX + rd + 1 (twisted only when the round reaches it, so the global stream ends
        // on the block holding its last word)
        qfl_window_to(sL, WL, haveL, c.qL + rd + (c.rL + lastE >= kMtN ? 1 : 0), lane);
        qfl_window_to(sG, WG, haveG, c.qG + rd + (c.rG + lastE >= kMtN ? 1 : 0), lane);
        wave_lds_fence();
        const int bL = (int)(((c.qL + rd) & 1) * kMtN) + c.rL, bG = (int)(((c.qG + rd) & 1) * kMtN) + c.rG;
        cr.ex = 0;
        cr.act = 0;
        cr.hp[0] = cr.hp[1] = cr.hp[2] = 0u;
        // AS:472-481: v, the exact mask, q = v / delta for the lane's ten elements at once
        // (exact elements' quotients are discarded, so they stay out of the division's guard)
        float vv[kMtGroups], qq[kMtGroups];
        uint32_t exm = 0;
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            vv[k] = cur.r[k] * c.sc;                                  // AS:472
            exm |= ((vv[k] > thr) || (vv[k] < -thr) ? 1u : 0u) << k;  // AS:478
        }
        div_n(vv, c.dp, qq, exm);
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const int e = 64 * k + lane;
            const int es = e < kMtN ? e : 0;
            const int pl = bL + es, pg = bG + es;
            const uint32_t wl = WL[pl >= 2 * kMtN ? pl - 2 * kMtN : pl];
            const uint32_t wg = WG[pg >= 2 * kMtN ? pg - 2 * kMtN : pg];
            // stage 1 (AS:472-487), branch-free: inactive elements compute on zeros, raise no
            // flags and store nothing
            const bool active = e < kMtN && (int64_t)i0 + e < D;
            cr.wg[k] = mt_temper(wg);
            const float v = vv[k];
            const bool ex = (exm >> k) & 1u;
            const float q = ex ? 0.f : qq[k];                         // AS:480-481 (= v / delta), q[exact] = 0
            const float fl = floorf(q);
            const float p = q - fl;                                   // AS:483
            flags |= (active && !(p >= 0.f && p <= 1.f)) ? UQ_QFL_BAD_P : 0;
            const float bern = (u24(mt_temper(wl)) < p) ? 1.f : 0.f;
            const float iq = fl + bern;                               // AS:484
            const float t1 = iq * c.fh;                               // AS:486 in f32 (no fma: -ffp-contract=off)
            const float t2 = t1 + (float)cur.h[k];
            const float it = truncf(t2 + c.fhalf);                    // .long() truncates
            const bool inr = it >= -c.fnumel && it < c.fnumel;        // torch.take's range (NaN: out)
            flags |= (active && !inr) ? UQ_QFL_BAD_INDEX : 0;
            int32_t idx = inr ? (int32_t)it : 0;
            idx = idx < 0 ? idx + c.numel : idx;                      // torch.take wraps negatives
            if (c.packed) {                                           // AS:486-487, one 4-byte gather
                cr.t[k][0] = __builtin_amdgcn_raw_buffer_load_b32(c.rt, (uint32_t)idx * 4u, 0, 0);
                cr.t[k][1] = 0u;
            } else {
                const auto t = __builtin_amdgcn_raw_buffer_load_b64(c.rt, (uint32_t)idx * 8u, 0, 0);
                cr.t[k][0] = t[0];
                cr.t[k][1] = t[1];
            }
            cr.v[k] = v;
            cr.ex |= (active && ex ? 1u : 0u) << k;
            cr.act |= (active ? 1u : 0u) << k;
            cr.hp[k >> 2] |= (cur.h[k] & 0xFFu) << (8 * (k & 3));
        }
    };
    if (LEAN) {
        // one register set each (two waves per SIMD hide the latencies instead): stage 1 of
        // round rd, the loads of round rd + 1, then stage 2 of round rd
        for (int64_t rd = c0; rd < c1; ++rd) {
            stage1(rd, I0, R0);
            load_in((uint32_t)((rd + 1) * kMtN), I0);                // (beyond D: the descriptor returns 0)
            finish(R0, (uint32_t)(rd * kMtN));
        }
        return etot;
    }
    // one round: loads for round rd + 1 into `nxt`, stage 1 of round rd from `cur` into `cr`
    // (its gathers issued), then stage 2 of round rd - 1 (`pr`) while those gathers fly
    auto round = [&](int64_t rd, const In& cur, In& nxt, QflRound& cr, const QflRound& pr, bool fin) {
        const uint32_t i0 = (uint32_t)(rd * kMtN);
        load_in(i0 + (uint32_t)kMtN, nxt);                           // (beyond D: the descriptor returns 0)
        stage1(rd, cur, cr);
        if (fin) finish(pr, i0 - (uint32_t)kMtN);
    };
    for (int64_t rd = c0; rd < c1; rd += 2) {
        round(rd, I0, I1, R0, R1, rd > c0);
        if (rd + 1 < c1) round(rd + 1, I1, I0, R1, R0, true);
    }
    if (c1 > c0) finish(((c1 - 1 - c0) & 1) ? R1 : R0, (uint32_t)((c1 - 1) * kMtN));
    return etot;
}

// The global generator's state after the message's D draws: the block holding word D - 1
// (sG after the last round) and ATen's (left, next) for it.
__device__ __forceinline__ void qfl_state_out(uint32_t* so, const uint32_t (&sG)[kMtGroups], int64_t D, int32_t gleft,
                                              int32_t gnext, int64_t vG, int lane) {
    uint32_t left1, next1;
    if (D <= (int64_t)gleft - 1) {                               // every draw from the current block
        left1 = (uint32_t)(gleft - D);
        next1 = (uint32_t)(gnext + D);
    } else {
        const int64_t pos = (vG + D - 1) % kMtN;
        next1 = (uint32_t)(pos + 1);
        left1 = (uint32_t)(kMtN - pos);
    }
    mt_store(sG, so + 2, lane);
    if (lane == 0) {
        so[0] = left1;
        so[1] = next1;
    }
}

// The global generator of message j into registers: ATen's state (left, next, words) or a
// fresh generator seeded with px_seeds[j] (init_genrand by one lane in `scratch`).
__device__ __forceinline__ void qfl_gen_init(const QflSendArgs& a, int64_t j, uint32_t (&sG)[kMtGroups],
                                             uint32_t* scratch, int32_t& gleft, int32_t& gnext, int lane) {
    gleft = 1;
    gnext = 0;
    if (a.px_state) {
        const uint32_t* st = a.px_state + j * kQfStateWords;
        gleft = (int32_t)st[0];
        gnext = (int32_t)st[1];
        mt_load(sG, st + 2, lane);
    } else {
        if (lane == 0) mt_seed(scratch, (uint32_t)a.px_seeds[j]);
        wave_lds_fence();
        mt_load(sG, scratch, lane);
    }
}

// KQ1 for batches: one wave per message.  XK: 0 = int64 X (the drop-in's X.long()), 1 = uint8 X.
template <int XK>
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_send_wave_kernel(QflSendArgs a) {
    __shared__ uint32_t WLsh[kQfWavesPerWG][2 * kMtN];    // local stream ring per wave (first: the seed scratch)
    __shared__ uint32_t WGsh[kQfWavesPerWG][2 * kMtN];    // global stream ring per wave
    __shared__ float rtab[kQflRecvTab];                   // the fused receiver's table
    if (XK == 2) {
        for (int i = threadIdx.x; i < a.rtab_n; i += 64 * kQfWavesPerWG) rtab[i] = a.rtab[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    if (j >= a.n) return;                                       // whole wave: no barrier below
    uint32_t* WL = WLsh[wv];
    uint32_t* WG = WGsh[wv];
    uint32_t sL[kMtGroups], sG[kMtGroups];
    int32_t gleft, gnext;
    qfl_gen_init(a, j, sG, WG, gleft, gnext, lane);
    if (lane == 0) mt_seed(WL, (uint32_t)a.prng_seeds[j]);
    wave_lds_fence();
    mt_load(sL, WL, lane);
    wave_lds_fence();
    const QflCtx c = qfl_ctx<XK>(a, j, gleft, gnext);
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    if (a.lstate)                                               // pass A done by KQ1a
        mt_load(sL, a.lstate + j * kMtN, lane);
    else
        qfl_pass_a(c, sL, 0, nch, lane);
    int64_t haveL = nch, haveG = 0;
    mt_store(sL, WL + (haveL & 1) * kMtN, lane);
    mt_store(sG, WG, lane);
    int32_t flags = 0;
    const int64_t etot = qfl_pass_b<XK>(c, a.ev, sL, WL, haveL, sG, WG, haveG, 0, nch, 0, flags, rtab, lane);
    for (int s = 32; s >= 1; s >>= 1) flags |= __shfl_xor(flags, s);
    if (a.px_state_out)
        qfl_state_out(a.px_state_out + j * kQfStateWords, sG, a.D, gleft, gnext, c.qG * kMtN + c.rG, lane);
    if (lane == 0) {
        if (a.ecount) a.ecount[j] = (int32_t)etot;
        if (a.scale) a.scale[j] = c.sc;
        a.info[j] = flags;
    }
}

// KQ1a: pass A of the one-wave kernel alone (h = randint(0, h_len, (D,), local), AS:465/469):
// it needs only the message seeds, so it runs on the side stream beside the sender's RHT and
// norm, and KQ1 starts pass B from the local block it leaves in lstate.
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_pass_a_kernel(QflSendArgs a, uint32_t* __restrict__ lstate) {
    __shared__ uint32_t WLsh[kQfWavesPerWG][kMtN];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    if (j >= a.n) return;
    uint32_t* WL = WLsh[wv];
    uint32_t sL[kMtGroups];
    if (lane == 0) mt_seed(WL, (uint32_t)a.prng_seeds[j]);
    wave_lds_fence();
    mt_load(sL, WL, lane);
    QflCtx c;                                                   // what pass A reads of the context
    c.D = a.D;
    c.row = j * a.D;
    c.rh = make_rsrc(a.hbuf + c.row, (uint32_t)a.D);
    c.h_len = (uint32_t)a.h_len;
    c.hpow2 = (c.h_len & (c.h_len - 1)) == 0;
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    qfl_pass_a(c, sL, 0, nch, lane);
    mt_store(sL, lstate + j * kMtN, lane);
}

// KQ1 for a few messages (the per-call drop-in): one 512-thread workgroup per message.  Wave
// 0 ("scout") runs the local stream from its seed through all 2D words, wave 1 the global stream
// through D words; neither does per-coordinate work.  The other 6 waves take contiguous runs of
// rounds: when a scout's stream reaches the block a run starts from, the scout stores that block
// into the run's LDS slice (pass A) or ring (pass B) and raises its flag, so each run generates
// only its own words.  The critical path is the scouts' 2D / 624 twists, not the coordinates'
// arithmetic.  Exact values are written per run and compacted into index order at the end.
// Flags are waited for with a bounded spin (UQ_QFL_TIMEOUT if it ever ran out: the scouts never
// wait on anyone).
constexpr int kQfTeamWaves = 8;                    // 2 scouts + 6 runs
constexpr int kQfRuns = kQfTeamWaves - 2;
// messages per call up to which the team kernels run: a workgroup per message while they fit
// the GPU about once (1024 x 2^20, bits 1: sender 128 / 256 messages 4.5 / 5.5 ms against
// 11.4 ms one-wave; 1024 messages 19.4 ms against 15.6 -- there the one-wave kernels win)
constexpr int64_t kQfTeamMaxN = 256;
// padded dims up to which it runs: the last run waits for the scouts' 2D/624 twists (about
// 15 ms at 2^23), far inside qfl_wait_flag's bound of 2^24 sleeps; longer vectors take the
// one-wave-per-message kernel, which never waits
constexpr int64_t kQfTeamMaxD = (int64_t)1 << 23;
constexpr float kQfRunRatio = 0.885f;
__device__ __forceinline__ void qfl_run_bounds(int64_t nch, int64_t (&cb)[kQfRuns + 1]) {
    float w[kQfRuns], tot = 0.f, x = 1.f;
    for (int r = 0; r < kQfRuns; ++r) {
        w[r] = x;
        tot += x;
        x *= kQfRunRatio;
    }
    float acc = 0.f;
    cb[0] = 0;
    for (int r = 1; r < kQfRuns; ++r) {
        acc += w[r - 1];
        int64_t b = (int64_t)((float)nch * (acc / tot) + 0.5f);
        b = b < cb[r - 1] ? cb[r - 1] : (b > nch ? nch : b);
        cb[r] = b;
    }
    cb[kQfRuns] = nch;
}
__device__ __forceinline__ bool qfl_wait_flag(int* f) {
    for (int it = 0; it < (1 << 24); ++it) {
        if (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
__device__ __forceinline__ void qfl_give(uint32_t* dst, const uint32_t (&s)[kMtGroups], int* f, int lane) {
    mt_store(s, dst, lane);
    wave_lds_fence();
    if (lane == 0) __hip_atomic_store(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int XK>
__global__ void __launch_bounds__(64 * kQfTeamWaves)
quicfl_send_team_kernel(QflSendArgs a) {
    __shared__ uint32_t LA[kQfRuns][kMtN];               // pass-A start block per run
    __shared__ uint32_t WL[kQfRuns][2 * kMtN], WG[kQfRuns][2 * kMtN];   // pass-B rings per run
    __shared__ uint32_t seed_scratch[2][kMtN];
    __shared__ int rdy[kQfRuns][3];
    __shared__ int64_t cnt[kQfRuns];
    __shared__ int32_t sflags;
    __shared__ float rtab[kQflRecvTab];                  // the fused receiver's table
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = blockIdx.x;
    if (XK == 2)
        for (int i = threadIdx.x; i < a.rtab_n; i += 64 * kQfTeamWaves) rtab[i] = a.rtab[i];
    const int64_t D = a.D;
    const int64_t nch = (D + kMtN - 1) / kMtN;
    // run r takes rounds [cb[r], cb[r + 1]): lengths shrinking by kQfRunRatio, since a later
    // run's pass B starts later (the scout reaches its block later) and a round of pass B
    // costs ~9 twists, so all runs end together
    int64_t cb[kQfRuns + 1];
    qfl_run_bounds(nch, cb);
    for (int i = threadIdx.x; i < kQfRuns * 3; i += 64 * kQfTeamWaves) (&rdy[0][0])[i] = 0;
    if (threadIdx.x < kQfRuns) cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) sflags = 0;
    uint32_t s[kMtGroups];                               // the scouts' stream block
    int32_t gleft = a.px_state ? (int32_t)a.px_state[j * kQfStateWords] : 1;
    int32_t gnext = a.px_state ? (int32_t)a.px_state[j * kQfStateWords + 1] : 0;
    if (wv == 1) qfl_gen_init(a, j, s, seed_scratch[1], gleft, gnext, lane);
    if (wv == 0) {
        if (lane == 0) mt_seed(seed_scratch[0], (uint32_t)a.prng_seeds[j]);
        wave_lds_fence();
        mt_load(s, seed_scratch[0], lane);
    }
    __syncthreads();
    const QflCtx c = qfl_ctx<XK>(a, j, gleft, gnext);
    int32_t flags = 0;
    if (wv == 0) {                                       // local scout: blocks 0 .. qL + start of the last run
        __builtin_amdgcn_s_setprio(3);
        int64_t last = 0;
        for (int r = 0; r < kQfRuns; ++r)
            if (cb[r] < cb[r + 1]) last = c.qL + cb[r];
        for (int64_t k = 0; k <= last; ++k) {
            if (k) mt_twist_reg(s, lane);
            const int64_t kb = k - c.qL;
            for (int r = 0; r < kQfRuns; ++r) {
                if (cb[r] >= cb[r + 1]) continue;
                if (k == cb[r]) qfl_give(LA[r], s, &rdy[r][0], lane);
                if (kb == cb[r]) qfl_give(WL[r] + (k & 1) * kMtN, s, &rdy[r][1], lane);
            }
        }
    } else if (wv == 1) {                                // global scout
        __builtin_amdgcn_s_setprio(3);
        int64_t last = 0;
        for (int r = 0; r < kQfRuns; ++r)
            if (cb[r] < cb[r + 1]) last = c.qG + cb[r];
        for (int64_t k = 0; k <= last; ++k) {
            if (k) mt_twist_reg(s, lane);
            const int64_t kg = k - c.qG;
            for (int r = 0; r < kQfRuns; ++r)
                if (cb[r] < cb[r + 1] && kg == cb[r]) qfl_give(WG[r] + (k & 1) * kMtN, s, &rdy[r][2], lane);
        }
    } else {                                             // run r: rounds [c0, c1)
        const int r = wv - 2;
        const int64_t c0 = cb[r], c1 = cb[r + 1];
        if (c0 < c1) {
            bool ok = !a.force_timeout && qfl_wait_flag(&rdy[r][0]);
            if (ok) {
                uint32_t sa[kMtGroups];
                mt_load(sa, LA[r], lane);
                qfl_pass_a(c, sa, c0, c1, lane);
            }
            ok = ok && qfl_wait_flag(&rdy[r][1]) && qfl_wait_flag(&rdy[r][2]);
            if (ok) {
                int64_t haveL = c.qL + c0, haveG = c.qG + c0;
                uint32_t sL[kMtGroups], sG[kMtGroups];
                mt_load(sL, WL[r] + (haveL & 1) * kMtN, lane);
                mt_load(sG, WG[r] + (haveG & 1) * kMtN, lane);
                const int64_t e = qfl_pass_b<XK>(c, a.ev, sL, WL[r], haveL, sG, WG[r], haveG, c0, c1, c0 * kMtN, flags,
                                                 rtab, lane);
                if (lane == 0) cnt[r] = e;
                if (c1 == nch && a.px_state_out)
                    qfl_state_out(a.px_state_out + j * kQfStateWords, sG, D, gleft, gnext, c.qG * kMtN + c.rG, lane);
            } else {
                flags |= UQ_QFL_TIMEOUT;
            }
        }
        for (int o = 32; o >= 1; o >>= 1) flags |= __shfl_xor(flags, o);
        if (lane == 0 && flags) atomicOr(&sflags, flags);
    }
    __syncthreads();
    if (wv == 0) {                                       // exact values of run r: [c0*624, +cnt) -> index order
        int64_t base = 0;
        for (int r = 0; r < kQfRuns && !c.fused; ++r) {
            const int64_t src = cb[r] * kMtN, n_r = cnt[r];
            for (int64_t i0 = 0; i0 < n_r; i0 += 64) {   // (base <= src: a downward move, chunk by chunk)
                const int64_t i = i0 + lane;
                const float v = i < n_r ? a.ev[c.row + src + i] : 0.f;
                if (i < n_r) a.ev[c.row + base + i] = v;
            }
            base += n_r;
        }
        if (lane == 0) {
            if (a.ecount) a.ecount[j] = (int32_t)base;
            if (a.scale) a.scale[j] = c.sc;
            a.info[j] = sflags;
        }
    }
}

// ---- jump path: the three streams' run starts by MT19937 jump-ahead (KQ0j), then every run
// at once (KQ1j) ------------------------------------------------------------------------------
// The team kernel's critical path is its scouts walking the streams (2D/624 twists of the local
// stream: ~13 ms at 2^22).  Instead, each run's starting blocks are computed directly: the
// state 624 b words ahead is the correlation window_J = XOR_{k : g_k = 1} x[k .. k + 623] of
// g = t^(624 (b - 1)) mod phi (uq_mt_poly.cpp) with the stream's first 19937 + 623 words, then
// one twist (the window's word 0 carries only its top bit).  Runs of L rounds then start
// together, R of them per message, each with the passes of KQ1 (pass A for its h, pass B for its
// coordinates), so a message takes ~(jump + L rounds) instead of ~2D/624 twists.
//   KQ0s quicfl_stream_kernel   one wave per (message, stream): the base block and 32 twists,
//        x[0 .. 33 * 624), to HBM (read by every jump of that stream from L2).
//   KQ0j quicfl_jump_kernel   four 256-thread workgroups per (message, run, stream), each taking a
//        quarter of the polynomial's 624 words (39 per wave) with the stream words they read
//        staged in LDS (22 KB: several workgroups per CU); a wave XORs 4-word quads of x per set
//        coefficient (one ds_read_b128 per quad, a scalar branch per coefficient nibble); the
//        partial windows go to HBM, and the run XORs the four and twists once.
//   KQ1j quicfl_send_runs_kernel   one wave per (message, run), four per workgroup: pass A over
//        its rounds from the local block c0 (run 0: the seed), pass B from local block qL + c0
//        and global block c0 (run 0: the generator's own state); flags per run.
//   KQ1f quicfl_send_fin_kernel   one wave per message: flags ORed, the runs' exact values moved
//        into index order, ecount, scale.
constexpr int kMjBlocks = 33;                 // x[0 .. 33 * 624) covers k + w <= 19936 + 623 (+ quad tails)
constexpr int kMjX = kMjBlocks * kMtN;        // stream words kept per (message, stream)
constexpr int kMjParts = 4;                   // workgroups per jump, 156 coefficient words each
constexpr int kMjSlice = 39;                  // coefficient words per wave (4 waves x 4 parts x 39 = 624)
constexpr int kMjPartWords = 4 * kMjSlice * 32 + 632;   // LDS words of a part: its coefficients + the window

struct QflJumpArgs {
    const int32_t* prng_seeds;  // local streams: init_genrand(prng_seeds[j])
    const uint32_t* px_state;   // global streams: ATen state (left, next, words) per message, or null
    const int32_t* px_seeds;    //   or fresh generators
    const uint32_t* polyA;      // [R][624]: row r = t^(624 (r L - 1)) mod phi (row 0 unused)
    const uint32_t* polyB;      // [R][624]: row r = t^(624 (qL + r L - 1)) mod phi
    uint32_t* xs;               // [n][nstreams][kMjX]: the local (and the global) stream's first words
    uint32_t* parts;            // [n][R][kinds][kMjParts][624]: partial windows (local r L, local qL + r L, global r L)
    int32_t R;
    int64_t n;
    int32_t nstreams;           // 2: the sender (local + global); 1: the receiver (local)
    int32_t kinds;              // 3: the sender's three blocks per run; 1: the receiver's local block r L
};

// KQ0s: x[0 .. kMjX) of each message's two streams (base block, then 32 twists), one wave each
__global__ void __launch_bounds__(256)
quicfl_stream_kernel(QflJumpArgs a) {
    __shared__ uint32_t scratch[4][kMtN];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t id = (int64_t)blockIdx.x * 4 + wv;
    const int64_t j = id / a.nstreams;
    const int s = (int)(id % a.nstreams);                // 0 local, 1 global
    if (j >= a.n) return;
    uint32_t st[kMtGroups];
    if (s == 1 && a.px_state) {
        mt_load(st, a.px_state + j * kQfStateWords + 2, lane);
    } else {
        if (lane == 0) mt_seed(scratch[wv], (uint32_t)(s == 1 ? a.px_seeds[j] : a.prng_seeds[j]));
        wave_lds_fence();
        mt_load(st, scratch[wv], lane);
    }
    uint32_t* x = a.xs + (j * a.nstreams + s) * kMjX;
    __builtin_amdgcn_s_setprio(3);
    mt_store(st, x, lane);
    for (int b = 1; b < kMjBlocks; ++b) {
        mt_twist_reg(st, lane);
        mt_store(st, x + b * kMtN, lane);
    }
}

// acc[i] ^= XOR over the set bits t of NIB of E[t + i], E = (E0, E1): coefficient k0 + t applied
// to the four window words w0 .. w0 + 3 (x[k0 + t + w0 + i]); two terms per v_bitop3 (XOR3)
__device__ __forceinline__ uint32_t mj_xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int NIB>
__device__ __forceinline__ void mj_apply(uint32_t (&acc)[4], const uint4& E0, const uint4& E1) {
    const uint32_t E[8] = {E0.x, E0.y, E0.z, E0.w, E1.x, E1.y, E1.z, E1.w};
    constexpr int t0 = (NIB & 1) ? 0 : (NIB & 2) ? 1 : (NIB & 4) ? 2 : 3;           // lowest set bit
    constexpr int R1 = NIB & (NIB - 1);                                              // the others
    constexpr int t1 = (R1 & 1) ? 0 : (R1 & 2) ? 1 : (R1 & 4) ? 2 : 3;
    constexpr int R2 = R1 & (R1 - 1);
    constexpr int t2 = (R2 & 1) ? 0 : (R2 & 2) ? 1 : (R2 & 4) ? 2 : 3;
    constexpr int R3 = R2 & (R2 - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (R1 == 0) {
            acc[i] ^= E[t0 + i];
        } else {
            acc[i] = mj_xor3(acc[i], E[t0 + i], E[t1 + i]);
            if (R2 != 0 && R3 == 0) acc[i] ^= E[t2 + i];
            if (R3 != 0) acc[i] = mj_xor3(acc[i], E[t2 + i], E[3 + i]);
        }
    }
}
template <int NIB>
__device__ __forceinline__ void mj_apply3(uint32_t (&acc)[3][4], const uint4 (&E0)[3], const uint4 (&E1)[3]) {
#pragma unroll
    for (int g = 0; g < 3; ++g) mj_apply<NIB>(acc[g], E0[g], E1[g]);
}
__device__ __forceinline__ uint4 mj_quad(const uint32_t* p) {      // one ds_read_b128, never split
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const volatile u32x4v lds_q;
    const u32x4v v = *(lds_q*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// KQ0j: one 256-thread workgroup per (message, run, stream, part); part p's wave v takes the
// polynomial's words [156 p + 39 v, + 39) against window words 0..623 (lane quads: w0 = 256 g +
// 4 lane, group 2 lanes < 28), the stream words it reads staged in LDS; the 4 waves' partial
// windows are XORed and written out (the runs XOR the 4 parts and twist once).
__global__ void __launch_bounds__(256)
quicfl_jump_kernel(QflJumpArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t X[kMjPartWords];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t bid = blockIdx.x;
    const int p = (int)(bid % kMjParts);
    const int64_t job = bid / kMjParts;
    const int s = (int)(job % a.kinds);
    const int64_t jr = job / a.kinds;
    const int r = (int)(jr % a.R);
    const int64_t j = jr / a.R;
    if (j >= a.n || (r == 0 && s != 1)) return;          // run 0's local-A and global blocks are the bases
    const uint32_t* poly = (s == 1 ? a.polyB : a.polyA) + (size_t)r * kMtN;
    const int wb0 = p * 4 * kMjSlice + wv * kMjSlice;
    const uint32_t pv = lane < kMjSlice ? poly[wb0 + lane] : 0u;           // the wave's coefficient words
    const int k_lo = p * 4 * kMjSlice * 32;
    const uint32_t* x = a.xs + (j * a.nstreams + (s == 2 ? 1 : 0)) * kMjX;
    {                                                    // stage x[k_lo ..): every load in flight at once
        constexpr int kQ = kMjPartWords / 4, kPer = (kQ + 255) / 256;
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        u32x4v v[kPer];
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
            const int q = threadIdx.x + 256 * t;
            v[t] = q < kQ && k_lo + 4 * q < kMjX ? *(const u32x4v*)(x + k_lo + 4 * q) : u32x4v{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
            const int q = threadIdx.x + 256 * t;
            if (q < kQ) *(u32x4v*)(X + 4 * q) = v[t];
        }
    }
    __syncthreads();
    uint32_t acc[3][4];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[g][i] = 0u;
    int w0[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) w0[g] = g < 2 || lane < 28 ? 256 * g + 4 * lane : 0;
    for (int wi = 0; wi < kMjSlice; ++wi) {
        const uint32_t pw = (uint32_t)__builtin_amdgcn_readlane((int)pv, wi);
        if (!pw) continue;
        const int k0 = (wb0 + wi) * 32 - k_lo;
        uint4 E0[3], E1[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) E0[g] = mj_quad(X + k0 + w0[g]);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
#pragma unroll
            for (int g = 0; g < 3; ++g) E1[g] = mj_quad(X + k0 + 4 * m + 4 + w0[g]);
            switch ((pw >> (4 * m)) & 15u) {
                case 1: mj_apply3<1>(acc, E0, E1); break;
                case 2: mj_apply3<2>(acc, E0, E1); break;
                case 3: mj_apply3<3>(acc, E0, E1); break;
                case 4: mj_apply3<4>(acc, E0, E1); break;
                case 5: mj_apply3<5>(acc, E0, E1); break;
                case 6: mj_apply3<6>(acc, E0, E1); break;
                case 7: mj_apply3<7>(acc, E0, E1); break;
                case 8: mj_apply3<8>(acc, E0, E1); break;
                case 9: mj_apply3<9>(acc, E0, E1); break;
                case 10: mj_apply3<10>(acc, E0, E1); break;
                case 11: mj_apply3<11>(acc, E0, E1); break;
                case 12: mj_apply3<12>(acc, E0, E1); break;
                case 13: mj_apply3<13>(acc, E0, E1); break;
                case 14: mj_apply3<14>(acc, E0, E1); break;
                case 15: mj_apply3<15>(acc, E0, E1); break;
                default: break;
            }
#pragma unroll
            for (int g = 0; g < 3; ++g) E0[g] = E1[g];
        }
    }
    __syncthreads();                                     // every wave is done with x
    uint32_t* P = X + wv * 640;                          // partial windows, 640 words apart
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const int w = 256 * g + 4 * lane;
        if (w < kMtN) *(uint4*)(P + w) = make_uint4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
    }
    __syncthreads();
    uint32_t* out = a.parts + (((j * a.R + r) * a.kinds + s) * kMjParts + p) * kMtN;
    for (int i = threadIdx.x; i < kMtN; i += 256) out[i] = X[i] ^ X[640 + i] ^ X[1280 + i] ^ X[1920 + i];
}

// A run's block from KQ0j's parts: the window (XOR of the parts), then one twist (block b - 1's
// word 0 carries only its top bit; every word of block b is exact)
__device__ __forceinline__ void mj_block(uint32_t (&st)[kMtGroups], const uint32_t* parts, int lane) {
#pragma unroll
    for (int g = 0; g < kMtGroups; ++g) {
        const int i = 64 * g + lane;
        const int ii = i < kMtN ? i : 0;
        st[g] = parts[ii] ^ parts[kMtN + ii] ^ parts[2 * kMtN + ii] ^ parts[3 * kMtN + ii];
    }
    mt_twist_reg(st, lane);
}

struct QflRunArgs {
    const uint32_t* parts;      // KQ0j's partial windows [n][R][3][kMjParts][624]
    int32_t* runinfo;           // [n][R][2]: exact values of the run (KQ1j / KQ2c), its UQ_QFL_* flags
    int32_t R;
    int64_t L;                  // rounds per run (the last run may have fewer)
    int32_t passa_done;         // KQ1ar wrote every run's h already (the side stream): KQ1j skips pass A
};

// KQ1ar: pass A of every run (h for its rounds, AS:465/469) from its jumped local block c0 (run
// 0: the seed), one wave per (message, run): issued on the side stream right behind KQ0j, so it
// runs beside the sender's RHT and norm and KQ1j is left with pass B.
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_pass_a_runs_kernel(QflSendArgs a, QflRunArgs ra) {
    __shared__ uint32_t WLsh[kQfWavesPerWG][kMtN];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t id = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    const int64_t j = id / ra.R;
    const int r = (int)(id % ra.R);
    if (j >= a.n) return;
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    const int64_t c0 = (int64_t)r * ra.L, c1 = min(nch, c0 + ra.L);
    if (c0 >= c1) return;
    uint32_t sL[kMtGroups];
    if (r == 0) {
        uint32_t* WL = WLsh[wv];
        if (lane == 0) mt_seed(WL, (uint32_t)a.prng_seeds[j]);
        wave_lds_fence();
        mt_load(sL, WL, lane);
    } else {
        mj_block(sL, ra.parts + (j * ra.R + r) * 3 * kMjParts * kMtN, lane);   // local block c0
    }
    QflCtx c;                                                   // what pass A reads of the context
    c.D = a.D;
    c.row = j * a.D;
    c.rh = make_rsrc(a.hbuf + c.row, (uint32_t)a.D);
    c.h_len = (uint32_t)a.h_len;
    c.hpow2 = (c.h_len & (c.h_len - 1)) == 0;
    qfl_pass_a(c, sL, c0, c1, lane);
}

// W2: two waves per SIMD (the registers capped at 256, a few spilled), for plans of more than
// 1024 run waves; otherwise one (no spills)
template <int XK, bool W2>
__global__ void __launch_bounds__(64 * kQfWavesPerWG, W2 ? 2 : 1)
quicfl_send_runs_kernel(QflSendArgs a, QflRunArgs ra) {
    __shared__ uint32_t WLsh[kQfWavesPerWG][2 * kMtN];
    __shared__ uint32_t WGsh[kQfWavesPerWG][2 * kMtN];
    __shared__ float rtab[kQflRecvTab];
    if (XK == 2) {
        for (int i = threadIdx.x; i < a.rtab_n; i += 64 * kQfWavesPerWG) rtab[i] = a.rtab[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t id = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    const int64_t j = id / ra.R;
    const int r = (int)(id % ra.R);
    if (j >= a.n) return;                                // whole wave: no barrier below
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    const int64_t c0 = (int64_t)r * ra.L, c1 = min(nch, c0 + ra.L);
    int32_t* info = ra.runinfo + (j * ra.R + r) * 2;
    if (c0 >= c1) {
        if (lane == 0) info[0] = info[1] = 0;
        return;
    }
    uint32_t* WL = WLsh[wv];
    uint32_t* WG = WGsh[wv];
    const uint32_t* st = ra.parts + (j * ra.R + r) * 3 * kMjParts * kMtN;
    int32_t gleft = a.px_state ? (int32_t)a.px_state[j * kQfStateWords] : 1;
    int32_t gnext = a.px_state ? (int32_t)a.px_state[j * kQfStateWords + 1] : 0;
    const QflCtx c = qfl_ctx<XK>(a, j, gleft, gnext);
    uint32_t sL[kMtGroups], sG[kMtGroups];
    if (!ra.passa_done) {
        if (r == 0) {                                    // local block 0: the seed itself
            if (lane == 0) mt_seed(WL, (uint32_t)a.prng_seeds[j]);
            wave_lds_fence();
            mt_load(sL, WL, lane);
            wave_lds_fence();
        } else {
            mj_block(sL, st, lane);                      // local block c0
        }
        qfl_pass_a(c, sL, c0, c1, lane);                 // AS:465 h for the run's rounds
    }
    int64_t haveL = c.qL + c0, haveG = c0;
    mj_block(sL, st + kMjParts * kMtN, lane);            // local block qL + c0
    if (r == 0) {
        qfl_gen_init(a, j, sG, WG, gleft, gnext, lane);  // the global generator's own block 0
        wave_lds_fence();
    } else {
        mj_block(sG, st + 2 * kMjParts * kMtN, lane);    // global block c0
    }
    mt_store(sL, WL + (haveL & 1) * kMtN, lane);
    mt_store(sG, WG + (haveG & 1) * kMtN, lane);
    // exact values into the run's own span of ev (from coordinate c0 * 624); KQ1f moves them
    // into index order behind the earlier runs' (~0.4 % of the coordinates: no counting pass
    // over rot before the runs)
    const int64_t ebase = c0 * kMtN;
    int32_t flags = 0;
    const int64_t ecnt = qfl_pass_b<XK, W2>(c, a.ev, sL, WL, haveL, sG, WG, haveG, c0, c1, ebase, flags, rtab, lane);
    if (lane == 0 && !c.fused) info[0] = (int32_t)ecnt;
    for (int o = 32; o >= 1; o >>= 1) flags |= __shfl_xor(flags, o);
    if (c1 == nch && a.px_state_out)
        qfl_state_out(a.px_state_out + j * kQfStateWords, sG, a.D, gleft, gnext, c.qG * kMtN + c.rG, lane);
    if (lane == 0) info[1] = flags;
}

__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_send_fin_kernel(QflSendArgs a, QflRunArgs ra) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    if (j >= a.n) return;
    const int32_t* info = ra.runinfo + j * ra.R * 2;
    int32_t flags = 0;
    int64_t tot = 0;
    for (int r = lane; r < ra.R; r += 64) {
        flags |= info[2 * r + 1];
        if (!a.pre) tot += info[2 * r];
    }
    for (int o = 32; o >= 1; o >>= 1) {
        flags |= __shfl_xor(flags, o);
        tot += __shfl_xor(tot, o);
    }
    if (!a.pre) {                                       // runs' exact values -> index order
        int64_t base = 0;
        const int64_t row = j * a.D;
        for (int r = 0; r < ra.R; ++r) {
            const int64_t src = (int64_t)r * ra.L * kMtN, n_r = info[2 * r];
            if (src != base)
                for (int64_t i0 = 0; i0 < n_r; i0 += 64) {   // (base < src: a downward move, chunk by chunk)
                    const int64_t i = i0 + lane;
                    const float v = i < n_r ? a.ev[row + src + i] : 0.f;
                    if (i < n_r) a.ev[row + base + i] = v;
                }
            base += n_r;
        }
    }
    if (lane == 0) {
        if (a.ecount) a.ecount[j] = (int32_t)tot;
        if (a.scale) a.scale[j] = (1.0f / a.nrm[j]) * a.sqrtD;      // AS:466/470, as qfl_ctx
        a.info[j] = flags;
    }
}

// ---- receiver: QuicFLReceiver.decompress before its inverse RHT (AS:526-532) -----------------
// h = torch.randint(0, h_len, (D,)) of a generator seeded with prng_seed (word % h_len), then
// v = recv_table.take(X * h_len + h) (AS:530: -numel <= index < numel, negatives wrap, anything
// else raises -> UQ_QFL_BAD_INDEX), exact coordinates overwritten (AS:531), v / scale (f32).
// One wave per message; the table (<= 1024 floats) sits in LDS, shared by the workgroup's waves.
// XK: X as int64 (0, the reference's X.long()), uint8 (1, the batch sender's) or int32 (2).
// Exact values dense (at their coordinate) or compact (the message's exact values in index
// order, as the sender writes them): a compact value's slot is the number of exact coordinates
// before it, from wave ballots over the round's mask and a running count.  Loads run ahead:
// X one round, the mask two rounds (its ballots give the next round's value slots, whose loads
// are then one round ahead too).
constexpr int kQflTab = 1024;
struct QflRecvArgs {
    const void* X;                  // [n][D] int64 / uint8 / int32 (XK)
    int64_t n, D;
    const float* table;             // [tab_n] receiver table
    int32_t tab_n, h_len;
    const int32_t* prng_seeds;
    const uint8_t* exact_mask;      // [n][D] or null
    const float* exact_vals;        // [n][D] dense or compact, or null
    int compact;
    const int32_t* exact_count;     // [n] or null (compact: checked against the mask)
    const float* scale;             // [n]
    float* out;                     // [n][D]
    int32_t* info;                  // [n] or null
    int32_t force_timeout;          // test hook (uq_test_set_quicfl_hooks): team runs skip their waits
};

// Rounds [c0, c1) of message j's receiver (AS:526-532): s holds the h stream's block c0 on
// entry; ebase = the message's exact coordinates before round c0 (compact layout).  Returns
// UQ_QFL_* flags; *eend = the exact count through the rounds slotted.
template <int XK>
__device__ __forceinline__ int32_t qfl_recv_rounds(const QflRecvArgs& a, const float* tab, int64_t j,
                                                   uint32_t (&sL)[kMtGroups], int64_t c0, int64_t c1, uint32_t ebase,
                                                   uint32_t* eend, int lane) {
    const int64_t D = a.D;
    const int64_t row = j * D;
    const uint32_t Du = (uint32_t)D;
    const DivPlan dp = div_plan_norm(a.scale[j]);               // v / scale (AS:532): exact quotient
    const uint32_t hl = (uint32_t)a.h_len;
    const int32_t tab_n = a.tab_n;
    const bool hpow2 = (hl & (hl - 1)) == 0;
    const bool compact = a.compact != 0;
    constexpr uint32_t xb = XK == 0 ? 8u : (XK == 1 ? 1u : 4u);  // bytes per X
    // buffer descriptors: branch-free loads (0 beyond D) and stores (dropped beyond D)
    const __amdgpu_buffer_rsrc_t rXs = make_rsrc((const char*)a.X + row * xb, Du * xb);
    const __amdgpu_buffer_rsrc_t rmk = make_rsrc(a.exact_mask ? (const void*)(a.exact_mask + row) : a.X,
                                                 a.exact_mask ? Du : 0u);
    const __amdgpu_buffer_rsrc_t rvl = make_rsrc(a.exact_vals ? (const void*)(a.exact_vals + row) : a.X,
                                                 a.exact_vals ? Du * 4u : 0u);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + row, Du * 4u);
    const uint64_t below = (1ull << lane) - 1ull;
    // Three register sets (X, mask, exact values of a round) used in rotation by the loop
    // unrolled by three, so no set is copied while its loads are in flight
    struct Set {
        int64_t x[kMtGroups];
        uint32_t m[kMtGroups];
        float v[kMtGroups];
    };
    Set S0, S1, S2;
    auto load_x = [&](uint32_t i0, Set& o) {
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const uint32_t i = i0 + 64u * k + lane;
            if (XK == 0) {
                const auto w = __builtin_amdgcn_raw_buffer_load_b64(rXs, i * 8u, 0, kAuxNT);
                o.x[k] = (int64_t)(((uint64_t)w[1] << 32) | w[0]);
            } else if (XK == 1) {
                o.x[k] = __builtin_amdgcn_raw_buffer_load_b8(rXs, i, 0, kAuxNT);
            } else {
                o.x[k] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rXs, i * 4u, 0, kAuxNT);
            }
        }
    };
    auto load_m = [&](uint32_t i0, Set& o) {
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) o.m[k] = __builtin_amdgcn_raw_buffer_load_b8(rmk, i0 + 64u * k + lane, 0, 0);
    };
    auto load_v = [&](uint32_t i0, Set& o) {                     // the round's exact values (0 elsewhere)
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const int e = 64 * k + lane;
            const bool m = o.m[k] != 0u && e < kMtN;
            uint32_t slot = i0 + (uint32_t)e;
            if (compact) {
                const uint64_t bal = __ballot(m);
                slot = ebase + (uint32_t)__popcll(bal & below);
                ebase += (uint32_t)__popcll(bal);
            }
            o.v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rvl, qf_off(m, slot * 4u), 0, 0));
        }
    };
    int32_t flags = 0;
    // round c: X of c + 1 and the mask of c + 2 loaded, the values of c + 1 slotted from its mask
    // (loaded a round earlier); then the h stream's block and the outputs of round c
    auto round = [&](int64_t c, const Set& cur, Set& nx, Set& nx2) {
        const uint32_t i0 = (uint32_t)(c * kMtN);
        load_x(i0 + kMtN, nx);
        load_m(i0 + 2u * kMtN, nx2);
        if (c + 1 < c1) load_v(i0 + kMtN, nx);
        mt_twist_reg(sL, lane);
        float vv[kMtGroups], qq[kMtGroups];
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const int e = 64 * k + lane;
            const bool act = e < kMtN && (int64_t)i0 + e < D;
            const uint32_t w = mt_temper(sL[k]);
            const uint32_t h = hpow2 ? (w & (hl - 1u)) : (w % hl);                     // AS:528 randint
            const int64_t it = (int64_t)((uint64_t)cur.x[k] * (uint64_t)hl + h);       // AS:530 (int64 arithmetic)
            const bool inr = it >= -(int64_t)tab_n && it < (int64_t)tab_n;
            flags |= (act && !inr) ? UQ_QFL_BAD_INDEX : 0;
            const int32_t idx = inr ? (int32_t)(it < 0 ? it + tab_n : it) : 0;        // take wraps negatives
            vv[k] = cur.m[k] ? cur.v[k] : (inr ? tab[idx] : 0.f);                      // AS:531
        }
        div_n(vv, dp, qq);                                                              // AS:532 v / scale
#pragma unroll
        for (int k = 0; k < kMtGroups; ++k) {
            const int e = 64 * k + lane;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(qq[k]), ro, qf_off(e < kMtN, (i0 + (uint32_t)e) * 4u), 0,
                                                  kAuxNT);
        }
    };
    const uint32_t b0 = (uint32_t)(c0 * kMtN);
    load_x(b0, S0);
    load_m(b0, S0);
    load_m(b0 + kMtN, S1);
    load_v(b0, S0);
    for (int64_t c = c0; c < c1; c += 3) {
        round(c, S0, S1, S2);
        if (c + 1 < c1) round(c + 1, S1, S2, S0);
        if (c + 2 < c1) round(c + 2, S2, S0, S1);
    }
    *eend = ebase;
    return flags;
}

// KQ2 for batches: one wave per message, the table (<= 1024 floats) in LDS for the
// workgroup's waves.
template <int XK>
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_recv_wave_kernel(QflRecvArgs a) {
    __shared__ uint32_t Lsh[kQfWavesPerWG][kMtN];                // seed scratch per wave
    __shared__ float tab[kQflTab];
    for (int i = threadIdx.x; i < a.tab_n; i += 64 * kQfWavesPerWG) tab[i] = a.table[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    if (j >= a.n) return;
    uint32_t* Ls = Lsh[wv];
    if (lane == 0) mt_seed(Ls, (uint32_t)a.prng_seeds[j]);
    wave_lds_fence();
    uint32_t sL[kMtGroups];                                      // the h stream's block in registers
    mt_load(sL, Ls, lane);
    uint32_t etot = 0;
    int32_t flags = qfl_recv_rounds<XK>(a, tab, j, sL, 0, (a.D + kMtN - 1) / kMtN, 0u, &etot, lane);
    for (int o = 32; o >= 1; o >>= 1) flags |= __shfl_xor(flags, o);
    // AS:531 vec[exact_indeces] = exact_values raises unless the counts agree
    if (a.compact && a.exact_count && (int64_t)etot != (int64_t)a.exact_count[j]) flags |= UQ_QFL_BAD_EXACT;
    if (a.info && lane == 0) a.info[j] = flags;
}

// KQ2t for a few messages (the drop-in): one 512-thread workgroup per message.  The runs
// first count the exact coordinates of their rounds (their compact slots start after the
// earlier runs'), then wave 0 twists the h stream from its seed and hands each of the 7 runs
// its first block (as the sender's scouts do); the runs twist onward from there.
constexpr int kQrRuns = kQfTeamWaves - 1;
template <int XK>
__global__ void __launch_bounds__(64 * kQfTeamWaves)
quicfl_recv_team_kernel(QflRecvArgs a) {
    __shared__ float tab[kQflTab];
    __shared__ uint32_t SA[kQrRuns][kMtN];
    __shared__ uint32_t seed[kMtN];
    __shared__ uint32_t ecnt[kQrRuns];
    __shared__ int rdy[kQrRuns];
    __shared__ int32_t sflags;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = blockIdx.x;
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    const int64_t per = (nch + kQrRuns - 1) / kQrRuns;
    for (int i = threadIdx.x; i < a.tab_n; i += 64 * kQfTeamWaves) tab[i] = a.table[i];
    if (threadIdx.x < kQrRuns) rdy[threadIdx.x] = 0;
    if (threadIdx.x == 0) sflags = 0;
    if (wv == 0) {
        if (lane == 0) mt_seed(seed, (uint32_t)a.prng_seeds[j]);
    } else {                                             // run r's exact coordinates (compact slots)
        const int r = wv - 1;
        const int64_t c0 = r * per, c1 = min(nch, c0 + per);
        uint32_t cnt = 0;
        if (a.compact && a.exact_mask) {
            const uint8_t* mk = a.exact_mask + j * a.D;
            const int64_t e1 = min(a.D, c1 * kMtN);
            for (int64_t i = c0 * kMtN + lane; i < e1; i += 64) cnt += mk[i] != 0;
            for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
        }
        if (lane == 0) ecnt[r] = cnt;
    }
    __syncthreads();
    int32_t flags = 0;
    if (wv == 0) {                                       // the scout: blocks 0 .. start of the last run
        __builtin_amdgcn_s_setprio(3);
        uint32_t s[kMtGroups];
        mt_load(s, seed, lane);
        int64_t last = 0;
        for (int r = 0; r < kQrRuns; ++r)
            if (r * per < nch) last = r * per;
        for (int64_t k = 0; k <= last; ++k) {
            if (k) mt_twist_reg(s, lane);
            if (k % per == 0) {
                mt_store(s, SA[k / per], lane);
                wave_lds_fence();
                if (lane == 0) __hip_atomic_store(&rdy[k / per], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    } else {
        const int r = wv - 1;
        const int64_t c0 = r * per, c1 = min(nch, c0 + per);
        if (c0 < c1) {
            if (!a.force_timeout && qfl_wait_flag(&rdy[r])) {
                uint32_t s[kMtGroups];
                mt_load(s, SA[r], lane);
                uint32_t base = 0, eend = 0;
                for (int q = 0; q < r; ++q) base += ecnt[q];
                flags = qfl_recv_rounds<XK>(a, tab, j, s, c0, c1, base, &eend, lane);
            } else {
                flags = UQ_QFL_TIMEOUT;
            }
        }
        for (int o = 32; o >= 1; o >>= 1) flags |= __shfl_xor(flags, o);
        if (lane == 0 && flags) atomicOr(&sflags, flags);
    }
    __syncthreads();
    if (threadIdx.x == 0 && a.info) {
        int32_t f = sflags;
        uint32_t tot = 0;
        for (int q = 0; q < kQrRuns; ++q) tot += ecnt[q];
        if (a.compact && a.exact_count && (int64_t)tot != (int64_t)a.exact_count[j]) f |= UQ_QFL_BAD_EXACT;
        a.info[j] = f;
    }
}

// ---- receiver jump path (few messages): the h stream's run starts by jump-ahead ---------------
// KQ0s + KQ0j on the local stream only (one block per run: local block c0, the sender's polyA),
// then KQ2c counts each run's exact coordinates (compact slots), KQ2j runs every run of every
// message at once (qfl_recv_rounds), KQ2f ORs the flags and checks the exact count.
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_recv_count_kernel(QflRecvArgs a, QflRunArgs ra) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t id = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    const int64_t j = id / ra.R;
    const int r = (int)(id % ra.R);
    if (j >= a.n) return;
    int32_t cnt = 0;
    if (a.compact && a.exact_mask) {
        const uint8_t* mk = a.exact_mask + j * a.D;
        const int64_t e0 = (int64_t)r * ra.L * kMtN, e1 = min(a.D, e0 + ra.L * kMtN);
        if ((((uintptr_t)(mk + e0) | (uintptr_t)(mk + e1)) & 15) == 0) {
            // 16 bytes per lane (a 1 KB wave load); nonzero bytes of a word: the top bit of
            // ((w & 0x7F..) + 0x7F..) | w
            for (int64_t i = e0 + 16 * lane; i < e1; i += 1024) {
                const u32x4v q = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(mk + i));
                const uint32_t ws[4] = {q[0], q[1], q[2], q[3]};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    cnt += __popc((((ws[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | ws[k]) & 0x80808080u);
            }
        } else {
            for (int64_t i = e0 + lane; i < e1; i += 64) cnt += mk[i] != 0;
        }
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
    }
    if (lane == 0) ra.runinfo[(j * ra.R + r) * 2] = cnt;
}

template <int XK>
__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_recv_runs_kernel(QflRecvArgs a, QflRunArgs ra) {
    __shared__ float tab[kQflTab];
    __shared__ uint32_t seed[kQfWavesPerWG][kMtN];
    for (int i = threadIdx.x; i < a.tab_n; i += 64 * kQfWavesPerWG) tab[i] = a.table[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t id = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    const int64_t j = id / ra.R;
    const int r = (int)(id % ra.R);
    if (j >= a.n) return;
    const int64_t nch = (a.D + kMtN - 1) / kMtN;
    const int64_t c0 = (int64_t)r * ra.L, c1 = min(nch, c0 + ra.L);
    int32_t* info = ra.runinfo + (j * ra.R + r) * 2;
    if (c0 >= c1) {
        if (lane == 0) info[1] = 0;
        return;
    }
    uint32_t sL[kMtGroups];
    if (r == 0) {                                        // the h stream's block 0: the seed itself
        if (lane == 0) mt_seed(seed[wv], (uint32_t)a.prng_seeds[j]);
        wave_lds_fence();
        mt_load(sL, seed[wv], lane);
    } else {
        mj_block(sL, ra.parts + (j * ra.R + r) * kMjParts * kMtN, lane);
    }
    uint32_t ebase = 0;                                  // compact slots of the earlier runs (KQ2c)
    if (a.compact && a.exact_mask) {
        for (int q = lane; q < r; q += 64) ebase += (uint32_t)ra.runinfo[(j * ra.R + q) * 2];
        for (int o = 32; o >= 1; o >>= 1) ebase += __shfl_xor(ebase, o);
    }
    uint32_t eend = 0;
    int32_t flags = qfl_recv_rounds<XK>(a, tab, j, sL, c0, c1, ebase, &eend, lane);
    for (int o = 32; o >= 1; o >>= 1) flags |= __shfl_xor(flags, o);
    if (lane == 0) info[1] = flags;
}

__global__ void __launch_bounds__(64 * kQfWavesPerWG)
quicfl_recv_fin_kernel(QflRecvArgs a, QflRunArgs ra) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kQfWavesPerWG + wv;
    if (j >= a.n) return;
    const int32_t* info = ra.runinfo + j * ra.R * 2;
    int32_t flags = 0;
    int64_t tot = 0;
    for (int r = lane; r < ra.R; r += 64) {
        flags |= info[2 * r + 1];
        tot += info[2 * r];
    }
    for (int o = 32; o >= 1; o >>= 1) {
        flags |= __shfl_xor(flags, o);
        tot += __shfl_xor(tot, o);
    }
    // AS:531 vec[exact_indeces] = exact_values raises unless the counts agree
    if (a.compact && a.exact_count && tot != (int64_t)a.exact_count[j]) flags |= UQ_QFL_BAD_EXACT;
    if (lane == 0 && a.info) a.info[j] = flags;
}
