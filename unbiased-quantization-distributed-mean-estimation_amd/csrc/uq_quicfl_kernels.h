// uq_quicfl_kernels.h — QUIC-FL sender.  Included by uq_dme.hip inside
// its anonymous namespace, after uq_eden_kernels.h (the sender's RHT and norm are EDEN's).
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
// Kernel:
//   KQ1 quicfl_send_kernel  one 640-thread workgroup per message.  Both generators run as
//       MT19937 in LDS (double-buffered 624-word blocks: block b in buf[b & 1], so the words
//       of blocks b - 1 and b are readable while b + 1 is twisted into the other buffer).
//       Pass A: the local stream's first D words -> h (u8 scratch).  Pass B: 624 elements per
//       round; the local stream (words D..2D-1) and the global stream twist together (three
//       dependency phases each, one shared set of barriers), then each thread runs its
//       element through AS:472-490; the (X, p) table gather is one 8-byte load.  The exact
//       values are compacted in index order (wave ballots, per-wave counts written to LDS and
//       consumed after the next barrier).  Barriers fence LDS only, so the next round's
//       vector loads stay in flight across them.
//   The global generator starts from ATen's mt19937 state (left, next, 624 words): the first
//   left - 1 words are state[next ..], then twisted blocks; the state after the D draws is
//   written back for the host to restore into torch's generator.

constexpr int kQfT = 640;              // threads per sender workgroup (10 waves)
constexpr int kMtN = 624;              // MT19937 state words
constexpr int kQfWaves = kQfT / 64;
constexpr float kQflExactT = 2.8856349124267573f;   // f32(norm.ppf(1 - 2^-9)) (AS:475-478)
constexpr int kQfStateWords = 2 + kMtN;             // (left, next, words) per generator state

// LDS-only barrier: orders LDS traffic between the waves without waiting for vector memory
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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

__device__ __forceinline__ void mt_seed(uint32_t* mt, uint32_t seed) {     // init_genrand, one lane
    mt[0] = seed;
    for (int i = 1; i < kMtN; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

// Twist block b of up to two streams (buf[b & 1] -> buf[(b + 1) & 1]).  Every thread calls
// it with the same flags.  The buffer written must be free (a barrier since its last
// readers); the call ends with a barrier, after which both blocks are readable.
__device__ __forceinline__ void mt_twist2(uint32_t (*s0)[kMtN], int64_t b0, bool do0, uint32_t (*s1)[kMtN],
                                          int64_t b1, bool do1, int tid) {
    const uint32_t* o0 = s0[b0 & 1];
    uint32_t* n0 = s0[(b0 + 1) & 1];
    const uint32_t* o1 = s1[b1 & 1];
    uint32_t* n1 = s1[(b1 + 1) & 1];
    uint32_t a0 = 0, c0 = 0, d0 = 0, a1 = 0, c1 = 0, d1 = 0;
    if (tid < kMtN) {
        if (do0) { a0 = o0[tid]; c0 = tid + 1 < kMtN ? o0[tid + 1] : 0u; d0 = tid < 227 ? o0[tid + 397] : 0u; }
        if (do1) { a1 = o1[tid]; c1 = tid + 1 < kMtN ? o1[tid + 1] : 0u; d1 = tid < 227 ? o1[tid + 397] : 0u; }
    }
    if (tid < 227) {                                            // from old words only
        if (do0) n0[tid] = mt_mix(a0, c0, d0);
        if (do1) n1[tid] = mt_mix(a1, c1, d1);
    }
    lds_sync();
    if (tid >= 227 && tid < 454) {                              // reads new[tid - 227]
        if (do0) n0[tid] = mt_mix(a0, c0, n0[tid - 227]);
        if (do1) n1[tid] = mt_mix(a1, c1, n1[tid - 227]);
    }
    lds_sync();
    if (tid >= 454 && tid < kMtN) {
        if (tid < kMtN - 1) {
            if (do0) n0[tid] = mt_mix(a0, c0, n0[tid - 227]);
            if (do1) n1[tid] = mt_mix(a1, c1, n1[tid - 227]);
        } else {                                                // the last word wraps to new[0]
            if (do0) n0[tid] = mt_mix(a0, n0[0], n0[396]);
            if (do1) n1[tid] = mt_mix(a1, n1[0], n1[396]);
        }
    }
    lds_sync();
}

struct QflSendArgs {
    const float* rot;           // [n][D] rotated vectors (the RHT's output)
    const float* nrm;           // [n] torch.norm of each
    const float2* tab;          // [numel] (table_X, table_p) pairs
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
};

__global__ void __launch_bounds__(kQfT)
quicfl_send_kernel(QflSendArgs a) {
    __shared__ uint32_t Ls[2][kMtN];      // local generator blocks
    __shared__ uint32_t Gs[2][kMtN];      // global generator blocks
    __shared__ int32_t wcnt[2][kQfWaves];
    __shared__ int32_t sflags;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int64_t j = blockIdx.x;
    const int64_t D = a.D;
    const int64_t row = j * D;
    int32_t gleft = 1, gnext = 0;
    if (a.px_state) {
        const uint32_t* st = a.px_state + j * kQfStateWords;
        gleft = (int32_t)st[0];
        gnext = (int32_t)st[1];
        for (int i = tid; i < kMtN; i += kQfT) Gs[0][i] = st[2 + i];
    } else if (tid == 64) {
        mt_seed(Gs[0], (uint32_t)a.px_seeds[j]);
    }
    if (tid == 0) {
        mt_seed(Ls[0], (uint32_t)a.prng_seeds[j]);
        sflags = 0;
    }
    const float nv = a.nrm[j];
    const float sc = (1.0f / nv) * a.sqrtD;                      // AS:466/470 (IEEE 1/x, then f32 mul)
    lds_sync();
    const int64_t nch = (D + kMtN - 1) / kMtN;
    const int h_len = a.h_len;
    uint8_t* hb = a.hbuf + row;

    // ---- pass A: h = randint(0, h_len, (D,), local) (AS:465/469): word i is block c + 1, slot tid
    int64_t haveL = 0;
    // (no barrier before a twist here: the buffer it writes held block c - 1, whose last
    // readers, round c - 2's lanes and round c - 1's twist, are behind that twist's barriers)
    for (int64_t c = 0; c < nch; ++c) {
        mt_twist2(Ls, haveL, true, Gs, 0, false, tid);
        ++haveL;
        const int64_t i = c * kMtN + tid;
        if (tid < kMtN && i < D) hb[i] = (uint8_t)(mt_temper(Ls[haveL & 1][tid]) % (uint32_t)h_len);
    }

    // ---- pass B: local words D + i (virtual position 624 + D + i), global words i
    const int64_t vL = (int64_t)kMtN + D;
    const int64_t qL = vL / kMtN, rL = vL % kMtN;
    const int64_t vG = gleft > 1 ? (int64_t)gnext : (int64_t)kMtN;     // the first left - 1 words are state[next ..]
    const int64_t qG = vG / kMtN, rG = vG % kMtN;
    int64_t haveG = 0;
    const float thr = kQflExactT;
    const float fdelta = a.delta;
    const float fh = (float)h_len;
    const float fhalf = (float)a.half;
    const int64_t numel = a.numel;
    int32_t flags = 0;
    int64_t etot = 0;                                            // exact values written so far
    bool pend = false;                                           // an exact value of the previous round
    float pend_v = 0.f;
    int pend_rank = 0;
    // loads of round c + 1 are issued before round c's twists
    float r_cur = 0.f, r_nxt = 0.f;
    uint32_t h_cur = 0, h_nxt = 0;
    if (tid < kMtN && tid < D) {
        r_cur = __builtin_nontemporal_load(a.rot + row + tid);
        h_cur = hb[tid];
    }
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t i0 = c * kMtN;
        const int64_t i = i0 + tid;
        const bool active = tid < kMtN && i < D;
        const int64_t in = i + kMtN;
        if (tid < kMtN && in < D) {
            r_nxt = __builtin_nontemporal_load(a.rot + row + in);
            h_nxt = hb[in];
        }
        lds_sync();                                              // round c-1's readers are done
        if (pend) {                                              // round c-1's exact values, in index order
            int64_t base = etot;
            for (int w = 0; w < wv; ++w) base += wcnt[(c - 1) & 1][w];
            a.ev[row + base + pend_rank] = pend_v;
        }
        if (c) {
            for (int w = 0; w < kQfWaves; ++w) etot += wcnt[(c - 1) & 1][w];
        }
        pend = false;
        const int64_t lastT = (D - 1 - i0) < (kMtN - 1) ? (D - 1 - i0) : (kMtN - 1);    // last slot used
        const int64_t needL = qL + c + ((rL + lastT) >= kMtN ? 1 : 0);
        const int64_t needG = qG + c + ((rG + lastT) >= kMtN ? 1 : 0);
        while (haveL < needL || haveG < needG) {
            const bool dl = haveL < needL, dg = haveG < needG;
            mt_twist2(Ls, haveL, dl, Gs, haveG, dg, tid);
            haveL += dl;
            haveG += dg;
        }
        bool ex = false;
        float v = 0.f;
        if (active) {
            const int64_t pL = rL + tid, pG = rG + tid;
            const int64_t bL = qL + c + (pL >= kMtN), bG = qG + c + (pG >= kMtN);
            const uint32_t wl = mt_temper(Ls[bL & 1][pL >= kMtN ? pL - kMtN : pL]);
            const uint32_t wg = mt_temper(Gs[bG & 1][pG >= kMtN ? pG - kMtN : pG]);
            v = r_cur * sc;                                          // AS:472
            ex = (v > thr) || (v < -thr);                            // AS:478
            const float q = ex ? 0.f : v / fdelta;                   // AS:480-481
            const float fl = floorf(q);
            const float p = q - fl;                                  // AS:483
            if (!(p >= 0.f && p <= 1.f)) flags |= UQ_QFL_BAD_P;
            const float bern = ((double)(wl & 0xFFFFFFu) * 0x1p-24 < (double)p) ? 1.f : 0.f;
            const float iq = fl + bern;                              // AS:484
            const float t1 = iq * fh;                                // AS:486 in f32 (no fma: -ffp-contract=off)
            const float t2 = t1 + (float)h_cur;
            const float idxf = t2 + fhalf;
            int64_t idx = 0;
            if (!(idxf > -9.0e18f && idxf < 9.0e18f)) {
                flags |= UQ_QFL_BAD_INDEX;
            } else {
                idx = (int64_t)idxf;                                 // .long(): truncation
                if (idx < -numel || idx >= numel) flags |= UQ_QFL_BAD_INDEX;
                else if (idx < 0) idx += numel;                      // torch.take wraps negatives
            }
            idx = idx < 0 ? 0 : (idx >= numel ? numel - 1 : idx);    // (flagged above; stay in bounds)
            const float2 t = a.tab[idx];                             // AS:486-487
            if (!(t.y >= 0.f && t.y <= 1.f)) flags |= UQ_QFL_BAD_PX;
            const float bx = ((double)(wg & 0xFFFFFFu) * 0x1p-24 < (double)t.y) ? 1.f : 0.f;
            const float xf = t.x + bx;                               // AS:489
            if (a.x_kind == 0) {
                int64_t xv = 0;
                if (xf > -9.2e18f && xf < 9.2e18f) xv = (int64_t)xf;  // AS:490 .long()
                else flags |= UQ_QFL_X_RANGE;
                __builtin_nontemporal_store(xv, (int64_t*)a.X + row + i);
            } else {
                int32_t xv = 0;
                if (xf > -1.0f && xf < 256.0f) xv = (int32_t)xf;
                else flags |= UQ_QFL_X_RANGE;
                ((uint8_t*)a.X)[row + i] = (uint8_t)xv;
            }
            a.mask[row + i] = ex ? 1 : 0;
        }
        // exact values: rank within the wave now, wave offsets after the next barrier
        const uint64_t bal = __ballot(ex);
        if (lane == 0) wcnt[c & 1][wv] = (int32_t)__popcll(bal);
        if (ex) {
            pend = true;
            pend_v = v;
            pend_rank = (int)__popcll(bal & ((1ull << lane) - 1ull));
        }
        r_cur = r_nxt;
        h_cur = h_nxt;
    }
    lds_sync();
    if (pend) {
        int64_t base = etot;
        for (int w = 0; w < wv; ++w) base += wcnt[(nch - 1) & 1][w];
        a.ev[row + base + pend_rank] = pend_v;
    }
    if (nch) {
        for (int w = 0; w < kQfWaves; ++w) etot += wcnt[(nch - 1) & 1][w];
    }
    if (flags) atomicOr(&sflags, flags);
    // the global generator after its D draws
    if (a.px_state_out) {
        uint32_t* so = a.px_state_out + j * kQfStateWords;
        const uint32_t* src;
        uint32_t left1, next1;
        if (D <= (int64_t)gleft - 1) {                           // every draw from the current block
            src = Gs[0];
            left1 = (uint32_t)(gleft - D);
            next1 = (uint32_t)(gnext + D);
        } else {
            const int64_t vlast = vG + D - 1;
            const int64_t bl = vlast / kMtN, pos = vlast % kMtN;
            src = Gs[bl & 1];
            next1 = (uint32_t)(pos + 1);
            left1 = (uint32_t)(kMtN - pos);
        }
        for (int i = tid; i < kMtN; i += kQfT) so[2 + i] = src[i];
        if (tid == 0) {
            so[0] = left1;
            so[1] = next1;
        }
    }
    lds_sync();
    if (tid == 0) {
        a.ecount[j] = (int32_t)etot;
        a.scale[j] = sc;
        a.info[j] = sflags;
    }
}
