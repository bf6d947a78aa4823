// Type-message codec "UQR1": rANS over the int8 type codes.
// Included by uq_dme.hip inside its anonymous namespace.  Format and symbol map: see the
// header of include/uq_dme.h (uq_tc_*) and codes.py; oracle/uq_codec.c restates it on the CPU
// byte for byte (tests compare whole messages).
//
//   KC1 tc_hist_kernel     code counts per client (SWAR nibble counters for codes -4..3,
//                          LDS atomics for the rest, per 64 Ki-code segment)
//   KC2 tc_table_kernel    one wave per client: code -> symbol counts, quantized frequencies
//                          (sum 2^12), cumulative table, header size
//   KC3 tc_encode_kernel   one wave per chunk (W interleaved rANS states x 1024 steps), 8 per
//                          workgroup: steps in reverse, renormalisation words pushed per step
//                          in lane order (ballot + popcount), final states; words go to a
//                          scratch stack
//   KC4 tc_layout_kernel   one wave per client: cumulative words per chunk, message size
//   KC5 tc_scan_kernel     message offsets (exclusive scan over clients)
//   KC6 tc_pack_kernel     header, tables, states and words into the packed messages
//   KC7 tc_decode_kernel   one wave per chunk, 8 per workgroup: LDS slot table, forward
//                          steps, words read per step in lane order; checks the chunk ends
//                          exactly
// Bytes: KC1 and KC3 read the codes (d per client each), KC3 writes <= 2 B per symbol of
// scratch, KC6 copies the words; KC7 reads the message and writes d code bytes.
constexpr int kTcProbBits = 12;
constexpr uint32_t kTcM = 1u << kTcProbBits;
constexpr uint32_t kTcL = 1u << 16;
constexpr int kTcSteps = 1024;
constexpr uint32_t kTcMagic = 0x31525155u;   // "UQR1"
constexpr int kTcHistSeg = 65536;
constexpr int kTcRing = 512;                 // decoder word-ring block (u16 words)

__host__ __device__ inline int tc_lanes(int64_t d) {
    int64_t w = (d + kTcSteps - 1) / kTcSteps;
    return (int)(w < 1 ? 1 : (w > 64 ? 64 : w));
}
__host__ __device__ inline int64_t tc_nchunks(int64_t d) {
    const int64_t csz = (int64_t)tc_lanes(d) * kTcSteps;
    return d > 0 ? (d + csz - 1) / csz : 0;
}
__host__ __device__ inline uint64_t tc_align4(uint64_t x) { return (x + 3u) & ~(uint64_t)3u; }
__host__ __device__ inline uint64_t tc_table_off(int nsym) { return tc_align4(40 + 2 * (uint64_t)nsym); }
__host__ __device__ inline uint64_t tc_header_bytes(int nsym, int64_t nch, int W) {
    return tc_table_off(nsym) + 4 * (uint64_t)nch + 4 * (uint64_t)nch * (uint64_t)W;
}
__host__ __device__ inline uint64_t tc_bound(int64_t d) {
    return tc_header_bytes(256, tc_nchunks(d), tc_lanes(d)) + tc_align4(2 * (uint64_t)d);
}
__device__ __forceinline__ int tc_sym(int c, bool exact) {       // c: the int8 code as int
    const int k = c < 0 ? -c - 1 : c;
    const int neg = c < 0 ? 1 : 0;
    return 2 * k + (exact ? neg : (neg & (k > 0 ? 1 : 0)));
}
__device__ __forceinline__ int8_t tc_code(int s) {
    const int k = s >> 1;
    return (s & 1) ? (int8_t)(-k - 1) : (int8_t)k;
}

struct TcTable {            // per client, in the workspace
    uint32_t nsym, hdr_bytes, total_words, pad;
    uint32_t f[256];
    uint32_t cum[256];
};

// KC1: histogram of the int8 CODES (KC2 maps codes to symbols).  Codes are heavily skewed
// (0 for ~80 % of the coordinates at R = 1, most of the rest in -4..3), so one LDS atomic per
// byte would serialise on a few bins, and per-byte branches load the CU's one scalar unit.
// Codes -4..3 are counted branch-free: a SWAR byte add maps them to 0..7, each byte adds
// 1 << 4q to one of two nibble accumulators (even / odd bytes: <= 8 per pass, no carry),
// unpacked after every 16 bytes into four registers of two 16-bit fields (bins q and q + 4;
// a lane sees <= 256 bytes per segment, a wave <= 16384, so no field carries); they are
// summed over the wave by shuffles.  A lane whose 16 bytes hold another code adds those to
// LDS atomically (rare).
__global__ void __launch_bounds__(256)
tc_hist_kernel(const int8_t* __restrict__ codes, int64_t d, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    h[tid] = 0u;
    __syncthreads();
    const int64_t vec = blockIdx.y;
    const int64_t b = (int64_t)blockIdx.x * kTcHistSeg;
    const int64_t e = min(d, b + kTcHistSeg);
    const int8_t* row = codes + vec * d;
    const bool al = ((((uintptr_t)(row + b)) & 15u) == 0u);
    uint32_t cq[4] = {0u, 0u, 0u, 0u};              // cq[j]: bins j (low half) and j + 4 (high)
    auto rare_add = [&](uint32_t byte) {
        if (((byte + 4u) & 0xFFu) >= 8u) atomicAdd(&h[byte], 1u);
    };
    auto pass = [&](const uint4& w) {
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        uint32_t acc[2] = {0u, 0u};
        uint32_t any = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = ((ws[k] & 0x7F7F7F7Fu) + 0x04040404u) ^ (ws[k] & 0x80808080u);   // bytes + 4
            any |= t & 0xF8F8F8F8u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = (t >> (8 * j)) & 0xFFu;
                acc[j & 1] += q < 8u ? (1u << (4 * q)) : 0u;
            }
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < 4; ++j) cq[j] += (acc[a] >> (4 * j)) & 0x000F000Fu;
        if (any) {
#pragma unroll 1
            for (int k = 0; k < 16; ++k) rare_add((ws[k >> 2] >> (8 * (k & 3))) & 0xFFu);
        }
    };
    if (al) {
        int64_t i = b + (int64_t)tid * 16;
        for (; i + 256 * 16 + 16 <= e; i += 2 * 256 * 16) {         // two loads in flight
            const uint4 w0 = *reinterpret_cast<const uint4*>(row + i);
            const uint4 w1 = *reinterpret_cast<const uint4*>(row + i + 256 * 16);
            pass(w0);
            pass(w1);
        }
        for (; i + 16 <= e; i += 256 * 16) pass(*reinterpret_cast<const uint4*>(row + i));
        for (; i < e; ++i) {                                          // ragged end: one thread
            const uint32_t byte = (uint32_t)(uint8_t)row[i];
            const uint32_t q = (byte + 4u) & 0xFFu;
            if (q < 8u) cq[q & 3u] += 1u << (16 * (q >> 2));
            else atomicAdd(&h[byte], 1u);
        }
    } else {
        for (int64_t i = b + tid; i < e; i += 256) {
            const uint32_t byte = (uint32_t)(uint8_t)row[i];
            const uint32_t q = (byte + 4u) & 0xFFu;
            if (q < 8u) cq[q & 3u] += 1u << (16 * (q >> 2));
            else atomicAdd(&h[byte], 1u);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        for (int o = 32; o > 0; o >>= 1) cq[j] += (uint32_t)__shfl_xor((int)cq[j], o, 64);
    if (lane < 8) {                                   // bin q = lane <-> code q - 4
        const uint32_t v = lane == 0 ? cq[0] : lane == 1 ? cq[1] : lane == 2 ? cq[2] : lane == 3 ? cq[3]
                         : lane == 4 ? cq[0] : lane == 5 ? cq[1] : lane == 6 ? cq[2] : cq[3];
        const uint32_t cnt = (v >> (16 * (lane >> 2))) & 0xFFFFu;
        if (cnt) atomicAdd(&h[(lane - 4) & 0xFF], cnt);
    }
    __syncthreads();
    if (h[tid]) atomicAdd(&hist[vec * 256 + tid], h[tid]);
}

// KC2: one wave per client.
__global__ void __launch_bounds__(64)
tc_table_kernel(const uint32_t* __restrict__ hist, int64_t d, int exact, TcTable* __restrict__ tabs) {
    __shared__ uint32_t sc[256];
    const int64_t vec = blockIdx.x;
    const int lane = threadIdx.x;
    const uint32_t* hc = hist + vec * 256;          // counts per code byte
    uint32_t c[4], f[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sc[lane + 64 * r] = 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {                   // symbol counts (value mode folds code -1 into 0)
        const int b = lane + 64 * r;
        const uint32_t n = hc[b];
        if (n) atomicAdd(&sc[tc_sym((int)(int8_t)b, exact != 0)], n);
    }
    __syncthreads();
    int smax = -1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int s = lane + 64 * r;
        c[r] = sc[s];
        if (c[r]) smax = s;
    }
    for (int o = 32; o > 0; o >>= 1) smax = max(smax, __shfl_xor(smax, o, 64));
    const int nsym = d > 0 ? 2 * (smax >> 1) + 2 : 0;
    int64_t sum = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        f[r] = c[r] ? (uint32_t)(((uint64_t)c[r] * kTcM) / (uint64_t)d) : 0u;
        if (c[r] && f[r] == 0u) f[r] = 1u;
        sum += f[r];
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    // normalisation (oracle/uq_codec.c uqc_normalize): adjust the most frequent symbol
    // (lowest index on ties) until the sum is M
    while (d > 0 && sum != (int64_t)kTcM) {
        uint32_t key = 0u;                         // (f << 8) | (255 - s): max = largest f, lowest s
#pragma unroll
        for (int r = 0; r < 4; ++r) key = max(key, (f[r] << 8) | (uint32_t)(255 - (lane + 64 * r)));
        for (int o = 32; o > 0; o >>= 1) key = max(key, (uint32_t)__shfl_xor((int)key, o, 64));
        const int best = 255 - (int)(key & 0xFFu);
        const uint32_t fb = key >> 8;
        int64_t delta;
        if (sum < (int64_t)kTcM) {
            delta = (int64_t)kTcM - sum;
        } else {
            delta = sum - (int64_t)kTcM;
            if (delta > (int64_t)fb - 1) delta = (int64_t)fb - 1;
            delta = -delta;
        }
        if ((best & 63) == lane) f[best >> 6] = (uint32_t)((int64_t)fb + delta);
        sum += delta;
    }
    // cumulative frequencies: symbol s = lane + 64 r, scanned in symbol order
    TcTable* t = tabs + vec;
    uint32_t base = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint32_t incl = f[r];
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)incl, o, 64);
            if (lane >= o) incl += u;
        }
        t->f[lane + 64 * r] = f[r];
        t->cum[lane + 64 * r] = base + incl - f[r];
        base += (uint32_t)__shfl((int)incl, 63, 64);
    }
    if (lane == 0) {
        const int64_t nch = tc_nchunks(d);
        t->nsym = (uint32_t)nsym;
        t->hdr_bytes = (uint32_t)tc_header_bytes(nsym, nch, tc_lanes(d));
    }
}

// KC3 layout: scratch [n][nch][csz] u16 (the chunk's words end at csz); cwords [n][nch] u32,
// states [n][nch][W] u32.  Steps run in reverse in blocks of 16 (tc_load_blk prefetches a
// lane's 16 code bytes of the next block in the generic path).  x / f uses the invariant
// divisor form of tc_div (exact for every 32-bit x; tools/tc_div_check.c).
constexpr int kTcBlk = 16;

__device__ __forceinline__ void tc_load_blk(uint32_t (&b)[kTcBlk], const int8_t* row, int64_t blk, int W, int lane,
                                            int64_t len) {
#pragma unroll
    for (int t = 0; t < kTcBlk; ++t) {
        const int64_t i = (blk * kTcBlk + t) * W + lane;
        b[t] = (lane < W && i < len) ? (uint32_t)(uint8_t)row[i] : 0u;
    }
}

__device__ __forceinline__ void tc_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// KC3: grid (ceil(nch / kTcEncWaves), n), one wave per chunk; the waves of a workgroup share
// the per-symbol constants, one 16-byte LDS entry {x_max, f | cum << 16, divisor magic}.  Full
// chunks (W = 64 lanes x 1024 steps: every chunk of d >= 65536 but a ragged last one) take a
// branch-free path: each block of 16 steps arrives as one 16-byte load per lane (1 KB per
// wave, loaded a block ahead) staged in LDS and read back one byte per step; words go to a
// per-wave LDS ring (non-renormalising lanes write a dummy slot instead of branching) and
// leave as 8-byte stores per lane, 256 words at a time, tested every 4 steps.  The words,
// their order and the final states are those of the generic path.
struct alignas(16) TcEnc {
    uint32_t xmax;      // renormalise while x > xmax: x >= f << 20 (f = 4096 never)
    uint32_t fc;        // f | cum << 16
    uint32_t mg;        // x / f = (t + ((x - t) >> s1)) >> s2, t = mulhi(mg, x)
    uint32_t sh;        // s1 | s2 << 8
};
// Division by the invariant f (Granlund & Montgomery 1994, fig. 4.1): exact for every
// 32-bit x; l = ceil(log2 f), mg = floor(2^32 (2^l - f) / f) + 1, s1 = min(l, 1),
// s2 = max(l - 1, 0).
__device__ __forceinline__ uint32_t tc_div(uint32_t x, uint32_t mg, uint32_t sh) {
    const uint32_t t = __umulhi(mg, x);
    return (t + ((x - t) >> (sh & 0xFFu))) >> (sh >> 8);
}
constexpr int kTcEncWaves = 8;
constexpr int kTcRingW = 1024;              // encoder word ring per wave (u16), power of two
constexpr int kTcFlush = 256;               // words per ring flush (one 8-byte store per lane)

__global__ void __launch_bounds__(64 * kTcEncWaves)
tc_encode_kernel(const int8_t* __restrict__ codes, int64_t d, int exact, const TcTable* __restrict__ tabs,
                 uint16_t* __restrict__ scratch, uint32_t* __restrict__ cwords, uint32_t* __restrict__ states) {
    __shared__ TcEnc se[256];
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[kTcEncWaves][kTcBlk * 64];
    __shared__ __attribute__((aligned(16))) uint16_t ring[kTcEncWaves][kTcRingW + 64];   // + dummy slots
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t vec = blockIdx.y;
    const TcTable* t = tabs + vec;
    for (int q = tid; q < 256; q += 64 * kTcEncWaves) {
        const uint32_t f = t->f[q];
        int l = 0;
        while (l < 31 && (1u << l) < f) ++l;                      // ceil(log2 f)
        TcEnc e;
        e.xmax = f >= 4096u ? 0xFFFFFFFFu : (f << 20) - 1u;
        e.fc = f | (t->cum[q] << 16);
        e.mg = f ? (uint32_t)((((uint64_t)((1u << l) - f)) << 32) / f + 1u) : 0u;
        e.sh = (uint32_t)(l < 1 ? l : 1) | ((uint32_t)(l > 1 ? l - 1 : 0) << 8);
        se[q] = e;
    }
    __syncthreads();
    const int W = tc_lanes(d);
    const int64_t nch = tc_nchunks(d);
    const int64_t c = (int64_t)blockIdx.x * kTcEncWaves + wv;
    if (c >= nch) return;                                           // no workgroup barriers below
    const int64_t csz = (int64_t)W * kTcSteps;
    const int64_t base = c * csz;
    const int64_t len = min(csz, d - base);
    const int8_t* row = codes + vec * d + base;
    uint16_t* stk = scratch + (vec * nch + c) * csz;
    uint32_t x = kTcL;
    const uint64_t below = (1ull << lane) - 1ull;
    if (W == 64 && len == csz) {
        uint8_t* sb = sbuf[wv];
        uint16_t* rg = ring[wv];
        // block b holds steps 16b .. 16b+15: bytes [1024 b, 1024 b + 1024) of the chunk
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        const bool al = (((uintptr_t)row) & 15u) == 0u;
        auto load = [&](int b) -> uint4 {
            if (al) return rv[b * 64 + lane];
            const int8_t* p = row + (int64_t)b * 1024 + 16 * lane;
            uint32_t w4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w4[q] = (uint32_t)(uint8_t)p[4 * q] | ((uint32_t)(uint8_t)p[4 * q + 1] << 8) |
                        ((uint32_t)(uint8_t)p[4 * q + 2] << 16) | ((uint32_t)(uint8_t)p[4 * q + 3] << 24);
            return make_uint4(w4[0], w4[1], w4[2], w4[3]);
        };
        constexpr int nblk = kTcSteps / kTcBlk;                     // 64
        int ptr = (int)csz, fl = (int)csz;                          // words [ptr, fl) are in the ring
        uint4 nx = load(nblk - 1);
        for (int b = nblk - 1; b >= 0; --b) {
            tc_wave_sync();
            reinterpret_cast<uint4*>(sb)[lane] = nx;
            tc_wave_sync();
            if (b > 0) nx = load(b - 1);
#pragma unroll
            for (int g = 3; g >= 0; --g) {
#pragma unroll
                for (int tt = 4 * g + 3; tt >= 4 * g; --tt) {
                    const TcEnc e = se[tc_sym((int)(int8_t)sb[tt * 64 + lane], exact != 0)];
                    const bool need = x > e.xmax;
                    const uint64_t mk = __ballot(need);
                    const int k = __popcll(mk);
                    const int slot = need ? ((ptr - k + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u))) & (kTcRingW - 1))
                                          : kTcRingW + lane;
                    rg[slot] = (uint16_t)(x & 0xFFFFu);
                    x = need ? x >> 16 : x;
                    ptr -= k;
                    const uint32_t f = e.fc & 0xFFFFu;
                    const uint32_t qd = tc_div(x, e.mg, e.sh);               // floor(x / f), exact
                    x = (qd << kTcProbBits) + (x - qd * f) + (e.fc >> 16);
                }
                if (fl - ptr >= kTcFlush) {                           // uniform; pending <= 256 + 7 + 256
                    tc_wave_sync();
                    const int o = fl - kTcFlush;                      // multiple of 4: 8-byte aligned
                    const uint2 w = *reinterpret_cast<const uint2*>(&rg[(o + 4 * lane) & (kTcRingW - 1)]);
                    *reinterpret_cast<uint2*>(stk + o + 4 * lane) = w;
                    fl = o;
                }
            }
        }
        tc_wave_sync();
        for (int p = ptr + lane; p < fl; p += 64) stk[p] = rg[p & (kTcRingW - 1)];
        states[(vec * nch + c) * W + lane] = x;
        if (lane == 0) cwords[vec * nch + c] = (uint32_t)(csz - ptr);
        return;
    }
    const int64_t steps = (len + W - 1) / W;
    int64_t ptr = csz;
    const int64_t nblk = (steps + kTcBlk - 1) / kTcBlk;
    uint32_t cur[kTcBlk], nxt[kTcBlk];
    tc_load_blk(cur, row, nblk - 1, W, lane, len);
    for (int64_t blk = nblk - 1; blk >= 0; --blk) {
        if (blk > 0) tc_load_blk(nxt, row, blk - 1, W, lane, len);
#pragma unroll
        for (int tt = kTcBlk - 1; tt >= 0; --tt) {
            const int64_t st = blk * kTcBlk + tt;
            if (st >= steps) continue;                                  // uniform
            const bool act = lane < W && st * W + lane < len;
            int s = 0;
            bool need = false;
            if (act) {
                s = tc_sym((int)(int8_t)cur[tt], exact != 0);
                need = x > se[s].xmax;
            }
            const uint64_t mk = __ballot(need);
            const int k = __popcll(mk);
            if (need) {
                stk[ptr - k + __popcll(mk & below)] = (uint16_t)(x & 0xFFFFu);
                x >>= 16;
            }
            ptr -= k;
            if (act) {
                const TcEnc e = se[s];
                const uint32_t f = e.fc & 0xFFFFu;
                const uint32_t qd = tc_div(x, e.mg, e.sh);          // floor(x / f), exact
                x = (qd << kTcProbBits) + (x - qd * f) + (e.fc >> 16);
            }
        }
#pragma unroll
        for (int tt = 0; tt < kTcBlk; ++tt) cur[tt] = nxt[tt];
    }
    if (lane < W) states[(vec * nch + c) * W + lane] = x;
    if (lane == 0) cwords[vec * nch + c] = (uint32_t)(csz - ptr);
}

// KC4: one wave per client: cumulative words per chunk (in place), total, message size.
__global__ void __launch_bounds__(64)
tc_layout_kernel(int64_t d, TcTable* __restrict__ tabs, uint32_t* __restrict__ cwords, uint64_t* __restrict__ sizes) {
    const int64_t vec = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t nch = tc_nchunks(d);
    uint32_t* cw = cwords + vec * nch;
    uint32_t carry = 0u;
    for (int64_t c0 = 0; c0 < nch; c0 += 64) {
        const bool in = c0 + lane < nch;
        uint32_t v = in ? cw[c0 + lane] : 0u;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)v, o, 64);
            if (lane >= o) v += u;
        }
        if (in) cw[c0 + lane] = carry + v;               // words_end[c]
        carry += (uint32_t)__shfl((int)v, 63, 64);
    }
    if (lane == 0) {
        tabs[vec].total_words = carry;
        sizes[vec] = (uint64_t)tabs[vec].hdr_bytes + tc_align4(2 * (uint64_t)carry);
    }
}

// KC5: offsets[j] = sum of sizes before j, offsets[n] = total (one workgroup).
__global__ void __launch_bounds__(1024)
tc_scan_kernel(const uint64_t* __restrict__ sizes, int64_t n, uint64_t* __restrict__ offsets) {
    __shared__ uint64_t s[1024];
    __shared__ uint64_t carry;
    const int tid = threadIdx.x;
    if (tid == 0) carry = 0ull;
    __syncthreads();
    for (int64_t j0 = 0; j0 < n; j0 += 1024) {
        const uint64_t v = j0 + tid < n ? sizes[j0 + tid] : 0ull;
        s[tid] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint64_t u = tid >= o ? s[tid - o] : 0ull;
            __syncthreads();
            s[tid] += u;
            __syncthreads();
        }
        if (j0 + tid < n) offsets[j0 + tid] = carry + s[tid] - v;
        __syncthreads();
        if (tid == 0) carry += s[1023];
        __syncthreads();
    }
    if (tid == 0) offsets[n] = carry;
}

__device__ __forceinline__ void tc_put32(uint8_t* p, uint32_t v) {   // 4-byte aligned
    *reinterpret_cast<uint32_t*>(p) = v;
}

// KC6: grid (nch, n), 256 threads.  Chunk c's workgroup writes words_end[c], its states and
// its words; chunk 0's also the fixed header and the frequency table; the last chunk's the
// padding word.
__global__ void __launch_bounds__(256)
tc_pack_kernel(int64_t d, int64_t m, int exact, const float* __restrict__ l1, const TcTable* __restrict__ tabs,
               const uint16_t* __restrict__ scratch, const uint32_t* __restrict__ cwords,
               const uint32_t* __restrict__ states, const uint64_t* __restrict__ offsets, uint8_t* __restrict__ msgs) {
    const int tid = threadIdx.x;
    const int64_t vec = blockIdx.y;
    const int64_t c = blockIdx.x;
    const TcTable* t = tabs + vec;
    const int W = tc_lanes(d);
    const int64_t nch = tc_nchunks(d);
    const int64_t csz = (int64_t)W * kTcSteps;
    const int nsym = (int)t->nsym;
    uint8_t* msg = msgs + offsets[vec];
    const uint64_t toff = tc_table_off(nsym);
    uint32_t* wend = reinterpret_cast<uint32_t*>(msg + toff);
    uint32_t* st = wend + nch;
    uint16_t* words = reinterpret_cast<uint16_t*>(msg + t->hdr_bytes);
    if (c < nch) {                                     // (d == 0: a header-only message)
        const uint32_t* cw = cwords + vec * nch;
        const uint32_t w0 = c ? cw[c - 1] : 0u, w1 = cw[c];
        if (tid == 0) wend[c] = w1;
        if (tid < W) st[c * W + tid] = states[(vec * nch + c) * W + tid];
        const uint16_t* src = scratch + (vec * nch + c) * csz + (csz - (int64_t)(w1 - w0));
        for (uint32_t k = tid; k < w1 - w0; k += 256) words[w0 + k] = src[k];
        if (c == nch - 1 && tid == 0 && (t->total_words & 1u)) words[t->total_words] = 0;
    }
    if (c == 0) {
        if (tid == 0) {
            const uint64_t size = offsets[vec + 1] - offsets[vec];
            tc_put32(msg + 0, kTcMagic);
            tc_put32(msg + 4, 1u | ((uint32_t)(exact ? 1 : 0) << 16));
            tc_put32(msg + 8, (uint32_t)(uint64_t)d);
            tc_put32(msg + 12, (uint32_t)((uint64_t)d >> 32));
            tc_put32(msg + 16, (uint32_t)(uint64_t)m);
            tc_put32(msg + 20, (uint32_t)((uint64_t)m >> 32));
            tc_put32(msg + 24, __float_as_uint(l1[vec]));
            tc_put32(msg + 28, (uint32_t)nsym | ((uint32_t)kTcProbBits << 16) | ((uint32_t)W << 24));
            tc_put32(msg + 32, (uint32_t)nch);
            tc_put32(msg + 36, (uint32_t)size);
        }
        uint16_t* ft = reinterpret_cast<uint16_t*>(msg + 40);
        for (int s = tid; s < nsym; s += 256) ft[s] = (uint16_t)t->f[s];
        if (tid == 0 && (nsym & 1)) ft[nsym] = 0;
    }
}

// KC7: grid (ceil(nch / kTcDecWaves), n), one wave per chunk; the waves of a workgroup
// share the client's slot table.  status[vec] |= 1 bad header, 2 table, 4 words overrun /
// underrun, 8 final state.
//   Slot table: one u32 per slot = code | (f - 1) << 8 | (slot - cum[s]) << 20, so a step is
//   one LDS read (x' = f (x >> 12) + slot - cum[s]) before the renormalisation read.
//   Words: a per-wave LDS ring of kTcDecRing words (word v in slot v mod kTcDecRing),
//   refilled 256 words at a time from registers loaded one refill ahead.  Full chunks (W =
//   64, 1024 steps) run groups of 4 steps: before a group the ring holds every word it can
//   take (<= 256) and the overrun test is made once; inside, no branches (the scalar unit,
//   one per CU, bounded the branchy form).  Codes of 16 steps (1 KB) are staged in LDS and
//   leave as one 16-byte store per lane.  Other chunks take the checked step by step path.
constexpr int kTcDecWaves = 8;
constexpr int kTcDecRing = 1024;            // ring words per wave
constexpr int kTcDecFill = 256;             // words per refill (4 per lane)

__global__ void __launch_bounds__(64 * kTcDecWaves)
tc_decode_kernel(const uint8_t* __restrict__ msgs, uint64_t msgs_bytes, const uint64_t* __restrict__ offsets,
                 int64_t d, int64_t m_expect, int8_t* __restrict__ codes, float* __restrict__ l1,
                 int32_t* __restrict__ kmax, int32_t* __restrict__ status) {
    __shared__ uint32_t tab[kTcM];
    __shared__ uint32_t sf[256], scum[257];
    __shared__ uint16_t ring[kTcDecWaves][kTcDecRing];
    __shared__ __attribute__((aligned(16))) uint8_t ob[kTcDecWaves][kTcBlk * 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t vec = blockIdx.y;
    // offsets come from the peer: nothing is read unless [o0, o1) lies inside the buffer
    const uint64_t o0 = offsets[vec], o1 = offsets[vec + 1];
    if (!(o0 <= o1 && o1 <= msgs_bytes && o1 - o0 >= 40 && (o0 & 3u) == 0u)) {
        if (tid == 0 && blockIdx.x == 0) atomicOr(&status[vec], 1);
        return;
    }
    const uint8_t* msg = msgs + o0;
    const uint64_t size = o1 - o0;
    const uint32_t* h = reinterpret_cast<const uint32_t*>(msg);
    // every header carries m (h[4..5]); a batch is decoded for one m (codes_mean / decode
    // apply it), so a message of another m is flagged (bit 4) instead of mis-scaled
    if (m_expect >= 0 && ((uint64_t)h[4] | ((uint64_t)h[5] << 32)) != (uint64_t)m_expect) {
        if (tid == 0 && blockIdx.x == 0) atomicOr(&status[vec], 16);
        return;
    }
    const int W = tc_lanes(d);
    const int64_t nch = tc_nchunks(d);
    const int64_t c = (int64_t)blockIdx.x * kTcDecWaves + wv;
    bool ok = h[0] == kTcMagic && (h[1] & 0xFFFFu) == 1u &&
              ((uint64_t)h[2] | ((uint64_t)h[3] << 32)) == (uint64_t)d && ((h[7] >> 16) & 0xFFu) == (uint32_t)kTcProbBits &&
              (int)(h[7] >> 24) == W && (int64_t)h[8] == nch && (uint64_t)h[9] == size;
    const int nsym = ok ? (int)(h[7] & 0xFFFFu) : 0;
    ok = ok && nsym <= 256 && (d == 0 || nsym >= 2) && tc_header_bytes(nsym, nch, W) <= size;
    if (!ok) {                                                      // uniform over the workgroup
        if (tid == 0 && blockIdx.x == 0) atomicOr(&status[vec], 1);
        return;
    }
    if (d == 0) {
        if (tid == 0) {
            l1[vec] = __uint_as_float(h[6]);
            kmax[vec] = 0;
        }
        return;
    }
    const uint16_t* ft = reinterpret_cast<const uint16_t*>(msg + 40);
    for (int q = tid; q < 256; q += 64 * kTcDecWaves) sf[q] = q < nsym ? (uint32_t)ft[q] : 0u;
    __syncthreads();
    if (tid == 0) {
        uint32_t a = 0u;
        for (int q = 0; q < 256; ++q) {
            scum[q] = a;
            a += sf[q];
        }
        scum[256] = a;
    }
    __syncthreads();
    if (scum[256] != kTcM) {
        if (tid == 0 && blockIdx.x == 0) atomicOr(&status[vec], 2);
        return;
    }
    // slot -> (code, f - 1, slot - cum[s]): the s with cum[s] <= slot < cum[s+1]
    for (uint32_t j = tid; j < kTcM; j += 64 * kTcDecWaves) {
        int lo = 0, hi = 255;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (scum[mid] <= j) lo = mid; else hi = mid - 1;
        }
        tab[j] = (uint32_t)(uint8_t)tc_code(lo) | ((sf[lo] - 1u) << 8) | ((j - scum[lo]) << 20);
    }
    __syncthreads();
    if (c >= nch) return;                                           // no workgroup barriers below
    const uint64_t toff = tc_table_off(nsym);
    const uint32_t* wend = reinterpret_cast<const uint32_t*>(msg + toff);
    const uint32_t* st = wend + nch;
    const uint16_t* words = reinterpret_cast<const uint16_t*>(msg + tc_header_bytes(nsym, nch, W));
    const uint64_t wmax = (size - tc_header_bytes(nsym, nch, W)) / 2;
    const int64_t csz = (int64_t)W * kTcSteps;
    const int64_t base = c * csz;
    const int64_t len = min(csz, d - base);
    const int64_t steps = (len + W - 1) / W;
    const uint32_t r0 = c ? wend[c - 1] : 0u;
    const uint32_t rend = wend[c];
    bool bad = rend > wmax || r0 > rend;
    const uint32_t nw = bad ? 0u : rend - r0;        // the chunk's words: words[r0 .. rend)
    const uint16_t* cwp = words + r0;
    uint16_t* rg = ring[wv];
    constexpr int kPF = kTcDecFill / 64;
    uint16_t pf[kPF];
    uint32_t fu = 0;                                 // words [fu - kTcDecRing, fu) are in the ring
    auto fetch = [&]() {                             // pf = words [fu, fu + kTcDecFill)
#pragma unroll
        for (int j = 0; j < kPF; ++j) {
            const uint32_t v = fu + (uint32_t)(lane + 64 * j);
            pf[j] = v < nw ? cwp[v] : (uint16_t)0;
        }
    };
    auto refill = [&]() {
        tc_wave_sync();
#pragma unroll
        for (int j = 0; j < kPF; ++j) rg[(fu + (uint32_t)(lane + 64 * j)) & (kTcDecRing - 1)] = pf[j];
        fu += kTcDecFill;
        fetch();
        tc_wave_sync();
    };
    fetch();
    refill();
    uint32_t u = 0;                                  // words consumed
    uint32_t x = lane < W ? st[c * W + lane] : kTcL;
    int8_t* row = codes + vec * d + base;
    // one step of a lane with a symbol; `chk`: test the word count (false on an overrun)
    auto step = [&](int8_t& code, bool act, bool chk) -> bool {
        if (act) {
            const uint32_t e = tab[x & (kTcM - 1u)];
            x = (((e >> 8) & 0xFFFu) + 1u) * (x >> kTcProbBits) + (e >> 20);
            code = (int8_t)(e & 0xFFu);
        }
        const bool need = act && x < kTcL;
        const uint64_t mk = __ballot(need);
        const uint32_t k = (uint32_t)__popcll(mk);
        if (chk && u + k > nw) return false;
        const uint32_t v = u + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
        const uint32_t wd = rg[v & (kTcDecRing - 1)];
        x = need ? ((x << 16) | wd) : x;
        u += k;
        return true;
    };
    if (W == 64 && len == csz) {
        uint8_t* obw = ob[wv];
        for (int b = 0; b < kTcSteps / kTcBlk && !bad; ++b) {
#pragma unroll
            for (int g = 0; g < kTcBlk / 4; ++g) {
                if (fu < u + 2 * kTcDecFill) refill();               // uniform; keeps fu <= u + 768
                if (fu < u + kTcDecFill) refill();
                const bool chk = u + (uint32_t)kTcDecFill > nw;      // near the end: test each step
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    int8_t code = 0;
                    if (!step(code, true, chk)) {
                        bad = true;
                        break;
                    }
                    obw[(4 * g + t) * 64 + lane] = (uint8_t)code;
                }
                if (bad) break;
            }
            if (bad) break;
            tc_wave_sync();
            reinterpret_cast<uint4*>(row + (int64_t)b * (kTcBlk * 64))[lane] = reinterpret_cast<const uint4*>(obw)[lane];
            tc_wave_sync();
        }
    } else {
        for (int64_t s0 = 0; s0 < steps && !bad; ++s0) {
            if (fu < u + 2 * kTcDecFill) refill();
            if (fu < u + kTcDecFill) refill();
            const int64_t i = s0 * W + lane;
            const bool act = lane < W && i < len;
            int8_t code = 0;
            if (!step(code, act, true)) {
                bad = true;
                break;
            }
            if (act) row[i] = code;
        }
    }
    const uint32_t r = r0 + u;
    const bool endbad = __ballot(lane < W && x != kTcL) != 0ull;
    if (lane == 0) {
        if (bad || r != rend) atomicOr(&status[vec], 4);
        else if (endbad) atomicOr(&status[vec], 8);
        if (c == 0) {
            l1[vec] = __uint_as_float(h[6]);
            kmax[vec] = d > 0 ? (nsym - 2) / 2 : 0;
        }
    }
}
