// uq_biased_kernels.h — device code of the biased type quantizer (Reznik rounding).
// Included by uq_dme.hip inside its anonymous namespace (shares the K1 cascade).
//
// Reference (paths relative to the reference root):
//   NMSE_Results/Codes/All_Schemes.py:669-687  Type_biased_quantize
//   NMSE_Results/Codes/All_Schemes.py:644-666  Reznik
//
// Per client j (one row of x):
//   KB1  L1 = |x|.sum()                  K1 cascade, AbsOp           (AS:680)
//   KB2  m' = k'.sum(), k' = floor(m p + 0.5)  K1 cascade, RezKOp    (AS:648-649)
//   KB3  Delta = int(m' - m) -> |Delta| selections                    (AS:651-656)
//   KB4a the bucket of the |Delta|-th largest selection value v (+delta' for Delta > 0,
//        -delta' for Delta < 0; delta' = k' - m p, AS:655-665) among KB2's 2048 "fine" bins,
//        linear in |v| over [-0.5, 0.5] (rez_fbin: ~0.1 % of a Gaussian row per bin at R = 1)
//   KB6f ("fine" clients, the bucket small) out for every coordinate: bins above the bucket
//        are selected, below are not, the bucket's coordinates provisionally unselected and
//        listed (index, key); KB4d radix-selects the threshold key among the listed keys and
//        KB6p patches the listed coordinates that are selected -- x is read three times in all
//   KB4b (other clients: a bucket too large, tie-heavy data) radix select (3 passes, 11/11/10-bit
//        digits of the order key) over the whole row, then KB6
//   KB5  (ambiguous clients only) tie counts per tile, for the index-order tie rank
//   KB6  out = (L1 * sign(x)) * (k'' / m), k'' = k' -+ 1 on the selected set (AS:661/665/687)
// torch.topk compares values (as doubles): equal values are ties whatever their index.
// When the threshold value occurs more often than it is selected ("ambiguous"), torch's
// choice is the one libstdc++'s nth_element / partial_sort makes; KB6 takes the lowest
// indices instead, and the torch choice is replayed by uq_biased_torch_ties.h.

constexpr int kRadixBins = 2048;
constexpr int kHistItems = 64;                      // elements per thread in a histogram pass
constexpr int kHistSpan = 256 * kHistItems;         // 16384 elements per workgroup
constexpr int kSelItems = 16;                       // contiguous elements per thread (KB5/KB6)
constexpr int kSelTile = 256 * kSelItems;           // 4096 elements per tile

enum RezFlags : int32_t {
    kRezAmbiguous = 1,     // threshold value shared by selected and unselected coordinates
    kRezNonFinite = 2,     // m' is NaN/inf: the reference raises in int(m' - m) (AS:656)
    kRezRange = 4,         // |Delta| > d: torch.topk raises (cannot happen for finite input)
    kRezTorchTies = 8,     // selection set replayed with torch's tie choice (KB7)
    kRezFine = 16,         // threshold found among the fine bucket's keys listed by KB6f
    kRezFull = 32,         // threshold found by full-row radix passes (bucket too large)
};

struct RezState {          // 32 bytes per client; (delta, flags) are the public info pair
    int32_t delta;         // AS:656; 0 when m' == m (AS:651) or on error
    int32_t flags;         // RezFlags
    float mprime;          // AS:649
    uint32_t prefix;       // threshold key bits decided so far
    uint32_t kleft;        // selections still to place at/below the prefix
    uint32_t eq;           // keys equal to the threshold (after the last pass)
    uint32_t need;         // how many of those are selected
    uint32_t fbin;         // kRezFine: the threshold's fine bin
};

// Order-preserving u32 image of the selection value (+delta' for Delta > 0, -delta'
// otherwise): larger value -> larger key.  -0 folds onto +0 (torch: -0 == +0 is a
// tie) and NaNs onto one key above +inf (ATen's topk comparator puts NaN first).
__device__ __forceinline__ uint32_t rez_key_of(float dp, bool up) {
    float v = up ? dp : -dp;
    v = v + 0.0f;
    uint32_t u = __float_as_uint(v);
    if (v != v) u = 0x7FC00000u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// The selection value a key encodes (its inverse image; NaN keys decode to NaN).
__device__ __forceinline__ float rez_key_val(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// k' and the key of one coordinate, exactly the reference's f32 ops (no contraction):
// p = |x| / (L1 + 1e-12) (AS:681), mp = m * p, k' = floor(mp + 0.5) (AS:648),
// delta' = k' - mp (AS:655).
__device__ __forceinline__ uint32_t rez_elem(float xv, const DivPlan& dp, float fm, bool up, float& kp) {
    const float mp = fm * div1(fabsf(xv), dp);      // RN(|x| / den), reciprocal + Markstein
    kp = floorf(mp + 0.5f);
    return rez_key_of(kp - mp, up);
}

// Four at a time: packed reciprocal division with one guard test per four (div4).
__device__ __forceinline__ void rez_elem4(const float (&xv)[4], const DivPlan& dp, float fm, bool up, float (&kp)[4],
                                          uint32_t (&key)[4]) {
    float a[4], p[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = fabsf(xv[c]);
    div4(a, dp, p);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float mp = fm * p[c];
        kp[c] = floorf(mp + 0.5f);
        key[c] = rez_key_of(kp[c] - mp, up);
    }
}

template <int PASS> struct RadixPass;
template <> struct RadixPass<0> { static constexpr int shift = 21; static constexpr uint32_t dmask = 0x7FF, hmask = 0u; };
template <> struct RadixPass<1> { static constexpr int shift = 10; static constexpr uint32_t dmask = 0x7FF, hmask = 0xFFE00000u; };
template <> struct RadixPass<2> { static constexpr int shift = 0; static constexpr uint32_t dmask = 0x3FF, hmask = 0xFFFFFC00u; };

// Block-wide exclusive scan of one u32 per thread (256 threads); returns the exclusive
// prefix, writes the total.  `lds` needs 4 u32.
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += t;
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t = lds[k];
        base += (k < w) ? t : 0u;
        all += t;
    }
    __syncthreads();
    *total = all;
    return base + inc - v;
}

// KB3: Delta and the selection count per client.
__global__ void __launch_bounds__(256)
rez_setup_kernel(const float* __restrict__ msum, float fm, int64_t d, int64_t n, RezState* __restrict__ st) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    RezState s{};
    s.mprime = msum[i];
    if (!(s.mprime == fm)) {                       // AS:651
        if (!isfinite(s.mprime)) {
            s.flags |= kRezNonFinite;
        } else {
            const float df = s.mprime - fm;        // AS:656 f32 subtract, int() truncates
            const long long D = (long long)df;
            const long long K = D > 0 ? D : -D;
            if (K > d) {
                s.flags |= kRezRange;
            } else {
                s.delta = (int32_t)D;
                s.kleft = (uint32_t)K;
            }
        }
    }
    st[i] = s;
}

// KB4a: histogram of the PASS-th digit over keys matching the prefix.
template <int PASS, bool VEC4>
__device__ __forceinline__ void rez_hist_one(const float* __restrict__ x, int64_t d, const float* __restrict__ l1,
                                             float fm, const RezState* __restrict__ st, uint32_t* __restrict__ hist,
                                             int64_t vec) {
    using RP = RadixPass<PASS>;
    const uint32_t kleft = st[vec].kleft;
    if (kleft == 0 || !(st[vec].flags & kRezFull)) return;
    const uint32_t prefix = st[vec].prefix;
    const bool up = st[vec].delta > 0;
    __shared__ uint32_t h[kRadixBins];
    const int tid = threadIdx.x;
    for (int b = tid; b < kRadixBins; b += 256) h[b] = 0u;
    __syncthreads();
    const DivPlan dp = div_plan(l1[vec]);
    const float* xv = x + vec * d;
    const int64_t b0 = (int64_t)blockIdx.x * kHistSpan;
    auto visit = [&](float v) {
        float kp;
        const uint32_t key = rez_elem(v, dp, fm, up, kp);
        if ((key & RP::hmask) == prefix) atomicAdd(&h[(key >> RP::shift) & RP::dmask], 1u);
    };
    if (VEC4) {
        const float4* x4 = reinterpret_cast<const float4*>(xv + b0);
        const int64_t n4 = (std::min<int64_t>(d - b0, kHistSpan)) / 4;
#pragma unroll 4
        for (int j = 0; j < kHistItems / 4; ++j) {
            const int64_t q = (int64_t)j * 256 + tid;
            if (q < n4) {
                const float4 t = x4[q];
                visit(t.x); visit(t.y); visit(t.z); visit(t.w);
            }
        }
    } else {
        for (int j = 0; j < kHistItems; ++j) {
            const int64_t i = b0 + (int64_t)j * 256 + tid;
            if (i < d) visit(xv[i]);
        }
    }
    __syncthreads();
    uint32_t* g = hist + ((size_t)vec * kHistSlots + PASS) * kRadixBins;
    for (int b = tid; b < kRadixBins; b += 256)
        if (h[b]) atomicAdd(&g[b], h[b]);
    __syncthreads();                                   // h is reused by the next listed client
}

// Grid (spans, <= list length): y strides over KB4a's list of full clients (flist[0] = count).
template <int PASS, bool VEC4>
__global__ void __launch_bounds__(256)
rez_hist_kernel(const float* __restrict__ x, int64_t d, const float* __restrict__ l1, float fm,
                const RezState* __restrict__ st, uint32_t* __restrict__ hist, const uint32_t* __restrict__ flist) {
    const uint32_t nf = flist[0];
    for (uint32_t li = blockIdx.y; li < nf; li += gridDim.y) rez_hist_one<PASS, VEC4>(x, d, l1, fm, st, hist, flist[1 + li]);
}

// KB4a / KB4b: pick the digit holding the kleft-th largest key (one workgroup per client).
// FINE (KB4a): KB2's fine bins of +delta', mirrored for Delta < 0 (zeros and NaNs counted
// apart in zn); a bucket of at most `capf` coordinates makes the client kRezFine (its keys are
// listed by KB6f), a larger one kRezFull.  Otherwise (KB4b) pass PASS of the key digits over
// the full row, kRezFull clients only.
template <int PASS, bool FINE>
__device__ __forceinline__ void rez_select_one(RezState* __restrict__ st, const uint32_t* __restrict__ hist,
                                               const uint32_t* __restrict__ zn, uint32_t capf,
                                               uint32_t* __restrict__ flist, int64_t vec) {
    using RP = RadixPass<PASS>;
    constexpr int nb = FINE ? kRadixBins : (int)RP::dmask + 1;
    constexpr int per = nb / 256;
    const uint32_t kleft = st[vec].kleft;
    if (kleft == 0) {                                  // no selection: KB6 writes it (listed with the full)
        if (FINE && threadIdx.x == 0) flist[1 + atomicAdd(&flist[0], 1u)] = (uint32_t)vec;
        return;
    }
    if (!FINE && !(st[vec].flags & kRezFull)) return;
    __shared__ uint32_t lds[4];
    __shared__ int s_found;
    const int tid = threadIdx.x;
    __syncthreads();                                   // the previous listed client's s_found / lds
    if (tid == 0) s_found = 0;
    const uint32_t* h = hist + ((size_t)vec * kHistSlots + (FINE ? kFineSlot : PASS)) * kRadixBins;
    const bool mirror = FINE && st[vec].delta < 0;
    const uint32_t z = FINE ? zn[vec * 2] : 0u, nn = FINE ? zn[vec * 2 + 1] : 0u;
    auto count = [&](int b) -> uint32_t {
        if (!mirror) return h[b];
        uint32_t c = h[nb - 1 - b];              // fbin(-v) = 2047 - fbin(v) but for 0 and NaN
        if (b == 1023) c -= z;
        if (b == 1024) c += z;
        if (b == 0) c -= nn;
        if (b == 2047) c += nn;
        return c;
    };
    // thread t owns bins [nb - (t+1)*per, nb - t*per): thread 0 the highest digits
    const int hi = nb - tid * per;
    uint32_t c[per], sum = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        c[k] = count(hi - 1 - k);
        sum += c[k];
    }
    uint32_t total;
    uint32_t above = block_excl_scan_u32(sum, lds, &total);
    if (above < kleft && above + sum >= kleft) {
#pragma unroll
        for (int k = 0; k < per; ++k) {
            if (above + c[k] >= kleft) {
                const uint32_t digit = (uint32_t)(hi - 1 - k);
                RezState s = st[vec];
                if (FINE) {
                    if (c[k] <= capf) {
                        s.flags |= kRezFine;
                        s.fbin = digit;
                        s.kleft = kleft - above;         // to select inside the bucket
                        s.eq = c[k];                     // its coordinates = the candidates KB6f lists
                    } else {
                        s.flags |= kRezFull;
                        flist[1 + atomicAdd(&flist[0], 1u)] = (uint32_t)vec;      // for KB4b's passes
                    }
                } else {
                    s.prefix |= digit << RP::shift;
                    s.kleft = kleft - above;
                    if (PASS == 2) {
                        s.eq = c[k];
                        s.need = s.kleft;
                        if (s.eq > s.need) s.flags |= kRezAmbiguous;
                    }
                }
                st[vec] = s;
                s_found = 1;
                break;
            }
            above += c[k];
        }
    }
    __syncthreads();
    if (FINE && tid == 0 && !s_found) {                  // (cannot happen: sum = d >= kleft)
        st[vec].flags |= kRezFull;
        flist[1 + atomicAdd(&flist[0], 1u)] = (uint32_t)vec;
    }
}

// FINE (KB4a): one workgroup per client, the full ones appended to flist; else (KB4b) the
// workgroups stride over flist.
template <int PASS, bool FINE>
__global__ void __launch_bounds__(256)
rez_select_kernel(RezState* __restrict__ st, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ zn,
                  uint32_t capf, uint32_t* __restrict__ flist) {
    if (FINE) {
        rez_select_one<PASS, FINE>(st, hist, zn, capf, flist, blockIdx.x);
        return;
    }
    const uint32_t nf = flist[0];
    for (uint32_t li = blockIdx.x; li < nf; li += gridDim.x) rez_select_one<PASS, FINE>(st, hist, zn, capf, flist, flist[1 + li]);
}

// KB4d: the threshold key among a fine client's listed candidates (key digits 11/11/10 over
// the (index, key) pairs KB6f wrote; the candidates share the fine bin, not a key prefix).
// cand_pick: the digit of candidate pass `pass` holding the kleft-th largest key, from the
// pass's histogram h; updates s in every thread.
__device__ __forceinline__ void cand_pick(const uint32_t* h, int pass, RezState& s, uint32_t* lds) {
    const int tid = threadIdx.x;
    const int shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
    const int nb = pass == 2 ? 1024 : 2048;
    const int per = nb / 256;
    const int hi = nb - tid * per;
    uint32_t c[8], sum = 0;
    for (int k = 0; k < per; ++k) {
        c[k] = h[hi - 1 - k];
        sum += c[k];
    }
    __shared__ uint32_t s_digit, s_above, s_eq;
    if (tid == 0) { s_digit = 0u; s_above = 0u; s_eq = 0u; }
    uint32_t total;
    uint32_t above = block_excl_scan_u32(sum, lds, &total);
    if (above < s.kleft && above + sum >= s.kleft) {
        for (int k = 0; k < per; ++k) {
            if (above + c[k] >= s.kleft) {
                s_digit = (uint32_t)(hi - 1 - k);
                s_above = above;
                s_eq = c[k];
                break;
            }
            above += c[k];
        }
    }
    __syncthreads();
    s.prefix |= s_digit << shift;
    s.kleft -= s_above;
    if (pass == 2) {
        s.eq = s_eq;
        s.need = s.kleft;
        if (s.eq > s.need) s.flags |= kRezAmbiguous;
    }
    __syncthreads();
}

__device__ __forceinline__ void cand_pass_masks(int pass, int& shift, uint32_t& dmask, uint32_t& hmask) {
    shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
    dmask = pass == 2 ? 0x3FFu : 0x7FFu;
    hmask = pass == 0 ? 0u : (pass == 1 ? 0xFFE00000u : 0xFFFFFC00u);
}

__global__ void __launch_bounds__(256)
rez_cand_select_kernel(RezState* __restrict__ st, const uint2* __restrict__ cand, const uint32_t* __restrict__ cand_n,
                       uint32_t capf) {
    const int64_t vec = blockIdx.x;
    if (st[vec].kleft == 0 || !(st[vec].flags & kRezFine)) return;
    __shared__ uint32_t h[kRadixBins];
    __shared__ uint32_t lds[4];
    const int tid = threadIdx.x;
    const uint32_t nc = std::min(cand_n[vec], capf);
    const uint2* cv = cand + (size_t)vec * capf;
    RezState s = st[vec];
    for (int pass = 0; pass <= 2; ++pass) {
        int shift;
        uint32_t dmask, hmask;
        cand_pass_masks(pass, shift, dmask, hmask);
        for (int b = tid; b < kRadixBins; b += 256) h[b] = 0u;
        __syncthreads();
        // 8 independent candidate loads in flight per thread, then their LDS atomics
        uint32_t i = tid;
        for (; i + 7 * 256 < nc; i += 8 * 256) {
            uint32_t kk[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kk[u] = cv[i + u * 256].y;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if ((kk[u] & hmask) == s.prefix) atomicAdd(&h[(kk[u] >> shift) & dmask], 1u);
        }
        for (; i < nc; i += 256) {
            const uint32_t key = cv[i].y;
            if ((key & hmask) == s.prefix) atomicAdd(&h[(key >> shift) & dmask], 1u);
        }
        __syncthreads();
        cand_pick(h, pass, s, lds);
    }
    if (tid == 0) st[vec] = s;
}

// The same three passes for a few clients with long candidate lists (tie-heavy rows in the
// per-call drop-in): KB4d1 histograms kCandSpan candidates per workgroup into the client's
// pass histogram (hist[vec][pass], zero until then: the full-row passes skip fine clients),
// KB4d2 picks the digit from it with cand_pick (same bits as rez_cand_select_kernel).
constexpr int kCandSpan = 256 * 32;
template <int PASS>
__global__ void __launch_bounds__(256)
rez_cand_hist_kernel(const RezState* __restrict__ st, const uint2* __restrict__ cand,
                     const uint32_t* __restrict__ cand_n, uint32_t capf, uint32_t* __restrict__ hist) {
    const int64_t vec = blockIdx.y;
    if (st[vec].kleft == 0 || !(st[vec].flags & kRezFine)) return;
    const uint32_t nc = std::min(cand_n[vec], capf);
    const uint32_t b0 = blockIdx.x * (uint32_t)kCandSpan;
    if (b0 >= nc) return;
    constexpr int shift = PASS == 0 ? 21 : (PASS == 1 ? 10 : 0);
    constexpr uint32_t dmask = PASS == 2 ? 0x3FFu : 0x7FFu;
    constexpr uint32_t hmask = PASS == 0 ? 0u : (PASS == 1 ? 0xFFE00000u : 0xFFFFFC00u);
    constexpr int nb = (int)dmask + 1;
    __shared__ uint32_t h[nb];
    const int tid = threadIdx.x;
    for (int b = tid; b < nb; b += 256) h[b] = 0u;
    __syncthreads();
    const uint32_t prefix = st[vec].prefix;
    const uint2* cv = cand + (size_t)vec * capf;
    uint32_t kk[kCandSpan / 256];
#pragma unroll
    for (int u = 0; u < kCandSpan / 256; ++u) {
        const uint32_t i = b0 + tid + 256u * u;
        kk[u] = i < nc ? cv[i].y : ~prefix;                   // ~prefix never matches (hmask != 0)
    }
#pragma unroll
    for (int u = 0; u < kCandSpan / 256; ++u) {
        const uint32_t i = b0 + tid + 256u * u;
        if (i < nc && (kk[u] & hmask) == prefix) atomicAdd(&h[(kk[u] >> shift) & dmask], 1u);
    }
    __syncthreads();
    uint32_t* g = hist + ((size_t)vec * kHistSlots + PASS) * kRadixBins;
    for (int b = tid; b < nb; b += 256)
        if (h[b]) atomicAdd(&g[b], h[b]);
}

template <int PASS>
__global__ void __launch_bounds__(256)
rez_cand_pick_kernel(RezState* __restrict__ st, const uint32_t* __restrict__ hist) {
    const int64_t vec = blockIdx.x;
    if (st[vec].kleft == 0 || !(st[vec].flags & kRezFine)) return;
    __shared__ uint32_t h[kRadixBins];
    __shared__ uint32_t lds[4];
    const int tid = threadIdx.x;
    const uint32_t* g = hist + ((size_t)vec * kHistSlots + PASS) * kRadixBins;
    for (int b = tid; b < kRadixBins; b += 256) h[b] = g[b];
    __syncthreads();
    RezState s = st[vec];
    cand_pick(h, PASS, s, lds);
    if (tid == 0) st[vec] = s;
}

// KB5: keys equal to the threshold per tile (ambiguous clients only), for the index-order
// ranks of the lowest-index rule.  Grid (tiles, <= list length): y strides over `list` (the
// ambiguous clients, rez_tie_list_kernel), not over n mostly-exiting client rows.
template <bool VEC4>
__device__ __forceinline__ void rez_tiecount_tile(const float* __restrict__ x, int64_t d, const float* __restrict__ l1,
                                                  float fm, const RezState* __restrict__ st,
                                                  uint32_t* __restrict__ tilecnt, int32_t tiles, int64_t vec) {
    const int32_t fl = st[vec].flags;
    if (!(fl & kRezAmbiguous) || (fl & kRezTorchTies)) return;
    const uint32_t tau = st[vec].prefix;
    const bool up = st[vec].delta > 0;
    const DivPlan dp = div_plan(l1[vec]);
    const float* xv = x + vec * d;
    const int tid = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kSelTile + (int64_t)tid * kSelItems;
    uint32_t cnt = 0;
    float kp;
    if (VEC4 && e0 + kSelItems <= d) {
        const float4* x4 = reinterpret_cast<const float4*>(xv + e0);
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) {
            const float4 t = x4[j];
            cnt += rez_elem(t.x, dp, fm, up, kp) == tau;
            cnt += rez_elem(t.y, dp, fm, up, kp) == tau;
            cnt += rez_elem(t.z, dp, fm, up, kp) == tau;
            cnt += rez_elem(t.w, dp, fm, up, kp) == tau;
        }
    } else {
        for (int j = 0; j < kSelItems; ++j)
            if (e0 + j < d) cnt += rez_elem(xv[e0 + j], dp, fm, up, kp) == tau;
    }
    __shared__ uint32_t lds[4];
    uint32_t total;
    (void)block_excl_scan_u32(cnt, lds, &total);
    if (tid == 0) tilecnt[vec * tiles + blockIdx.x] = total;
    __syncthreads();                                   // lds is reused by the next listed client
}

template <bool VEC4>
__global__ void __launch_bounds__(256)
rez_tiecount_kernel(const float* __restrict__ x, int64_t d, const float* __restrict__ l1, float fm,
                    const RezState* __restrict__ st, uint32_t* __restrict__ tilecnt, int32_t tiles,
                    const uint32_t* __restrict__ list) {
    const uint32_t nl = list[0];
    for (uint32_t li = blockIdx.y; li < nl; li += gridDim.y)
        rez_tiecount_tile<VEC4>(x, d, l1, fm, st, tilecnt, tiles, list[1 + li]);
}

__device__ __forceinline__ float torch_signf(float v) {
    return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
}

// KB6: apply the selection and dequantize.  Selected = key > tau, or key == tau and
// (all ties are selected | rank among ties in index order < need | marked by KB7).
template <bool VEC4>
__device__ __forceinline__ void rez_output_tile(const float* __restrict__ x, float* __restrict__ out, int64_t d,
                                                const float* __restrict__ l1, float fm, const RezState* __restrict__ st,
                                                const uint32_t* __restrict__ tilecnt, int32_t tiles,
                                                const uint32_t* __restrict__ tie_bits, int part, int64_t vec) {
    const RezState s = st[vec];
    const bool on = s.kleft != 0;
    const bool amb = on && (s.flags & kRezAmbiguous);
    // part 0: every client; 1: clients without a tie at the threshold (run while KB7 replays
    // the others on a side stream); 2: only those with one (after KB7); 3: only the fine ones
    // with one (the lowest-index rule's second, list-strided launch).  Fine clients without
    // a tie were written by KB6f + KB6p; with a replayed tie KB6t patches them; with an
    // index-order tie (a failed replay, or the lowest-index rule) this kernel rewrites them:
    // the ranks need the whole row
    if ((part == 1 && amb) || (part == 2 && !amb)) return;
    if (part == 3 && !(amb && (s.flags & kRezFine))) return;   // (the listed full clients took part 0)
    if (on && (s.flags & kRezFine) && !amb) return;
    const bool replay = amb && (s.flags & kRezTorchTies);
    if (replay && (s.flags & kRezFine)) return;
    const bool up = s.delta > 0;
    const float L = l1[vec];
    const DivPlan dp = div_plan(L);
    const DivPlan dpm = div_plan_m(fm);
    const float adj = up ? -1.f : 1.f;
    const uint32_t tau = s.prefix;
    const float* xv = x + vec * d;
    float* ov = out + vec * d;
    const int tid = threadIdx.x;
    const int64_t tb = (int64_t)blockIdx.x * kSelTile;
    if (VEC4 && !(amb && !replay) && tb + kSelTile <= d) {
        // no index-order rank needed (block-uniform): lane-interleaved float4s, one
        // coalesced 1 KB row per wave per load, non-temporal loads and stores
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v* x4 = reinterpret_cast<const f4v*>(xv + tb);
        f4v* o4 = reinterpret_cast<f4v*>(ov + tb);
        const uint32_t* tbw = tie_bits + vec * ((d + 31) / 32);
        f4v a[kSelItems / 4];
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) a[j] = __builtin_nontemporal_load(x4 + j * 256 + tid);
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) {
            const float v4[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
            float k4[4], r4[4];
            uint32_t y4[4];
            rez_elem4(v4, dp, fm, up, k4, y4);
            const int64_t i0 = tb + 4 * ((int64_t)j * 256 + tid);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                bool sel = false;
                if (on) {
                    if (y4[c] > tau) sel = true;
                    else if (y4[c] == tau) sel = !amb || ((tbw[(i0 + c) >> 5] >> ((i0 + c) & 31)) & 1u);
                }
                k4[c] = sel ? k4[c] + adj : k4[c];             // k''
            }
            div4(k4, dpm, r4);                                 // RN(k'' / m)
            f4v o;
            o.x = (L * torch_signf(v4[0])) * r4[0];            // AS:687 (L1 * signs) * (k'' / m)
            o.y = (L * torch_signf(v4[1])) * r4[1];
            o.z = (L * torch_signf(v4[2])) * r4[2];
            o.w = (L * torch_signf(v4[3])) * r4[3];
            __builtin_nontemporal_store(o, o4 + j * 256 + tid);
        }
        return;
    }
    const int64_t e0 = tb + (int64_t)tid * kSelItems;
    const bool full = VEC4 && e0 + kSelItems <= d;
    float v[kSelItems];
    if (full) {
        const float4* x4 = reinterpret_cast<const float4*>(xv + e0);
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) {
            const float4 t = x4[j];
            v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kSelItems; ++j) v[j] = (e0 + j < d) ? xv[e0 + j] : 0.f;
    }
    float kp[kSelItems];
    uint32_t key[kSelItems];
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < kSelItems / 4; ++j) {
        const float v4[4] = {v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
        float k4[4];
        uint32_t y4[4];
        rez_elem4(v4, dp, fm, up, k4, y4);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            kp[4 * j + c] = k4[c];
            key[4 * j + c] = y4[c];
        }
    }
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) cnt += (key[j] == tau && e0 + j < d);
    uint32_t rank = 0;
    if (amb && !replay) {              // block-uniform
        __shared__ uint32_t lds[4];
        __shared__ uint32_t tile_base;
        uint32_t part = 0;
        for (int t = tid; t < (int)blockIdx.x; t += 256) part += tilecnt[vec * tiles + t];
        uint32_t ptot;
        (void)block_excl_scan_u32(part, lds, &ptot);
        if (tid == 0) tile_base = ptot;
        uint32_t ctot;
        rank = block_excl_scan_u32(cnt, lds, &ctot);
        rank += tile_base;
    }
    // KB7's replayed set: one bit per coordinate, rows of ceil(d/32) words
    const uint32_t* tbv = tie_bits + vec * ((d + 31) / 32);
    float q[kSelItems];
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        bool sel = false;
        if (on) {
            if (key[j] > tau) {
                sel = true;
            } else if (key[j] == tau) {
                if (!amb) sel = true;
                else if (replay) sel = (tbv[(e0 + j) >> 5] >> ((e0 + j) & 31)) & 1u;
                else sel = (rank++ < s.need);
            }
        }
        q[j] = sel ? kp[j] + adj : kp[j];                 // k''
    }
#pragma unroll
    for (int j = 0; j < kSelItems / 4; ++j) {
        const float k4[4] = {q[4 * j], q[4 * j + 1], q[4 * j + 2], q[4 * j + 3]};
        float r4[4];
        div4(k4, dpm, r4);                                 // RN(k'' / m)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            q[4 * j + c] = (L * torch_signf(v[4 * j + c])) * r4[c];   // AS:687 (L1 * signs) * (k'' / m)
    }
    if (full) {
        float4* o4 = reinterpret_cast<float4*>(ov + e0);
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) o4[j] = make_float4(q[4 * j], q[4 * j + 1], q[4 * j + 2], q[4 * j + 3]);
    } else {
#pragma unroll
        for (int j = 0; j < kSelItems; ++j)
            if (e0 + j < d) ov[e0 + j] = q[j];
    }
}

// list: null -- client blockIdx.y; else the clients list[1 ..= list[0]] (KB7's, part 2), the
// grid's y dimension striding over them, so the launch is not n x tiles mostly idle workgroups
template <bool VEC4>
__global__ void __launch_bounds__(256)
rez_output_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t d, const float* __restrict__ l1,
                  float fm, const RezState* __restrict__ st, const uint32_t* __restrict__ tilecnt, int32_t tiles,
                  const uint32_t* __restrict__ tie_bits, int part, const uint32_t* __restrict__ list) {
    if (!list) {
        rez_output_tile<VEC4>(x, out, d, l1, fm, st, tilecnt, tiles, tie_bits, part, blockIdx.y);
        return;
    }
    const uint32_t nl = list[0];
    for (uint32_t li = blockIdx.y; li < nl; li += gridDim.y) {
        rez_output_tile<VEC4>(x, out, d, l1, fm, st, tilecnt, tiles, tie_bits, part, list[1 + li]);
        __syncthreads();                               // the rank scans' LDS, reused by the next client
    }
}

// KB6f: fine clients (kRezFine) -- out for every coordinate with the selection decided by the
// fine bin (above the threshold's bin: selected; below: not); the threshold bin's coordinates
// are written unselected and listed as (index, key) pairs for KB4d: staged in LDS by LDS
// atomics, then one global atomic per workgroup reserves the list range (a per-thread list
// indexed by a running count lived in scratch: 1.77 ms against 1.72-1.74 here, the batch
// 0.01-0.05 ms faster, profiles/r5p_exp_biased_kb6f_lds.jsonl).  The same arithmetic as KB6, so
// KB6p's patch gives KB6's bits.
constexpr uint32_t kFineStage = 256;
template <bool VEC4>
__global__ void __launch_bounds__(256)
rez_output_fine_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t d, const float* __restrict__ l1,
                       float fm, const RezState* __restrict__ st, uint2* __restrict__ cand,
                       uint32_t* __restrict__ cand_n, uint32_t capf) {
    const int64_t vec = blockIdx.y;
    const RezState s = st[vec];
    if (s.kleft == 0 || !(s.flags & kRezFine)) return;
    const bool up = s.delta > 0;
    const float L = l1[vec];
    const DivPlan dp = div_plan(L);
    const DivPlan dpm = div_plan_m(fm);
    const float adj = up ? -1.f : 1.f;
    const uint32_t fb = s.fbin;
    const float* xv = x + vec * d;
    float* ov = out + vec * d;
    const int tid = threadIdx.x;
    const int64_t tb = (int64_t)blockIdx.x * kSelTile;
    // past kFineStage pairs (tie-heavy tiles), straight to the global list
    __shared__ uint2 stage[kFineStage];
    __shared__ uint32_t s_cnt, s_base;
    if (tid == 0) s_cnt = 0u;
    __syncthreads();
    auto one = [&](float v, float kp, uint32_t key, int64_t i, float& kq) {
        const uint32_t b = rez_fbin(rez_key_val(key));
        kq = b > fb ? kp + adj : kp;                           // k'' (the bucket provisionally unselected)
        if (b == fb) {
            const uint32_t slot = atomicAdd(&s_cnt, 1u);
            if (slot < kFineStage) {
                stage[slot] = make_uint2((uint32_t)i, key);
            } else {
                const uint32_t g = atomicAdd(&cand_n[vec], 1u);
                if (g < capf) cand[(size_t)vec * capf + g] = make_uint2((uint32_t)i, key);
            }
        }
    };
    if (VEC4 && tb + kSelTile <= d) {
        // lane-interleaved float4s (one coalesced 1 KB row per wave per load), non-temporal
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v* x4 = reinterpret_cast<const f4v*>(xv + tb);
        f4v* o4 = reinterpret_cast<f4v*>(ov + tb);
        f4v a[kSelItems / 4];
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) a[j] = __builtin_nontemporal_load(x4 + j * 256 + tid);
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) {
            const float v4[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
            float k4[4], q4[4], r4[4];
            uint32_t y4[4];
            rez_elem4(v4, dp, fm, up, k4, y4);
            const int64_t i0 = tb + 4 * ((int64_t)j * 256 + tid);
#pragma unroll
            for (int c = 0; c < 4; ++c) one(v4[c], k4[c], y4[c], i0 + c, q4[c]);
            div4(q4, dpm, r4);                                 // RN(k'' / m)
            f4v o;
            o.x = (L * torch_signf(v4[0])) * r4[0];            // AS:687 (L1 * signs) * (k'' / m)
            o.y = (L * torch_signf(v4[1])) * r4[1];
            o.z = (L * torch_signf(v4[2])) * r4[2];
            o.w = (L * torch_signf(v4[3])) * r4[3];
            __builtin_nontemporal_store(o, o4 + j * 256 + tid);
        }
    } else {
        const int64_t e0 = tb + (int64_t)tid * kSelItems;
#pragma unroll
        for (int j = 0; j < kSelItems / 4; ++j) {
            float v4[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v4[c] = (e0 + 4 * j + c < d) ? xv[e0 + 4 * j + c] : 0.f;
            float k4[4], q4[4], r4[4];
            uint32_t y4[4];
            rez_elem4(v4, dp, fm, up, k4, y4);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (e0 + 4 * j + c < d) one(v4[c], k4[c], y4[c], e0 + 4 * j + c, q4[c]);
                else q4[c] = 0.f;
            }
            div4(q4, dpm, r4);
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (e0 + 4 * j + c < d) ov[e0 + 4 * j + c] = (L * torch_signf(v4[c])) * r4[c];
        }
    }
    __syncthreads();
    const uint32_t tot = min(s_cnt, (uint32_t)kFineStage);
    if (tot == 0) return;                                      // block-uniform
    if (tid == 0) s_base = atomicAdd(&cand_n[vec], tot);
    __syncthreads();
    uint2* cv = cand + (size_t)vec * capf;
    for (uint32_t t = tid; t < tot; t += 256)
        if (s_base + t < capf) cv[s_base + t] = stage[t];
}

// KB6p: the listed coordinates of a fine client without a threshold tie that are selected
// (key >= the threshold key: every tie is selected) get k'' = k' -+ 1.
constexpr int kPatchBlocks = 4;
constexpr int64_t kListedGridY = 64;      // list-strided launches after KB7: y extent
__global__ void __launch_bounds__(256)
rez_fine_patch_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t d, const float* __restrict__ l1,
                      float fm, const RezState* __restrict__ st, const uint2* __restrict__ cand,
                      const uint32_t* __restrict__ cand_n, uint32_t capf) {
    const int64_t vec = blockIdx.y;
    const RezState s = st[vec];
    if (s.kleft == 0 || !(s.flags & kRezFine) || (s.flags & kRezAmbiguous)) return;
    const uint32_t nc = std::min(cand_n[vec], capf);
    const uint2* cv = cand + (size_t)vec * capf;
    const bool up = s.delta > 0;
    const float L = l1[vec];
    const DivPlan dp = div_plan(L);
    const DivPlan dpm = div_plan_m(fm);
    const float adj = up ? -1.f : 1.f;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nc; i += gridDim.x * 256) {
        const uint2 c = cv[i];
        if (c.y < s.prefix) continue;
        const float v = x[vec * d + c.x];
        float kp;
        (void)rez_elem(v, dp, fm, up, kp);
        out[vec * d + c.x] = (L * torch_signf(v)) * div1(kp + adj, dpm);     // AS:687 with k''
    }
}

// KB6t: the fine clients whose threshold ties KB7 replayed.  KB6f wrote their rows with the
// threshold's bin unselected and listed the bin; the listed coordinates that are selected (key
// above the threshold key, or equal to it with KB7's bit) get k'' = k' -+ 1.  Grid (blocks,
// <= list length): y strides over KB7's client list.
__global__ void __launch_bounds__(256)
rez_tie_patch_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t d, const float* __restrict__ l1,
                     float fm, const RezState* __restrict__ st, const uint2* __restrict__ cand,
                     const uint32_t* __restrict__ cand_n, uint32_t capf, const uint32_t* __restrict__ tie_bits,
                     const uint32_t* __restrict__ list) {
    const uint32_t nl = list[0];
    for (uint32_t li = blockIdx.y; li < nl; li += gridDim.y) {
        const int64_t vec = list[1 + li];
        const RezState s = st[vec];
        constexpr int32_t want = kRezFine | kRezAmbiguous | kRezTorchTies;
        if (s.kleft == 0 || (s.flags & want) != want) continue;
        const uint32_t nc = std::min(cand_n[vec], capf);
        const uint2* cv = cand + (size_t)vec * capf;
        const uint32_t* bits = tie_bits + vec * ((d + 31) / 32);
        const bool up = s.delta > 0;
        const float L = l1[vec];
        const DivPlan dp = div_plan(L);
        const DivPlan dpm = div_plan_m(fm);
        const float adj = up ? -1.f : 1.f;
        for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nc; i += gridDim.x * 256) {
            const uint2 c = cv[i];
            if (c.y < s.prefix) continue;
            if (c.y == s.prefix && !((bits[c.x >> 5] >> (c.x & 31)) & 1u)) continue;
            const float v = x[vec * d + c.x];
            float kp;
            (void)rez_elem(v, dp, fm, up, kp);
            out[vec * d + c.x] = (L * torch_signf(v)) * div1(kp + adj, dpm);     // AS:687 with k''
        }
    }
}

// KB-small: the whole AS:644-687 for vectors shorter than GRAIN in ONE launch (the reference
// harness's d = 1024 / 2048 per-vector calls): one 256-thread workgroup per client computes
// L1 and m' in torch's cascade order (block_torch_sum), Delta, the |Delta|-th largest key by
// three radix passes over the client's keys held in LDS (dynamic, 4 d bytes), and the outputs.
// Threshold ties are resolved by the lowest-index rule (index-order ranks: one block scan
// over contiguous per-thread segments); with UQ_TIES_TORCH an ambiguous client is only flagged
// (kRezAmbiguous without kRezTorchTies) and the host reruns the multi-kernel path for it.
// Writes l1buf[vec], st[vec] (delta, flags: the info pair) and out.
constexpr int64_t kSmallBiasedMax = kGrain - 1;
__global__ void __launch_bounds__(256)
biased_small_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t d, float fm,
                    const float* __restrict__ l1in, float* __restrict__ l1buf, RezState* __restrict__ st) {
    extern __shared__ uint32_t keys[];                // [d] keys of the client
    __shared__ float scr[64 * 32 + 64];
    __shared__ uint32_t h[kRadixBins];
    __shared__ uint32_t lds[4];
    __shared__ uint32_t sel_digit, sel_above, sel_cnt;
    const int tid = threadIdx.x;
    const int64_t vec = blockIdx.x;
    const float* xv = x + vec * d;
    float* ov = out + vec * d;
    const float L = l1in ? l1in[vec] : block_torch_sum(xv, d, scr, [](float v) { return fabsf(v); });   // AS:680
    const DivPlan dp = div_plan(L);
    const float mprime = block_torch_sum(xv, d, scr, [&](float v) {                                 // AS:648-649
        return floorf(fm * div1(fabsf(v), dp) + 0.5f);
    });
    RezState s{};                                     // KB3 (AS:651-656)
    s.mprime = mprime;
    if (!(mprime == fm)) {
        if (!isfinite(mprime)) {
            s.flags |= kRezNonFinite;
        } else {
            const float df = mprime - fm;
            const long long D = (long long)df;
            const long long K = D > 0 ? D : -D;
            if (K > d) s.flags |= kRezRange;
            else {
                s.delta = (int32_t)D;
                s.kleft = (uint32_t)K;
            }
        }
    }
    const bool up = s.delta > 0;
    const bool on = s.kleft != 0;
    if (on) {                                         // KB4: keys, then the 3 radix digits from the top
        for (int64_t i = tid; i < d; i += 256) {
            float kp;
            keys[i] = rez_elem(xv[i], dp, fm, up, kp);
        }
        uint32_t prefix = 0, kleft = s.kleft, eq = 0;
        auto pass = [&](int shift, uint32_t dmask, uint32_t hmask) {
            const int nb = (int)dmask + 1;
            for (int b = tid; b < kRadixBins; b += 256) h[b] = 0u;
            __syncthreads();
            for (int64_t i = tid; i < d; i += 256) {
                const uint32_t k = keys[i];
                if ((k & hmask) == prefix) atomicAdd(&h[(k >> shift) & dmask], 1u);
            }
            __syncthreads();
            const int per = nb / 256;
            const int hi = nb - tid * per;            // thread 0 the highest digits
            uint32_t sum = 0;
            for (int k = 0; k < per; ++k) sum += h[hi - 1 - k];
            uint32_t total;
            uint32_t above = block_excl_scan_u32(sum, lds, &total);
            if (above < kleft && above + sum >= kleft) {
                for (int k = 0; k < per; ++k) {
                    const uint32_t c = h[hi - 1 - k];
                    if (above + c >= kleft) {
                        sel_digit = (uint32_t)(hi - 1 - k);
                        sel_above = above;
                        sel_cnt = c;
                        break;
                    }
                    above += c;
                }
            }
            __syncthreads();
            prefix |= sel_digit << shift;
            kleft -= sel_above;
            eq = sel_cnt;
            __syncthreads();
        };
        pass(RadixPass<0>::shift, RadixPass<0>::dmask, RadixPass<0>::hmask);
        pass(RadixPass<1>::shift, RadixPass<1>::dmask, RadixPass<1>::hmask);
        pass(RadixPass<2>::shift, RadixPass<2>::dmask, RadixPass<2>::hmask);
        s.prefix = prefix;
        s.kleft = kleft;
        s.eq = eq;
        s.need = kleft;
        if (eq > kleft) s.flags |= kRezAmbiguous;
    }
    const bool amb = on && (s.flags & kRezAmbiguous);
    const uint32_t tau = s.prefix;
    const DivPlan dpm = div_plan_m(fm);
    const float adj = up ? -1.f : 1.f;
    auto emit = [&](int64_t i, bool sel) {            // KB6 (AS:661/665/687)
        float kp;
        (void)rez_elem(xv[i], dp, fm, up, kp);
        const float k2 = sel ? kp + adj : kp;          // k''
        ov[i] = (L * torch_signf(xv[i])) * div1(k2, dpm);
    };
    if (!amb) {
        for (int64_t i = tid; i < d; i += 256) emit(i, on && keys[i] >= tau);
    } else {                                          // lowest indices among the ties
        const int64_t seg = (d + 255) / 256, b0 = tid * seg, b1 = b0 + seg < d ? b0 + seg : d;
        uint32_t cnt = 0;
        for (int64_t i = b0; i < b1; ++i) cnt += keys[i] == tau;
        uint32_t total;
        uint32_t rank = block_excl_scan_u32(cnt, lds, &total);
        for (int64_t i = b0; i < b1; ++i) {
            const uint32_t k = keys[i];
            emit(i, k > tau || (k == tau && rank++ < s.need));
        }
    }
    if (tid == 0) {
        l1buf[vec] = L;
        st[vec] = s;
    }
}
