// uq_biased_torch_ties.h — KB7: replay torch CPU's topk tie choice for ambiguous clients.
// Included by uq_dme.hip after uq_biased_kernels.h (anonymous namespace).
//
// torch.topk on a CPU f32 vector (ATen TopKImpl.h; torch is built against libstdc++)
// fills a queue of (value, index) pairs in index order and runs
//     std::partial_sort(q, q + k, end, comp)        if k * 64 <= d
//     std::nth_element(q, q + k - 1, end, comp)     otherwise
// with comp(a, b) = "a is NaN and b is not, or a > b"; the selected indices are q[0..k).
// Among coordinates whose value equals the threshold, which ones land in q[0..k) depends
// on the exact element moves of those algorithms, so KB7 replays them on the u32 keys of
// KB4 (key order == comp order, NaN and -0 folded as comp sees them):
//   * nth_element = introselect: median-of-3 pivot, unguarded Hoare partition, depth
//     limit 2*floor(log2 d) then heap_select, insertion sort of the last <= 3 elements.
//     Each Hoare partition runs data-parallel: the j-th left stop (key <= pivot, scanning
//     up from first+1) is swapped with the j-th right stop (key >= pivot, scanning down;
//     the pivot at `first` guards it) for every j with L_j < R_j; the cut is
//     min(L_{J+1}, R_J).  The stops come from one block-wide scan over the range.
//     (tools/nth_emul.cpp checks this restatement against std::nth_element itself.)
//   * partial_sort's set = heap_select: make_heap on q[0..k), then every later element
//     that beats the heap top replaces it (pop_heap).  Sequential by nature; one wave
//     skips 64 non-candidates per ballot, lane 0 runs the heap moves.
// The heap routines restate libstdc++'s __make_heap / __adjust_heap / __push_heap.
// Each workgroup owns one scratch slot (keys[d], indices[d] = the queue in SoA form, plus
// two position lists) and walks the clients blockIdx.x, +gridDim.x, ...; clients without
// an ambiguous tie are skipped.  Ranges of <= kTieLdsPairs finish in LDS.

constexpr int kTieSlots = 256;       // workgroups (and scratch slots) of KB7: one per CU
constexpr int kTieThreads = 1024;    // 16 waves per client (full replays)
constexpr int kTieWaves = kTieThreads / kWave;
constexpr int kTieU = 8;             // independent loads in flight per lane
constexpr int kTieLdsPairs = 8192;   // ranges this short finish in LDS (96 KB with the stop lists)
constexpr int kTieWaveMax = 1024;    // ... the last levels, below this, in one wave (no barriers)

#define TT_DECL() do {} while (0)
#define TT_T0() do {} while (0)
#define TT_ACC(k) do {} while (0)
#define TT_CNT(k) do {} while (0)

struct TieShared {
    uint32_t wl[kTieWaves], wr[kTieWaves];   // per-wave stop counts of one partition
    int64_t first, last;
    int depth, ret;
    uint32_t piv;
    uint32_t marked;
};

// The (value, index) queue in SoA form; element i = (K[i], I[i]).  The same code runs on
// the global slot and on the LDS copy of a short range.
struct Queue {
    uint32_t* K;
    uint32_t* I;
    __device__ uint32_t key(int64_t i) const { return K[i]; }
    __device__ uint64_t get(int64_t i) const { return ((uint64_t)K[i] << 32) | I[i]; }
    __device__ void set(int64_t i, uint64_t v) const { K[i] = (uint32_t)(v >> 32); I[i] = (uint32_t)v; }
    __device__ void swap(int64_t a, int64_t b) const {
        const uint32_t ka = K[a], ia = I[a];
        K[a] = K[b]; I[a] = I[b];
        K[b] = ka; I[b] = ia;
    }
    __device__ uint4 key4(int64_t q) const { return *reinterpret_cast<const uint4*>(K + q); }   // q % 4 == 0
};

// The same queue in LDS, through address-space-3 pointers: ds_read / ds_write (a generic
// pointer to LDS compiles to flat accesses, several times their latency).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
struct LdsQueue {
    lds_u32* K;
    lds_u32* I;
    __device__ uint32_t key(int64_t i) const { return K[i]; }
    __device__ uint64_t get(int64_t i) const { return ((uint64_t)K[i] << 32) | I[i]; }
    __device__ void set(int64_t i, uint64_t v) const { K[i] = (uint32_t)(v >> 32); I[i] = (uint32_t)v; }
    __device__ void swap(int64_t a, int64_t b) const {
        const uint32_t ka = K[a], ia = I[a];
        K[a] = K[b]; I[a] = I[b];
        K[b] = ka; I[b] = ia;
    }
    __device__ uint4 key4(int64_t q) const {                 // q % 4 == 0: one ds_read_b128
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) const u32x4v lds_q;
        const u32x4v v = *(lds_q*)(K + q);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
};

__device__ __forceinline__ uint32_t pkey(uint64_t p) { return (uint32_t)(p >> 32); }

template <class Q>
__device__ void tt_adjust_heap(const Q& A, int64_t f, int64_t hole, int64_t len, uint64_t value) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (A.key(f + second) > A.key(f + second - 1)) second--;
        A.set(f + hole, A.get(f + second));
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        A.set(f + hole, A.get(f + second - 1));
        hole = second - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && A.key(f + parent) > pkey(value)) {
        A.set(f + hole, A.get(f + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A.set(f + hole, value);
}

template <class Q>
__device__ void tt_make_heap(const Q& A, int64_t f, int64_t len) {
    if (len < 2) return;
    for (int64_t parent = (len - 2) / 2;; --parent) {
        tt_adjust_heap(A, f, parent, len, A.get(f + parent));
        if (parent == 0) break;
    }
}

// heap_select(A + f, A + m, A + l) by one wave (lanes 0..63 of the caller).
template <class Q>
__device__ void tt_heap_select_wave(const Q& A, int64_t f, int64_t m, int64_t l, int lane) {
    if (lane == 0) tt_make_heap(A, f, m - f);
    uint32_t top = __shfl(lane == 0 ? A.key(f) : 0u, 0, kWave);
    for (int64_t base = m; base < l; base += kWave) {
        const int64_t i = base + lane;
        const bool cand = i < l;
        const uint32_t ki = cand ? A.key(i) : 0u;
        uint64_t mask = __ballot(cand && ki > top);
        while (mask) {
            const int j = __builtin_ctzll(mask);
            uint32_t nt = 0;
            if (lane == 0) {                       // pop_heap(f, m, base + j)
                const uint64_t v = A.get(base + j);
                A.set(base + j, A.get(f));
                tt_adjust_heap(A, f, 0, m - f, v);
                nt = A.key(f);
            }
            top = __shfl(nt, 0, kWave);
            const uint64_t later = (j == 63) ? 0ull : (~0ull << (j + 1));
            mask = __ballot(cand && ki > top) & later;
        }
    }
}

template <class Q>
__device__ void tt_move_median_to_first(const Q& A, int64_t r, int64_t a, int64_t b, int64_t c) {
    const uint32_t ka = A.key(a), kb = A.key(b), kc = A.key(c);
    if (ka > kb) {
        if (kb > kc) A.swap(r, b);
        else if (ka > kc) A.swap(r, c);
        else A.swap(r, a);
    } else if (ka > kc) A.swap(r, a);
    else if (kb > kc) A.swap(r, c);
    else A.swap(r, b);
}

template <class Q>
__device__ void tt_insertion_sort(const Q& A, int64_t f, int64_t l) {
    if (f == l) return;
    for (int64_t i = f + 1; i != l; ++i) {
        const uint64_t v = A.get(i);
        if (pkey(v) > A.key(f)) {
            for (int64_t j = i; j > f; --j) A.set(j, A.get(j - 1));
            A.set(f, v);
        } else {
            int64_t j = i;
            while (pkey(v) > A.key(j - 1)) {
                A.set(j, A.get(j - 1));
                --j;
            }
            A.set(j, v);
        }
    }
}

__device__ __forceinline__ int floor_log2_i64(int64_t n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

// Stops of [s0, s1) (one wave's segment) in index order: FN(i, left, right) per element,
// lanes own i = b + u*64 + lane, kTieU loads in flight.  (Indices are 32-bit: d < 2^31.)
template <class Q, class FN>
__device__ __forceinline__ void tt_scan_segment(const Q& A, int32_t first, int32_t s0, int32_t s1, uint32_t piv,
                                                int lane, FN&& fn) {
    for (int32_t b = s0; b < s1; b += kWave * kTieU) {
        uint32_t k[kTieU];
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int32_t i = b + u * kWave + lane;
            k[u] = i < s1 ? A.key(i) : 0u;
        }
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int32_t i = b + u * kWave + lane;
            const bool valid = i < s1 && i >= first;
            fn(i, valid && i > first && k[u] <= piv,      // left stop:  !comp(A[i], pivot)
               valid && k[u] >= piv);                     // right stop: !comp(pivot, A[i])
        }
    }
}

// One unguarded Hoare partition of [first+1, last) around the pivot at `first` (indices
// relative to the queue view; positions listed as PosT).  Each wave lists the stops of
// its contiguous segment: one counting pass, a 16-entry prefix, one listing pass.
// Returns the cut, or -1 on an internal inconsistency.  32-bit index arithmetic (d < 2^31).
template <class Q, typename PosT, typename PosPtr, int NT>
__device__ int64_t tt_partition(const Q& A, PosPtr Lpos, PosPtr Rpos, int64_t first64, int64_t last64,
                                uint32_t piv, TieShared& sh) {
    TT_DECL();
    TT_T0();
    const int32_t first = (int32_t)first64, last = (int32_t)last64;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // segments start at multiples of 4 (16-byte aligned in the 16-byte aligned view); indices
    // below `first` belong to no stop list
    const int32_t a0 = first & ~3;
    constexpr int NW = NT / kWave;
    const int32_t seg = ((((last - a0) + NW - 1) / NW) + 4 * kWave - 1) & ~(4 * kWave - 1);
    const int32_t s0 = min(last, a0 + w * seg);
    const int32_t s1 = min(last, s0 + seg);
    uint32_t cl = 0, cr = 0;
    {   // counting pass: 4 keys per lane and load, lane-local counts, one wave reduction
        constexpr int kCU = 4;
        for (int32_t b = s0; b < s1; b += kWave * 4 * kCU) {
            uint4 kv[kCU];
#pragma unroll
            for (int u = 0; u < kCU; ++u) {
                const int32_t q = b + 4 * (u * kWave + lane);
                kv[u] = q < s1 ? A.key4(q) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < kCU; ++u) {
                const int32_t q = b + 4 * (u * kWave + lane);
                const uint32_t k4[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int32_t i = q + c;
                    const bool in = i < s1 && i >= first;
                    cl += (in && i > first && k4[c] <= piv) ? 1u : 0u;
                    cr += (in && k4[c] >= piv) ? 1u : 0u;
                }
            }
        }
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) {
            cl += __shfl_xor(cl, o, kWave);
            cr += __shfl_xor(cr, o, kWave);
        }
    }
    if (lane == 0) {
        sh.wl[w] = cl;
        sh.wr[w] = cr;
    }
    __syncthreads();
    uint32_t ol = 0, orr = 0, nL = 0, nR = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        const uint32_t a = sh.wl[q], b = sh.wr[q];
        ol += q < w ? a : 0u;
        orr += q < w ? b : 0u;
        nL += a;
        nR += b;
    }
    tt_scan_segment(A, first, s0, s1, piv, lane, [&](int32_t i, bool lf, bool rf) {
        const uint64_t ml = __ballot(lf), mr = __ballot(rf);
        if (lf) Lpos[ol + __popcll(ml & lt)] = (PosT)i;
        if (rf) Rpos[orr + __popcll(mr & lt)] = (PosT)i;
        ol += (uint32_t)__popcll(ml);
        orr += (uint32_t)__popcll(mr);
    });
    __syncthreads();
    TT_ACC(1);
    // J = number of swaps = largest J with L_J < R_J (1-based; R counted from the right),
    // found by a block-parallel search (the predicate holds for a prefix of J).
    int32_t lo = 0, hi = (int32_t)(nL < nR ? nL : nR);
    const int32_t nRi = (int32_t)nR;
    while (lo < hi) {
        const int32_t step = (hi - lo + NT - 1) / NT;
        const int32_t cand = lo + (tid + 1) * step;
        const bool f = cand <= hi && (int32_t)Lpos[cand - 1] < (int32_t)Rpos[nRi - cand];
        const int cnt = __syncthreads_count(f);
        if (cnt == 0) {
            hi = lo + step - 1;
        } else {
            lo = lo + cnt * step;
            hi = min(hi, lo + step - 1);
        }
    }
    TT_ACC(2);
    const int32_t J = lo;
    int32_t cut = INT32_MAX;
    if (J < (int32_t)nL) cut = (int32_t)Lpos[J];
    if (J > 0) cut = min(cut, (int32_t)Rpos[nRi - J]);
    // the J swaps are disjoint pairs: kTieU of them per lane, independent loads
    for (int32_t j0 = 0; j0 < J; j0 += NT * kTieU) {
        int32_t a[kTieU], b[kTieU];
        uint32_t ka[kTieU], kb[kTieU], ia[kTieU], ib[kTieU];
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int32_t j = j0 + u * NT + tid;
            a[u] = j < J ? (int32_t)Lpos[j] : -1;
            b[u] = j < J ? (int32_t)Rpos[nRi - 1 - j] : -1;
        }
#pragma unroll
        for (int u = 0; u < kTieU; ++u)
            if (a[u] >= 0) {
                ka[u] = A.K[a[u]]; ia[u] = A.I[a[u]];
                kb[u] = A.K[b[u]]; ib[u] = A.I[b[u]];
            }
#pragma unroll
        for (int u = 0; u < kTieU; ++u)
            if (a[u] >= 0) {
                A.K[a[u]] = kb[u]; A.I[a[u]] = ib[u];
                A.K[b[u]] = ka[u]; A.I[b[u]] = ia[u];
            }
    }
    __syncthreads();
    TT_ACC(3);
    return (cut <= first || cut >= last) ? -1 : (int64_t)cut;
}

// introselect's main loop on the queue view (element i of the vector at view index i - o)
// while the range is longer than `stop`.  Returns 0 (range now <= stop), 1 (finished
// through the heap fallback) or -1 (internal inconsistency).
template <class Q, typename PosT, typename PosPtr, int NT>
__device__ int tt_select_loop(const Q& A, PosPtr Lpos, PosPtr Rpos, int64_t o, int64_t nth, int64_t stop,
                              TieShared& sh) {
    TT_DECL();
    const int tid = threadIdx.x;
    for (;;) {
        const int64_t first = sh.first - o, last = sh.last - o;
        const int depth = sh.depth;
        if (last - first <= stop) return 0;
        if (depth == 0) {                                   // heap_select(first, nth+1, last)
            if (tid < kWave) tt_heap_select_wave(A, first, nth - o + 1, last, tid);
            __syncthreads();
            if (tid == 0) A.swap(first, nth - o);
            __syncthreads();
            return 1;
        }
        __syncthreads();
        TT_T0();
        if (tid == 0) {
            const int64_t mid = first + (last - first) / 2;
            tt_move_median_to_first(A, first, first + 1, mid, last - 1);
            sh.piv = A.key(first);
        }
        __syncthreads();
        TT_ACC(4);
        const int64_t cut = tt_partition<Q, PosT, PosPtr, NT>(A, Lpos, Rpos, first, last, sh.piv, sh);
        if (cut < 0) return -1;
        if (tid == 0) {
            if (cut + o <= nth) sh.first = cut + o; else sh.last = cut + o;
            sh.depth = depth - 1;
        }
        __syncthreads();
    }
}

// LDS operations of one wave are performed in order; this keeps the compiler from moving
// them across the points where lanes read what other lanes wrote
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// introselect's loop on the LDS window (view index = vector index - o) by ONE wave, down to
// ranges of 3 (tt_select_loop's moves, without a barrier per step: a workgroup-wide
// partition of a few thousand keys is a dozen barriers and serial lane-0 steps, the wave's
// one ordered pass appends its stops directly).  first / last / depth in and out (vector
// indices).  Returns 0 (range <= 3), 1 (finished through the heap fallback), -1 (internal
// inconsistency).
__device__ int tt_select_wave(const LdsQueue& A, lds_u16* lL, lds_u16* lR, int64_t o, int64_t nth, int64_t& first_io,
                              int64_t& last_io, int& depth_io, int lane) {
    constexpr int kU = 4;                                   // keys in flight per lane
    int32_t first = (int32_t)(first_io - o), last = (int32_t)(last_io - o);
    const int32_t nv = (int32_t)(nth - o);
    int depth = depth_io;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int ret = 0;
    TT_DECL();
    TT_T0();
    for (;;) {
        if (last - first <= 3) break;
        TT_CNT(11);
        if (depth == 0) {                                   // heap_select(first, nth+1, last)
            tt_heap_select_wave(A, first, nv + 1, last, lane);
            wave_lds_sync();
            if (lane == 0) A.swap(first, nv);
            wave_lds_sync();
            ret = 1;
            break;
        }
        if (lane == 0) tt_move_median_to_first(A, first, first + 1, first + (last - first) / 2, last - 1);
        wave_lds_sync();
        const uint32_t piv = A.key(first);
        uint32_t nL = 0, nR = 0;
        TT_ACC(15);
        for (int32_t b = first; b < last; b += kWave * kU) {        // stops in index order
            uint32_t k[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t i = b + u * kWave + lane;
                k[u] = i < last ? A.key(i) : 0u;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t i = b + u * kWave + lane;
                const bool in = i < last;
                const bool lf = in && i > first && k[u] <= piv;     // !comp(A[i], pivot)
                const bool rf = in && k[u] >= piv;                  // !comp(pivot, A[i])
                const uint64_t ml = __ballot(lf), mr = __ballot(rf);
                if (lf) lL[nL + (uint32_t)__popcll(ml & lt)] = (uint16_t)i;
                if (rf) lR[nR + (uint32_t)__popcll(mr & lt)] = (uint16_t)i;
                nL += (uint32_t)__popcll(ml);
                nR += (uint32_t)__popcll(mr);
            }
        }
        wave_lds_sync();
        TT_ACC(12);
        int32_t lo = 0, hi = (int32_t)(nL < nR ? nL : nR);  // J: L_J < R_J holds for a prefix
        while (lo < hi) {
            const int32_t step = (hi - lo + kWave - 1) / kWave;
            const int32_t cand = lo + (lane + 1) * step;
            const bool f = cand <= hi && (int32_t)lL[cand - 1] < (int32_t)lR[nR - cand];
            const int c = __popcll(__ballot(f));
            if (c == 0) {
                hi = lo + step - 1;
            } else {
                lo = lo + c * step;
                hi = min(hi, lo + step - 1);
            }
        }
        const int32_t J = lo;
        int32_t cut = INT32_MAX;
        if (J < (int32_t)nL) cut = lL[J];
        if (J > 0) cut = min(cut, (int32_t)lR[nR - J]);
        TT_ACC(13);
        for (int32_t j0 = 0; j0 < J; j0 += kWave * kU) {              // J disjoint swaps
            int32_t pa[kU], pb[kU];
            uint32_t ka[kU], kb[kU], ia[kU], ib[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t j = j0 + u * kWave + lane;
                pa[u] = j < J ? (int32_t)lL[j] : -1;
                pb[u] = j < J ? (int32_t)lR[nR - 1 - j] : -1;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (pa[u] >= 0) {
                    ka[u] = A.K[pa[u]]; ia[u] = A.I[pa[u]];
                    kb[u] = A.K[pb[u]]; ib[u] = A.I[pb[u]];
                }
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (pa[u] >= 0) {
                    A.K[pa[u]] = kb[u]; A.I[pa[u]] = ib[u];
                    A.K[pb[u]] = ka[u]; A.I[pb[u]] = ia[u];
                }
        }
        wave_lds_sync();
        TT_ACC(14);
        if (cut <= first || cut >= last) {
            ret = -1;
            break;
        }
        if (cut <= nv) first = cut; else last = cut;
        --depth;
    }
    first_io = first + o;
    last_io = last + o;
    depth_io = depth;
    return ret;
}

// std::nth_element(A, A + nth, A + d) by the whole workgroup (false on an inconsistency),
// from introselect's state (first, last, depth) -- (0, d, 2 floor(log2 d)) at the start, or
// where the multi-workgroup levels (KB7a, below) left it.
template <int NT>
__device__ bool tt_introselect(const Queue& A, uint32_t* Lpos, uint32_t* Rpos, int64_t d, int64_t nth,
                               TieShared& sh, uint32_t* lK, uint32_t* lI, uint16_t* lL, uint16_t* lR,
                               int64_t first0, int64_t last0, int depth0) {
    TT_DECL();
    const int tid = threadIdx.x;
    if (tid == 0) {
        sh.first = first0;
        sh.last = last0;
        sh.depth = depth0;
    }
    __syncthreads();
    int r = tt_select_loop<Queue, uint32_t, uint32_t*, NT>(A, Lpos, Rpos, 0, nth, kTieLdsPairs, sh);
    if (r < 0) return false;
    TT_T0();
    if (r == 0 && sh.last - sh.first > 3) {                // finish the short range in LDS
        const int64_t f0 = sh.first, len = sh.last - sh.first;
        for (int64_t i = tid; i < len; i += NT) {
            lK[i] = A.K[f0 + i];
            lI[i] = A.I[f0 + i];
        }
        __syncthreads();
        TT_ACC(8);
        const LdsQueue L{(lds_u32*)lK, (lds_u32*)lI};
        // the whole workgroup while the range is long, one wave below kTieWaveMax
        r = tt_select_loop<LdsQueue, uint16_t, lds_u16*, NT>(L, (lds_u16*)lL, (lds_u16*)lR, f0, nth, kTieWaveMax, sh);
        __syncthreads();                                     // every wave has read sh's range
        TT_ACC(7);
        if (r == 0 && tid < kWave) {
            int64_t f = sh.first, l = sh.last;
            int dep = sh.depth;
            const int rw = tt_select_wave(L, (lds_u16*)lL, (lds_u16*)lR, f0, nth, f, l, dep, tid);
            if (tid == 0) {
                sh.first = f;
                sh.last = l;
                sh.depth = dep;
                sh.ret = rw;
            }
        }
        if (r != 0 && tid == 0) sh.ret = r;
        __syncthreads();
        TT_ACC(9);
        r = sh.ret;
        for (int64_t i = tid; i < len; i += NT) {
            A.K[f0 + i] = lK[i];
            A.I[f0 + i] = lI[i];
        }
        __syncthreads();
        if (r < 0) return false;
    }
    TT_ACC(5);
    if (r == 0 && tid == 0) tt_insertion_sort(A, sh.first, sh.last);
    __syncthreads();
    TT_ACC(10);
    return true;
}

// ---- KB7a: introselect's first levels over many workgroups ----------------------------
// The long partitions (range > kTieLevelMin) of all replayed clients run level by level
// as separate launches over (segments x slots), so every CU works on them instead of one
// workgroup per client: queue fill; per level the pivot (median of 3 to `first`), stop
// counts per segment, stop lists in index order, J and the cut, the J swaps.  The element
// moves are those of tt_partition (the stop lists are defined by index order, not by who
// scans), so rez_ties_kernel resumes from the saved (first, last, depth) with the same
// queue it would have built itself.  Slot a serves list entry a (a < kTieSlots).
constexpr int64_t kTieLevelMin = kTieLdsPairs;   // shorter ranges finish in rez_ties_kernel's LDS
// KB7a's levels run while a range is longer than kTieLevelStop, level count ceil(log2(d /
// stop)) + kTieLevelMargin (median-of-3 pivots halve a range per level on average; an idle
// level is five dependent ~6 us launches).  The 1024-thread replays (part 1, right after the
// levels on the side stream) take every slot KB7a resumed from where it stopped: global-memory
// levels while longer than kTieLdsPairs, then the LDS levels (workgroup-wide, the last ones in
// one wave).  Stop / margin on one box (ms per C2-sized torch-tie batch, tools/exp/run_r5x.sh,
// run_r5z.sh): 16384 / 2 4.57, 16384 / 3 4.55, 8192 / 3 4.54, 32768 / 2 4.58, 65536 / 2 4.60.
// (Round 3 stopped at 2^14 after levels for 0.6 per level + 2 and ran the LDS tails with
// 256 threads through generic pointers: 4.63 on the same box as this form's 4.59.)
constexpr int64_t kTieLevelStop = 16384;
constexpr int kTieLevelMargin = 3;
// KB6's first part waits for this many KB7a levels (launch_torch_ties' `mid`)
constexpr int kTieHeavyLevels = 2;
constexpr int64_t kTieLevelMinClients = 32;      // KB7a for batches of at least this many clients
// ... and for any batch of vectors this long: one replay workgroup walking 2^22 keys took
// ~9 ms (a 6-client batch at d = 2^22 with one ambiguous client), KB7a's idle launches 0.35 ms
constexpr int64_t kTieLevelBigD = (int64_t)1 << 21;
constexpr int kTieSegs = 256;               // segments per partition (one wave each)
constexpr int kTieMarkSegs = 64;            // workgroups per client for kt_mark

struct TieLevelState {
    int64_t first, last, nth;
    int64_t J, nL, nR;
    int64_t mpos;               // the median's position before its move to `first` (-1: moved)
    int32_t depth, active, filled, err;
    uint32_t piv, kfirst;       // the pivot; the key at `first` before the move
    uint32_t marked;            // ties at the threshold in [0, first) (kt_mark_kernel)
};

// tt_move_median_to_first's choice: which of a, b, c (keys ka, kb, kc) moves to `first`
__device__ __forceinline__ int64_t tt_median_pos(uint32_t ka, uint32_t kb, uint32_t kc, int64_t a, int64_t b,
                                                 int64_t c) {
    if (ka > kb) {
        if (kb > kc) return b;
        return ka > kc ? c : a;
    }
    if (ka > kc) return a;
    return kb > kc ? c : b;
}

constexpr int kTieGrid = 2048;              // workgroups of the per-level launches (4 waves each)

// segment s of [first, last) for one wave
__device__ __forceinline__ void kt_seg(int64_t first, int64_t last, int s, int64_t& s0, int64_t& s1) {
    const int64_t len = last - first;
    const int64_t seg = (((len + kTieSegs - 1) / kTieSegs) + 63) & ~(int64_t)63;
    s0 = min(last, first + (int64_t)s * seg);
    s1 = min(last, s0 + seg);
}

// A slot's introselect state at this level: level 0 from the client (queue [0, d), depth
// 2 floor(log2 d); listed nth_element clients only -- partial_sort's heap path and unused
// slots stay unfilled, rez_ties_kernel part 2 replays those), later levels from tls.
struct KtLevel {
    int64_t vec, k, first, last;
    int depth;
    bool filled, act;
};
__device__ __forceinline__ KtLevel kt_level(int a, int64_t d, uint32_t nlist, const RezState* __restrict__ st,
                                            const uint32_t* __restrict__ list, const TieLevelState* __restrict__ tls,
                                            int64_t stop, bool level0) {
    KtLevel v{};
    if (a >= (int)nlist) return v;
    v.vec = list[1 + a];
    if (level0) {
        const int32_t delta = st[v.vec].delta;
        v.k = delta > 0 ? delta : -(int64_t)delta;
        v.first = 0;
        v.last = d;
        v.depth = 2 * floor_log2_i64(d);
        v.filled = v.k * 64 > d;
        v.act = v.filled && v.depth > 0 && d > stop;
    } else {
        const TieLevelState& t = tls[a];
        v.first = t.first;
        v.last = t.last;
        v.depth = t.depth;
        v.filled = t.filled != 0;
        v.act = v.filled && !t.err && v.depth > 0 && v.last - v.first > stop;
    }
    return v;
}

// One wave's segment [s0, s1) of a level: its stop counts with the median move substituted
// (sub: the segment holds `first` or mpos); L0: keys from x, and the queue written (d < 2^31:
// 32-bit indices; the 64-bit index arithmetic was most of this loop's VALU work).
template <bool L0>
__device__ __forceinline__ void kt_count_seg(const float* __restrict__ xv, const DivPlan& dp, float fm, bool up,
                                             uint32_t* __restrict__ K, uint32_t* __restrict__ I, int32_t s0, int32_t s1,
                                             int32_t first, int32_t mpos, uint32_t piv, uint32_t kfirst, bool sub,
                                             int lane, uint32_t& cl, uint32_t& cr) {
    for (int32_t b = s0; b < s1; b += 64 * kTieU) {
        uint32_t kk[kTieU];
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int32_t i = b + u * 64 + lane;
            float kp;
            kk[u] = i < s1 ? (L0 ? rez_elem(xv[i], dp, fm, up, kp) : K[i]) : 0u;
        }
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int32_t i = b + u * 64 + lane;
            if (i >= s1) continue;
            uint32_t key = kk[u], idx = (uint32_t)i;
            if (sub) {
                if (i == first) { key = piv; idx = (uint32_t)mpos; }
                else if (i == mpos) { key = kfirst; idx = (uint32_t)first; }
            }
            if (L0) {
                K[i] = key;
                I[i] = idx;
            }
            cl += ((!sub || i > first) && key <= piv) ? 1u : 0u;
            cr += (key >= piv) ? 1u : 0u;
        }
    }
}

// level step 1: the pivot and the left / right stop counts per segment (cnt [slots][kTieSegs]
// [2]); at level 0 also the queue fill from x (the tie bits of the listed clients cleared
// beside it: no other row is read).  Workgroup 0 (one thread per slot) keeps the slots'
// state (level 0: sets it up), their active flags and the compacted active list (alist[0] =
// count) that the level's other launches spread over.  Items (slot, segment), one per wave:
// every wave of a slot computes the median of 3 itself, so the pivot costs no launch of its
// own.  The move of the median to `first` is written by the fill at level 0; at later levels
// the counts and the lists see it as a substitution (positions first and mpos) and kt_jcut
// moves the pair in memory, when no kernel reads the keys.
__global__ void __launch_bounds__(256)
kt_count_kernel(const float* __restrict__ x, int64_t d, const float* __restrict__ l1, float fm,
                const RezState* __restrict__ st, uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ list,
                TieLevelState* __restrict__ tls, uint32_t* __restrict__ cnt, uint32_t* __restrict__ alist,
                uint32_t* __restrict__ tie_bits, int slots, int64_t stop, int level0) {
    const uint32_t nlist = list[0];
    const int lane = threadIdx.x & 63;
    const int64_t dpad = (d + 3) & ~(int64_t)3;
    if (blockIdx.x == 0) {
        __shared__ uint32_t wc[kTieSlots / 64];
        const int a = threadIdx.x, w = a >> 6;
        bool act = false;
        if (a < slots) {
            const KtLevel v = kt_level(a, d, nlist, st, list, tls, stop, level0 != 0);
            act = v.act;
            TieLevelState& t = tls[a];
            if (level0) {                           // field by field: piv is the segment-0 wave's
                t.first = 0;
                t.last = d;
                t.nth = v.k - 1;
                t.J = t.nL = t.nR = 0;
                t.depth = v.depth;
                t.filled = v.filled ? 1 : 0;
                t.err = 0;
                t.marked = 0u;
            }
            t.active = act ? 1 : 0;
        }
        const uint64_t m = __ballot(act);
        if (lane == 0) wc[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = 0, tot = 0;
        for (int q = 0; q < kTieSlots / 64; ++q) {
            off += q < w ? wc[q] : 0u;
            tot += wc[q];
        }
        if (act) alist[1 + off + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)a;
        if (a == 0) alist[0] = tot;
    }
    const int nsl = min((int)nlist, slots);
    const int64_t items = (int64_t)nsl * kTieSegs;
    for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < items; it += (int64_t)gridDim.x * 4) {
        const int a = (int)(it / kTieSegs), sg = (int)(it % kTieSegs);
        if (level0) {
            const int64_t words = (d + 31) / 32;
            const int64_t wseg = (words + kTieSegs - 1) / kTieSegs;
            const int64_t w0 = (int64_t)sg * wseg, w1 = min(words, w0 + wseg);
            for (int64_t e = a; e < (int64_t)nlist; e += slots) {
                uint32_t* row = tie_bits + (int64_t)list[1 + e] * words;
                for (int64_t i = w0 + lane; i < w1; i += 64) row[i] = 0u;
            }
        }
        const KtLevel v = kt_level(a, d, nlist, st, list, tls, stop, level0 != 0);
        if (!v.filled || (!level0 && !v.act)) continue;
        uint32_t* K = qbuf + (size_t)a * 2 * dpad;
        uint32_t* I = K + dpad;
        const float* xv = x ? x + v.vec * d : nullptr;
        DivPlan dp{};
        bool up = false;
        if (level0) {
            dp = div_plan(l1[v.vec]);
            up = st[v.vec].delta > 0;
        }
        auto key_at = [&](int64_t i) -> uint32_t {
            float kp;
            return level0 ? rez_elem(xv[i], dp, fm, up, kp) : K[i];
        };
        // the median of 3 to `first` (tt_move_median_to_first), when this level runs
        int64_t mpos = -1;
        uint32_t piv = 0u, kfirst = 0u;
        if (v.act) {
            const int64_t mid = v.first + (v.last - v.first) / 2;
            kfirst = key_at(v.first);
            const uint32_t ka = key_at(v.first + 1), kb = key_at(mid), kc = key_at(v.last - 1);
            mpos = tt_median_pos(ka, kb, kc, v.first + 1, mid, v.last - 1);
            piv = mpos == v.first + 1 ? ka : (mpos == mid ? kb : kc);
        }
        int64_t s0, s1;
        kt_seg(v.first, v.last, sg, s0, s1);
        const bool sub = mpos >= 0 && ((v.first >= s0 && v.first < s1) || (mpos >= s0 && mpos < s1));
        uint32_t cl = 0, cr = 0;
        if (level0)
            kt_count_seg<true>(xv, dp, fm, up, K, I, (int32_t)s0, (int32_t)s1, (int32_t)v.first, (int32_t)mpos, piv,
                               kfirst, sub, lane, cl, cr);
        else
            kt_count_seg<false>(xv, dp, fm, up, K, I, (int32_t)s0, (int32_t)s1, (int32_t)v.first, (int32_t)mpos, piv,
                                kfirst, sub, lane, cl, cr);
        if (!v.act) continue;                           // level 0 fill of a slot whose range is short
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cl += __shfl_xor(cl, o, 64);
            cr += __shfl_xor(cr, o, 64);
        }
        if (lane == 0) {
            cnt[((size_t)a * kTieSegs + sg) * 2] = cl;
            cnt[((size_t)a * kTieSegs + sg) * 2 + 1] = cr;
            if (sg == 0) {
                tls[a].piv = piv;
                tls[a].kfirst = kfirst;
                tls[a].mpos = level0 ? -1 : mpos;
            }
        }
    }
}

// level step 3: stop lists in index order
__global__ void __launch_bounds__(256)
kt_list_kernel(int64_t d, const uint32_t* __restrict__ qbuf, uint32_t* __restrict__ pos,
               const TieLevelState* __restrict__ tls, const uint32_t* __restrict__ cnt,
               const uint32_t* __restrict__ alist) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t items = (int64_t)alist[0] * kTieSegs;
    for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < items; it += (int64_t)gridDim.x * 4) {
        const int a = (int)alist[1 + it / kTieSegs], sg = (int)(it % kTieSegs);
        const TieLevelState& t = tls[a];
        const int64_t dpad = (d + 3) & ~(int64_t)3;
        const uint32_t* K = qbuf + (size_t)a * 2 * dpad;
        uint32_t* Lpos = pos + (size_t)a * 2 * d;
        uint32_t* Rpos = Lpos + d;
        uint32_t ol = 0, orr = 0;
        for (int q = lane; q < sg; q += 64) {
            ol += cnt[((size_t)a * kTieSegs + q) * 2];
            orr += cnt[((size_t)a * kTieSegs + q) * 2 + 1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            ol += __shfl_xor(ol, o, 64);
            orr += __shfl_xor(orr, o, 64);
        }
        const int64_t first = t.first, mpos = t.mpos;
        const uint32_t piv = t.piv, kfirst = t.kfirst;
        int64_t s0, s1;
        kt_seg(first, t.last, sg, s0, s1);
        // the median move as a substitution: only the (at most two) segments holding `first`
        // or mpos take the slow form (wave-uniform)
        const bool sub = (first >= s0 && first < s1) || (mpos >= s0 && mpos < s1);
        const int32_t e1 = (int32_t)s1, f32 = (int32_t)first, m32 = (int32_t)mpos;      // d < 2^31
        for (int32_t b = (int32_t)s0; b < e1; b += 64 * kTieU) {
            uint32_t kk[kTieU];
#pragma unroll
            for (int u = 0; u < kTieU; ++u) {
                const int32_t i = b + u * 64 + lane;
                kk[u] = i < e1 ? K[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kTieU; ++u) {
                const int32_t i = b + u * 64 + lane;
                uint32_t key = kk[u];
                if (sub) key = i == f32 ? piv : (i == m32 ? kfirst : key);
                const bool lf = i < e1 && (!sub || i > f32) && key <= piv;
                const bool rf = i < e1 && key >= piv;
                const uint64_t ml = __ballot(lf), mr = __ballot(rf);
                if (lf) Lpos[ol + __popcll(ml & lt)] = (uint32_t)i;
                if (rf) Rpos[orr + __popcll(mr & lt)] = (uint32_t)i;
                ol += (uint32_t)__popcll(ml);
                orr += (uint32_t)__popcll(mr);
            }
        }
    }
}

// level step 4 (one 256-thread workgroup per slot): J = the largest J with L_J < R_J (R
// counted from the right), the cut, and introselect's next range -- as tt_partition /
// tt_select_loop.  Small workgroups, so that the step is dispatched between KB6's
// workgroups instead of waiting for a whole CU to drain (KB7a runs beside KB6).
constexpr int kJcutThreads = 256;

__global__ void __launch_bounds__(kJcutThreads)
kt_jcut_kernel(int64_t d, uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ pos, TieLevelState* __restrict__ tls,
               const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ alist) {
    constexpr int kW = kJcutThreads / kWave;
    __shared__ uint32_t red[2][kW];
    if (blockIdx.x >= alist[0]) return;
    const int a = (int)alist[1 + blockIdx.x], tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    TieLevelState& t = tls[a];
    const uint32_t* Lpos = pos + (size_t)a * 2 * d;
    const uint32_t* Rpos = Lpos + d;
    uint32_t cl = 0, cr = 0;
    for (int q = tid; q < kTieSegs; q += kJcutThreads) {
        cl += cnt[((size_t)a * kTieSegs + q) * 2];
        cr += cnt[((size_t)a * kTieSegs + q) * 2 + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cl += __shfl_xor(cl, o, 64);
        cr += __shfl_xor(cr, o, 64);
    }
    if (lane == 0) {
        red[0][w] = cl;
        red[1][w] = cr;
    }
    __syncthreads();
    uint32_t nL = 0, nR = 0;
    for (int q = 0; q < kW; ++q) {
        nL += red[0][q];
        nR += red[1][q];
    }
    int64_t lo = 0, hi = nL < nR ? nL : nR;
    while (lo < hi) {
        const int64_t step = (hi - lo + kJcutThreads - 1) / kJcutThreads;
        const int64_t cand = lo + (int64_t)(tid + 1) * step;
        const bool f = cand <= hi && (int64_t)Lpos[cand - 1] < (int64_t)Rpos[nR - cand];
        const int c = __syncthreads_count(f);
        if (c == 0) {
            hi = lo + step - 1;
        } else {
            lo = lo + (int64_t)c * step;
            hi = std::min<int64_t>(hi, lo + step - 1);
        }
    }
    if (tid == 0) {
        if (t.mpos >= 0) {                  // the median's move to `first` (kt_count_kernel)
            const int64_t dpad = (d + 3) & ~(int64_t)3;
            uint32_t* K = qbuf + (size_t)a * 2 * dpad;
            uint32_t* I = K + dpad;
            const uint32_t im = I[t.mpos], i0 = I[t.first];
            K[t.first] = t.piv;
            I[t.first] = im;
            K[t.mpos] = t.kfirst;
            I[t.mpos] = i0;
        }
        const int64_t J = lo;
        int64_t cut = INT64_MAX;
        if (J < (int64_t)nL) cut = (int64_t)Lpos[J];
        if (J > 0) cut = std::min<int64_t>(cut, (int64_t)Rpos[nR - J]);
        t.J = J;
        t.nL = nL;
        t.nR = nR;
        if (cut <= t.first || cut >= t.last) {
            t.err = 1;
        } else {
            if (cut <= t.nth) t.first = cut; else t.last = cut;
            t.depth -= 1;
        }
    }
}

// level step 5: the J disjoint swaps
__global__ void __launch_bounds__(256)
kt_swap_kernel(int64_t d, uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ pos,
               const TieLevelState* __restrict__ tls, const uint32_t* __restrict__ alist) {
    // few VGPRs (u32 positions, 4 swaps in flight per lane): this runs beside KB6, whose
    // 40-VGPR waves leave only small holes to dispatch into.  The grid is dealt out over the
    // active slots (workgroup b serves slot b mod nA), so a workgroup reads its slot's state
    // once and strides over that slot's swaps.
    constexpr int kB = 4;
    const uint32_t nA = alist[0];
    if (blockIdx.x >= (gridDim.x / nA) * nA) return;             // also nA == 0
    const int a = (int)alist[1 + blockIdx.x % nA];
    const int64_t c = blockIdx.x / nA, C = gridDim.x / nA;
    const TieLevelState& t = tls[a];
    const int64_t dpad = (d + 3) & ~(int64_t)3;
    uint32_t* K = qbuf + (size_t)a * 2 * dpad;
    uint32_t* I = K + dpad;
    const uint32_t* Lpos = pos + (size_t)a * 2 * d;
    const uint32_t* Rpos = Lpos + d;
    const int32_t J = (int32_t)t.J, nR = (int32_t)t.nR;      // d < 2^31
    const int tid = threadIdx.x;
    for (int32_t j0 = (int32_t)c * 256 * kB; j0 < J; j0 += (int32_t)C * 256 * kB) {
        uint32_t pa[kB], pb[kB], ka[kB], kb[kB], ia[kB], ib[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int32_t j = j0 + u * 256 + tid;
            pa[u] = j < J ? Lpos[j] : 0u;
            pb[u] = j < J ? Rpos[nR - 1 - j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kB; ++u)
            if (j0 + u * 256 + tid < J) {
                ka[u] = K[pa[u]]; ia[u] = I[pa[u]];
                kb[u] = K[pb[u]]; ib[u] = I[pb[u]];
            }
#pragma unroll
        for (int u = 0; u < kB; ++u)
            if (j0 + u * 256 + tid < J) {
                K[pa[u]] = kb[u]; I[pa[u]] = ib[u];
                K[pb[u]] = ka[u]; I[pb[u]] = ia[u];
            }
    }
}

// After the levels, queue[0, first) is final (introselect only works inside [first, last)):
// the ties at the threshold there are marked here over (segments x slots) workgroups, so the
// LDS-tail replay marks only [first, k).
__global__ void __launch_bounds__(256)
kt_mark_kernel(int64_t d, const uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ list,
               const RezState* __restrict__ st, TieLevelState* __restrict__ tls, uint32_t* __restrict__ tie_bits) {
    __shared__ uint32_t wsum[4];
    const int64_t a = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    TieLevelState& t = tls[a];
    if (!t.filled || t.err) return;
    const int64_t vec = list[1 + a];
    const uint32_t tau = st[vec].prefix;
    const int64_t dpad = (d + 3) & ~(int64_t)3;
    const uint32_t* K = qbuf + (size_t)a * 2 * dpad;
    const uint32_t* I = K + dpad;
    uint32_t* bits = tie_bits + vec * ((d + 31) / 32);
    const int64_t end = t.first;
    const int64_t seg = (((end + gridDim.x - 1) / gridDim.x) + 255) & ~(int64_t)255;
    const int64_t b = min(end, (int64_t)blockIdx.x * seg), e = min(end, b + seg);
    uint32_t mine = 0;
    for (int64_t p0 = b; p0 < e; p0 += 256 * kTieU) {
        uint32_t kk[kTieU];
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int64_t p = p0 + (int64_t)u * 256 + tid;
            kk[u] = p < e ? K[p] : ~tau;
        }
#pragma unroll
        for (int u = 0; u < kTieU; ++u) {
            const int64_t p = p0 + (int64_t)u * 256 + tid;
            if (p < e && kk[u] == tau) {
                const uint32_t ii = I[p];
                atomicOr(&bits[ii >> 5], 1u << (ii & 31));
                ++mine;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (lane == 0) wsum[w] = mine;
    __syncthreads();
    if (tid == 0) {
        const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (tot) atomicAdd(&t.marked, tot);
    }
}

// The clients KB7 replays, in client order: list[0] = count, list[1 + i] = client.  With one
// replay per workgroup (up to kTieSlots of them) no workgroup runs two replays back to back,
// which a client-strided walk did whenever two ambiguous clients shared a residue mod the
// grid.
__global__ void __launch_bounds__(1024)
rez_tie_list_kernel(const RezState* __restrict__ st, int64_t n, uint32_t* __restrict__ list) {
    __shared__ uint32_t wc[16];
    __shared__ uint32_t base;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) base = 0u;
    __syncthreads();
    for (int64_t j0 = 0; j0 < n; j0 += 1024) {
        const int64_t j = j0 + tid;
        bool f = false;
        if (j < n) {
            const RezState s = st[j];
            f = s.kleft != 0 && (s.flags & kRezAmbiguous);
        }
        const uint64_t m = __ballot(f);
        if (lane == 0) wc[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = base;
        for (int q = 0; q < w; ++q) off += wc[q];
        if (f) list[1 + off + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)j;
        __syncthreads();
        if (tid == 0) {
            uint32_t t = 0u;
            for (int q = 0; q < 16; ++q) t += wc[q];
            base += t;
        }
        __syncthreads();
    }
    if (tid == 0) list[0] = base;
}

// Defined fallback of a replay that failed its consistency checks (internal error,
// reported through the status word): the client keeps kRezAmbiguous without kRezTorchTies,
// so KB6 ranks its threshold ties in index order (the UQ_TIES_LOWEST_INDEX choice) from
// per-tile tie counts -- which rez_tiecount_kernel skips for listed clients, so the
// workgroup counts them here (a wave per 4096-tile).
template <int NT>
__device__ void tt_fallback_tilecounts(const float* __restrict__ xv, int64_t d, const DivPlan& dp, float fm, bool up,
                                       uint32_t tau, uint32_t* __restrict__ trow, int32_t tiles) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    for (int32_t t = w; t < tiles; t += NT / kWave) {
        const int64_t b = (int64_t)t * kSelTile, e = min(d, b + (int64_t)kSelTile);
        uint32_t c = 0;
        for (int64_t i = b + lane; i < e; i += kWave) {
            float kp;
            c += rez_elem(xv[i], dp, fm, up, kp) == tau ? 1u : 0u;
        }
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
        if (lane == 0) trow[t] = c;
    }
}

// NT threads per workgroup.  part 0: every listed client (slots walk the list).  With
// KB7a's level state `tls`: part 1 finishes the clients KB7a resumed (slot a = list entry a),
// part 2 every other listed client.
template <int NT>
__global__ void __launch_bounds__(NT)
rez_ties_kernel(const float* __restrict__ x, int64_t d, const float* __restrict__ l1, float fm,
                RezState* __restrict__ st, uint32_t* __restrict__ tie_bits, uint32_t* __restrict__ qbuf,
                uint32_t* __restrict__ pos, const uint32_t* __restrict__ list, uint32_t* __restrict__ ctrl,
                const TieLevelState* __restrict__ tls, int part, uint32_t* __restrict__ tilecnt, int32_t tiles,
                int force_fail) {
    TT_DECL();
    // force_fail != 0 (test hook uq_test_force_replay_failure, never set by the library itself)
    // sends every replay down the failure path below, so its fallback can be checked against
    // the lowest-index rule
    const int64_t dpad = (d + 3) & ~(int64_t)3;              // 16-byte aligned K and I rows
    const Queue A{qbuf + (size_t)blockIdx.x * 2 * dpad, qbuf + (size_t)blockIdx.x * 2 * dpad + dpad};
    uint32_t* Lpos = pos + (size_t)blockIdx.x * 2 * d;
    uint32_t* Rpos = Lpos + d;
    const int tid = threadIdx.x;
    __shared__ TieShared sh;
    __shared__ __attribute__((aligned(16))) uint32_t lK[kTieLdsPairs + 4];
    __shared__ uint32_t lI[kTieLdsPairs];
    __shared__ uint16_t lL[kTieLdsPairs], lR[kTieLdsPairs];
    const uint32_t nlist = list[0];
    for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
        const int64_t vec = list[1 + li];
        const RezState s = st[vec];
        if (s.kleft == 0 || !(s.flags & kRezAmbiguous)) continue;
        const bool up = s.delta > 0;
        const int64_t k = up ? s.delta : -(int64_t)s.delta;
        const DivPlan dp = div_plan(l1[vec]);
        const float* xv = x + vec * d;
        TT_T0();
        // resumed: KB7a filled this slot's queue and ran introselect's first levels
        const bool resumed = tls && li == blockIdx.x && tls[li].filled;
        // part 1: resumed slots (from KB7a's saved state); part 2: everything else
        if ((part == 1 && !resumed) || (part == 2 && resumed)) continue;
        // queue[j] = (value, j) (TopKImpl.h); 4 coordinates per lane and load
        const bool xv4 = ((uintptr_t)xv & 15u) == 0;
        for (int64_t i0 = 0; i0 < (resumed ? 0 : d); i0 += (int64_t)NT * 4 * kTieU) {
            float4 v[kTieU];
#pragma unroll
            for (int u = 0; u < kTieU; ++u) {
                const int64_t i = i0 + 4 * ((int64_t)u * NT + tid);
                if (xv4 && i + 3 < d) {
                    v[u] = *reinterpret_cast<const float4*>(xv + i);
                } else {
                    v[u].x = i < d ? xv[i] : 0.f;
                    v[u].y = i + 1 < d ? xv[i + 1] : 0.f;
                    v[u].z = i + 2 < d ? xv[i + 2] : 0.f;
                    v[u].w = i + 3 < d ? xv[i + 3] : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < kTieU; ++u) {
                const int64_t i = i0 + 4 * ((int64_t)u * NT + tid);
                if (i >= d) continue;
                float kp;
                uint4 kk, ii;
                kk.x = rez_elem(v[u].x, dp, fm, up, kp);
                kk.y = rez_elem(v[u].y, dp, fm, up, kp);
                kk.z = rez_elem(v[u].z, dp, fm, up, kp);
                kk.w = rez_elem(v[u].w, dp, fm, up, kp);
                ii = make_uint4((uint32_t)i, (uint32_t)i + 1, (uint32_t)i + 2, (uint32_t)i + 3);
                if (i + 3 < d) {
                    *reinterpret_cast<uint4*>(A.K + i) = kk;
                    *reinterpret_cast<uint4*>(A.I + i) = ii;
                } else {
                    const uint32_t ka[4] = {kk.x, kk.y, kk.z, kk.w};
                    for (int c = 0; i + c < d; ++c) {
                        A.K[i + c] = ka[c];
                        A.I[i + c] = (uint32_t)(i + c);
                    }
                }
            }
        }
        if (tid == 0) sh.marked = 0;
        __syncthreads();
        TT_ACC(0);
        bool ok = true;
        if (k * 64 <= d) {                                  // std::partial_sort's selection
            if (tid < kWave) tt_heap_select_wave(A, 0, k, d, tid);
            __syncthreads();
        } else {                                            // std::nth_element
            if (resumed && tls[li].err) ok = false;
            else if (resumed) ok = tt_introselect<NT>(A, Lpos, Rpos, d, k - 1, sh, lK, lI, lL, lR, tls[li].first, tls[li].last,
                                                  tls[li].depth);
            else ok = tt_introselect<NT>(A, Lpos, Rpos, d, k - 1, sh, lK, lI, lL, lR, 0, d, 2 * floor_log2_i64(d));
        }
        ok = ok && !force_fail;
        uint32_t* bits = tie_bits + vec * ((d + 31) / 32);
        TT_T0();
        if (ok) {
            uint32_t mine = 0;
            const int64_t pb = resumed ? tls[li].first : 0;   // [0, first) marked by kt_mark_kernel
            if (resumed && tid == 0) atomicAdd(&sh.marked, tls[li].marked);
            for (int64_t p0 = pb; p0 < k; p0 += (int64_t)NT * kTieU) {
                uint32_t kk[kTieU], ii[kTieU];
#pragma unroll
                for (int u = 0; u < kTieU; ++u) {
                    const int64_t p = p0 + (int64_t)u * NT + tid;
                    kk[u] = p < k ? A.K[p] : 0u;
                    ii[u] = p < k ? A.I[p] : 0u;
                }
#pragma unroll
                for (int u = 0; u < kTieU; ++u) {
                    const int64_t p = p0 + (int64_t)u * NT + tid;
                    if (p < k && kk[u] == s.prefix) {
                        atomicOr(&bits[ii[u] >> 5], 1u << (ii[u] & 31));
                        ++mine;
                    }
                }
            }
            if (mine) atomicAdd(&sh.marked, mine);
        }
        __syncthreads();
        TT_ACC(6);
        const bool good = __syncthreads_count(!(ok && sh.marked == s.need)) == 0;
        if (tid == 0) {
            if (good) {
                st[vec].flags = s.flags | kRezTorchTies;
            } else {
                __hip_atomic_store(ctrl + 2, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!good) tt_fallback_tilecounts<NT>(xv, d, dp, fm, up, s.prefix, tilecnt + vec * tiles, tiles);
        __syncthreads();
    }
}
