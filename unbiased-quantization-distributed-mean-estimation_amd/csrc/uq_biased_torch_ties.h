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
// Each workgroup owns one scratch slot (pairs[d] + two position lists) and walks the
// clients blockIdx.x, +gridDim.x, ...; clients without an ambiguous tie are skipped.

constexpr int kTieSlots = 64;        // workgroups (and scratch slots) of KB7
constexpr int kTieItems = 16;        // pairs per thread per partition chunk
constexpr int kTieChunk = 256 * kTieItems;

__device__ __forceinline__ uint32_t pkey(uint64_t p) { return (uint32_t)(p >> 32); }

__device__ void tt_adjust_heap(uint64_t* A, int64_t f, int64_t hole, int64_t len, uint64_t value) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (pkey(A[f + second]) > pkey(A[f + second - 1])) second--;
        A[f + hole] = A[f + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        A[f + hole] = A[f + second - 1];
        hole = second - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && pkey(A[f + parent]) > pkey(value)) {
        A[f + hole] = A[f + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[f + hole] = value;
}

__device__ void tt_make_heap(uint64_t* A, int64_t f, int64_t len) {
    if (len < 2) return;
    for (int64_t parent = (len - 2) / 2;; --parent) {
        tt_adjust_heap(A, f, parent, len, A[f + parent]);
        if (parent == 0) break;
    }
}

// heap_select(A + f, A + m, A + l) by one wave (lanes 0..63 of the caller).
__device__ void tt_heap_select_wave(uint64_t* A, int64_t f, int64_t m, int64_t l, int lane) {
    if (lane == 0) tt_make_heap(A, f, m - f);
    uint32_t top = __shfl(lane == 0 ? pkey(A[f]) : 0u, 0, kWave);
    for (int64_t base = m; base < l; base += kWave) {
        const int64_t i = base + lane;
        const uint32_t ki = i < l ? pkey(A[i]) : 0u;
        const bool cand = i < l;
        uint64_t mask = __ballot(cand && ki > top);
        while (mask) {
            const int j = __builtin_ctzll(mask);
            uint32_t nt = 0;
            if (lane == 0) {                       // pop_heap(f, m, base + j)
                const uint64_t v = A[base + j];
                A[base + j] = A[f];
                tt_adjust_heap(A, f, 0, m - f, v);
                nt = pkey(A[f]);
            }
            top = __shfl(nt, 0, kWave);
            const uint64_t later = (j == 63) ? 0ull : (~0ull << (j + 1));
            mask = __ballot(cand && ki > top) & later;
        }
    }
}

__device__ __forceinline__ void tt_swap(uint64_t* A, int64_t a, int64_t b) {
    const uint64_t t = A[a];
    A[a] = A[b];
    A[b] = t;
}

__device__ void tt_move_median_to_first(uint64_t* A, int64_t r, int64_t a, int64_t b, int64_t c) {
    const uint32_t ka = pkey(A[a]), kb = pkey(A[b]), kc = pkey(A[c]);
    if (ka > kb) {
        if (kb > kc) tt_swap(A, r, b);
        else if (ka > kc) tt_swap(A, r, c);
        else tt_swap(A, r, a);
    } else if (ka > kc) tt_swap(A, r, a);
    else if (kb > kc) tt_swap(A, r, c);
    else tt_swap(A, r, b);
}

__device__ void tt_insertion_sort(uint64_t* A, int64_t f, int64_t l) {
    if (f == l) return;
    for (int64_t i = f + 1; i != l; ++i) {
        const uint64_t v = A[i];
        if (pkey(v) > pkey(A[f])) {
            for (int64_t j = i; j > f; --j) A[j] = A[j - 1];
            A[f] = v;
        } else {
            int64_t j = i;
            while (pkey(v) > pkey(A[j - 1])) {
                A[j] = A[j - 1];
                --j;
            }
            A[j] = v;
        }
    }
}

__device__ __forceinline__ int floor_log2_i64(int64_t n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

// std::nth_element(A, A + nth, A + d) by the whole workgroup.  Returns false on an
// internal inconsistency (never expected; reported through the status word).
__device__ bool tt_introselect(uint64_t* A, uint32_t* Lpos, uint32_t* Rpos, int64_t d, int64_t nth) {
    __shared__ int64_t s_first, s_last, s_cut, s_J;
    __shared__ int s_depth, s_bad;
    __shared__ uint32_t s_piv;
    __shared__ uint32_t lds[4];
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_first = 0;
        s_last = d;
        s_depth = 2 * floor_log2_i64(d);
        s_bad = 0;
    }
    __syncthreads();
    for (;;) {
        const int64_t first = s_first, last = s_last;
        const int depth = s_depth;
        if (last - first <= 3) break;
        if (depth == 0) {                                   // introselect's heap fallback
            if (tid < kWave) tt_heap_select_wave(A, first, nth + 1, last, tid);
            __syncthreads();
            if (tid == 0) tt_swap(A, first, nth);
            __syncthreads();
            return true;
        }
        if (tid == 0) {
            const int64_t mid = first + (last - first) / 2;
            tt_move_median_to_first(A, first, first + 1, mid, last - 1);
            s_piv = pkey(A[first]);
        }
        __syncthreads();
        const uint32_t piv = s_piv;
        // stops of both scans in index order, positions listed in Lpos / Rpos
        uint32_t nL = 0, nR = 0;
        for (int64_t c0 = first; c0 < last; c0 += kTieChunk) {
            const int64_t i0 = c0 + (int64_t)tid * kTieItems;
            uint32_t flags = 0, cl = 0, cr = 0;
#pragma unroll
            for (int j = 0; j < kTieItems; ++j) {
                const int64_t i = i0 + j;
                if (i < last) {
                    const uint32_t k = pkey(A[i]);
                    const bool lf = i > first && k <= piv;      // !comp(A[i], pivot)
                    const bool rf = k >= piv;                   // !comp(pivot, A[i])
                    flags |= (lf ? 1u : 0u) << j;
                    flags |= (rf ? 1u : 0u) << (16 + j);
                    cl += lf;
                    cr += rf;
                }
            }
            uint32_t tot;
            const uint32_t ex = block_excl_scan_u32(cl | (cr << 16), lds, &tot);
            uint32_t pl = nL + (ex & 0xFFFFu), pr = nR + (ex >> 16);
#pragma unroll
            for (int j = 0; j < kTieItems; ++j) {
                if (flags & (1u << j)) Lpos[pl++] = (uint32_t)(i0 + j);
                if (flags & (1u << (16 + j))) Rpos[pr++] = (uint32_t)(i0 + j);
            }
            nL += tot & 0xFFFFu;
            nR += tot >> 16;
        }
        __syncthreads();
        if (tid == 0) {
            // J = number of swaps: largest J with L_J < R_J (1-based; R counted from the right)
            int64_t lo = 0, hi = nL < nR ? nL : nR;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) / 2;
                if (Lpos[mid - 1] < Rpos[nR - mid]) lo = mid; else hi = mid - 1;
            }
            int64_t cut = INT64_MAX;
            if (lo < (int64_t)nL) cut = Lpos[lo];
            if (lo > 0) cut = std::min<int64_t>(cut, Rpos[nR - lo]);
            if (cut <= first || cut >= last) s_bad = 1;
            s_J = lo;
            s_cut = cut;
        }
        __syncthreads();
        if (s_bad) return false;
        const int64_t J = s_J;
        for (int64_t j = tid; j < J; j += 256) tt_swap(A, Lpos[j], Rpos[nR - 1 - j]);
        __syncthreads();
        if (tid == 0) {
            if (s_cut <= nth) s_first = s_cut; else s_last = s_cut;
            s_depth = depth - 1;
        }
        __syncthreads();
    }
    if (tid == 0) tt_insertion_sort(A, s_first, s_last);
    __syncthreads();
    return true;
}

__global__ void __launch_bounds__(256)
rez_ties_kernel(const float* __restrict__ x, int64_t d, const float* __restrict__ l1, float fm,
                RezState* __restrict__ st, uint32_t* __restrict__ tie_bits, uint64_t* __restrict__ pairs,
                uint32_t* __restrict__ pos, int64_t n, uint32_t* __restrict__ ctrl) {
    uint64_t* A = pairs + (size_t)blockIdx.x * d;
    uint32_t* Lpos = pos + (size_t)blockIdx.x * 2 * d;
    uint32_t* Rpos = Lpos + d;
    const int tid = threadIdx.x;
    __shared__ uint32_t s_marked;
    for (int64_t vec = blockIdx.x; vec < n; vec += gridDim.x) {
        const RezState s = st[vec];
        if (s.kleft == 0 || !(s.flags & kRezAmbiguous)) continue;
        const bool up = s.delta > 0;
        const int64_t k = up ? s.delta : -(int64_t)s.delta;
        const float den = l1[vec] + 1e-12f;
        const float* xv = x + vec * d;
        for (int64_t i = tid; i < d; i += 256) {           // queue[j] = (value, j) (TopKImpl.h)
            float kp;
            A[i] = ((uint64_t)rez_elem(xv[i], den, fm, up, kp) << 32) | (uint64_t)i;
        }
        if (tid == 0) s_marked = 0;
        __syncthreads();
        bool ok = true;
        if (k * 64 <= d) {                                  // std::partial_sort's selection
            if (tid < kWave) tt_heap_select_wave(A, 0, k, d, tid);
            __syncthreads();
        } else {                                            // std::nth_element
            ok = tt_introselect(A, Lpos, Rpos, d, k - 1);
        }
        uint32_t* bits = tie_bits + vec * ((d + 31) / 32);
        if (ok) {
            uint32_t mine = 0;
            for (int64_t p = tid; p < k; p += 256) {
                const uint64_t e = A[p];
                if (pkey(e) == s.prefix) {
                    const uint32_t idx = (uint32_t)e;
                    atomicOr(&bits[idx >> 5], 1u << (idx & 31));
                    ++mine;
                }
            }
            atomicAdd(&s_marked, mine);
        }
        __syncthreads();
        if (tid == 0) {
            if (ok && s_marked == s.need) {
                st[vec].flags = s.flags | kRezTorchTies;
            } else {
                __hip_atomic_store(ctrl + 2, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
}
