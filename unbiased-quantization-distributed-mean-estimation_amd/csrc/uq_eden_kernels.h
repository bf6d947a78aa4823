// uq_eden_kernels.h — EDEN with the randomized Hadamard transform.
// Included by uq_dme.hip inside its anonymous namespace.
//
// Reference (AS = NMSE_Results/Codes/All_Schemes.py):
//   AS:100-115  Hadamard.hadamard: stages h = 2..D, a' = a + b, b' = a' - 2b (f32), then
//               v / f32(sqrt(D))
//   AS:117-120  random_diagonal: torch CPU generator (MT19937) seeded per call,
//               2 * bernoulli(1/2) - 1: one 32-bit word per coordinate, -1 iff its low
//               24 bits are >= 2^23
//   AS:123-153  RHT sender (zero-pad to D = 2^p, * diag, H) / receiver (H, * diag)
//   AS:324-376  EdenSender: bins = bucketize(v * f32(sqrt(D)) / ||v||, boundaries),
//               scale = ||v||^2 / dot(centroids[bins], v)
//   AS:378-413  EdenReceiver: scale * RHT^-1(centroids[bins])[:dim]
// Kernels:
//   KE0 rht_signs_kernel   MT19937 per seed -> int8 diagonal rows (cached by the caller)
//   KE1 fwht_pass_kernel   up to 12 (first pass) / 8 (later passes) butterfly stages in
//                          LDS; the first pass fuses pad * diag (sender) or the centroid
//                          lookup (receiver), the last pass / sqrt(D) (and * diag * scale,
//                          truncation to dim on the receiver)
//   KE2 eden_norm_kernel   torch.norm(v, 2) in torch CPU order: 8 lanes of fma, lanes in order
//   KE3 eden_bins_kernel   bucketize -> u8 bins, fp64 partial dot per tile
//   KE4 eden_scale_kernel  dot partials in tile order, scale = f32(nrm*nrm) / f32(dot)

constexpr int kFwhtT = 256;            // threads per FWHT workgroup
constexpr int kFwhtLowBits = 12;       // first pass: contiguous tiles of 4096
constexpr int kFwhtHighBits = 8;       // later passes: 2^8 rows x 32 columns
constexpr int kFwhtCols = 32;
constexpr int kEdenTile = 4096;        // KE3 tile (256 threads x 16)

// AS:302-306 centroids and AS:311-315 boundaries (the update on AS:315 overwrites the
// 1-bit entry with the midpoint list [0.0]).
struct EdenTables {
    float c[4];      // centroids, 2^nbits entries
    float b[3];      // boundaries, 2^nbits - 1 entries
    int nb;          // number of boundaries
};

// ---- KE0: MT19937 -> diagonal ---------------------------------------------------------
// One workgroup per seed; the in-place twist runs in its three dependency phases
// ([0,227) from old words, [227,454) and [454,624) reading words updated earlier).
__global__ void __launch_bounds__(640)
rht_signs_kernel(const int32_t* __restrict__ seeds, int64_t D, int8_t* __restrict__ signs) {
    __shared__ uint32_t mt[624];
    const int tid = threadIdx.x;
    int8_t* row = signs + (int64_t)blockIdx.x * D;
    if (tid == 0) {
        mt[0] = (uint32_t)seeds[blockIdx.x];
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    }
    __syncthreads();
    auto twist_word = [&](int i) -> uint32_t {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7FFFFFFFu);
        return mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
    };
    for (int64_t base = 0; base < D; base += 624) {
        uint32_t nv = 0;
        if (tid < 227) nv = twist_word(tid);
        __syncthreads();
        if (tid < 227) mt[tid] = nv;
        __syncthreads();
        if (tid >= 227 && tid < 454) nv = twist_word(tid);
        __syncthreads();
        if (tid >= 227 && tid < 454) mt[tid] = nv;
        __syncthreads();
        if (tid >= 454 && tid < 624) nv = twist_word(tid);
        __syncthreads();
        if (tid >= 454 && tid < 624) mt[tid] = nv;
        __syncthreads();
        if (tid < 624 && base + tid < D) {
            uint32_t y = mt[tid];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9D2C5680u;
            y ^= (y << 15) & 0xEFC60000u;
            y ^= y >> 18;
            row[base + tid] = ((y & 0xFFFFFFu) < 0x800000u) ? (int8_t)1 : (int8_t)-1;   // u < 1/2 -> +1
        }
    }
}

// ---- KE1: one FWHT pass ----------------------------------------------------------------
// Stages for index bits [lo, lo + k).  lo == 0: tiles of 2^k contiguous elements.
// lo > 0: tiles of 2^k rows x 32 columns (row r, column c -> hi + (r << lo) + c0 + c).
// MODE 0: plain (in -> out, f32).  MODE 1 (first sender pass): in = x rows of length
// `dim`, zero-padded, times the diagonal.  MODE 2 (first receiver pass): in = u8 bins,
// value = centroid.  LAST: divide by sqrt(D) as f32 (AS:114); RECV_LAST additionally
// multiplies by the diagonal and the per-client scale and writes only [0, dim).
struct FwhtArgs {
    const void* in;
    float* out;
    const int8_t* signs;        // [rows][D] diagonal rows
    const int32_t* sign_row;    // [n] row of each client
    const float* scale;         // [n] (receiver last pass)
    int64_t D, dim;
    float sqrtD;
    EdenTables tab;
};

template <int MODE, bool LAST, bool RECV_LAST>
__global__ void __launch_bounds__(kFwhtT)
fwht_pass_kernel(FwhtArgs a, int lo, int k) {
    __shared__ float s[1 << (kFwhtHighBits + 5)];        // 4096 (first pass) or 256 x 32
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t D = a.D;
    const int cols = lo == 0 ? 1 : kFwhtCols;
    const int rows = 1 << k;
    const int tile_elems = rows * cols;
    const int64_t lowspan = (int64_t)1 << lo;                 // columns available below lo
    const int64_t col_groups = lo == 0 ? 1 : lowspan / kFwhtCols;
    const int64_t t = blockIdx.x;
    const int64_t hi = (t / col_groups) << (lo + k);
    const int64_t c0 = (t % col_groups) * kFwhtCols;
    const int8_t* sg = a.signs + (int64_t)(a.sign_row ? a.sign_row[vec] : 0) * D;
    auto gidx = [&](int e) -> int64_t {                       // tile element -> vector index
        const int r = lo == 0 ? e : e / kFwhtCols;
        const int c = lo == 0 ? 0 : e % kFwhtCols;
        return hi + ((int64_t)r << lo) + c0 + c;
    };
    // load (lanes walk columns fastest: 128-byte rows)
    for (int e = tid; e < tile_elems; e += kFwhtT) {
        const int64_t i = gidx(e);
        float v;
        if (MODE == 1) {
            const float* x = (const float*)a.in + vec * a.dim;
            v = i < a.dim ? x[i] : 0.f;
            v = v * (float)sg[i];                               // AS:132/137 * diag
        } else if (MODE == 2) {
            const uint8_t* bins = (const uint8_t*)a.in + vec * D;
            v = a.tab.c[bins[i]];                               // AS:383 take(centroids, bins)
        } else {
            v = ((const float*)a.in)[vec * D + i];
        }
        s[e] = v;
    }
    __syncthreads();
    // butterflies over the row bits: rows (r, r + 2^j), bit j of r clear (AS:107-112)
    const int pairs = (rows >> 1) * cols;
    for (int j = 0; j < k; ++j) {
        for (int q = tid; q < pairs; q += kFwhtT) {
            const int c = q % cols;
            const int pr = q / cols;
            const int r = ((pr >> j) << (j + 1)) | (pr & ((1 << j) - 1));
            const int ea = r * cols + c, eb = (r + (1 << j)) * cols + c;
            const float av = s[ea], bv = s[eb];
            const float na = av + bv;
            s[ea] = na;
            s[eb] = na - 2.f * bv;
        }
        __syncthreads();
    }
    for (int e = tid; e < tile_elems; e += kFwhtT) {
        const int64_t i = gidx(e);
        float v = s[e];
        if (LAST) v = v / a.sqrtD;                              // AS:114 vec /= sqrt(d)
        if (RECV_LAST) {
            if (i < a.dim) {
                v = v * (float)sg[i];                           // AS:152 * diag
                a.out[vec * a.dim + i] = a.scale[vec] * v;      // AS:413 scale * vec, [:dim]
            }
        } else {
            a.out[vec * D + i] = v;
        }
    }
}

// ---- KE2: torch.norm(v, 2) -------------------------------------------------------------
// 8 clients per 64-thread block, lane l of a client accumulates v[8i + l] with fma in
// order; the 8 lane sums are added 0..7, then sqrt (f32).  D is a power of two >= 8 or
// smaller (then the scalar tail path applies to all of it).
__global__ void __launch_bounds__(64)
eden_norm_kernel(const float* __restrict__ v, int64_t n, int64_t D, float* __restrict__ nrm) {
    const int l = threadIdx.x & 7;
    const int64_t vec = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 3);
    const bool live = vec < n;
    const float* p = v + (live ? vec : 0) * D;
    const int64_t nv = D - D % 8;
    float acc = 0.f;
    if (live) {
        int64_t i = l;
        for (; i + 8 * 15 < nv; i += 8 * 16) {
            float t[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) t[u] = p[i + 8 * u];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = fmaf(t[u], t[u], acc);
        }
        for (; i < nv; i += 8) acc = fmaf(p[i], p[i], acc);
    }
    // lanes 0..7 in order, then the scalar tail
    float tot = __shfl(acc, (threadIdx.x & ~7), kWave);
    for (int j = 1; j < 8; ++j) tot = tot + __shfl(acc, (threadIdx.x & ~7) + j, kWave);
    if (live && l == 0) {
        for (int64_t i = nv; i < D; ++i) tot = tot + p[i] * p[i];
        nrm[vec] = sqrtf(tot);
    }
}

// ---- KE3: bins and partial dots ---------------------------------------------------------
__global__ void __launch_bounds__(256)
eden_bins_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm,
                 EdenTables tab, uint8_t* __restrict__ bins, double* __restrict__ part, int32_t tiles) {
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const float nv = nrm[vec];
    const float* p = v + vec * D;
    uint8_t* bp = bins + vec * D;
    double dot = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kEdenTile + tid; i < std::min<int64_t>(D, (int64_t)(blockIdx.x + 1) * kEdenTile);
         i += 256) {
        const float x = p[i];
        const float z = (x * sqrtD) / nv;                   // AS:329 vec * sqrt(D) / norm
        int b = 0;
        for (int j = 0; j < tab.nb; ++j) b += (tab.b[j] < z) ? 1 : 0;    // bucketize, right=False
        bp[i] = (uint8_t)b;
        dot += (double)tab.c[b] * (double)x;                // AS:335 dot(centroids[bins], vec)
    }
    __shared__ double red[256];
    red[tid] = dot;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    if (tid == 0) part[vec * tiles + blockIdx.x] = red[0];
}

// ---- KE4: scale per client ---------------------------------------------------------------
__global__ void __launch_bounds__(256)
eden_scale_kernel(const double* __restrict__ part, int32_t tiles, const float* __restrict__ nrm, int64_t n,
                  float* __restrict__ scale) {
    const int64_t vec = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (vec >= n) return;
    double dot = 0.0;
    for (int t = 0; t < tiles; ++t) dot += part[vec * tiles + t];
    const float nv = nrm[vec];
    scale[vec] = (nv * nv) / (float)dot;                    // AS:335 norm ** 2 / dot
}
