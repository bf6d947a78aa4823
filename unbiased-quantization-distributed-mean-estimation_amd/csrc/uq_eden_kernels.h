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
//   KE4 eden_dotbins_kernel bucketize -> u8 bins and AS:335 torch.dot(centroids[bins], v) in
//                          MKL sdot's order (one wave per client, a lane per accumulator
//                          lane), scale = f32(nrm*nrm) / dot; the receiver's first pass reads
//                          the bins (MODE 2)

// Orders one wave's LDS accesses across lanes: the compiler sees single-lane addresses only
// (s[i] and s[i + 1] never alias for ONE lane) and could otherwise move a read past another
// lane's write; the wave's LDS operations themselves execute in program order.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
}

constexpr int kFwhtT = 256;            // threads per FWHT workgroup
constexpr int kFwhtLowBits = 12;       // first pass: contiguous tiles of 4096
constexpr int kFwhtLow16Bits = 14;     // ... of 16384 when D = 2^22 (14 + 8)
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

// torch.bucketize(z, boundaries) (right=False: boundaries strictly below z; NaN -> nb) and
// take(centroids, bin) with the table in registers: a dynamically indexed kernel-argument array
// is read from memory per element, and the compiler turns a select chain over its entries back
// into such a load unless the values are opaque (the empty asm)
struct EdenCents {
    float c0, c1, c2, c3;
};
__device__ __forceinline__ EdenCents eden_cents(const EdenTables& t) {
    EdenCents r{t.c[0], t.c[1], t.c[2], t.c[3]};
    __asm__ volatile("" : "+v"(r.c0), "+v"(r.c1), "+v"(r.c2), "+v"(r.c3));
    return r;
}
__device__ __forceinline__ int eden_bin(const EdenTables& t, float z) {
    int b = !(t.b[0] >= z) ? 1 : 0;
    if (t.nb > 1) b += (!(t.b[1] >= z) ? 1 : 0) + (!(t.b[2] >= z) ? 1 : 0);
    return b;
}
__device__ __forceinline__ float eden_cent(const EdenCents& t, int b) {
    // bit masks instead of selects (a select chain is rewritten into an indexed table load)
    const uint32_t m0 = 0u - (uint32_t)(b == 0), m1 = 0u - (uint32_t)(b == 1), m2 = 0u - (uint32_t)(b == 2),
                   m3 = 0u - (uint32_t)(b == 3);
    return __uint_as_float((__float_as_uint(t.c0) & m0) | (__float_as_uint(t.c1) & m1) |
                           (__float_as_uint(t.c2) & m2) | (__float_as_uint(t.c3) & m3));
}

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

// KE0b: the diagonal rows as bits (bit i % 32 of word i / 32 set where the sign is -1), so the
// passes that apply the diagonal read 1/8 byte per coordinate instead of 1
__global__ void __launch_bounds__(256)
rht_sign_bits_kernel(const int8_t* __restrict__ signs, int64_t rows, int64_t D, uint32_t* __restrict__ bits) {
    const int64_t W = (D + 31) / 32;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= rows * W) return;
    const int64_t r = q / W, w = q % W;
    const int8_t* s = signs + r * D + 32 * w;
    const int n = (int)min((int64_t)32, D - 32 * w);
    uint32_t b = 0;
    for (int k = 0; k < n; ++k) b |= (s[k] < 0 ? 1u : 0u) << k;
    bits[q] = b;
}

// +-1.0f from bit 0 (set: -1) as an opaque operand, so that the multiply stays a v_mul_f32 as
// with the int8 rows (the compiler would otherwise fold x * (b ? -1 : 1) into a sign flip,
// which differs from the multiply on NaN inputs)
__device__ __forceinline__ float sign_pm1(uint32_t b) {
    float m = (b & 1u) ? -1.0f : 1.0f;
    asm volatile("" : "+v"(m));
    return m;
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
    const uint32_t* sbits;      // [rows][ceil(D / 32)] the same rows as bits (KE0b), or null
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
            v = eden_cent(eden_cents(a.tab), bins[i]);          // AS:383 take(centroids, bins)
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
                a.out[vec * a.dim + i] = a.scale ? a.scale[vec] * v : v;   // AS:413 scale * vec, [:dim]
            }
        } else {
            a.out[vec * D + i] = v;
        }
    }
}

// ---- KE1': register-radix passes for the two common shapes -----------------------------
// Same stages in the same order as fwht_pass_kernel (so the same bits), with 16 (low pass)
// or 32 (high pass) elements per thread in registers and padded LDS transposes between
// rounds of register-local stages.
__device__ __forceinline__ void bfly(float& a, float& b) {   // AS:109-110
    const float na = a + b;
    b = na - 2.f * b;
    a = na;
}

// stages over the 4 bits of a 16-element register array (index bit j of i)
__device__ __forceinline__ void stages16(float* v) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!(i & (1 << j))) bfly(v[i], v[i | (1 << j)]);
}

__device__ __forceinline__ int pad17(int e) { return e + (e >> 4); }

// Low pass over 4096 contiguous elements, index e = b0 + 16 b1 + 256 b2: round 1 thread
// (b1, b2) holds b0 = 0..15 (bits 0-3), round 2 thread (b0, b2) holds b1 (bits 4-7),
// round 3 thread (b0, b1) holds b2 (bits 8-11).
template <int MODE, bool LAST, bool RECV_LAST>
__global__ void __launch_bounds__(256)
fwht_low4096_kernel(FwhtArgs a) {
    __shared__ float s[4096 + 256];
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t D = a.D;
    const EdenCents cs = eden_cents(a.tab);
    const int64_t base = (int64_t)blockIdx.x * 4096;
    const int8_t* sg = a.signs + (int64_t)(a.sign_row ? a.sign_row[vec] : 0) * D;
    float v[16];
    {   // round-1 layout: 16 contiguous elements
        const int64_t i0 = base + (int64_t)tid * 16;
        if (MODE == 1) {
            const float* x = (const float*)a.in + vec * a.dim;
            const bool full = i0 + 16 <= a.dim && (((uintptr_t)(x + i0)) & 15) == 0;
            if (full) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = *reinterpret_cast<const float4*>(x + i0 + 4 * q);
                    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i0 + i < a.dim) ? x[i0 + i] : 0.f;
            }
            if (a.sbits) {                                                     // 16 signs as bits
                const int64_t W = (D + 31) / 32;
                const uint32_t bw = a.sbits[(int64_t)(a.sign_row ? a.sign_row[vec] : 0) * W + (i0 >> 5)] >> (i0 & 31);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = v[i] * sign_pm1(bw >> i);      // AS:132/137 * diag
            } else {
                const int4 sgv = *reinterpret_cast<const int4*>(sg + i0);       // 16 signs
                const int8_t* sb = reinterpret_cast<const int8_t*>(&sgv);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = v[i] * (float)sb[i];            // AS:132/137 * diag
            }
        } else if (MODE == 2) {
            const int4 bv = *reinterpret_cast<const int4*>((const uint8_t*)a.in + vec * D + i0);
            const uint8_t* bb = reinterpret_cast<const uint8_t*>(&bv);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = eden_cent(cs, bb[i]);            // AS:383
        } else {
            const float* p = (const float*)a.in + vec * D + i0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);
                v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
            }
        }
    }
    stages16(v);                                                   // bits 0-3
    const int b1r1 = tid & 15, b2r1 = tid >> 4;
#pragma unroll
    for (int i = 0; i < 16; ++i) s[pad17(i + 16 * b1r1 + 256 * b2r1)] = v[i];
    __syncthreads();
    const int b0 = tid & 15, b2 = tid >> 4;                        // round 2: (b0, b2)
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = s[pad17(b0 + 16 * i + 256 * b2)];
    stages16(v);                                                   // bits 4-7
#pragma unroll
    for (int i = 0; i < 16; ++i) s[pad17(b0 + 16 * i + 256 * b2)] = v[i];
    __syncthreads();
    const int b1 = tid >> 4;                                       // round 3: (b0, b1)
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = s[pad17(b0 + 16 * b1 + 256 * i)];
    stages16(v);                                                   // bits 8-11
    if (!RECV_LAST) {
        // back through LDS so that each lane stores 16 contiguous bytes (float4 stores
        // of 1 KB per wave instead of 16 dword stores of 256 B)
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) s[pad17(b0 + 16 * b1 + 256 * i)] = LAST ? v[i] / a.sqrtD : v[i];   // AS:114
        __syncthreads();
        float* o = a.out + vec * D + base;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * (tid + 256 * j);
            const int pe = pad17(e);
            const f32x4 t = {s[pe], s[pe + 1], s[pe + 2], s[pe + 3]};
            __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(o + e));
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t gi = base + b0 + 16 * b1 + 256 * i;          // lanes: consecutive b0 + 16 b1
        float r = v[i];
        if (LAST) r = r / a.sqrtD;                                 // AS:114
        if (RECV_LAST) {
            if (gi < a.dim) {
                r = r * (float)sg[gi];                             // AS:152
                a.out[vec * a.dim + gi] = a.scale ? a.scale[vec] * r : r;
            }
        } else {
            a.out[vec * D + gi] = r;
        }
    }
}

// First pass over 16384 contiguous elements (bits 0-13), for D = 2^22: 14 + 8 bits instead of
// 12 + 8 + 2, one pass fewer each way.  1024 threads; index e = b0 + 16 b1 + 256 b2 + 4096 b3
// (b3: 2 bits).  Rounds as fwht_low4096_kernel (b0, b1, b2 in registers in turn, padded LDS
// transposes), then bits 12-13: a thread takes four columns p = b0 + 16 b1 + 256 b2 and their
// four b3 values.  The same stages in the same order, so the same bits as 12 + 8 + 2.
// MODE 0: plain (QUIC-FL's receiver, in place), 1: sender (pad, * diag), 2: receiver (centroids
// of the bins); never the last pass.
template <int MODE>
__global__ void __launch_bounds__(1024)
fwht_low16k_kernel(FwhtArgs a) {
    __shared__ float s[16384 + 1024];
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t D = a.D;
    const EdenCents cs = eden_cents(a.tab);
    const int64_t base = (int64_t)blockIdx.x * 16384;
    float v[16];
    {   // round-1 layout: 16 contiguous elements
        const int64_t i0 = base + (int64_t)tid * 16;
        if (MODE == 0) {
            const float* p = (const float*)a.in + vec * D + i0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);
                v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
            }
        } else if (MODE == 1) {
            const int8_t* sg = a.signs + (int64_t)(a.sign_row ? a.sign_row[vec] : 0) * D;
            const float* x = (const float*)a.in + vec * a.dim;
            const bool full = i0 + 16 <= a.dim && (((uintptr_t)(x + i0)) & 15) == 0;
            if (full) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = *reinterpret_cast<const float4*>(x + i0 + 4 * q);
                    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i0 + i < a.dim) ? x[i0 + i] : 0.f;
            }
            if (a.sbits) {                                                     // 16 signs as bits
                const int64_t W = (D + 31) / 32;
                const uint32_t bw = a.sbits[(int64_t)(a.sign_row ? a.sign_row[vec] : 0) * W + (i0 >> 5)] >> (i0 & 31);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = v[i] * sign_pm1(bw >> i);      // AS:132/137 * diag
            } else {
                const int4 sgv = *reinterpret_cast<const int4*>(sg + i0);       // 16 signs
                const int8_t* sb = reinterpret_cast<const int8_t*>(&sgv);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = v[i] * (float)sb[i];            // AS:132/137 * diag
            }
        } else {
            const int4 bv = *reinterpret_cast<const int4*>((const uint8_t*)a.in + vec * D + i0);
            const uint8_t* bb = reinterpret_cast<const uint8_t*>(&bv);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = eden_cent(cs, bb[i]);            // AS:383
        }
    }
    const int b3 = tid >> 8, o3 = 4096 * b3;
    stages16(v);                                                   // bits 0-3
    {
        const int b1 = tid & 15, b2 = (tid >> 4) & 15;
#pragma unroll
        for (int i = 0; i < 16; ++i) s[pad17(i + 16 * b1 + 256 * b2 + o3)] = v[i];
    }
    __syncthreads();
    const int b0 = tid & 15;
    {
        const int b2 = (tid >> 4) & 15;                            // round 2: (b0, b2, b3)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = s[pad17(b0 + 16 * i + 256 * b2 + o3)];
        stages16(v);                                               // bits 4-7
#pragma unroll
        for (int i = 0; i < 16; ++i) s[pad17(b0 + 16 * i + 256 * b2 + o3)] = v[i];
    }
    __syncthreads();
    {
        const int b1 = (tid >> 4) & 15;                            // round 3: (b0, b1, b3)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = s[pad17(b0 + 16 * b1 + 256 * i + o3)];
        stages16(v);                                               // bits 8-11
#pragma unroll
        for (int i = 0; i < 16; ++i) s[pad17(b0 + 16 * b1 + 256 * i + o3)] = v[i];
    }
    __syncthreads();
    float* o = a.out + vec * D + base;
#pragma unroll
    for (int j = 0; j < 4; ++j) {                                  // round 4: bits 12-13
        const int p = tid + 1024 * j;
        float w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = s[pad17(p + 4096 * k)];
        bfly(w[0], w[1]);                                          // bit 12
        bfly(w[2], w[3]);
        bfly(w[0], w[2]);                                          // bit 13
        bfly(w[1], w[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(w[k], o + p + 4096 * k);
    }
}

// High pass: 256 rows (index bits lo..lo+7) x 64 columns, 512 threads (a wave reads one
// row's 64 contiguous floats, 256 B).  Round 1: thread (c, g), c = tid % 64, g = tid / 64,
// holds rows 32 g + m (m = 0..31; row bits 0-4).  Round 2: thread (c, h) holds rows
// a + 32 u for a in 4h..4h+3, u = 0..7 (row bits 5-7).
constexpr int kHighCols = 64;
constexpr int kHighT = 512;
template <bool LAST, bool RECV_LAST>
__global__ void __launch_bounds__(kHighT)
fwht_high256_kernel(FwhtArgs a, int lo) {
    __shared__ float s[256 * (kHighCols + 1)];
    const int64_t vec = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t D = a.D;
    const int64_t lowspan = (int64_t)1 << lo;
    const int64_t col_groups = lowspan / kHighCols;
    const int64_t t = blockIdx.x;
    const int64_t hi = (t / col_groups) << (lo + 8);
    const int64_t c0 = (t % col_groups) * kHighCols;
    const int8_t* sg = a.signs + (int64_t)(a.sign_row ? a.sign_row[vec] : 0) * D;
    const int c = tid & (kHighCols - 1), g = tid / kHighCols;
    const float* in = (const float*)a.in + vec * D;
    const float sc = (RECV_LAST && a.scale) ? a.scale[vec] : 1.0f;
    // the tile's diagonal as sign bits (2 KB of LDS keeps two workgroups per CU): thread
    // tid packs the 32 sign bytes of half a row
    __shared__ uint32_t sgb[RECV_LAST ? 2 * 256 : 1];
    if (RECV_LAST && a.sbits) {                          // the bits as they are (64 columns: 2 words)
        const int row = tid >> 1, half = tid & 1;
        const int64_t W = (D + 31) / 32;
        sgb[tid] = a.sbits[(int64_t)(a.sign_row ? a.sign_row[vec] : 0) * W +
                           ((hi + ((int64_t)row << lo) + c0 + 32 * half) >> 5)];
    } else if (RECV_LAST) {
        const int row = tid >> 1, half = tid & 1;
        const int4* sr = reinterpret_cast<const int4*>(sg + hi + ((int64_t)row << lo) + c0 + 32 * half);
        const int4 w0 = sr[0], w1 = sr[1];
        const uint32_t wv[8] = {(uint32_t)w0.x, (uint32_t)w0.y, (uint32_t)w0.z, (uint32_t)w0.w,
                                (uint32_t)w1.x, (uint32_t)w1.y, (uint32_t)w1.z, (uint32_t)w1.w};
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w = wv[k];
            bits |= (((w >> 7) & 1u) | ((w >> 14) & 2u) | ((w >> 21) & 4u) | ((w >> 28) & 8u)) << (4 * k);
        }
        sgb[tid] = bits;
    }
    float v[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) v[m] = __builtin_nontemporal_load(in + hi + ((int64_t)(32 * g + m) << lo) + c0 + c);
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int m = 0; m < 32; ++m)
            if (!(m & (1 << j))) bfly(v[m], v[m | (1 << j)]);
#pragma unroll
    for (int m = 0; m < 32; ++m) s[(32 * g + m) * (kHighCols + 1) + c] = v[m];
    __syncthreads();
    const int h = g;
#pragma unroll
    for (int aa = 0; aa < 4; ++aa)
#pragma unroll
        for (int u = 0; u < 8; ++u) v[aa * 8 + u] = s[(4 * h + aa + 32 * u) * (kHighCols + 1) + c];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int aa = 0; aa < 4; ++aa)
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (!(u & (1 << j))) bfly(v[aa * 8 + u], v[aa * 8 + (u | (1 << j))]);
#pragma unroll
    for (int aa = 0; aa < 4; ++aa)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int row = 4 * h + aa + 32 * u;
            const int64_t gi = hi + ((int64_t)row << lo) + c0 + c;
            float r = v[aa * 8 + u];
            if (LAST) r = r / a.sqrtD;                             // AS:114
            if (RECV_LAST) {
                if (gi < a.dim) {
                    r = r * (((sgb[2 * row + (c >> 5)] >> (c & 31)) & 1u) ? -1.0f : 1.0f);   // AS:152 (diag = +-1)
                    __builtin_nontemporal_store(a.scale ? sc * r : r, a.out + vec * a.dim + gi);
                }
            } else {
                __builtin_nontemporal_store(r, a.out + vec * D + gi);
            }
        }
}

// ---- KE1'': a pass of at most 6 bits after the first (D = 2^13..2^18: 12 + 1..6; 2^21, 2^22: 12 + 8 + 1..2)
// fwht_pass_kernel would stage 2^K x 32 elements per 256-thread workgroup; here a thread owns
// one column j below 2^lo and keeps its 2^K rows (stride 2^lo) in registers: coalesced rows,
// the same stages in the same order (so the same bits), the same epilogue.
template <int K, bool LAST, bool RECV_LAST>
__global__ void __launch_bounds__(256)
fwht_small_kernel(FwhtArgs a, int lo) {
    const int64_t vec = blockIdx.y;
    const int64_t D = a.D;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= (D >> K)) return;
    const int64_t base = ((q >> lo) << (lo + K)) + (q & (((int64_t)1 << lo) - 1));
    const float* in = (const float*)a.in + vec * D;
    float v[1 << K];
#pragma unroll
    for (int r = 0; r < (1 << K); ++r) v[r] = in[base + ((int64_t)r << lo)];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int r = 0; r < (1 << K); ++r)
            if (!(r & (1 << j))) bfly(v[r], v[r | (1 << j)]);         // AS:107-112
    const int8_t* sg = a.signs + (int64_t)(a.sign_row ? a.sign_row[vec] : 0) * D;
#pragma unroll
    for (int r = 0; r < (1 << K); ++r) {
        const int64_t i = base + ((int64_t)r << lo);
        float x = v[r];
        if (LAST) x = x / a.sqrtD;                                  // AS:114 vec /= sqrt(d)
        if (RECV_LAST) {
            if (i < a.dim) {
                x = x * (float)sg[i];                               // AS:152 * diag
                a.out[vec * a.dim + i] = a.scale ? a.scale[vec] * x : x;   // AS:413 scale * vec, [:dim]
            }
        } else {
            a.out[vec * D + i] = x;
        }
    }
}

// ---- KE2: torch.norm(v, 2) -------------------------------------------------------------
// torch CPU order: 8 interleaved lanes, acc_l = fma(v[8i + l], v[8i + l], acc_l) in i order,
// then acc_0 + acc_1 + ... + acc_7, the scalar tail, sqrt (f32).  One workgroup serves 4
// clients: wave 0 runs the 32 chains (client k = lane / 8, torch lane l = lane % 8) and never
// touches global memory; waves 1-4 stream 1024-float chunks of the 4 clients into a
// triple-buffered LDS image laid out [client][l][i], so a chain lane reads 4 consecutive
// steps with one ds_read_b128.
constexpr int kNormClients = 4;
constexpr int kNormChunk = 2048;                    // floats per client per chunk (1024: EDEN batch +0.05 ms, 512: +0.4 ms; profiles/r3j_exp_eden_norm_chunk.jsonl)
constexpr int kNormRow = kNormChunk / 8 + 4;        // one torch lane's 128 steps (+4 pad)
constexpr int kNormClientStride = 8 * kNormRow;
constexpr int kNormBuf = kNormClients * kNormClientStride;
constexpr int kNormThreads = 64 + 256;
// Loads run two chunks ahead in two register sets (the loop is unrolled by two so the set is
// static): chunk ch + 2's loads stay in flight across iteration ch + 1 (0.86 -> 0.77 ms at
// 1024 x 2^20 in tools/exp/norm_nc.py).  Whole chunks load without per-element guards.
__global__ void __launch_bounds__(kNormThreads)
eden_norm_kernel(const float* __restrict__ v, int64_t n, int64_t D, float* __restrict__ nrm) {
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nv = D - D % 8;
    const int64_t nchunks = (nv + kNormChunk - 1) / kNormChunk;
    const bool chain = tid < kWave;
    // loaders: thread t' = tid - 64 owns client k = t' / 64 and float4 slots (t' % 64) + 64 q
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = !chain && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * D;
    constexpr int kLQ = kNormChunk / 256;             // float4 per loader thread
    float4 na[kLQ], nb[kLQ];
    auto load = [&](float4 (&nx)[kLQ], int64_t ch) {
        if (ch >= nchunks) return;                       // uniform
        if (lvalid && (ch + 1) * kNormChunk <= nv) {     // wave-uniform: a whole chunk, no guards
#pragma unroll
            for (int q = 0; q < kLQ; ++q)
                nx[q] = ld_stream(reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q)));
            return;
        }
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int64_t i = ch * kNormChunk + 4 * (lj + 64 * q);
            nx[q].x = (lvalid && i < nv) ? lp[i] : 0.f;
            nx[q].y = (lvalid && i + 1 < nv) ? lp[i + 1] : 0.f;
            nx[q].z = (lvalid && i + 2 < nv) ? lp[i + 2] : 0.f;
            nx[q].w = (lvalid && i + 3 < nv) ? lp[i + 3] : 0.f;
        }
    };
    auto store = [&](const float4 (&nx)[kLQ], float* sb) {      // element e = 8 i + l -> [k][l][i]
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int e = 4 * (lj + 64 * q);
            const int i = e >> 3, l = e & 7;
            float* base = sb + lk * kNormClientStride + i;
            base[(l + 0) * kNormRow] = nx[q].x;
            base[(l + 1) * kNormRow] = nx[q].y;
            base[(l + 2) * kNormRow] = nx[q].z;
            base[(l + 3) * kNormRow] = nx[q].w;
        }
    };
    const int ck = (tid >> 3) & (kNormClients - 1), cl = tid & 7;   // lanes >= 32 mirror 0..31
    float acc = 0.f;
    auto chain_chunk = [&](int64_t ch) {
        const int cnt = (int)(std::min<int64_t>(kNormChunk, nv - ch * kNormChunk) / 8);
        const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
        int i = 0;
        for (; i + 16 <= cnt; i += 16) {
            float4 t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(row + i + 4 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = fmaf(t[u].x, t[u].x, acc);
                acc = fmaf(t[u].y, t[u].y, acc);
                acc = fmaf(t[u].z, t[u].z, acc);
                acc = fmaf(t[u].w, t[u].w, acc);
            }
        }
        for (; i < cnt; ++i) acc = fmaf(row[i], row[i], acc);
    };
    if (nchunks > 0 && !chain) {
        load(na, 0);
        store(na, s[0]);
        load(na, 1);                                   // chunk 1 -> na, chunk 2 -> nb
        load(nb, 2);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunks; ch += 2) {
        // iteration ch: chain on chunk ch; chunk ch + 1 (na) into LDS, chunk ch + 3 -> na
        if (chain) chain_chunk(ch);
        else if (ch + 1 < nchunks) {
            store(na, s[(ch + 1) % 3]);
            load(na, ch + 3);
        }
        __syncthreads();
        if (ch + 1 >= nchunks) break;
        // iteration ch + 1: chain on chunk ch + 1; chunk ch + 2 (nb) into LDS, ch + 4 -> nb
        if (chain) chain_chunk(ch + 1);
        else if (ch + 2 < nchunks) {
            store(nb, s[(ch + 2) % 3]);
            load(nb, ch + 4);
        }
        __syncthreads();
    }
    if (chain) {
        const int base = tid & ~7;
        float tot = __shfl(acc, base, kWave);
        for (int j = 1; j < 8; ++j) tot = tot + __shfl(acc, base + j, kWave);
        const int64_t vec = v0 + ck;
        if (tid < 8 * kNormClients && cl == 0 && vec < n) {
            const float* p = v + vec * D;
            // torch's CPU norm below one 8-wide vector (EDEN's D = 1, 2, 4): |x| for one
            // element, fma for two, mul + add for four (measured on torch 2.10)
            if (D == 2) tot = fmaf(p[1], p[1], fmaf(p[0], p[0], 0.0f));
            else for (int64_t i = nv; i < D; ++i) tot = tot + p[i] * p[i];
            nrm[vec] = D == 1 ? fabsf(p[0]) : sqrtf(tot);
        }
    }
}

// The same kernel when every chunk is whole (D a multiple of kNormChunk: D >= 1024), with
// no guards anywhere: with the guarded loads and the general chunk count of the kernel
// above the compiler's waits cost the two-ahead overlap (0.87-0.98 against 0.79 ms at
// 1024 x 2^20, tools/exp/norm_in_pipeline.py).  Same adds in the same order.
__global__ void __launch_bounds__(kNormThreads)
eden_norm_whole_kernel(const float* __restrict__ v, int64_t n, int64_t D, float* __restrict__ nrm) {
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nchunks = D / kNormChunk;
    const bool chain = tid < kWave;
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = !chain && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * D;
    constexpr int kLQ = kNormChunk / 256;
    float4 na[kLQ], nb[kLQ];
    auto load = [&](float4 (&nx)[kLQ], int64_t ch) {
        if (!lvalid || ch >= nchunks) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) nx[q] = ld_stream(reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q)));
    };
    auto store = [&](const float4 (&nx)[kLQ], float* sb) {
        if (chain) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int e = 4 * (lj + 64 * q);
            const int i = e >> 3, l = e & 7;
            float* base = sb + lk * kNormClientStride + i;
            base[(l + 0) * kNormRow] = nx[q].x;
            base[(l + 1) * kNormRow] = nx[q].y;
            base[(l + 2) * kNormRow] = nx[q].z;
            base[(l + 3) * kNormRow] = nx[q].w;
        }
    };
    const int ck = (tid >> 3) & (kNormClients - 1), cl = tid & 7;
    float acc = 0.f;
    auto chainstep = [&](int64_t ch) {
        const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
        for (int i = 0; i < kNormChunk / 8; i += 16) {
            float4 t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(row + i + 4 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = fmaf(t[u].x, t[u].x, acc);
                acc = fmaf(t[u].y, t[u].y, acc);
                acc = fmaf(t[u].z, t[u].z, acc);
                acc = fmaf(t[u].w, t[u].w, acc);
            }
        }
    };
    if (!chain) {
        load(na, 0);
        store(na, s[0]);
        load(na, 1);                    // chunk 1 -> na, chunk 2 -> nb
        load(nb, 2);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunks; ch += 2) {
        if (chain) chainstep(ch);
        else if (ch + 1 < nchunks) {
            store(na, s[(ch + 1) % 3]);
            load(na, ch + 3);
        }
        __syncthreads();
        if (ch + 1 >= nchunks) break;
        if (chain) chainstep(ch + 1);
        else if (ch + 2 < nchunks) {
            store(nb, s[(ch + 2) % 3]);
            load(nb, ch + 4);
        }
        __syncthreads();
    }
    if (chain) {
        const int base = tid & ~7;
        float tot = __shfl(acc, base, kWave);
        for (int j = 1; j < 8; ++j) tot = tot + __shfl(acc, base + j, kWave);
        const int64_t vec = v0 + ck;
        if (tid < 8 * kNormClients && cl == 0 && vec < n) nrm[vec] = sqrtf(tot);
    }
}

// ---- KE2s: the same norm for small batches, its chains cut into segments -----------------
// KE2 runs each client's 8 chains of D/8 dependent fmas end to end: with few clients the
// chain IS the kernel (0.64 ms at n = 1, D = 2^20: 80 % of the per-call EDEN drop-in).  The
// segmented form gives the same bits with the chains cut into segments of kSegSteps steps:
//   KE2a  fp64 sum of v^2 per (lane, segment)                                  (approximate)
//   KE2b  guess g = f32(fp64 exclusive prefix of those sums) per segment        (approximate)
//   KE2c  e = the segment's f32 fma chain run from g.  Inside one binade the f32 grid is
//         uniform, so RN(a + p) = RN(b + p) + (a - b) for grid points a, b when a + p and
//         b + p stay in that binade and are not midpoints (a - b shifts a midpoint onto a
//         midpoint, so the two chains meet ties at the same steps).  Hence any start A in
//         g's binade ends at A + (e - g) exactly, if the guess chain met no tie and stayed in
//         the binade and A + (e - g) is still in it.  Segments whose guess chain crosses a
//         binade edge, meets a tie (or cannot rule one out), or starts / ends within
//         kSegTab/2 grid steps of an edge are listed for a table:
//   KE2t  the chain run from each of the kSegTab f32 starts whose bit patterns surround g's.
//   KE2d  one wave per torch lane walks its segments in order from A = 0: a wave prefix sum
//         of e - g resolves every segment up to the first one that does not translate
//         (exact: one binade range, checked), that one is resolved by its table or, when A
//         is outside the table, by running its kSegSteps steps.  The lanes are then added
//         in order as in KE2.  Every end value is the sequential chain's, bit for bit.
constexpr int kSegSteps = 64;                          // chain steps per segment
constexpr int kSegBlock = 8 * kSegSteps;               // floats of one segment (all 8 lanes)
constexpr int kSegPerWG = 32;                          // segments per KE2a / KE2c workgroup
constexpr int kSegPad = kSegBlock + 8;                 // LDS row of a segment (8 floats apart: banks)
constexpr int kSegTab = 1024;                          // table starts per listed segment
constexpr int kSegTabCap = 256;                        // tables per client at most (beyond: KE2d runs the steps)
// tables per client for a vector of D: the table region is cap * 4 KB per client, so short
// vectors get fewer (a 2^14 vector is 64 KB; beyond the cap a segment's 64 steps run in KE2d)
__host__ __device__ inline int seg_tab_cap(int64_t D) {
    const int64_t c = D / 512;
    return (int)(c < 32 ? 32 : (c > kSegTabCap ? kSegTabCap : c));
}
constexpr int64_t kSegMinD = (int64_t)kSegBlock * kSegPerWG;
static_assert(kSegSteps == 64, "KE2d's step path loads one segment as one value per lane of a wave");

__device__ __forceinline__ uint32_t fbits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ int fexp(float x) { return (int)((__float_as_uint(x) >> 23) & 0xFFu); }

// kSegPerWG segments of one client from v into LDS rows [segment][8 * step + lane]
__device__ __forceinline__ void seg_stage(const float* __restrict__ v, int64_t D, int64_t client, int64_t seg0,
                                          float* s, int tid) {
    const float4* src = reinterpret_cast<const float4*>(v + client * D + seg0 * kSegBlock);
#pragma unroll
    for (int j = 0; j < kSegBlock * kSegPerWG / 4 / 256; ++j) {
        const int q = tid + 256 * j;
        const int e = 4 * q;
        *reinterpret_cast<float4*>(s + (e / kSegBlock) * kSegPad + (e % kSegBlock)) = src[q];
    }
}

__global__ void __launch_bounds__(256)
eden_segsum_kernel(const float* __restrict__ v, int64_t D, double* __restrict__ segsum) {
    __shared__ __attribute__((aligned(16))) float s[kSegPerWG * kSegPad];
    const int tid = threadIdx.x;
    const int64_t client = blockIdx.y;
    const int64_t K = D / kSegBlock;
    const int64_t seg0 = (int64_t)blockIdx.x * kSegPerWG;
    seg_stage(v, D, client, seg0, s, tid);
    __syncthreads();
    const int sl = tid >> 3, l = tid & 7;
    const float* row = s + sl * kSegPad + l;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};              // an approximation: any order will do
#pragma unroll 16
    for (int i = 0; i < kSegSteps; ++i) {
        const double x = row[8 * i];
        acc[i & 3] += x * x;
    }
    segsum[(client * 8 + l) * K + seg0 + sl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// one workgroup per (lane, client): the exclusive prefix of the lane's K segment sums, in
// rounds of 1024 (4 per thread, coalesced); lane 0's workgroup zeroes the table count
__global__ void __launch_bounds__(256)
eden_segscan_kernel(const double* __restrict__ segsum, int64_t K, float* __restrict__ g, int32_t* __restrict__ tabcnt) {
    __shared__ double wsum[256 / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int l = blockIdx.x;
    const int64_t client = blockIdx.y;
    if (tid == 0 && l == 0) tabcnt[client] = 0;
    const double* src = segsum + (client * 8 + l) * K;
    float* dst = g + (client * 8 + l) * K;
    double carry = 0.0;
    for (int64_t r0 = 0; r0 < K; r0 += 1024) {
        double x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = r0 + 4 * tid + k;
            x[k] = i < K ? src[i] : 0.0;
        }
        const double t = (x[0] + x[1]) + (x[2] + x[3]);
        const double incl = wave_incl_scan(t, lane);
        if (lane == kWave - 1) wsum[wid] = incl;
        __syncthreads();
        double run = carry + wave_prev(incl), tot = carry;
#pragma unroll
        for (int w = 0; w < 256 / kWave; ++w) {
            if (w < wid) run += wsum[w];
            tot += wsum[w];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = r0 + 4 * tid + k;
            if (i < K) dst[i] = (float)run;
            run += x[k];
        }
        carry = tot;
    }
}

__global__ void __launch_bounds__(256)
eden_segchain_kernel(const float* __restrict__ v, int64_t D, const float* __restrict__ g, float* __restrict__ e,
                     int32_t* __restrict__ kind, int32_t* __restrict__ tabcnt, int32_t* __restrict__ tabseg, int cap) {
    __shared__ __attribute__((aligned(16))) float s[kSegPerWG * kSegPad];
    const int tid = threadIdx.x;
    const int64_t client = blockIdx.y;
    const int64_t K = D / kSegBlock;
    const int64_t seg0 = (int64_t)blockIdx.x * kSegPerWG;
    seg_stage(v, D, client, seg0, s, tid);
    __syncthreads();
    const int sl = tid >> 3, l = tid & 7;
    const int64_t idx = (client * 8 + l) * K + seg0 + sl;
    const float* row = s + sl * kSegPad + l;
    const float g0 = g[idx];
    float b = g0;
    bool tie = false;
#pragma unroll 16
    for (int i = 0; i < kSegSteps; ++i) {                 // (unrolled: LDS reads ahead of the chain)
        const float x = row[8 * i];
        const float r = fmaf(x, x, b);
        // (b + x*x) - r exactly (fp64: b - r is exact when their exponents are within 28, and
        // the fma returns the residual exactly whenever it is one of the values tested): a
        // midpoint is half a grid step, u/2, or u/4 just below a power of two
        const int er = fexp(r);
        const double u = __longlong_as_double((long long)((uint64_t)(std::max(er, 1) - 150 + 1023) << 52));
        const double res = fabs(fma((double)x, (double)x, (double)b - (double)r));
        tie = tie || res == 0.5 * u || res == 0.25 * u || (b != 0.0f && er - fexp(b) > 28);
        b = r;
    }
    const int eg = fexp(g0);
    const bool finite = eg < 255 && fexp(b) < 255;
    const bool cross = fexp(b) != eg;
    const bool near_bottom = eg > 0 && (fbits(g0) & 0x7FFFFFu) < (uint32_t)(kSegTab / 2);
    const bool near_top = !cross && (((uint32_t)(eg + 1) << 23) - fbits(b)) <= (uint32_t)(kSegTab / 2);
    int32_t k = 0;
    if (!finite || cross || tie || near_bottom || near_top) {
        const int slot = atomicAdd(&tabcnt[client], 1);
        if (slot < cap) {
            k = slot + 1;
            tabseg[client * cap + slot] = (int32_t)((seg0 + sl) * 8 + l);
        } else {
            k = -1;                                    // no table: KE2d runs its steps
        }
    }
    e[idx] = b;
    kind[idx] = k;
}

__global__ void __launch_bounds__(256)
eden_segtab_kernel(const float* __restrict__ v, int64_t D, const float* __restrict__ g, const int32_t* __restrict__ tabcnt,
                   const int32_t* __restrict__ tabseg, float* __restrict__ tab, int cap) {
    __shared__ float xs[kSegSteps];
    const int64_t client = blockIdx.y;
    const int slot = blockIdx.x;
    if (slot >= std::min(tabcnt[client], cap)) return;                   // uniform
    const int tid = threadIdx.x;
    const int32_t code = tabseg[client * cap + slot];
    const int64_t seg = code >> 3;
    const int l = code & 7;
    const int64_t K = D / kSegBlock;
    if (tid < kSegSteps) xs[tid] = v[client * D + 8 * (seg * kSegSteps + tid) + l];
    __syncthreads();
    const int64_t gb = fbits(g[(client * 8 + l) * K + seg]);
    constexpr int kPer = kSegTab / 256;
    float a[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int64_t sb = gb + tid + 256 * k - kSegTab / 2;
        a[k] = sb < 0 ? __uint_as_float(0x7FC00000u) : __uint_as_float((uint32_t)sb);   // (never looked up)
    }
    for (int i = 0; i < kSegSteps; ++i) {
        const float x = xs[i];
#pragma unroll
        for (int k = 0; k < kPer; ++k) a[k] = fmaf(x, x, a[k]);
    }
    float* out = tab + ((int64_t)client * cap + slot) * kSegTab;
#pragma unroll
    for (int k = 0; k < kPer; ++k) out[tid + 256 * k] = a[k];
}

// one workgroup per client, wave l walks torch lane l's chain.  A wave holds kWalkChunks
// chunks of 64 segments in registers (lane j: segment 64 q + j of chunk q) and loads the next
// tile of chunks while it walks this one.
constexpr int kWalkChunks = 8;
__global__ void __launch_bounds__(512)
eden_segwalk_kernel(const float* __restrict__ v, int64_t D, const float* __restrict__ g, const float* __restrict__ e,
                    const int32_t* __restrict__ kind, const float* __restrict__ tab, float* __restrict__ nrm, int cap) {
    __shared__ float accs[8];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), l = tid / kWave;
    const int64_t client = blockIdx.x;
    const int64_t K = D / kSegBlock;
    const int64_t base = (client * 8 + l) * K;
    float cg[kWalkChunks], ce[kWalkChunks], ng[kWalkChunks] = {}, ne[kWalkChunks] = {};
    int32_t ck[kWalkChunks], nk[kWalkChunks] = {};
    auto fetch = [&](int64_t tile, float (&fg)[kWalkChunks], float (&fe)[kWalkChunks], int32_t (&fk)[kWalkChunks]) {
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            const int64_t s = (tile * kWalkChunks + q) * kWave + lane;
            fg[q] = s < K ? g[base + s] : 0.0f;
            fe[q] = s < K ? e[base + s] : 0.0f;
            fk[q] = s < K ? kind[base + s] : 0;
        }
    };
    float A = 0.0f;                                    // wave-uniform
    int64_t s0 = 0;
    // resolve segment s0 of chunk c (registers: this lane's segment of the chunk) and, when
    // it translates, every following one of the chunk that does
    auto step = [&](int64_t c, float sg, float se, int32_t sk) {
        const int o = (int)(s0 - c * kWave);
        const bool inb = lane >= o && c * kWave + lane < K;
        const bool fin = fexp(sg) < 255 && fexp(se) < 255;
        const double tau = (inb && fin) ? (double)se - (double)sg : 0.0;   // >= 0: chains never decrease
        const double Aj = (double)A + wave_prev(wave_incl_scan(tau, lane));
        // the partial sums are exact while they stay below 2^28 times A's binade (multiples of
        // its grid step, 51 bits); A = 0 (or not finite) resolves one segment at a time
        const bool span = A > 0.0f && fexp(A) < 255;
        const double lim = __longlong_as_double((long long)((uint64_t)(std::max(fexp(A), 1) - 127 + 28 + 1023) << 52));
        const float af = (float)Aj;
        const float r = af + (float)tau;
        const bool valid = inb && fin && (lane == o || (span && Aj + tau < lim)) && (double)af == Aj &&
                           (af == sg || (sk == 0 && fexp(af) == fexp(sg) && fexp(r) == fexp(sg)));
        const uint64_t bad = __ballot(inb && !valid);
        const uint64_t inm = __ballot(inb);
        const int first = bad ? __builtin_ctzll(bad) : 64 - __builtin_clzll(inm);
        if (first > o) {                               // segments o .. first - 1 resolved
            const float res = af == sg ? se : r;
            A = __shfl(res, first - 1, kWave);
            s0 = c * kWave + first;
            return;
        }
        // segment s0 does not translate: its table, or its steps
        const int32_t kk = __shfl(sk, o, kWave);
        const float gg = __shfl(sg, o, kWave);
        bool done = false;
        if (kk > 0) {
            const int64_t d = (int64_t)fbits(A) - (int64_t)fbits(gg) + kSegTab / 2;
            if (d >= 0 && d < kSegTab) {
                A = tab[((int64_t)client * cap + (kk - 1)) * kSegTab + d];
                done = true;
            }
        }
        if (!done) {
            const float x = v[client * D + 8 * (s0 * kSegSteps + lane) + l];
            for (int i = 0; i < kSegSteps; ++i) {
                const float xi = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)fbits(x), i));
                A = fmaf(xi, xi, A);
            }
        }
        s0 += 1;
    };
    fetch(0, cg, ce, ck);
    const int64_t tiles = (K + kWalkChunks * kWave - 1) / (kWalkChunks * kWave);
    for (int64_t t = 0; t < tiles; ++t) {
        if (t + 1 < tiles) fetch(t + 1, ng, ne, nk);
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            const int64_t c = t * kWalkChunks + q;
            const int64_t cend = std::min<int64_t>(K, (c + 1) * kWave);
            while (s0 < cend) step(c, cg[q], ce[q], ck[q]);
        }
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            cg[q] = ng[q];
            ce[q] = ne[q];
            ck[q] = nk[q];
        }
    }
    if (lane == 0) accs[l] = A;
    __syncthreads();
    if (tid == 0) {
        float tot = accs[0];
        for (int j = 1; j < 8; ++j) tot = tot + accs[j];
        nrm[client] = sqrtf(tot);
    }
}

// ---- KE4: bins and the scale's dot product in MKL sdot's order ---------------------------
// AS:329-335 bins = bucketize(vec * sqrt(D) / norm, boundaries); scale = norm ** 2 /
// torch.dot(take(centroids, bins), vec).  torch's CPU dot is MKL's sdot; its order on the
// fixtures' host (oracle/uq_eden.py:torch_dot, tools/dot_order_probe.py, pinned by
// tests/golden/dot_vectors.json and every EDEN scale the reference recorded): 4 accumulators x
// 16 lanes over 64-element blocks, each lane a sequential fma chain, so element i belongs to
// chain i % 64 at step i / 64; of a remainder below 64, a 32-element block into accumulators 0
// and 1 and then 16-element chunks into accumulator 0 (the last masked: 0 * 0); then
// (acc0 + acc1) + (acc2 + acc3) lane-wise and the 16 lanes as i + (i + 8), i + (i + 4),
// (0 + 1) + (2 + 3).  One wave per client: lane l runs chain l over the client's rotated
// vector (64 consecutive floats per step: one coalesced 256-byte load per wave), writes each
// coordinate's bin (u8) and folds c[bin] * v into its chain; two register sets of kDotU steps of
// loads in flight (32: with few clients one wave's loads in flight bound the kernel, round 6:
// 256 x 2^22 EDEN 10.98 -> 10.48 ms, profiles/r6k_ab_c4_eden_ke4u32.jsonl).  The bin needs no division per element: y = v * f32(sqrt D) (AS:329) falls
// in bin sum_j [!(y <= T_j)] where T_j is the largest f32 y with RN(y / norm) <= boundary j --
// y -> RN(y / norm) is non-decreasing for a positive finite norm, so this is exactly
// torch.bucketize of the quotient (NaN included); T_j is found once per client by bisection
// over the floats' order.  Other norms (0, inf, NaN) take the per-element division.
constexpr int kDotWaves = 4;
constexpr int kDotU = 32;

__device__ __forceinline__ uint32_t ford_key(float y) {          // order-preserving u32 image
    const uint32_t u = __float_as_uint(y);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ford_val(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
// the largest f32 y with RN(y / nv) <= b (nv positive and finite)
__device__ __forceinline__ float eden_thresh(float b, float nv) {
    uint32_t lo = ford_key(-INFINITY), hi = ford_key(INFINITY);   // lo satisfies, hi does not
    while (hi - lo > 1u) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (ford_val(mid) / nv <= b) lo = mid;
        else hi = mid;
    }
    return ford_val(lo);
}

// One client's bins and chains (lane l: chain l); THR: bins by the thresholds T, else by the
// per-element division (norms that are not positive and finite).  Returns the lane's chain.
template <int NB, bool THR>
__device__ __forceinline__ float dotbins_chains(const float* __restrict__ vj, int64_t D, float sqrtD, float nv,
                                                const EdenTables& tab, const EdenCents& cs, const float (&T)[NB],
                                                uint8_t* __restrict__ bj, int lane) {
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(vj, (uint32_t)(D * 4));
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(bj, (uint32_t)D);
    float acc = 0.f;
    auto step = [&](float x, int64_t i) {                                  // bins[i], acc = fma(c[bin], x, acc)
        const float y = x * sqrtD;                                          // AS:329 vec * sqrt(D)
        int b;
        if (THR) {
            b = !(y <= T[0]) ? 1 : 0;
#pragma unroll
            for (int q = 1; q < NB; ++q) b += !(y <= T[q]) ? 1 : 0;
        } else {
            b = eden_bin(tab, y / nv);
        }
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, rb, (uint32_t)i, 0, 0);
        acc = fmaf(eden_cent(cs, b), x, acc);                               // AS:335
    };
    const int64_t steps = D / 64;
    auto pipelined = [&](auto u) {                                         // u steps per register set
        constexpr int U = decltype(u)::value;
        float A[U], B[U];
        auto load = [&](float (&R)[U], int64_t s0) {
#pragma unroll
            for (int k = 0; k < U; ++k)
                R[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    rv, (uint32_t)((s0 + k) * 64 + lane) * 4u, 0, kAuxNT));     // beyond D: 0, unused
        };
        auto run = [&](const float (&R)[U], int64_t s0) {
#pragma unroll
            for (int k = 0; k < U; ++k) step(R[k], (s0 + k) * 64 + lane);
        };
        load(A, 0);
        for (int64_t s0 = 0; s0 < steps; s0 += 2 * U) {
            load(B, s0 + U);
            run(A, s0);
            load(A, s0 + 2 * U);
            run(B, s0 + U);
        }
    };
    if (steps >= 2 * kDotU && steps % (2 * kDotU) == 0) {
        pipelined(std::integral_constant<int, kDotU>{});
        return acc;
    }
    if (steps >= kDotU && steps % kDotU == 0) {                            // e.g. D = 2048
        pipelined(std::integral_constant<int, kDotU / 2>{});
        return acc;
    }
    int64_t i0 = 0;
    for (; i0 + 64 <= D; i0 += 64) step(vj[i0 + lane], i0 + lane);
    if (D - i0 >= 32) {                                                    // remainder: acc 0 and 1
        if (lane < 32) step(vj[i0 + lane], i0 + lane);
        i0 += 32;
    }
    for (; i0 < D; i0 += 16)                                               // then acc 0, masked
        if (lane < 16) {
            if (i0 + lane < D) step(vj[i0 + lane], i0 + lane);
            else acc = fmaf(0.f, 0.f, acc);
        }
    return acc;
}

template <int NB>       // boundaries: 1 (1 bit) or 3 (2 bits)
__global__ void __launch_bounds__(64 * kDotWaves)
eden_dotbins_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm, EdenTables tab,
                    uint8_t* __restrict__ bins, float* __restrict__ scale, int64_t n, const int32_t* __restrict__ redo) {
    __shared__ float red[kDotWaves][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * kDotWaves + wv;
    if (j >= n) return;                                                    // whole wave
    if (redo && !redo[j]) return;                                          // (after KE2+4: its flagged clients)
    const float nv = nrm[j];
    const EdenCents cs = eden_cents(tab);
    const bool thr = nv > 0.f && nv < INFINITY;                            // wave-uniform
    float T[NB];
    {
        const float t = (thr && lane < NB) ? eden_thresh(tab.b[lane < NB ? lane : 0], nv) : 0.f;
#pragma unroll
        for (int q = 0; q < NB; ++q) T[q] = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(t), q));
    }
    const float acc = thr ? dotbins_chains<NB, true>(v + j * D, D, sqrtD, nv, tab, cs, T, bins + j * D, lane)
                          : dotbins_chains<NB, false>(v + j * D, D, sqrtD, nv, tab, cs, T, bins + j * D, lane);
    red[wv][lane] = acc;
    wave_lds_fence();
    if (lane == 0) {
        const float* a = red[wv];
        float w[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) w[l] = (a[l] + a[16 + l]) + (a[32 + l] + a[48 + l]);
#pragma unroll
        for (int l = 0; l < 8; ++l) w[l] = w[l] + w[l + 8];
#pragma unroll
        for (int l = 0; l < 4; ++l) w[l] = w[l] + w[l + 4];
        const float dot = (w[0] + w[1]) + (w[2] + w[3]);
        scale[j] = (nv * nv) / dot;                                        // AS:335 norm ** 2 / dot
    }
}

// ---- KE4s: the same bins and dot for small batches, its chains cut into segments ----------
// eden_dotbins_kernel runs each client's 64 chains of D/64 dependent fmas on one wave: with a
// few clients the chain is the kernel (D/64 steps of ~6-19 VALU each: 0.35 ms at n = 1,
// D = 2^20).  As KE2s does for the norm, the chains are cut into segments of kSegSteps steps;
// a segment of all 64 chains is one 4096-element tile (chain l, step 64 k + i = element
// 4096 k + 64 i + l).  Every chain here is non-decreasing (c[bin] has the sign of v, so each
// product is >= 0), and the KE2s argument applies unchanged with p = c * v instead of v * v:
//   KE4a  bins, and the fp64 sum of c * v per (chain, segment)                (approximate)
//   KE4b  guesses g = f32(fp64 exclusive prefix) per segment (eden_segscan_kernel<64>)
//   KE4c  the segment's f32 fma chain from g -> e; segments whose chain crosses a binade,
//         meets (or cannot rule out) a tie, or starts / ends near a binade edge are listed
//   KE4t  the chain run from each of the kSegTab starts around g for the listed segments
//   KE4d  one wave per chain walks its segments from 0 (wave scans of e - g, tables, steps)
//   KE4f  the 64 chains in MKL's order, scale = f32(nrm * nrm) / dot
// The per-client thresholds of the bins (eden_thresh) are computed once by KE4p.
constexpr int kDSegTiles = 4;                            // KE4c: tiles (segments) per workgroup

struct DotElem {                                         // c[bin(v)] of one client
    float sqrtD, nv, T0, T1, T2;
    bool thr;
    EdenTables tab;
    EdenCents cs;
    __device__ __forceinline__ int bin(float x) const {
        const float y = x * sqrtD;                       // AS:329 vec * sqrt(D)
        if (!thr) return eden_bin(tab, y / nv);
        int b = !(y <= T0) ? 1 : 0;
        if (tab.nb > 1) b += (!(y <= T1) ? 1 : 0) + (!(y <= T2) ? 1 : 0);
        return b;
    }
    __device__ __forceinline__ float cent(float x) const { return eden_cent(cs, bin(x)); }
};
__device__ __forceinline__ DotElem dot_elem(const float* thr4, const float* nrm, int64_t j, float sqrtD,
                                            const EdenTables& tab) {
    DotElem e;
    e.sqrtD = sqrtD;
    e.nv = nrm[j];
    e.T0 = thr4[j * 4];
    e.T1 = thr4[j * 4 + 1];
    e.T2 = thr4[j * 4 + 2];
    e.thr = thr4[j * 4 + 3] != 0.f;
    e.tab = tab;
    e.cs = eden_cents(tab);
    return e;
}

// KE4p: thresholds per client (lane q: boundary q), thr4[j] = (T0, T1, T2, valid)
__global__ void __launch_bounds__(64)
eden_thresh_kernel(const float* __restrict__ nrm, EdenTables tab, float* __restrict__ thr4) {
    const int64_t j = blockIdx.x;
    const int lane = threadIdx.x;
    const float nv = nrm[j];
    const bool ok = nv > 0.f && nv < INFINITY;
    if (lane < 3) thr4[j * 4 + lane] = (ok && lane < tab.nb) ? eden_thresh(tab.b[lane], nv) : 0.f;
    if (lane == 3) thr4[j * 4 + 3] = ok ? 1.f : 0.f;
}

// KE4a: one tile per workgroup; thread (g, l) sums steps 16 g .. 16 g + 15 of chain l
__global__ void __launch_bounds__(256)
eden_dseg_sum_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm,
                     const float* __restrict__ thr4, EdenTables tab, uint8_t* __restrict__ bins,
                     double* __restrict__ segsum) {
    __shared__ double part[4][64];
    const int tid = threadIdx.x, l = tid & 63, g = tid >> 6;
    const int64_t client = blockIdx.y, k = blockIdx.x, K = D / kEdenTile;
    const DotElem de = dot_elem(thr4, nrm, client, sqrtD, tab);
    const float* t = v + client * D + k * kEdenTile;
    uint8_t* bt = bins + client * D + k * kEdenTile;
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = t[64 * (16 * g + i) + l];
    double acc = 0.0;                                    // an approximation: any order will do
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int b = de.bin(x[i]);
        bt[64 * (16 * g + i) + l] = (uint8_t)b;
        acc += (double)eden_cent(de.cs, b) * (double)x[i];
    }
    part[g][l] = acc;
    __syncthreads();
    if (tid < 64) segsum[(client * 64 + l) * K + k] = (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
}

// KE4b: exclusive prefix per (chain, client) of its K segment sums (the norm's scan, 64 chains)
template <int L>
__global__ void __launch_bounds__(256)
eden_segscan_l_kernel(const double* __restrict__ segsum, int64_t K, float* __restrict__ g, int32_t* __restrict__ tabcnt) {
    __shared__ double wsum[256 / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int l = blockIdx.x;
    const int64_t client = blockIdx.y;
    if (tid == 0 && l == 0) tabcnt[client] = 0;
    const double* src = segsum + (client * L + l) * K;
    float* dst = g + (client * L + l) * K;
    double carry = 0.0;
    for (int64_t r0 = 0; r0 < K; r0 += 1024) {
        double xs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = r0 + 4 * tid + q;
            xs[q] = i < K ? src[i] : 0.0;
        }
        const double t = (xs[0] + xs[1]) + (xs[2] + xs[3]);
        const double incl = wave_incl_scan(t, lane);
        if (lane == kWave - 1) wsum[wid] = incl;
        __syncthreads();
        double run = carry + wave_prev(incl), tot = carry;
#pragma unroll
        for (int w = 0; w < 256 / kWave; ++w) {
            if (w < wid) run += wsum[w];
            tot += wsum[w];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = r0 + 4 * tid + q;
            if (i < K) dst[i] = (float)run;
            run += xs[q];
        }
        carry = tot;
    }
}

// KE4c: thread (tile k, chain l) runs its segment's 64 steps from the guess (the KE2c tests)
__global__ void __launch_bounds__(256)
eden_dseg_chain_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm,
                       const float* __restrict__ thr4, EdenTables tab, const float* __restrict__ g,
                       float* __restrict__ e, int32_t* __restrict__ kind, int32_t* __restrict__ tabcnt,
                       int32_t* __restrict__ tabseg, int cap) {
    const int tid = threadIdx.x, l = tid & 63;
    const int64_t client = blockIdx.y, K = D / kEdenTile;
    const int64_t k = (int64_t)blockIdx.x * kDSegTiles + (tid >> 6);
    const DotElem de = dot_elem(thr4, nrm, client, sqrtD, tab);
    const float* t = v + client * D + k * kEdenTile + l;
    const int64_t idx = (client * 64 + l) * K + k;
    const float g0 = g[idx];
    float b = g0;
    bool tie = false;
#pragma unroll 16
    for (int i = 0; i < kSegSteps; ++i) {
        const float x = t[64 * i];
        const float c = de.cent(x);
        // a negative product (a tiny v whose quotient underflowed into the lowest bin) breaks
        // the chain's monotonicity: list the segment (its table or its steps are sequential)
        tie = tie || (((fbits(c) ^ fbits(x)) >> 31) && x != 0.0f && c != 0.0f);
        const float r = fmaf(c, x, b);
        // (b + c*x) - r exactly: a midpoint is u/2, or u/4 just below a power of two (KE2c)
        const int er = fexp(r);
        const double u = __longlong_as_double((long long)((uint64_t)(std::max(er, 1) - 150 + 1023) << 52));
        const double res = fabs(fma((double)c, (double)x, (double)b - (double)r));
        tie = tie || res == 0.5 * u || res == 0.25 * u || (b != 0.0f && er - fexp(b) > 28);
        b = r;
    }
    const int eg = fexp(g0);
    const bool finite = eg < 255 && fexp(b) < 255;
    const bool cross = fexp(b) != eg;
    const bool near_bottom = eg > 0 && (fbits(g0) & 0x7FFFFFu) < (uint32_t)(kSegTab / 2);
    const bool near_top = !cross && (((uint32_t)(eg + 1) << 23) - fbits(b)) <= (uint32_t)(kSegTab / 2);
    int32_t kk = 0;
    if (!finite || cross || tie || near_bottom || near_top) {
        const int slot = atomicAdd(&tabcnt[client], 1);
        if (slot < cap) {
            kk = slot + 1;
            tabseg[client * cap + slot] = (int32_t)(k * 64 + l);
        } else {
            kk = -1;                                     // no table: KE4d runs its steps
        }
    }
    e[idx] = b;
    kind[idx] = kk;
}

// KE4t: the listed segment's chain from each of the kSegTab starts around its guess
__global__ void __launch_bounds__(256)
eden_dseg_tab_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm,
                     const float* __restrict__ thr4, EdenTables tab, const float* __restrict__ g,
                     const int32_t* __restrict__ tabcnt, const int32_t* __restrict__ tabseg, float* __restrict__ tabv,
                     int cap) {
    __shared__ float xs[kSegSteps], cs_[kSegSteps];
    const int64_t client = blockIdx.y;
    const int slot = blockIdx.x;
    if (slot >= std::min(tabcnt[client], cap)) return;                   // uniform
    const int tid = threadIdx.x;
    const int32_t code = tabseg[client * cap + slot];
    const int64_t k = code >> 6;
    const int l = code & 63;
    const int64_t K = D / kEdenTile;
    if (tid < kSegSteps) {
        const DotElem de = dot_elem(thr4, nrm, client, sqrtD, tab);
        const float x = v[client * D + k * kEdenTile + 64 * tid + l];
        xs[tid] = x;
        cs_[tid] = de.cent(x);
    }
    __syncthreads();
    const int64_t gb = fbits(g[(client * 64 + l) * K + k]);
    constexpr int kPer = kSegTab / 256;
    float a[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int64_t sb = gb + tid + 256 * q - kSegTab / 2;
        a[q] = sb < 0 ? __uint_as_float(0x7FC00000u) : __uint_as_float((uint32_t)sb);   // (never looked up)
    }
    for (int i = 0; i < kSegSteps; ++i) {
        const float x = xs[i], c = cs_[i];
#pragma unroll
        for (int q = 0; q < kPer; ++q) a[q] = fmaf(c, x, a[q]);
    }
    float* out = tabv + ((int64_t)client * cap + slot) * kSegTab;
#pragma unroll
    for (int q = 0; q < kPer; ++q) out[tid + 256 * q] = a[q];
}

// KE4d: wave w of workgroup b walks chain 8 b + w of client blockIdx.y (KE2d's walk); the
// chain's end goes to acc64[client][chain]
__global__ void __launch_bounds__(512)
eden_dseg_walk_kernel(const float* __restrict__ v, int64_t D, float sqrtD, const float* __restrict__ nrm,
                      const float* __restrict__ thr4, EdenTables tab, const float* __restrict__ g,
                      const float* __restrict__ e, const int32_t* __restrict__ kind, const float* __restrict__ tabv,
                      float* __restrict__ acc64, int cap) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    const int l = blockIdx.x * 8 + tid / kWave;
    const int64_t client = blockIdx.y;
    const int64_t K = D / kEdenTile;
    const int64_t base = (client * 64 + l) * K;
    const DotElem de = dot_elem(thr4, nrm, client, sqrtD, tab);
    float cg[kWalkChunks], ce[kWalkChunks], ng[kWalkChunks] = {}, ne[kWalkChunks] = {};
    int32_t ck[kWalkChunks], nk[kWalkChunks] = {};
    auto fetch = [&](int64_t tile, float (&fg)[kWalkChunks], float (&fe)[kWalkChunks], int32_t (&fk)[kWalkChunks]) {
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            const int64_t s = (tile * kWalkChunks + q) * kWave + lane;
            fg[q] = s < K ? g[base + s] : 0.0f;
            fe[q] = s < K ? e[base + s] : 0.0f;
            fk[q] = s < K ? kind[base + s] : 0;
        }
    };
    float A = 0.0f;                                    // wave-uniform
    int64_t s0 = 0;
    auto step = [&](int64_t c, float sg, float se, int32_t sk) {
        const int o = (int)(s0 - c * kWave);
        const bool inb = lane >= o && c * kWave + lane < K;
        const bool fin = fexp(sg) < 255 && fexp(se) < 255;
        const double tau = (inb && fin) ? (double)se - (double)sg : 0.0;   // >= 0: chains never decrease
        const double Aj = (double)A + wave_prev(wave_incl_scan(tau, lane));
        const bool span = A > 0.0f && fexp(A) < 255;
        const double lim = __longlong_as_double((long long)((uint64_t)(std::max(fexp(A), 1) - 127 + 28 + 1023) << 52));
        const float af = (float)Aj;
        const float r = af + (float)tau;
        const bool valid = inb && fin && (lane == o || (span && Aj + tau < lim)) && (double)af == Aj &&
                           (af == sg || (sk == 0 && fexp(af) == fexp(sg) && fexp(r) == fexp(sg)));
        const uint64_t bad = __ballot(inb && !valid);
        const uint64_t inm = __ballot(inb);
        const int first = bad ? __builtin_ctzll(bad) : 64 - __builtin_clzll(inm);
        if (first > o) {
            const float res = af == sg ? se : r;
            A = __shfl(res, first - 1, kWave);
            s0 = c * kWave + first;
            return;
        }
        const int32_t kk = __shfl(sk, o, kWave);
        const float gg = __shfl(sg, o, kWave);
        bool done = false;
        if (kk > 0) {
            const int64_t dd = (int64_t)fbits(A) - (int64_t)fbits(gg) + kSegTab / 2;
            if (dd >= 0 && dd < kSegTab) {
                A = tabv[((int64_t)client * cap + (kk - 1)) * kSegTab + dd];
                done = true;
            }
        }
        if (!done) {
            const float x = v[client * D + s0 * kEdenTile + 64 * lane + l];
            const float c = de.cent(x);
            for (int i = 0; i < kSegSteps; ++i) {
                const float xi = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)fbits(x), i));
                const float ci = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)fbits(c), i));
                A = fmaf(ci, xi, A);
            }
        }
        s0 += 1;
    };
    fetch(0, cg, ce, ck);
    const int64_t tiles = (K + kWalkChunks * kWave - 1) / (kWalkChunks * kWave);
    for (int64_t t = 0; t < tiles; ++t) {
        if (t + 1 < tiles) fetch(t + 1, ng, ne, nk);
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            const int64_t c = t * kWalkChunks + q;
            const int64_t cend = std::min<int64_t>(K, (c + 1) * kWave);
            while (s0 < cend) step(c, cg[q], ce[q], ck[q]);
        }
#pragma unroll
        for (int q = 0; q < kWalkChunks; ++q) {
            cg[q] = ng[q];
            ce[q] = ne[q];
            ck[q] = nk[q];
        }
    }
    if (lane == 0) acc64[client * 64 + l] = A;
}

// KE4f: the 64 chains in MKL's order, scale = f32(nrm * nrm) / dot (AS:335)
__global__ void __launch_bounds__(64)
eden_dseg_final_kernel(const float* __restrict__ acc64, const float* __restrict__ nrm, float* __restrict__ scale) {
    const int64_t j = blockIdx.x;
    if (threadIdx.x != 0) return;
    const float* a = acc64 + j * 64;
    float w[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) w[l] = (a[l] + a[16 + l]) + (a[32 + l] + a[48 + l]);
#pragma unroll
    for (int l = 0; l < 8; ++l) w[l] = w[l] + w[l + 8];
#pragma unroll
    for (int l = 0; l < 4; ++l) w[l] = w[l] + w[l + 4];
    const float dot = (w[0] + w[1]) + (w[2] + w[3]);
    const float nv = nrm[j];
    scale[j] = (nv * nv) / dot;
}

// ---- KE2+4: the 1-bit norm, bins and dot in one read (batches of more than 256 clients) --
// With one boundary at 0, bucketize(v * sqrt(D) / norm) is v's sign -- 1 for v > 0 (and NaN),
// else 0 -- unless the quotient underflows to 0 (a positive v below ~2^-149 * norm / sqrt(D))
// or the norm is not positive and finite.  So the bins, and with them the dot's chains, need no
// norm: KE2's workgroup (4 clients, loader waves staging chunks in LDS, one wave on the
// norm's 32 chains) gets one more wave per client that runs that client's 64 dot chains from
// the same LDS image, and the loaders write the bins and track the smallest positive v * sqrt(D).
// At the end the norm is known: a client whose norm is not positive and finite, or whose
// smallest positive product underflows, is flagged and recomputed by the exact KE4
// (eden_dotbins_kernel with `redo`); every other client's bins and scale are KE4's bits.
constexpr int kNDThreads = 64 + 256 + 64 * kNormClients;
__global__ void __launch_bounds__(kNDThreads)
eden_normdot1_kernel(const float* __restrict__ v, int64_t n, int64_t D, float sqrtD, EdenTables tab,
                     float* __restrict__ nrm, uint8_t* __restrict__ bins, float* __restrict__ scale,
                     int32_t* __restrict__ redo) {
    __shared__ __attribute__((aligned(16))) float s[3][kNormBuf];
    __shared__ float dacc[kNormClients][64];
    __shared__ uint32_t minpos[kNormClients];
    const int tid = threadIdx.x;
    const int64_t v0 = (int64_t)blockIdx.x * kNormClients;
    const int64_t nchunks = D / kNormChunk;
    const bool chain = tid < kWave;
    const bool loader = tid >= kWave && tid < kWave + 256;
    const bool dotw = tid >= kWave + 256;
    const int lt = tid - kWave, lk = lt >> 6, lj = lt & 63;
    const bool lvalid = loader && v0 + lk < n;
    const float* lp = v + (lvalid ? v0 + lk : 0) * D;
    uint8_t* lb = bins + (lvalid ? v0 + lk : 0) * D;
    if (tid < kNormClients) minpos[tid] = 0x7F800000u;                 // +inf
    constexpr int kLQ = kNormChunk / 256;
    float4 na[kLQ], nb[kLQ];
    uint32_t mymin = 0x7F800000u;                                      // bits of the smallest positive y
    auto load = [&](float4 (&nx)[kLQ], int64_t ch) {
        if (!lvalid || ch >= nchunks) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) nx[q] = ld_stream(reinterpret_cast<const float4*>(lp + ch * kNormChunk + 4 * (lj + 64 * q)));
    };
    // The bins of a chunk are computed when it is staged, kept in LDS (sbins, two chunks), and
    // written after the next barrier by the loaders as 16-byte non-temporal stores (a wave
    // writes 1 KB of one client's bins per instruction), issued after the next loads: vmcnt
    // retires in issue order, so a store issued just before a load would make the wait for
    // that load also wait for the store's acknowledgement.  (1-bit 1024 x 2^20 round trip:
    // dword stores before the loads 6.58 ms, after them 6.44 ms, profiles/r6c_ab_eden.jsonl;
    // no bins stores at all 6.08 ms, r6b_eden_ab.jsonl.)
    __shared__ __attribute__((aligned(16))) uint32_t sbins[2][kNormClients][kNormChunk / 4];
    auto store = [&](const float4 (&nx)[kLQ], float* sb, int64_t ch) {
        if (!loader) return;
#pragma unroll
        for (int q = 0; q < kLQ; ++q) {
            const int e = 4 * (lj + 64 * q);
            const int i = e >> 3, l = e & 7;
            float* base = sb + lk * kNormClientStride + i;
            base[(l + 0) * kNormRow] = nx[q].x;
            base[(l + 1) * kNormRow] = nx[q].y;
            base[(l + 2) * kNormRow] = nx[q].z;
            base[(l + 3) * kNormRow] = nx[q].w;
            const float xs[4] = {nx[q].x, nx[q].y, nx[q].z, nx[q].w};   // the bins of these 4 (sign rule)
            uint32_t w = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float y = xs[c] * sqrtD;
                w |= (!(y <= 0.f) ? 1u : 0u) << (8 * c);
                if (lvalid && y > 0.f) mymin = min(mymin, __float_as_uint(y));
            }
            sbins[ch & 1][lk][lj + 64 * q] = w;
        }
    };
    auto flush_bins = [&](int64_t ch) {          // chunk ch's bins, staged before the last barrier
        if (!lvalid) return;
        typedef uint32_t u32x4b __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int r = 0; r < kNormChunk / 4 / 256; ++r) {
            const int w0 = 4 * (lj + 64 * r);
            const u32x4b t = *reinterpret_cast<const u32x4b*>(&sbins[ch & 1][lk][w0]);
            __builtin_nontemporal_store(t, reinterpret_cast<u32x4b*>(lb + ch * kNormChunk + 4 * w0));
        }
    };
    const int ck = (tid >> 3) & (kNormClients - 1), cl = tid & 7;
    float acc = 0.f;
    const int dk = (tid - kWave - 256) >> 6, dl = tid & 63;           // dot wave: client dk, chain dl
    const EdenCents cs = eden_cents(tab);
    auto chainstep = [&](int64_t ch) {
        if (chain) {
            const float* row = s[ch % 3] + ck * kNormClientStride + cl * kNormRow;
            for (int i = 0; i < kNormChunk / 8; i += 16) {
                float4 t[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(row + i + 4 * u);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc = fmaf(t[u].x, t[u].x, acc);
                    acc = fmaf(t[u].y, t[u].y, acc);
                    acc = fmaf(t[u].z, t[u].z, acc);
                    acc = fmaf(t[u].w, t[u].w, acc);
                }
            }
        } else if (dotw) {
            // element 64 s + dl of the chunk sits at lane (dl % 8), step 8 s + dl / 8 of the image
            const float* row = s[ch % 3] + dk * kNormClientStride + (dl & 7) * kNormRow + (dl >> 3);
#pragma unroll 8
            for (int st = 0; st < kNormChunk / 64; ++st) {
                const float x = row[8 * st];
                const float c = !(x * sqrtD <= 0.f) ? cs.c1 : cs.c0;   // AS:335 take(centroids, bins)
                acc = fmaf(c, x, acc);
            }
        }
    };
    if (loader) {
        load(na, 0);
        store(na, s[0], 0);
        load(na, 1);
        load(nb, 2);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunks; ch += 2) {
        chainstep(ch);
        if (loader && ch + 1 < nchunks) {
            store(na, s[(ch + 1) % 3], ch + 1);
            load(na, ch + 3);
        }
        if (loader) flush_bins(ch);
        __syncthreads();
        if (ch + 1 >= nchunks) break;
        chainstep(ch + 1);
        if (loader && ch + 2 < nchunks) {
            store(nb, s[(ch + 2) % 3], ch + 2);
            load(nb, ch + 4);
        }
        if (loader) flush_bins(ch + 1);
        __syncthreads();
    }
    if (lvalid) atomicMin(&minpos[lk], mymin);
    if (dotw) dacc[dk][dl] = acc;
    float nv = 0.f;
    if (chain) {
        const int base = tid & ~7;
        float tot = __shfl(acc, base, kWave);
        for (int j = 1; j < 8; ++j) tot = tot + __shfl(acc, base + j, kWave);
        nv = sqrtf(tot);
        const int64_t vec = v0 + ck;
        if (tid < 8 * kNormClients && cl == 0 && vec < n) nrm[vec] = nv;
    }
    __syncthreads();
    if (chain && tid < 8 * kNormClients && cl == 0 && v0 + ck < n) {
        const int64_t vec = v0 + ck;
        const float* a = dacc[ck];
        float w[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) w[l] = (a[l] + a[16 + l]) + (a[32 + l] + a[48 + l]);
#pragma unroll
        for (int l = 0; l < 8; ++l) w[l] = w[l] + w[l + 8];
#pragma unroll
        for (int l = 0; l < 4; ++l) w[l] = w[l] + w[l + 4];
        const float dot = (w[0] + w[1]) + (w[2] + w[3]);
        scale[vec] = (nv * nv) / dot;                                  // AS:335 norm ** 2 / dot
        const float mp = __uint_as_float(minpos[ck]);
        const bool ok = nv > 0.f && nv < INFINITY && (mp == INFINITY || mp / nv > 0.f);
        redo[vec] = ok ? 0 : 1;
    }
}
