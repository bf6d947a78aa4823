/* CPU ORACLE (C) — test infrastructure only, never the product path.
 *
 * Same restatement as oracle/uq_oracle.py, in plain C so the checker and the
 * bench's cpu_baseline leg run at d = 2^20 in reasonable time.  Built by
 * oracle/Makefile with -O2 -ffp-contract=off (no FMA contraction, IEEE f32
 * division, denormals kept), loaded through ctypes by tests/ and bench.py only.
 *
 * Reference semantics followed (paths relative to the reference root):
 *   NMSE_Results/Codes/All_Schemes.py:609-641  Type_unbiased_quantize
 *     :624  L1 = |x|.sum()  -> torch CPU cascade order (ATen SumKernel)
 *     :625-631 den, v, p, mp, floor, frac           (f32, IEEE)
 *     :635  cumsum(frac) -> sequential fp64 accumulate, each prefix -> f32
 *     :636-637 crossing test, :640 output
 *   NMSE_Results/Codes/Normal_dist.py:137-138  est += q / n
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TORCH_GRAIN 32768
#define VEC_LANES 8
#define ILP 4
#define NUM_LEVELS 4

static int ceil_log2_i64(int64_t x) {
    if (x <= 1) return 0;
    int r = 0;
    uint64_t v = (uint64_t)(x - 1);
    while (v) { r++; v >>= 1; }
    return r;
}

/* ATen multi_row_sum over R rows of width W (row stride W), f32 accumulate. */
static void cascade(const float* a, int64_t R, int W, float* out) {
    int lp = ceil_log2_i64(R) / NUM_LEVELS;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp;
    const int64_t mask = step - 1;
    float acc[NUM_LEVELS][VEC_LANES * ILP];
    memset(acc, 0, sizeof(acc));
    int64_t i = 0;
    for (; i + step <= R;) {
        for (int64_t j = 0; j < step; ++j, ++i)
            for (int k = 0; k < W; ++k) acc[0][k] += a[i * W + k];
        for (int j = 1; j < NUM_LEVELS; ++j) {
            for (int k = 0; k < W; ++k) { acc[j][k] += acc[j - 1][k]; acc[j - 1][k] = 0.0f; }
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < R; ++i)
        for (int k = 0; k < W; ++k) acc[0][k] += a[i * W + k];
    for (int j = 1; j < NUM_LEVELS; ++j)
        for (int k = 0; k < W; ++k) acc[0][k] += acc[j][k];
    for (int k = 0; k < W; ++k) out[k] = acc[0][k];
}

static float row_sum_scalar(const float* x, int64_t s) {
    int64_t nilp = s / ILP;
    float p[ILP] = {0, 0, 0, 0};
    if (nilp) cascade(x, nilp, ILP, p);
    for (int64_t k = nilp * ILP; k < s; ++k) p[0] += x[k];
    for (int k = 1; k < ILP; ++k) p[0] += p[k];
    return p[0];
}

static float chunk_sum(const float* x, int64_t s) {
    if (s < VEC_LANES) return row_sum_scalar(x, s);
    int64_t vs = s / VEC_LANES, nilp = vs / ILP;
    float p[ILP * VEC_LANES];
    memset(p, 0, sizeof(p));
    if (nilp) cascade(x, nilp, ILP * VEC_LANES, p);
    float p0[VEC_LANES];
    for (int l = 0; l < VEC_LANES; ++l) p0[l] = p[l];
    for (int64_t v = nilp * ILP; v < vs; ++v)
        for (int l = 0; l < VEC_LANES; ++l) p0[l] += x[v * VEC_LANES + l];
    for (int k = 1; k < ILP; ++k)
        for (int l = 0; l < VEC_LANES; ++l) p0[l] += p[k * VEC_LANES + l];
    float acc = 0.0f;
    for (int64_t k = vs * VEC_LANES; k < s; ++k) acc += x[k];
    for (int l = 0; l < VEC_LANES; ++l) acc += p0[l];
    return acc;
}

/* torch CPU f32 `sum` of a contiguous vector for `torch_threads` intra-op threads
 * (ATen TensorIteratorBase::parallel_reduce).  d < GRAIN or T == 1: one cascade.
 * Otherwise two_pass_reduction: nt = min(T, ceil(d/GRAIN)) chunks of ceil(d/nt)
 * (invoke_parallel), thread t adds its chunk's cascade sum into buffer[t] of a T-element
 * zero buffer, and the result is 0 + the cascade sum of that buffer (checked against
 * torch 2.10 for T = 1..39, 47, 63..65, 96, 128, 200, 256; the chunk sums are NOT added
 * sequentially unless T is 1, 2, 3, 4 or 8). */
float uqo_torch_sum(const float* v, int64_t d, int torch_threads) {
    if (d <= 0) return 0.0f;
    int T = torch_threads < 1 ? 1 : torch_threads;
    if (d < TORCH_GRAIN || T == 1) return 0.0f + chunk_sum(v, d);
    int64_t nt = (d + TORCH_GRAIN - 1) / TORCH_GRAIN;
    if (nt > T) nt = T;
    int64_t cs = (d + nt - 1) / nt;
    float* buf = (float*)calloc((size_t)T, sizeof(float));
    if (!buf) return NAN;
    for (int64_t c = 0; c < nt; ++c) {
        int64_t b = c * cs, e = b + cs < d ? b + cs : d;
        if (e > b) buf[c] = 0.0f + chunk_sum(v + b, e - b);
    }
    float r = 0.0f + chunk_sum(buf, T);
    free(buf);
    return r;
}

/* |x| into scratch, then torch's chunking by intra-op thread count. */
float uqo_l1_torch_order(const float* x, int64_t d, int torch_threads, float* scratch) {
    if (d <= 0) return 0.0f;
    for (int64_t i = 0; i < d; ++i) scratch[i] = fabsf(x[i]);
    return uqo_torch_sum(scratch, d, torch_threads);
}

static inline float torch_sign(float v) {
    if (v > 0.0f) return 1.0f;
    if (v < 0.0f) return -1.0f;
    return 0.0f;  /* +-0 -> +0, NaN -> 0 */
}

/* One client vector.  l1 < 0 (or NaN-safe flag use_l1=0) -> compute. */
float uqo_quantize(const float* x, float* out, int64_t d, int64_t m, float X,
                   int torch_threads, int use_l1, float l1_in, float* scratch) {
    float L = use_l1 ? l1_in : uqo_l1_torch_order(x, d, torch_threads, scratch);
    const float den = L + 1e-12f;
    const float fm = (float)m;
    double acc = 0.0;
    float c_prev = 0.0f;
    for (int64_t i = 0; i < d; ++i) {
        float v = x[i] / den;
        float p = fabsf(v);
        float mp = fm * p;
        float fl = floorf(mp);
        float fr = mp - fl;
        acc += (double)fr;
        float c = (float)acc;
        float diff = floorf(c - X) - floorf(c_prev - X);
        float r = (diff == 1.0f) ? 1.0f : 0.0f;
        float t = (L * torch_sign(v)) * (fl + r);
        out[i] = t / fm;
        c_prev = c;
    }
    return L;
}

void uqo_quantize_batch(const float* x, float* out, int64_t n, int64_t d, int64_t m,
                        const float* X, int torch_threads, float* l1_out, float* scratch) {
    for (int64_t j = 0; j < n; ++j) {
        float L = uqo_quantize(x + j * d, out + j * d, d, m, X[j], torch_threads, 0, 0.0f, scratch);
        if (l1_out) l1_out[j] = L;
    }
}

/* The same batch with clients spread over `nthreads` OpenMP threads (each client is
 * independent, AS:609-641): the all-cores CPU baseline.  Returns the threads used. */
int uqo_quantize_batch_mt(const float* x, float* out, int64_t n, int64_t d, int64_t m,
                          const float* X, int torch_threads, float* l1_out, int nthreads) {
    int used = 1;
#pragma omp parallel num_threads(nthreads)
    {
#pragma omp single
        used = omp_get_num_threads();
        float* scratch = (float*)malloc((size_t)(d > 0 ? d : 1) * sizeof(float));
#pragma omp for schedule(dynamic, 1)
        for (int64_t j = 0; j < n; ++j) {
            float L = uqo_quantize(x + j * d, out + j * d, d, m, X[j], torch_threads, 0, 0.0f, scratch);
            if (l1_out) l1_out[j] = L;
        }
        free(scratch);
    }
    return used;
}

/* Normal_dist.py:137 — est += q / n, client order, f32. */
void uqo_client_mean(const float* q, int64_t n, int64_t d, float n_div, float* est) {
    for (int64_t i = 0; i < d; ++i) est[i] = 0.0f;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < d; ++i) est[i] += q[j * d + i] / n_div;
}

/* The same sum continued from est (clients fed in order over several calls: one call over
 * all of them gives the same bits). */
void uqo_client_mean_acc(const float* q, int64_t n, int64_t d, float n_div, float* est) {
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < d; ++i) est[i] += q[j * d + i] / n_div;
}

/* torch.norm(v, 2) on CPU f32, the EDEN sender's norm (NMSE_Results/Codes/All_Schemes.py:329):
 * 8 lanes of fma chains over the first d - d % 8 elements, lanes added in order, the tail
 * as f32 v*v adds, sqrt.  The C form of oracle/uq_eden.py:torch_norm2 (pinned there against
 * torch; tests/test_oracle_golden.py checks both against torch.norm). */
float uqo_torch_norm2(const float* v, int64_t d) {
    float acc[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    const int64_t nv = d - d % 8;
    for (int64_t i = 0; i < nv; i += 8)
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(v[i + l], v[i + l], acc[l]);
    float s = acc[0];
    for (int l = 1; l < 8; ++l) s = s + acc[l];
    /* below one 8-wide vector torch takes other paths (measured, torch 2.10): |x| for one
     * element, fma for two, mul + add for four; ragged tails after whole vectors are not
     * pinned (EDEN's D is a power of two) */
    if (d == 1) return fabsf(v[0]);
    if (d == 2) return sqrtf(fmaf(v[1], v[1], fmaf(v[0], v[0], 0.0f)));
    for (int64_t i = nv; i < d; ++i) {
        const float p = v[i] * v[i];
        s = s + p;
    }
    return sqrtf(s);
}

/* torch.dot(x, y) on CPU f32 (All_Schemes.py:335, EDEN's scale), MKL's sdot on the fixtures'
 * host (oracle/uq_eden.py:torch_dot, tools/dot_order_probe.py): 4 accumulators x 16 lanes over
 * 64-element blocks, fma chains; of the remainder, a 32-element block into accumulators 0
 * and 1, then 16-element chunks into accumulator 0 (the last one masked: lanes beyond n add
 * 0 * 0); (acc0 + acc1) + (acc2 + acc3) lane-wise; lanes i + (i + 8), i + (i + 4), then
 * (0 + 1) + (2 + 3). */
float uqo_torch_dot(const float* x, const float* y, int64_t n) {
    float acc[64];
    for (int l = 0; l < 64; ++l) acc[l] = 0.0f;
    const int64_t nb = n / 64;
    for (int64_t b = 0; b < nb; ++b)
        for (int l = 0; l < 64; ++l) acc[l] = fmaf(x[64 * b + l], y[64 * b + l], acc[l]);
    int64_t i0 = nb * 64;
    if (n - i0 >= 32) {                          /* a 32-element block: accumulators 0 and 1 */
        for (int l = 0; l < 32; ++l) acc[l] = fmaf(x[i0 + l], y[i0 + l], acc[l]);
        i0 += 32;
    }
    for (; i0 < n; i0 += 16)                     /* 16-element chunks, the last masked: acc 0 */
        for (int l = 0; l < 16; ++l)
            acc[l] = i0 + l < n ? fmaf(x[i0 + l], y[i0 + l], acc[l]) : fmaf(0.0f, 0.0f, acc[l]);
    float v[16];
    for (int l = 0; l < 16; ++l) v[l] = (acc[l] + acc[16 + l]) + (acc[32 + l] + acc[48 + l]);
    for (int l = 0; l < 8; ++l) v[l] = v[l] + v[l + 8];
    for (int l = 0; l < 4; ++l) v[l] = v[l] + v[l + 4];
    return (v[0] + v[1]) + (v[2] + v[3]);
}
