/* CPU ORACLE (C) for the type-message codec "UQR1" -- test infrastructure only, never the
 * product path.  Restates, symbol for symbol and byte for byte, what the HIP codec kernels
 * (csrc/uq_codec_kernels.h) write, so tests can check GPU messages byte-identical and
 * decode messages independently.
 *
 * The reference has no wire format ("parity unpinned"); its output is
 * the dequantized vector of All_Schemes.py:640, out = L1 * sign(v) * k / m.  A client is
 * fully described by (L1, m, signed counts k), i.e. by the int8 type codes of codes.py
 * (code = k for sign(v) >= 0, ~k for sign(v) < 0).  This codec entropy-codes those codes:
 *
 *   symbol   s = 2k + neg   (exact mode: neg = sign(v) < 0, so -0.0 outputs round-trip)
 *            s = 2k + (neg && k > 0)   (value mode: the sign of a zero count is dropped;
 *                                        the decoded q equals the reference's values, with
 *                                        +0.0 where the reference has -0.0)
 *   model    per-client static frequencies, M = 2^12, from the client's symbol counts
 *   coder    rANS, 32-bit state, L = 2^16, 16-bit renormalisation words; W interleaved
 *            states (W = min(64, ceil(d/1024))), chunks of W x 1024 symbols; symbol i of a
 *            chunk belongs to lane i % W, step i / W.
 *
 * Message (little endian, sections 4-byte aligned):
 *   0  u32 magic "UQR1"       4  u16 version = 1, u16 flags (bit 0: exact zero signs)
 *   8  u64 d                  16 u64 m
 *   24 u32 L1 (f32 bits)      28 u16 nsym (= 2*kmax + 2), u8 prob_bits = 12, u8 lanes W
 *   32 u32 nchunks            36 u32 total bytes of the message
 *   40 u16 freq[nsym] (+ pad to 4)
 *      u32 words_end[nchunks] (cumulative 16-bit word counts)
 *      u32 state[nchunks][W]  (final encoder states = initial decoder states)
 *      u16 words[...]         (chunk 0's words, chunk 1's, ...; + pad to 4)
 * Word order inside a chunk: decoder step j reads the words of the lanes that renormalise
 * at step j, in ascending lane order, before step j+1's.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TC_MAGIC 0x31525155u /* "UQR1" */
#define TC_PROB_BITS 12
#define TC_M (1u << TC_PROB_BITS)
#define TC_L (1u << 16)
#define TC_STEPS 1024

static int tc_lanes(int64_t d) {
    int64_t w = (d + TC_STEPS - 1) / TC_STEPS;
    if (w < 1) w = 1;
    if (w > 64) w = 64;
    return (int)w;
}

static inline int code_sym(int8_t c, int exact) {
    const int k = c < 0 ? -(int)c - 1 : (int)c;
    const int neg = c < 0;
    return 2 * k + (exact ? neg : (neg && k > 0));
}
static inline int8_t sym_code(int s) {
    const int k = s >> 1;
    return (s & 1) ? (int8_t)(-k - 1) : (int8_t)k;
}

/* Quantized frequencies (sum M): f = max(1, cnt*M/d) for present symbols; a shortfall goes
 * to the most frequent symbol (lowest index on ties); an excess is taken from the most
 * frequent symbols in turn, never below 1. */
void uqc_normalize(const uint32_t* cnt, int nsym, uint64_t total, uint32_t* f) {
    int64_t sum = 0;
    for (int s = 0; s < nsym; ++s) {
        f[s] = cnt[s] ? (uint32_t)(((uint64_t)cnt[s] * TC_M) / total) : 0u;
        if (cnt[s] && f[s] == 0u) f[s] = 1u;
        sum += f[s];
    }
    if (sum == 0) return;
    while (sum != (int64_t)TC_M) {
        int best = 0;
        for (int s = 1; s < nsym; ++s)
            if (f[s] > f[best]) best = s;
        if (sum < (int64_t)TC_M) {
            f[best] += (uint32_t)((int64_t)TC_M - sum);
            sum = TC_M;
        } else {
            int64_t dec = sum - (int64_t)TC_M;
            if (dec > (int64_t)f[best] - 1) dec = (int64_t)f[best] - 1;
            f[best] -= (uint32_t)dec;
            sum -= dec;
        }
    }
}

static inline uint64_t align4(uint64_t x) { return (x + 3u) & ~(uint64_t)3u; }

/* Header bytes before the words (also where the words start). */
uint64_t uqc_header_bytes(int nsym, int64_t nchunks, int lanes) {
    return align4(40 + 2 * (uint64_t)nsym) + 4 * (uint64_t)nchunks + 4 * (uint64_t)nchunks * lanes;
}

/* Upper bound of one message: every symbol emits at most one word. */
uint64_t uqc_bound(int64_t d) {
    const int W = tc_lanes(d);
    const int64_t nch = d > 0 ? (d + (int64_t)W * TC_STEPS - 1) / ((int64_t)W * TC_STEPS) : 0;
    return uqc_header_bytes(256, nch, W) + align4(2 * (uint64_t)d);
}

/* Encode one client.  Returns the message size, or 0 on a bad argument. */
uint64_t uqc_encode(const int8_t* codes, int64_t d, int64_t m, float l1, int exact, uint8_t* out) {
    uint32_t cnt[256] = {0}, f[256] = {0}, cum[257] = {0};
    int kmax = 0;
    for (int64_t i = 0; i < d; ++i) {
        const int k = codes[i] < 0 ? -(int)codes[i] - 1 : (int)codes[i];
        if (k > kmax) kmax = k;
        cnt[code_sym(codes[i], exact)]++;
    }
    const int nsym = d > 0 ? 2 * kmax + 2 : 0;
    if (d > 0) uqc_normalize(cnt, nsym, (uint64_t)d, f);
    for (int s = 0; s < nsym; ++s) cum[s + 1] = cum[s] + f[s];
    const int W = tc_lanes(d);
    const int64_t csz = (int64_t)W * TC_STEPS;
    const int64_t nch = d > 0 ? (d + csz - 1) / csz : 0;
    const uint64_t hdr = uqc_header_bytes(nsym, nch, W);
    uint32_t* wend = (uint32_t*)(out + align4(40 + 2 * (uint64_t)nsym));
    uint32_t* states = wend + nch;
    uint16_t* words = (uint16_t*)(out + hdr);
    uint16_t* tmp = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(csz > 0 ? csz : 1));
    uint64_t nw = 0;
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t base = c * csz;
        const int64_t len = d - base < csz ? d - base : csz;
        const int64_t steps = (len + W - 1) / W;
        uint32_t x[64];
        for (int l = 0; l < W; ++l) x[l] = TC_L;
        int64_t ptr = csz;                      /* stack of this chunk's words, grows down */
        for (int64_t st = steps - 1; st >= 0; --st) {
            int need[64], nneed = 0;
            int sy[64];
            for (int l = 0; l < W; ++l) {
                const int64_t i = st * W + l;
                need[l] = 0;
                if (i >= len) continue;
                sy[l] = code_sym(codes[base + i], exact);
                const uint64_t xmax = ((uint64_t)(TC_L >> TC_PROB_BITS) << 16) * f[sy[l]];
                if ((uint64_t)x[l] >= xmax) {
                    need[l] = 1;
                    ++nneed;
                }
            }
            int r = 0;
            for (int l = 0; l < W; ++l) {
                if (!need[l]) continue;
                tmp[ptr - nneed + r] = (uint16_t)(x[l] & 0xFFFFu);
                x[l] >>= 16;
                ++r;
            }
            ptr -= nneed;
            for (int l = 0; l < W; ++l) {
                const int64_t i = st * W + l;
                if (i >= len) continue;
                const uint32_t fs = f[sy[l]];
                x[l] = ((x[l] / fs) << TC_PROB_BITS) + (x[l] % fs) + cum[sy[l]];
            }
        }
        const uint64_t cw = (uint64_t)(csz - ptr);
        memcpy(words + nw, tmp + ptr, cw * sizeof(uint16_t));
        nw += cw;
        wend[c] = (uint32_t)nw;
        for (int l = 0; l < W; ++l) states[c * W + l] = x[l];
    }
    free(tmp);
    const uint64_t total = hdr + align4(2 * nw);
    if (2 * nw < align4(2 * nw)) words[nw] = 0;    /* padding */
    uint32_t u32;
    u32 = TC_MAGIC; memcpy(out + 0, &u32, 4);
    uint16_t u16 = 1; memcpy(out + 4, &u16, 2);
    u16 = (uint16_t)(exact ? 1 : 0); memcpy(out + 6, &u16, 2);
    uint64_t u64 = (uint64_t)d; memcpy(out + 8, &u64, 8);
    u64 = (uint64_t)m; memcpy(out + 16, &u64, 8);
    memcpy(out + 24, &l1, 4);
    u16 = (uint16_t)nsym; memcpy(out + 28, &u16, 2);
    out[30] = TC_PROB_BITS;
    out[31] = (uint8_t)W;
    u32 = (uint32_t)nch; memcpy(out + 32, &u32, 4);
    u32 = (uint32_t)total; memcpy(out + 36, &u32, 4);
    for (int s = 0; s < nsym; ++s) { u16 = (uint16_t)f[s]; memcpy(out + 40 + 2 * s, &u16, 2); }
    if (nsym & 1) memset(out + 40 + 2 * nsym, 0, 2);
    return total;
}

/* Decode one client.  Returns 0, or a negative value for a malformed message. */
int uqc_decode(const uint8_t* msg, uint64_t size, int8_t* codes, int64_t d_expect, float* l1, int64_t* m) {
    uint32_t magic, nch, total;
    uint16_t ver, flags, nsym;
    uint64_t d, mm;
    if (size < 40) return -1;
    memcpy(&magic, msg, 4); memcpy(&ver, msg + 4, 2); memcpy(&flags, msg + 6, 2);
    memcpy(&d, msg + 8, 8); memcpy(&mm, msg + 16, 8); memcpy(l1, msg + 24, 4);
    memcpy(&nsym, msg + 28, 2); memcpy(&nch, msg + 32, 4); memcpy(&total, msg + 36, 4);
    const int W = msg[31];
    (void)flags;
    if (magic != TC_MAGIC || ver != 1 || msg[30] != TC_PROB_BITS || (int64_t)d != d_expect || total != size) return -1;
    if (W != tc_lanes((int64_t)d) || nsym > 256) return -1;
    *m = (int64_t)mm;
    uint32_t f[256] = {0}, cum[257] = {0};
    for (int s = 0; s < nsym; ++s) {
        uint16_t t;
        memcpy(&t, msg + 40 + 2 * s, 2);
        f[s] = t;
        cum[s + 1] = cum[s] + f[s];
    }
    if (d > 0 && cum[nsym] != TC_M) return -2;
    uint8_t lut[TC_M];
    for (int s = 0; s < nsym; ++s)
        for (uint32_t j = cum[s]; j < cum[s + 1]; ++j) lut[j] = (uint8_t)s;
    const uint32_t* wend = (const uint32_t*)(msg + align4(40 + 2 * (uint64_t)nsym));
    const uint32_t* states = wend + nch;
    const uint16_t* words = (const uint16_t*)(msg + uqc_header_bytes(nsym, nch, W));
    const int64_t csz = (int64_t)W * TC_STEPS;
    for (int64_t c = 0; c < (int64_t)nch; ++c) {
        const int64_t base = c * csz;
        const int64_t len = (int64_t)d - base < csz ? (int64_t)d - base : csz;
        const int64_t steps = (len + W - 1) / W;
        uint64_t r = c ? wend[c - 1] : 0;
        uint32_t x[64];
        for (int l = 0; l < W; ++l) x[l] = states[c * W + l];
        for (int64_t st = 0; st < steps; ++st) {
            for (int l = 0; l < W; ++l) {
                const int64_t i = st * W + l;
                if (i >= len) continue;
                const uint32_t slot = x[l] & (TC_M - 1);
                const int s = lut[slot];
                x[l] = f[s] * (x[l] >> TC_PROB_BITS) + slot - cum[s];
                codes[base + i] = sym_code(s);
            }
            for (int l = 0; l < W; ++l) {
                const int64_t i = st * W + l;
                if (i >= len || x[l] >= TC_L) continue;
                if (r >= wend[c]) return -3;
                x[l] = (x[l] << 16) | words[r++];
            }
        }
        if (r != wend[c]) return -3;
        for (int l = 0; l < W; ++l)
            if (x[l] != TC_L) return -4;
    }
    return 0;
}
