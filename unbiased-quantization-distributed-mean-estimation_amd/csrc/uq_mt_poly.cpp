// uq_mt_poly.cpp — host side of the MT19937 jump-ahead behind the QUIC-FL sender's jump path
// (uq_quicfl_kernels.h, KQ0j / KQ1j).  Plain C++ (g++), linked into libuq_dme.so.
//
// Why: QuicFLSender.compress (All_Schemes.py:455-490) draws h and bernoulli(p) from a local
// torch generator and bernoulli(p_X) from the global one: three MT19937 streams of D words
// each, serial by construction (a 624-word block is twisted from the previous one).  The
// state transition F of MT19937 is linear over GF(2) on its 19937-bit state, so the state J
// steps ahead is g(F) s with g = t^J mod phi, phi the characteristic polynomial of F
// (degree 19937, primitive).  In the sliding-window form x[k .. k+623] of the word sequence,
// state_k is window k, so window J = XOR over the set coefficients g_k of window k: a
// correlation of g with the first 19937 + 623 words of the stream, which the GPU computes
// (KQ0j).  This file supplies g:
//   * phi: Berlekamp-Massey over GF(2) on bit 0 of 2 * 19937 + 64 successive MT19937 words
//     (the minimal polynomial of any nonzero linear output sequence of a primitive
//     recurrence is its characteristic polynomial; the degree is checked);
//   * residues mod phi as 312 u64 words (bit k = coefficient of t^k); products by carry-less
//     multiplication (PCLMULQDQ when the CPU has it, a portable shift-and-xor otherwise) and
//     Barrett reduction one 64-bit chunk at a time (mu = floor(t^(19937+64) / phi));
//   * P_b = t^(624 b) mod phi (window 624 b = block b of the stream) from a table of
//     t^(624 * 2^i) by squaring, and arithmetic progressions of b by one product per term.
// Everything is computed once per process and cached (thread-safe).
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>
#include <wmmintrin.h>

namespace {

constexpr int kDeg = 19937;       // degree of phi
constexpr int kW = 312;           // u64 words per residue (19968 bits)
constexpr int kMtN = 624;

struct Poly {
    uint64_t w[kW];
};

// ---- host MT19937 (ATen / init_genrand), untempered words -------------------------------
struct HostMt {
    uint32_t s[kMtN];
    explicit HostMt(uint32_t seed) {
        s[0] = seed;
        for (int i = 1; i < kMtN; ++i) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
    }
    void twist() {
        for (int i = 0; i < kMtN; ++i) {
            const uint32_t y = (s[i] & 0x80000000u) | (s[(i + 1) % kMtN] & 0x7FFFFFFFu);
            s[i] = s[(i + 397) % kMtN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
        }
    }
};

inline uint64_t extract64(const std::vector<uint64_t>& v, int64_t pos) {   // bits [pos, pos + 64)
    const int64_t q = pos >> 6;
    const int sh = (int)(pos & 63);
    const uint64_t lo = q < (int64_t)v.size() ? v[q] : 0;
    if (!sh) return lo;
    const uint64_t hi = q + 1 < (int64_t)v.size() ? v[q + 1] : 0;
    return (lo >> sh) | (hi << (64 - sh));
}

// ---- carry-less products ------------------------------------------------------------------
__attribute__((target("pclmul"))) void prod_clmul(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    std::memset(r, 0, sizeof(uint64_t) * (2 * kW + 2));
    for (int i = 0; i < kW; ++i) {
        if (!a[i]) continue;
        const __m128i ai = _mm_set_epi64x(0, (long long)a[i]);
        for (int j = 0; j < kW; j += 2) {
            const __m128i bj = _mm_set_epi64x((long long)b[j + 1], (long long)b[j]);
            const __m128i p0 = _mm_clmulepi64_si128(ai, bj, 0x00);
            const __m128i p1 = _mm_clmulepi64_si128(ai, bj, 0x10);
            r[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p0);
            r[i + j + 1] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p0, p0)) ^ (uint64_t)_mm_cvtsi128_si64(p1);
            r[i + j + 2] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p1, p1));
        }
    }
}

inline void clmul64_soft(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    while (b) {
        const int i = __builtin_ctzll(b);
        b &= b - 1;
        lo ^= a << i;
        if (i) hi ^= a >> (64 - i);
    }
}

void prod_soft(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    std::memset(r, 0, sizeof(uint64_t) * (2 * kW + 2));
    for (int i = 0; i < kW; ++i) {
        if (!a[i]) continue;
        for (int j = 0; j < kW; ++j) {
            uint64_t lo, hi;
            clmul64_soft(a[i], b[j], lo, hi);
            r[i + j] ^= lo;
            r[i + j + 1] ^= hi;
        }
    }
}

__attribute__((target("pclmul"))) inline void clmul64_hw(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
    const __m128i p = _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)a), _mm_set_epi64x(0, (long long)b), 0x00);
    lo = (uint64_t)_mm_cvtsi128_si64(p);
    hi = (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p, p));
}

// acc[w] ^= x[k + w] for every set coefficient k of g: the jump's correlation (AVX2 where the
// CPU has it: 624 words are 78 ymm XORs per coefficient, ~10^4 coefficients per jump)
__attribute__((target_clones("avx2", "default"))) void correlate(const uint64_t* g, const uint32_t* x,
                                                                 uint32_t* acc) {
    for (int k = 0; k < kDeg; ++k)
        if ((g[k >> 6] >> (k & 63)) & 1u) {
            const uint32_t* xk = x + k;
            for (int w = 0; w < kMtN; ++w) acc[w] ^= xk[w];
        }
}

class MtPoly {
  public:
    static MtPoly& get() {
        static MtPoly inst;
        return inst;
    }
    bool ok() const { return ok_; }

    // out[c] = t^(624 (b0 + c * step)) mod phi, c < count, as 624 u32 words each
    void progression(int64_t b0, int64_t step, int count, uint32_t* out) {
        std::lock_guard<std::mutex> g(mu_);
        if (count <= 0) return;
        Poly cur = pow_blocks(b0);
        const Poly st = pow_blocks(step);
        for (int c = 0; c < count; ++c) {
            if (c) cur = mulmod(cur, st);
            std::memcpy(out + (size_t)c * kMtN, cur.w, sizeof(cur.w));
        }
    }

    // the state (624 words, block-aligned) b blocks ahead, entirely on the host: the same
    // correlation the GPU's KQ0j computes (the CPU tests check it against direct twisting)
    void jump_host(const uint32_t* st, int64_t b, uint32_t* out) {
        if (b == 0) {
            std::memcpy(out, st, kMtN * 4);
            return;
        }
        Poly g;
        {
            std::lock_guard<std::mutex> lk(mu_);
            g = pow_blocks(b - 1);
        }
        // x[0 .. 33 * 624): the stream's first words from the base block
        std::vector<uint32_t> x((size_t)33 * kMtN);
        HostMt m(0);
        std::memcpy(m.s, st, kMtN * 4);
        std::memcpy(x.data(), m.s, kMtN * 4);
        for (int blk = 1; blk < 33; ++blk) {
            m.twist();
            std::memcpy(x.data() + (size_t)blk * kMtN, m.s, kMtN * 4);
        }
        uint32_t acc[kMtN] = {};
        correlate(g.w, x.data(), acc);
        std::memcpy(m.s, acc, sizeof(acc));           // block b - 1 (word 0's low 31 bits aside)
        m.twist();                                    // block b: every word exact
        std::memcpy(out, m.s, kMtN * 4);
    }

  private:
    MtPoly() {
        hw_ = __builtin_cpu_supports("pclmul");
        ok_ = find_phi();
        if (!ok_) return;
        // mu = floor(t^(kDeg + 64) / phi): degree 64, the t^64 term implicit
        std::vector<uint64_t> rem(kW + 2, 0);
        rem[(kDeg + 64) >> 6] |= 1ull << ((kDeg + 64) & 63);
        uint64_t q = 0;
        for (int p = kDeg + 64; p >= kDeg; --p) {
            if (!((rem[p >> 6] >> (p & 63)) & 1u)) continue;
            if (p - kDeg < 64) q |= 1ull << (p - kDeg);
            xor_shifted_phi(rem.data(), p - kDeg);
        }
        mu_lo_ = q;
        Poly t624{};
        t624.w[kMtN >> 6] = 1ull << (kMtN & 63);     // t^624 (below the degree: reduced)
        pow2_.push_back(t624);
    }

    void xor_shifted_phi(uint64_t* r, int sh) {       // r ^= phi * t^sh
        const int q = sh >> 6, b = sh & 63;
        for (int i = 0; i <= kW; ++i) {
            const uint64_t v = phi_[i];
            if (!v) continue;
            r[q + i] ^= v << b;
            if (b) r[q + i + 1] ^= v >> (64 - b);
        }
    }

    bool find_phi() {
        const int N = 2 * kDeg + 64;
        std::vector<uint8_t> s(N);
        HostMt m(5489u);
        int t = 0;
        while (t < N) {
            m.twist();
            for (int i = 0; i < kMtN && t < N; ++i) s[t++] = m.s[i] & 1u;
        }
        const int RW = (N + 63) / 64 + 2;
        std::vector<uint64_t> rv(RW, 0);               // rv bit i = s[N - 1 - i]
        for (int i = 0; i < N; ++i)
            if (s[N - 1 - i]) rv[i >> 6] |= 1ull << (i & 63);
        const int CW = kW + 4;
        std::vector<uint64_t> C(CW, 0), B(CW, 0), T(CW, 0);
        C[0] = B[0] = 1;
        int L = 0, mm = 1;
        for (int n = 0; n < N; ++n) {
            // discrepancy: sum_{i=0..L} C_i s[n - i] = sum_i C_i rv[N - 1 - n + i]
            const int64_t off = (int64_t)N - 1 - n;
            uint64_t acc = 0;
            for (int wi = 0; wi <= (L >> 6) && wi < CW; ++wi) acc ^= C[wi] & extract64(rv, off + 64 * wi);
            if (!(__builtin_popcountll(acc) & 1)) {
                ++mm;
                continue;
            }
            const bool grow = 2 * L <= n;
            if (grow) T = C;
            const int q = mm >> 6, b = mm & 63;        // C ^= t^mm B
            for (int i = CW - 1; i >= 0; --i) {
                uint64_t v = 0;
                if (i - q >= 0) v = B[i - q] << b;
                if (b && i - q - 1 >= 0) v |= B[i - q - 1] >> (64 - b);
                C[i] ^= v;
            }
            if (grow) {
                L = n + 1 - L;
                B = T;
                mm = 1;
            } else {
                ++mm;
            }
        }
        if (L != kDeg) return false;
        std::memset(phi_, 0, sizeof(phi_));
        for (int k = 0; k <= kDeg; ++k) {              // phi_k = C_{L - k}
            const int i = kDeg - k;
            if ((C[i >> 6] >> (i & 63)) & 1u) phi_[k >> 6] |= 1ull << (k & 63);
        }
        return (phi_[kDeg >> 6] >> (kDeg & 63)) & 1u;
    }

    Poly mulmod(const Poly& a, const Poly& b) {
        uint64_t r[2 * kW + 2];
        if (hw_) prod_clmul(a.w, b.w, r);
        else prod_soft(a.w, b.w, r);
        // Barrett, top chunk first: bits [kDeg + 64 k, + 64) cancelled by q * phi * t^(64 k),
        // q = floor(C * mu / t^64) = hi(C * mu_lo) ^ C
        for (int k = (2 * kDeg - 2 - kDeg) / 64; k >= 0; --k) {
            const int64_t pos = kDeg + 64 * (int64_t)k;
            const int qw = (int)(pos >> 6), sh = (int)(pos & 63);
            const uint64_t c = (r[qw] >> sh) | (sh ? r[qw + 1] << (64 - sh) : 0);
            if (!c) continue;
            uint64_t lo, hi;
            if (hw_) clmul64_hw(c, mu_lo_, lo, hi);
            else clmul64_soft(c, mu_lo_, lo, hi);
            const uint64_t q = hi ^ c;
            for (int i = 0; i <= kDeg / 64; ++i) {
                if (!phi_[i]) continue;
                if (hw_) clmul64_hw(q, phi_[i], lo, hi);
                else clmul64_soft(q, phi_[i], lo, hi);
                r[k + i] ^= lo;
                r[k + i + 1] ^= hi;
            }
        }
        Poly out;
        std::memcpy(out.w, r, sizeof(out.w));
        return out;
    }

    Poly pow_blocks(int64_t b) {                       // t^(624 b) mod phi
        auto it = cache_.find(b);
        if (it != cache_.end()) return it->second;
        Poly r{};
        r.w[0] = 1;
        bool one = true;
        for (int i = 0; (b >> i) != 0; ++i) {
            while ((int)pow2_.size() <= i) pow2_.push_back(mulmod(pow2_.back(), pow2_.back()));
            if (!((b >> i) & 1)) continue;
            r = one ? pow2_[i] : mulmod(r, pow2_[i]);
            one = false;
        }
        if (cache_.size() < 4096) cache_.emplace(b, r);
        return r;
    }

    std::mutex mu_;
    bool ok_ = false, hw_ = false;
    uint64_t phi_[kW + 1];
    uint64_t mu_lo_ = 0;
    std::vector<Poly> pow2_;                           // t^(624 * 2^i) mod phi
    std::unordered_map<int64_t, Poly> cache_;
};

}  // namespace

// Internal entry points (declared in uq_dme.hip; uq_mt_jump_host is also in include/uq_dme.h).
extern "C" int uq_mtpoly_progression(int64_t b0, int64_t step, int32_t count, uint32_t* out) {
    MtPoly& m = MtPoly::get();
    if (!m.ok() || b0 < 0 || step < 0 || count < 0 || !out) return -1;
    m.progression(b0, step, count, out);
    return 0;
}

extern "C" int uq_mt_jump_host(const uint32_t* state624, int64_t blocks, uint32_t* out624) {
    MtPoly& m = MtPoly::get();
    if (!m.ok() || blocks < 0 || !state624 || !out624) return -1;
    m.jump_host(state624, blocks, out624);
    return 0;
}
