// Host check of the fast exact f32 division used on the GPU (uq_dme.hip div_rn):
// q64 = (double)a * RN64(1/(double)b); RN32(q64) unless q64 is within 2 ulp64 of an
// f32 rounding midpoint or outside the f32 normal range, where a / b is used.
// Compile: g++ -O2 -ffp-contract=off tools/divcheck.cpp -o /tmp/divcheck
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <random>
static inline bool uncertain(double q) {
    uint64_t b; std::memcpy(&b, &q, 8);
    uint32_t low = (uint32_t)b & 0x1FFFFFFFu;
    uint32_t dist = low > 0x10000000u ? low - 0x10000000u : 0x10000000u - low;
    double aq = std::fabs(q);
    return !(aq >= 0x1p-126 && aq < 0x1p127) || dist <= 2u;
}
static inline float div_rn(float a, float b, double rb, long* slow) {
    double q = (double)a * rb;
    if (uncertain(q)) { ++*slow; return a / b; }
    return (float)q;
}
int main() {
    std::mt19937_64 g(1);
    long bad = 0, slow = 0, n = 0;
    auto rf = [&](int emin, int emax) {
        uint32_t m = g() & 0x7FFFFF; int e = emin + (int)(g() % (uint64_t)(emax - emin + 1));
        uint32_t s = (g() & 1) << 31; uint32_t bits = s | ((uint32_t)(e + 127) << 23) | m; float f; std::memcpy(&f, &bits, 4); return f; };
    for (int rep = 0; rep < 4; ++rep) {
        for (long i = 0; i < 50000000; ++i) {
            float a, b;
            switch (i % 4) {
                case 0: a = rf(-20, 20); b = rf(-20, 20); break;          // generic
                case 1: a = rf(-126, 127); b = rf(-126, 127); break;      // full range
                case 2: a = rf(-3, 3); b = (float)(1 + (g() % 5000000)); break;  // x / L1-like, out / m-like
                default: { a = (float)(int)(g() % 3000000) * rf(-2, 2); b = rf(10, 24); }
            }
            if (i % 1000 == 7) { uint32_t t = g() & 0xFFFF; std::memcpy(&b, &t, 4); }   // subnormal divisors
            double rb = 1.0 / (double)b;
            float q = div_rn(a, b, rb, &slow), r = a / b;
            uint32_t x, y; std::memcpy(&x, &q, 4); std::memcpy(&y, &r, 4);
            if (x != y && !(std::isnan(q) && std::isnan(r))) { if (bad < 5) printf("BAD a=%a b=%a q=%a r=%a\n", a, b, q, r); ++bad; }
            ++n;
        }
    }
    printf("checked %ld, mismatches %ld, slow-path %ld (%.2e)\n", n, bad, slow, (double)slow / n);
    return bad != 0;
}
