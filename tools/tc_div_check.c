/* The encoder's x / f (csrc/uq_codec_kernels.h tc_div: Granlund & Montgomery 1994, fig. 4.1)
 * against C's unsigned division, for every f = 1..4096, on x sampled densely across [0, 2^32)
 * plus every x within 2 of a multiple of f near the top and 2^32 - 1 (the theorem covers all x).
 *     gcc -O2 -o /tmp/tc_div_check tools/tc_div_check.c && /tmp/tc_div_check */
#include <stdint.h>
#include <stdio.h>

static uint32_t tc_div(uint32_t x, uint32_t f) {
    int l = 0;
    while (l < 31 && (1u << l) < f) ++l;
    const uint32_t mg = (uint32_t)((((uint64_t)((1u << l) - f)) << 32) / f + 1u);
    const uint32_t s1 = l < 1 ? (uint32_t)l : 1u, s2 = l > 1 ? (uint32_t)(l - 1) : 0u;
    const uint32_t t = (uint32_t)(((uint64_t)mg * x) >> 32);
    return (t + ((x - t) >> s1)) >> s2;
}

int main(void) {
    uint64_t bad = 0, n = 0;
    for (uint32_t f = 1; f <= 4096; ++f) {
        for (uint64_t x = 0; x < (1ull << 32); x += (f < 64 ? 9973 : 99991))
            for (int dd = -2; dd <= 2; ++dd) {
                const uint32_t y = (uint32_t)x + (uint32_t)dd;
                ++n;
                bad += tc_div(y, f) != y / f;
            }
        const uint32_t q = 0xFFFFFFFFu / f;
        for (int dd = -2; dd <= 2; ++dd) {
            const uint32_t y = q * f + (uint32_t)dd;
            ++n;
            bad += tc_div(y, f) != y / f;
        }
        ++n;
        bad += tc_div(0xFFFFFFFFu, f) != 0xFFFFFFFFu / f;
    }
    printf("tc_div: %llu quotients, %llu mismatches\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
