// Host check of the generated bit-sliced finder test (csrc/hip/kraft_bits.hpp): every position of
// seeded random bit streams (three bit densities) against a direct per-position Kraft sum.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#define KRAFT_FN static inline
static inline uint32_t bop3_host(uint32_t a, uint32_t b, uint32_t c, int imm) {
    uint32_t r = 0;
    for (int i = 0; i < 8; i++)
        if ((imm >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}
#define NDFL_BOP3(a, b, c, imm) bop3_host((a), (b), (c), (imm))
#include "kraft_bits.hpp"

static uint32_t bit(const uint32_t* w, uint64_t p) { return (w[p >> 5] >> (p & 31)) & 1; }

int main(int argc, char** argv) {
    const int nw = argc > 1 ? atoi(argv[1]) : (1 << 16);
    std::mt19937_64 rng(12345);
    uint32_t* w = (uint32_t*)malloc((nw + 8) * 4);
    long total = 0, pos = 0, bad = 0;
    for (int rep = 0; rep < 3; rep++) {
        for (int i = 0; i < nw + 8; i++) {
            uint32_t v = (uint32_t)rng();
            if (rep == 1) v &= (uint32_t)rng();
            if (rep == 2) v |= (uint32_t)rng() & (uint32_t)rng();
            w[i] = v;
        }
        for (int t = 0; t < nw; t++) {
            const uint32_t m = kraft_complete_mask(w[t], w[t + 1], w[t + 2], w[t + 3]);
            for (int i = 0; i < 32; i++) {
                const uint64_t p = (uint64_t)t * 32 + i;
                uint32_t hclen = 0, kr = 0;
                for (int k = 0; k < 4; k++) hclen |= bit(w, p + 13 + k) << k;
                for (uint32_t f = 0; f < hclen + 4; f++) {
                    uint32_t l = 0;
                    for (int k = 0; k < 3; k++) l |= bit(w, p + 17 + 3 * f + k) << k;
                    if (l) kr += 128u >> l;
                }
                const uint32_t ref = kr == 128;
                total++;
                pos += ref;
                if (ref != ((m >> i) & 1)) bad++;
            }
        }
    }
    printf("%ld %ld %ld\n", total, pos, bad);
    return bad != 0;
}
