// Round 5 analysis tool (not product code, not a checker): replays the header finder's stage-1
// filter and the strict stage's per-survivor code-length loop (inflate_kernels.hip,
// ndfl_inflate_strict_kernel) on the CPU over a raw DEFLATE stream, and reports how many
// code-length steps each survivor takes and which check ends it.
//   gcc -O2 -o /tmp/strict_sim scripts/r05/strict_sim.c && /tmp/strict_sim stream.defl
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const uint8_t* B;
static uint64_t NB;
static uint32_t bits(uint64_t p, uint32_t n) {        // n <= 25, LSB-first, zero past the end
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t q = p + i;
        if (q < NB && (B[q >> 3] >> (q & 7) & 1)) v |= 1u << i;
    }
    return v;
}
static const int CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
enum { R_BAD16, R_OVERRUN, R_LITK, R_DISTK, R_EOI, R_EOB0, R_LITINC, R_DIST, R_ACCEPT, R_N };
static const char* RN[R_N] = {"16 first", "run past HLIT+HDIST", "lit/len Kraft > 1", "dist Kraft > 1",
                              "input end", "end: EOB length 0", "end: lit/len incomplete", "end: dist code",
                              "accepted"};

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* buf = malloc(n + 16);
    if (fread(buf, 1, n, f) != (size_t)n) return 1;
    B = buf; NB = (uint64_t)n * 8;
    uint64_t surv = 0, steps_tot = 0, cnt[R_N] = {0}, steps_by[R_N] = {0};
    uint64_t hist[400] = {0};
    uint64_t eob_early = 0;       // survivors that pass position 256 with EOB length 0 (an early reject)
    uint64_t eob_steps_saved = 0;
    for (uint64_t p = 0; p + 17 <= NB; p++) {
        uint32_t h = bits(p, 17);
        if ((h & 1) || ((h >> 1) & 3) != 2) continue;
        uint32_t hlit = (h >> 3) & 31, hdist = (h >> 8) & 31, hclen = (h >> 13) & 15;
        if (hlit >= 30 || hdist >= 30) continue;
        uint32_t ncl = hclen + 4;
        if (p + 17 + 3 * ncl > NB) continue;
        uint32_t len[19] = {0};
        uint32_t kr = 0;
        for (uint32_t j = 0; j < ncl; j++) { len[CLO[j]] = bits(p + 17 + 3 * j, 3); kr += len[CLO[j]] ? 128u >> len[CLO[j]] : 0; }
        if (kr != 128) continue;
        surv++;
        // canonical code -> 7-bit MSB-first table
        uint8_t tab[128];
        uint32_t pos = 0;
        for (uint32_t l = 1; l <= 7; l++)
            for (uint32_t s = 0; s < 19; s++)
                if (len[s] == l) { uint32_t run = 128u >> l; for (uint32_t r = 0; r < run; r++) tab[pos + r] = (uint8_t)(s | l << 5); pos += run; }
        uint32_t numLit = hlit + 257, numDist = hdist + 1, total = numLit + numDist;
        uint64_t q = p + 17 + 3 * ncl;
        uint32_t i = 0, litK = 0, distK = 0, ones = 0, other = 0, eob = 0, d0 = 0, d31 = 0, steps = 0;
        int runVal = -1, reason = -1;
        uint32_t eob_seen_at = 0;
        for (;;) {
            steps++;
            uint32_t b = bits(q, 14);
            uint32_t rev = 0;
            for (int k = 0; k < 7; k++) rev |= ((b >> k) & 1) << (6 - k);
            uint32_t te = tab[rev], sym = te & 31, cl = te >> 5;
            uint32_t nx = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
            uint32_t ex = (b >> cl) & ((1u << nx) - 1);
            uint32_t run = sym < 16 ? 1 : ex + (sym == 18 ? 11 : 3);
            int bad = sym == 16 && runVal < 0;
            runVal = sym < 16 ? (int)sym : sym == 16 ? runVal : 0;
            q += cl + nx;
            uint32_t en = i + run, v = (uint32_t)runVal, wt = v ? 32768u >> v : 0;
            litK += ((en < numLit ? en : numLit) - (i < numLit ? i : numLit)) * wt;
            uint32_t da = (i > numLit ? i : numLit) - numLit, db = (en > numLit ? en : numLit) - numLit, cd = db - da;
            distK += cd * wt;
            ones += v == 1 ? cd : 0;
            other += v > 1 ? cd : 0;
            if (i <= 256 && 256 < en) { eob = v; eob_seen_at = steps; }
            if (cd && da == 0) d0 = v;
            if (da <= 31 && 31 < db) d31 = v;
            i = en;
            if (bad) { reason = R_BAD16; break; }
            if (en > total) { reason = R_OVERRUN; break; }
            if (q > NB) { reason = R_EOI; break; }
            if (litK > 32768u) { reason = R_LITK; break; }
            if (distK > 32768u) { reason = R_DISTK; break; }
            if (i >= total) {
                if (eob == 0) reason = R_EOB0;
                else if (litK != 32768u) reason = R_LITINC;
                else if (numDist == 1 && d0 == 0) reason = R_ACCEPT;
                else if (ones == 1 && other == 0) reason = (numDist == 32 && d31 == 1) ? R_DIST : R_ACCEPT;
                else reason = distK == 32768u ? R_ACCEPT : R_DIST;
                break;
            }
        }
        if (reason == R_EOB0 && eob_seen_at) { eob_early++; eob_steps_saved += steps - eob_seen_at; }
        cnt[reason]++; steps_by[reason] += steps; steps_tot += steps;
        hist[steps < 399 ? steps : 399]++;
    }
    printf("stream %lu bytes, %lu survivors, %.2f steps per survivor\n", n, surv, (double)steps_tot / surv);
    for (int r = 0; r < R_N; r++)
        printf("  %-26s %9lu (%5.1f %%)  %7.1f steps each\n", RN[r], cnt[r], 100.0 * cnt[r] / surv, cnt[r] ? (double)steps_by[r] / cnt[r] : 0.0);
    printf("  EOB-length-0 rejects decidable at position 256: %lu, steps after it %lu (%.1f %% of all steps)\n",
           eob_early, eob_steps_saved, 100.0 * eob_steps_saved / steps_tot);
    uint64_t c = 0;
    printf("  steps cdf:");
    for (int s = 0; s < 400; s++) { c += hist[s]; if (s == 2 || s == 5 || s == 10 || s == 20 || s == 40 || s == 80 || s == 160) printf(" <=%d: %.1f%%", s, 100.0 * c / surv); }
    printf("\n");
    return 0;
}
