// Round 5 analysis tool (not product code): how much of the count pass's phase-mapped work is
// redundant.  For every "phased" dynamic block of a raw DEFLATE stream (>= 192 of the 288
// literal/length code lengths are 8, the count pass's switch), the block's data bits are cut into
// 448-bit lane segments; each segment is decoded from its 8 bit phases to the first token boundary
// at or past its end, as the count pass does.  Two runs that land on the same boundary decode
// identically from there; the tool reports the token steps of all runs against the steps left if a
// run stopped at the first boundary it shares with a lower phase's run.
//   gcc -O2 -o /tmp/phase_merge_sim scripts/r05/phase_merge_sim.c && /tmp/phase_merge_sim stream.defl
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const uint8_t* B;
static uint64_t NB;
static uint32_t bitsat(uint64_t p, uint32_t n) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; i++) { uint64_t q = p + i; if (q < NB && ((B[q >> 3] >> (q & 7)) & 1)) v |= 1u << i; }
    return v;
}
typedef struct { uint16_t cnt[16], sym[320]; } Code;
static void build(Code* c, const uint8_t* len, int n) {
    memset(c, 0, sizeof *c);
    for (int i = 0; i < n; i++) c->cnt[len[i]]++;
    c->cnt[0] = 0;
    uint16_t off[16]; off[1] = 0;
    for (int i = 1; i < 15; i++) off[i + 1] = off[i] + c->cnt[i];
    for (int i = 0; i < n; i++) if (len[i]) c->sym[off[len[i]]++] = (uint16_t)i;
}
static int decode(const Code* c, uint64_t* p) {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)bitsat(*p, 1); (*p)++;
        int count = c->cnt[l];
        if (code - count < first) return c->sym[index + (code - first)];
        index += count; first += count; first <<= 1; code <<= 1;
    }
    return -1;
}
static const int CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
static const uint8_t LEXT[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
// one token from *p; returns 0 ok, 1 end of block, 2 error
static int token(const Code* lc, const Code* dc, uint64_t* p) {
    int s = decode(lc, p);
    if (s < 0 || s > 285) return 2;
    if (s < 256) return 0;
    if (s == 256) return 1;
    *p += LEXT[s - 257];
    int d = decode(dc, p);
    if (d < 0 || d > 29) return 2;
    if (d >= 4) *p += (uint64_t)(d >> 1) - 1;
    return 0;
}

#define MAXB 2048
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t* buf = calloc(n + 16, 1);
    if (fread(buf, 1, n, f) != (size_t)n) return 1;
    B = buf; NB = (uint64_t)n * 8;
    uint64_t P = 0, phased_blocks = 0, blocks = 0, segs = 0, steps_all = 0, steps_merged = 0, runs_merged = 0, runs = 0;
    uint64_t hist_alive[9] = {0};                  // distinct runs alive at the segment's end
    static uint64_t bnd[8][MAXB];
    static int nbnd[8];
    for (;;) {
        uint32_t fin = bitsat(P, 1), type = bitsat(P + 1, 2);
        P += 3;
        blocks++;
        if (type == 0) { P = (P + 7) & ~7ull; uint32_t len = bitsat(P, 16); P += 32 + 8ull * len; if (fin) break; continue; }
        uint8_t lens[320] = {0};
        Code lc, dc;
        if (type == 1) {
            for (int i = 0; i < 288; i++) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
            uint8_t dl[32]; for (int i = 0; i < 32; i++) dl[i] = 5;
            build(&lc, lens, 288); build(&dc, dl, 32);
        } else {
            int nl = (int)bitsat(P, 5) + 257, nd = (int)bitsat(P + 5, 5) + 1, ncl = (int)bitsat(P + 10, 4) + 4;
            P += 14;
            uint8_t cl[19] = {0};
            for (int i = 0; i < ncl; i++) { cl[CLO[i]] = (uint8_t)bitsat(P, 3); P += 3; }
            Code cc; build(&cc, cl, 19);
            int i = 0;
            while (i < nl + nd) {
                int s = decode(&cc, &P);
                if (s < 16) lens[i++] = (uint8_t)s;
                else if (s == 16) { int r = 3 + (int)bitsat(P, 2); P += 2; uint8_t v = lens[i - 1]; while (r--) lens[i++] = v; }
                else if (s == 17) { int r = 3 + (int)bitsat(P, 3); P += 3; while (r--) lens[i++] = 0; }
                else { int r = 11 + (int)bitsat(P, 7); P += 7; while (r--) lens[i++] = 0; }
            }
            uint8_t dl[32] = {0};
            for (int k = 0; k < nd; k++) dl[k] = lens[nl + k];
            for (int k = nl; k < 320; k++) lens[k] = 0;
            build(&lc, lens, nl); build(&dc, dl, nd);
        }
        int n8 = 0;
        for (int i = 0; i < 288; i++) n8 += lens[i] == 8;
        const uint64_t d0 = P;
        uint64_t q = P;                            // the true decode: the block's end
        for (;;) { int r = token(&lc, &dc, &q); if (r) break; }
        const uint64_t dend = q;
        P = q;
        if (type == 2 && n8 >= 192) {
            phased_blocks++;
            for (uint64_t s = d0; s + 8 < dend; s += 448) {
                const uint64_t e = s + 448 < dend ? s + 448 : dend;
                segs++;
                for (int k = 0; k < 8; k++) {
                    uint64_t p = s + k;
                    nbnd[k] = 0;
                    while (p < e && nbnd[k] < MAXB) {
                        int r = token(&lc, &dc, &p);
                        bnd[k][nbnd[k]++] = p;
                        if (r) break;
                    }
                }
                // merged accounting: run k stops at its first boundary that a lower run also has
                int alive = 0;
                for (int k = 0; k < 8; k++) {
                    runs++;
                    steps_all += (uint64_t)nbnd[k];
                    int stop = nbnd[k];
                    for (int i = 0; i < nbnd[k] && stop == nbnd[k]; i++)
                        for (int j = 0; j < k && stop == nbnd[k]; j++) {
                            // boundaries are increasing: binary search run j's list
                            int lo = 0, hi = nbnd[j];
                            while (lo < hi) { int m = (lo + hi) / 2; if (bnd[j][m] < bnd[k][i]) lo = m + 1; else hi = m; }
                            if (lo < nbnd[j] && bnd[j][lo] == bnd[k][i]) stop = i + 1;
                        }
                    if (stop < nbnd[k]) runs_merged++; else alive++;
                    steps_merged += (uint64_t)stop;
                }
                hist_alive[alive]++;
            }
        }
        if (fin || P >= NB) break;
    }
    printf("blocks %llu, phased %llu, segments %llu, runs %llu (merged before the end %llu)\n",
           (unsigned long long)blocks, (unsigned long long)phased_blocks, (unsigned long long)segs,
           (unsigned long long)runs, (unsigned long long)runs_merged);
    printf("token steps: all 8 runs %llu, stopping at the first shared boundary %llu (%.1f %%)\n",
           (unsigned long long)steps_all, (unsigned long long)steps_merged, 100.0 * steps_merged / (steps_all ? steps_all : 1));
    printf("distinct runs at the segment end:");
    for (int a = 1; a <= 8; a++) printf(" %d:%.1f%%", a, 100.0 * hist_alive[a] / (segs ? segs : 1));
    printf("\n");
    return 0;
}
