// Round 5 analysis tool (not product code): decodes a raw DEFLATE stream (dynamic / fixed / stored
// blocks) and counts its tokens by literal/length code length and distance code length, to size
// how often a decode lane needs a code longer than the primary tables (10-bit literal/length,
// 8-bit distance) of the GPU decoder's count and emit passes.
//   gcc -O2 -o /tmp/code_len_stats scripts/r05/code_len_stats.c && /tmp/code_len_stats stream.defl
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static const uint8_t* B;
static uint64_t NB, P;
static uint32_t get(uint32_t n) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; i++, P++) v |= (uint32_t)((B[P >> 3] >> (P & 7)) & 1) << i;
    return v;
}
typedef struct { uint16_t cnt[16], sym[320]; uint8_t len[320]; } Code;
static void build(Code* c, const uint8_t* len, int n) {
    for (int i = 0; i < 16; i++) c->cnt[i] = 0;
    for (int i = 0; i < n; i++) { c->cnt[len[i]]++; c->len[i] = len[i]; }
    c->cnt[0] = 0;
    uint16_t off[16]; off[1] = 0;
    for (int i = 1; i < 15; i++) off[i + 1] = off[i] + c->cnt[i];
    for (int i = 0; i < n; i++) if (len[i]) c->sym[off[len[i]]++] = (uint16_t)i;
}
static int decode(const Code* c, uint32_t* L) {   // canonical, bit by bit (puff style)
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (int)get(1);
        int count = c->cnt[l];
        if (code - count < first) { *L = (uint32_t)l; return c->sym[index + (code - first)]; }
        index += count; first += count; first <<= 1; code <<= 1;
    }
    return -1;
}
static const int CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
static const uint16_t LBASE[29] = {3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
static const uint8_t LEXT[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t* buf = calloc(n + 16, 1);
    if (fread(buf, 1, n, f) != (size_t)n) return 1;
    B = buf; NB = (uint64_t)n * 8; P = 0;
    uint64_t lit_by_len[16] = {0}, len_by_len[16] = {0}, dist_by_len[16] = {0}, blocks[3] = {0}, tokens = 0, out = 0;
    for (;;) {
        uint32_t fin = get(1), type = get(2);
        blocks[type < 3 ? type : 0]++;
        if (type == 0) {
            P = (P + 7) & ~7ull;
            uint32_t len = get(16); get(16);
            P += 8ull * len; out += len;
        } else {
            uint8_t lens[320] = {0};
            Code lc, dc;
            int nl = 288, nd = 32;
            if (type == 1) {
                for (int i = 0; i < 288; i++) lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
                for (int i = 0; i < 32; i++) lens[288 + i] = 5;
                build(&lc, lens, 288); build(&dc, lens + 288, 32);
            } else {
                nl = (int)get(5) + 257; nd = (int)get(5) + 1; int ncl = (int)get(4) + 4;
                uint8_t cl[19] = {0};
                for (int i = 0; i < ncl; i++) cl[CLO[i]] = (uint8_t)get(3);
                Code cc; build(&cc, cl, 19);
                int i = 0;
                while (i < nl + nd) {
                    uint32_t L; int s = decode(&cc, &L);
                    if (s < 16) lens[i++] = (uint8_t)s;
                    else if (s == 16) { int r = 3 + (int)get(2); uint8_t v = lens[i - 1]; while (r--) lens[i++] = v; }
                    else if (s == 17) { int r = 3 + (int)get(3); while (r--) lens[i++] = 0; }
                    else { int r = 11 + (int)get(7); while (r--) lens[i++] = 0; }
                }
                uint8_t dl[32] = {0};
                for (int k = 0; k < nd; k++) dl[k] = lens[nl + k];
                build(&lc, lens, nl); build(&dc, dl, nd);
            }
            for (;;) {
                uint32_t L; int s = decode(&lc, &L);
                if (s < 0) { fprintf(stderr, "bad code at %llu\n", (unsigned long long)P); return 1; }
                if (s == 256) break;
                tokens++;
                if (s < 256) { lit_by_len[L]++; out++; continue; }
                len_by_len[L]++;
                uint32_t ml = LBASE[s - 257] + get(LEXT[s - 257]);
                uint32_t DL; int d = decode(&dc, &DL);
                dist_by_len[DL]++;
                if (d >= 4) get((uint32_t)(d >> 1) - 1);
                out += ml;
            }
        }
        if (fin || P >= NB) break;
    }
    printf("blocks stored/fixed/dynamic %llu/%llu/%llu, tokens %llu, output %llu\n", (unsigned long long)blocks[0],
           (unsigned long long)blocks[1], (unsigned long long)blocks[2], (unsigned long long)tokens, (unsigned long long)out);
    uint64_t lit = 0, lng = 0, dst = 0, litL = 0, lenL = 0, dL = 0;
    for (int l = 0; l < 16; l++) { lit += lit_by_len[l]; lng += len_by_len[l]; dst += dist_by_len[l];
        if (l > 10) { litL += lit_by_len[l]; lenL += len_by_len[l]; } if (l > 8) dL += dist_by_len[l]; }
    printf("literal tokens %llu, length tokens %llu\n", (unsigned long long)lit, (unsigned long long)lng);
    printf("lit/len codes longer than 10 bits: %llu literals + %llu lengths = %.3f %% of tokens; distance codes longer than 8 bits: %llu\n",
           (unsigned long long)litL, (unsigned long long)lenL, 100.0 * (litL + lenL) / tokens, (unsigned long long)dL);
    printf("literal code length histogram:");
    for (int l = 1; l < 16; l++) printf(" %d:%.2f%%", l, 100.0 * lit_by_len[l] / lit);
    printf("\n");
    return 0;
}
