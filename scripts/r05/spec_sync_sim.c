// gcc -O2 -o /tmp/spec_sync_sim scripts/r05/spec_sync_sim.c && /tmp/spec_sync_sim stream.defl
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


// Round 5 analysis tool (not product code): how often a lane's speculative run (decoding from its
// 448-bit segment start) fails to meet the true token path inside the segment, per dynamic block,
// classified by the block's literal/length code (used symbols, codes of length 8).
#define SEGB 448
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t* buf = calloc(n + 16, 1);
    if (fread(buf, 1, n, f) != (size_t)n) return 1;
    B = buf; NB = (uint64_t)n * 8;
    uint8_t* isb = calloc(NB / 8 + 64, 1);        // true token boundaries of the current block (bitmap)
    uint64_t P = 0;
    int nblk = 0;
    printf("block  bits  used  n8  segs  unsynced  unsync%%  mean_sync_bits  unsync_by64%%  no_phase_by64%%\n");
    for (;;) {
        uint32_t fin = bitsat(P, 1), type = bitsat(P + 1, 2);
        P += 3;
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
        int n8 = 0, used = 0;
        for (int i = 0; i < 288; i++) { n8 += lens[i] == 8; used += lens[i] != 0; }
        const uint64_t d0 = P;
        uint64_t q = P;
        for (;;) { isb[q >> 3] |= 1 << (q & 7); int r = token(&lc, &dc, &q); if (r) break; }
        const uint64_t dend = q;
        uint64_t segs = 0, unsync = 0, syncsum = 0, unsync64 = 0, unsyncph = 0;
        for (uint64_t s = d0 + SEGB; s + SEGB < dend; s += SEGB) {
            segs++;
            uint64_t p = s; int ok = 0;
            while (p < s + SEGB) {
                if ((isb[p >> 3] >> (p & 7)) & 1) { ok = 1; break; }
                if (token(&lc, &dc, &p)) break;
            }
            if (ok) syncsum += p - s; else unsync++;
            if (!ok || p >= s + 64) unsync64++;
            // the count pass's phase runs: starts s..s+7, on the true path by the first checkpoint (s + 64)
            int okp = 0;
            for (int f = 0; f < 8 && !okp; f++) {
                uint64_t q = s + f;
                while (q < s + 64) {
                    if ((isb[q >> 3] >> (q & 7)) & 1) { okp = 1; break; }
                    if (token(&lc, &dc, &q)) break;
                }
                if (!okp && ((isb[q >> 3] >> (q & 7)) & 1)) okp = 1;
            }
            if (!okp) unsyncph++;
        }
        for (uint64_t b = d0; b <= dend; b++) isb[b >> 3] &= ~(1 << (b & 7));
        P = dend;
        if (segs) printf("%5d %6llu %4d %4d %5llu %6llu %7.1f %8.1f %7.1f %7.1f\n", nblk, (unsigned long long)(dend - d0), used, n8,
                         (unsigned long long)segs, (unsigned long long)unsync, 100.0 * unsync / segs,
                         segs > unsync ? (double)syncsum / (segs - unsync) : 0.0, 100.0 * unsync64 / segs,
                         100.0 * unsyncph / segs);
        nblk++;
        if (fin || P >= NB) break;
    }
    return 0;
}
