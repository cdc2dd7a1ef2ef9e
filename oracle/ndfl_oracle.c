/*
 * ndfl_oracle.c -- CPU restatement of nayuki/DEFLATE-library-Java's DEFLATE path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + cpu_baseline).  Never linked by the product.
 * Each function cites the reference file:line it restates; D/ = /root/reference/src/io/nayuki/deflate/.
 * Pinning: see ndfl_oracle.h header and tests/test_oracle_*.py.
 */
#include "ndfl_oracle.h"
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* Bit writer: restates DeflaterOutputStream.BitOut (D/DeflaterOutputStream.java:141-171).      */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint8_t* out; uint64_t cap, n;
    uint64_t buf; int len; int overflow;
} bw_t;

static void bw_put(bw_t* w, uint8_t b) {
    if (w->n < w->cap) w->out[w->n] = b; else w->overflow = 1;
    w->n++;
}
/* writeBits: flush whole bytes only when the value does not fit (:147-156). */
static void bw_bits(bw_t* w, uint32_t v, int nb) {
    if (nb > 64 - w->len) {
        for (; w->len >= 8; w->len -= 8, w->buf >>= 8) bw_put(w, (uint8_t)w->buf);
    }
    if (nb > 0) w->buf |= (uint64_t)v << w->len;
    w->len += nb;
}
static int bw_pos(const bw_t* w) { return w->len % 8; }            /* getBitPosition :159-161 */
static void bw_finish(bw_t* w) {                                    /* finish :164-169 */
    bw_bits(w, 0, (8 - bw_pos(w)) % 8);
    for (; w->len >= 8; w->len -= 8, w->buf >>= 8) bw_put(w, (uint8_t)w->buf);
}

/* Counting writer: CountingBitOutputStream (D/comp/CountingBitOutputStream.java:14-33). */
typedef struct { bw_t* real; uint64_t count; } sink_t;
static void sk_bits(sink_t* s, uint32_t v, int nb) {
    if (s->real) bw_bits(s->real, v, nb); else s->count += (uint64_t)nb;
}
static int sk_pos(const sink_t* s) { return s->real ? bw_pos(s->real) : (int)(s->count % 8); }

/* ------------------------------------------------------------------------------------------ */
/* Huffman code construction: Lz77Huffman.calcHuffmanCodeLengths (D/comp/Lz77Huffman.java:309-364) */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint64_t freq; int32_t sym; int32_t a, b; } pm_node;

/* Stable merge sort by frequency (Collections.sort with a Long.compare comparator, :321). */
static void pm_stable_sort(int32_t* idx, int32_t* tmp, int n, const pm_node* pool) {
    if (n < 2) return;
    int h = n / 2;
    pm_stable_sort(idx, tmp, h, pool);
    pm_stable_sort(idx + h, tmp, n - h, pool);
    int i = 0, j = h, k = 0;
    while (i < h && j < n) {
        if (pool[idx[j]].freq < pool[idx[i]].freq) tmp[k++] = idx[j++];
        else tmp[k++] = idx[i++];                       /* ties keep the earlier element first */
    }
    while (i < h) tmp[k++] = idx[i++];
    while (j < n) tmp[k++] = idx[j++];
    memcpy(idx, tmp, sizeof(int32_t) * (size_t)n);
}

static void pm_count(const pm_node* pool, int32_t id, uint8_t* hist) {  /* countOccurrences :339-363 */
    const pm_node* nd = &pool[id];
    if (nd->sym >= 0) { hist[nd->sym]++; return; }
    pm_count(pool, nd->a, hist);
    pm_count(pool, nd->b, hist);
}

static void calc_code_lengths(const uint32_t* hist, int n, int max_len, uint8_t* out_lens) {
    int32_t nleaves = 0;
    pm_node* pool = (pm_node*)malloc(sizeof(pm_node) * (size_t)(n + (size_t)max_len * 2 * (size_t)(n + 1) + 4));
    int32_t* leaves = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t npool = 0;
    for (int s = 0; s < n; s++) {                         /* leaves in symbol order (:310-315) */
        if (hist[s] > 0) {
            pool[npool].freq = hist[s]; pool[npool].sym = s; pool[npool].a = pool[npool].b = -1;
            leaves[nleaves++] = npool++;
        }
    }
    int cap = 2 * (n + 1) + 4;
    int32_t* nodes = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int nn = 0;
    for (int it = 0; it < max_len; it++) {               /* package-merge (:318-332) */
        for (int k = 0; k < nleaves; k++) nodes[nn + k] = leaves[k];
        nn += nleaves;
        pm_stable_sort(nodes, tmp, nn, pool);
        int m = 0;
        for (int j = 0; j + 2 <= nn; j += 2) {
            pm_node* p = &pool[npool];
            p->freq = pool[nodes[j]].freq + pool[nodes[j + 1]].freq;
            p->sym = -1; p->a = nodes[j]; p->b = nodes[j + 1];
            tmp[m++] = npool++;
        }
        memcpy(nodes, tmp, sizeof(int32_t) * (size_t)m);
        nn = m;
    }
    memset(out_lens, 0, (size_t)n);
    for (int i = 0; i < nleaves - 1; i++) pm_count(pool, nodes[i], out_lens);   /* :334-335 */
    free(pool); free(leaves); free(nodes); free(tmp);
}

/* codeLengthsToCodes (:372-391): rev(code) << 4 | len, or -1 on an over/under-full code. */
static int lengths_to_codes(const uint8_t* lens, int n, int max_len, int32_t* out) {
    uint32_t next = 0;
    for (int cl = 1; cl <= max_len; cl++) {
        next <<= 1;
        for (int s = 0; s < n; s++) {
            if (lens[s] != cl) continue;
            if ((next >> cl) != 0) return -1;
            uint32_t rev = 0;
            for (int b = 0; b < cl; b++) rev |= ((next >> b) & 1u) << (cl - 1 - b);
            out[s] = (int32_t)(rev << 4 | (uint32_t)cl);
            next++;
        }
    }
    if (next != (1u << max_len)) return -1;
    return 0;
}

static const int CLC_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int32_t STATIC_LIT[288], STATIC_DIST[32];
static int static_ready = 0;
static void init_static(void) {                            /* :394-410 */
    if (static_ready) return;
    uint8_t l[288], d[32];
    int i = 0;
    for (; i < 144; i++) l[i] = 8;
    for (; i < 256; i++) l[i] = 9;
    for (; i < 280; i++) l[i] = 7;
    for (; i < 288; i++) l[i] = 8;
    for (i = 0; i < 32; i++) d[i] = 5;
    lengths_to_codes(l, 288, 9, STATIC_LIT);
    lengths_to_codes(d, 32, 5, STATIC_DIST);
    static_ready = 1;
}

/* ------------------------------------------------------------------------------------------ */
/* Lz77Huffman.decide/compressTo (D/comp/Lz77Huffman.java:42-286)                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int dynamic, min_run, max_run, min_dist, max_dist; } lz_params;

typedef struct {            /* exact-prefix candidate chains (equivalent to the exhaustive loop) */
    int64_t* head; int64_t* prev; int64_t base, inserted;
} chain_t;

static uint32_t key3(const uint8_t* b, int64_t j) { return (uint32_t)b[j] | (uint32_t)b[j + 1] << 8 | (uint32_t)b[j + 2] << 16; }
static uint32_t hash3(uint32_t k) { return (k * 2654435761u) >> 17; }   /* 15-bit bucket */

/* One search step at `index`: returns best run and distance exactly as :68-84. */
static void lz_search(const uint8_t* b, int64_t off, int64_t index, int64_t end, const lz_params* P,
                      int brute, chain_t* ch, int* best_run, int* best_dist) {
    int bestRun = 0, bestDist = 0;
    int64_t distEnd = P->max_dist;
    if (index - off < distEnd) distEnd = index - off;
    if (brute || P->max_dist <= 2) {
        for (int64_t dist = P->min_dist; dist <= distEnd && bestRun < P->max_run; dist++) {
            int run = 0;
            int64_t hi = index - dist, di = index;
            for (; run < P->max_run && di < end && b[di] == b[hi]; run++, di++) {
                hi++;
                if (hi == index) hi -= dist;
            }
            if (run > bestRun || (run == bestRun && dist < bestDist)) { bestRun = run; bestDist = (int)dist; }
        }
    } else if (index + 2 < end && distEnd >= P->min_dist) {
        /* Only candidates whose run reaches min_run (>= 3) can be chosen; they share the 3-byte
         * prefix.  Walk nearest-first (ascending distance), keep strictly longer runs only, stop
         * at max_run: identical to the ascending exhaustive loop. */
        for (; ch->inserted < index; ch->inserted++) {
            int64_t j = ch->inserted;
            if (j + 2 >= end) continue;
            uint32_t h = hash3(key3(b, j));
            ch->prev[j - ch->base] = ch->head[h];
            ch->head[h] = j;
        }
        uint32_t k = key3(b, index);
        for (int64_t j = ch->head[hash3(k)]; j >= off; j = ch->prev[j - ch->base]) {
            int64_t dist = index - j;
            if (dist > distEnd) break;
            if (dist < P->min_dist) continue;
            if (key3(b, j) != k) continue;
            int run = 0;
            while (run < P->max_run && index + run < end && b[index + run] == b[j + run]) run++;
            if (run > bestRun) {
                bestRun = run; bestDist = (int)dist;
                if (bestRun >= P->max_run) break;
            }
        }
    }
    *best_run = bestRun; *best_dist = bestDist;
}

/* Returns 0, or -1 if the parameters make an unencodable block (mirrors an exception). */
static int lz_compress(const uint8_t* b, int64_t off, int64_t histLen, int64_t dataLen,
                       const lz_params* P, int isFinal, sink_t* out, int brute) {
    int64_t index = off + histLen;
    const int64_t end = index + dataLen;
    int64_t tcap = dataLen * 2 + 4;
    uint16_t* tok = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)tcap);
    int64_t nt = 0;
    uint32_t litHist[286]; uint32_t distHist[30];
    memset(litHist, 0, sizeof litHist); memset(distHist, 0, sizeof distHist);

    chain_t ch = {0};
    if (!brute && P->max_dist > 2) {
        ch.head = (int64_t*)malloc(sizeof(int64_t) * 32768);
        for (int i = 0; i < 32768; i++) ch.head[i] = -1;
        ch.prev = (int64_t*)malloc(sizeof(int64_t) * (size_t)(end - off + 1));
        ch.base = off; ch.inserted = off;
    }

    while (index < end) {                                  /* :68-130 */
        int bestRun, bestDist;
        lz_search(b, off, index, end, P, brute, &ch, &bestRun, &bestDist);
        if (bestRun == 0 || bestRun < P->min_run) {
            int sym = b[index];
            index++;
            tok[nt++] = (uint16_t)(sym << 4);
            litHist[sym]++;
        } else {
            {   /* length symbol :92-111 */
                int r = bestRun - 3, numExtra, sym, extra;
                if (bestRun < 11) { numExtra = 0; sym = r + 257; extra = 0; }
                else if (bestRun == 258) { numExtra = 0; sym = 285; extra = 0; }
                else {
                    numExtra = 29 - __builtin_clz((unsigned)r);
                    sym = (numExtra << 2) + (r >> numExtra) + 257;
                    extra = r & ((1 << numExtra) - 1);
                }
                tok[nt++] = (uint16_t)(sym << 4 | numExtra);
                litHist[sym]++;
                tok[nt++] = (uint16_t)extra;
            }
            {   /* distance symbol :112-127 */
                int d = bestDist - 1, numExtra, sym, extra;
                if (bestDist < 5) { numExtra = 0; sym = d; extra = 0; }
                else {
                    numExtra = 30 - __builtin_clz((unsigned)d);
                    sym = (numExtra << 1) + (d >> numExtra);
                    extra = d & ((1 << numExtra) - 1);
                }
                tok[nt++] = (uint16_t)(sym << 4 | numExtra);
                distHist[sym]++;
                tok[nt++] = (uint16_t)extra;
            }
            index += bestRun;
        }
    }
    tok[nt++] = (uint16_t)(256 << 4);                      /* :131-132 */
    litHist[256]++;
    if (ch.head) { free(ch.head); free(ch.prev); }

    sk_bits(out, isFinal ? 1u : 0u, 1);                    /* :134-135 */
    sk_bits(out, P->dynamic ? 2u : 1u, 2);

    int32_t litCode[288], distCodeArr[32];
    const int32_t* litLenCode; const int32_t* distCode;
    int rc = 0;
    if (!P->dynamic) {
        init_static();
        litLenCode = STATIC_LIT; distCode = STATIC_DIST;
    } else {
        if (dataLen == 0) litHist[0]++;                    /* :146-147 */
        int litN = 286;
        while (litN > 257 && litHist[litN - 1] == 0) litN--;   /* :148-151 */
        uint8_t litLen[286];
        calc_code_lengths(litHist, litN, 15, litLen);       /* :153 */

        int used = 0;
        for (int i = 0; i < 30; i++) if (distHist[i] > 0) used++;
        if (used == 1) {                                    /* :157-170 */
            for (int i = 0; i < 30; i++) {
                if (distHist[i] > 0) {
                    if (30 - i > 1) distHist[i + 1] = 1; else distHist[i - 1] = 1;
                    break;
                }
            }
        }
        int distN = 30;
        while (distN > 1 && distHist[distN - 1] == 0) distN--;   /* :172-175 */
        uint8_t distLen[30];
        int emptyDist = (distN == 1 && distHist[0] == 0);
        if (emptyDist) distLen[0] = 0;                       /* :177-181 */
        else calc_code_lengths(distHist, distN, 15, distLen);

        int nc = litN + distN;                               /* :183-185 */
        uint8_t codeLens[316];
        memcpy(codeLens, litLen, (size_t)litN);
        memcpy(codeLens + litN, distLen, (size_t)distN);

        int clSym[316], clExtra[316], ncs = 0;              /* greedy RLE :187-223 */
        for (int i = 0; i < nc;) {
            int val = codeLens[i];
            if (val == 0) {
                int runLength = 1;
                for (; runLength < 138 && i + runLength < nc && codeLens[i + runLength] == 0; runLength++);
                if (runLength < 3) { clSym[ncs] = val; clExtra[ncs++] = 0; i++; }
                else if (runLength < 11) { clSym[ncs] = 17; clExtra[ncs++] = runLength - 3; i += runLength; }
                else { clSym[ncs] = 18; clExtra[ncs++] = runLength - 11; i += runLength; }
                continue;
            }
            if (i > 0) {
                int runLength = 0;
                for (; runLength < 6 && i + runLength < nc && codeLens[i + runLength] == codeLens[i - 1]; runLength++);
                if (runLength >= 3) { clSym[ncs] = 16; clExtra[ncs++] = runLength - 3; i += runLength; continue; }
            }
            clSym[ncs] = val; clExtra[ncs++] = 0; i++;
        }
        uint32_t clHist[19]; memset(clHist, 0, sizeof clHist);
        for (int k = 0; k < ncs; k++) clHist[clSym[k]]++;
        uint8_t clLen[19];
        calc_code_lengths(clHist, 19, 7, clLen);            /* :225 */
        int reordered[19];
        for (int i = 0; i < 19; i++) reordered[i] = clLen[CLC_ORDER[i]];
        int ncl = 19;
        for (; ncl > 4 && reordered[ncl - 1] == 0; ncl--);  /* :230-234 */

        sk_bits(out, (uint32_t)(litN - 257), 5);            /* :236-238 */
        sk_bits(out, (uint32_t)(distN - 1), 5);
        sk_bits(out, (uint32_t)(ncl - 4), 4);
        for (int i = 0; i < ncl; i++) sk_bits(out, (uint32_t)reordered[i], 3);

        int32_t clCode[19];
        if (lengths_to_codes(clLen, 19, 7, clCode) != 0) { rc = -1; goto done; }
        for (int k = 0; k < ncs; k++) {                     /* :243-258 */
            int32_t pair = clCode[clSym[k]];
            sk_bits(out, (uint32_t)pair >> 4, pair & 0xF);
            if (clSym[k] >= 16)
                sk_bits(out, (uint32_t)clExtra[k], clSym[k] == 16 ? 2 : clSym[k] == 17 ? 3 : 7);
        }
        if (lengths_to_codes(litLen, litN, 15, litCode) != 0) { rc = -1; goto done; }
        litLenCode = litCode;
        if (emptyDist) distCode = NULL;
        else {
            if (lengths_to_codes(distLen, distN, 15, distCodeArr) != 0) { rc = -1; goto done; }
            distCode = distCodeArr;
        }
    }
    for (int64_t k = 0; k < nt;) {                         /* token emission :267-285 */
        int litLenPair = tok[k++];
        int sym = litLenPair >> 4, lenNumExtra = litLenPair & 0xF;
        int32_t cp = litLenCode[sym];
        sk_bits(out, (uint32_t)cp >> 4, cp & 0xF);
        if (sym > 256) {
            sk_bits(out, tok[k++], lenNumExtra);
            int distPair = tok[k++];
            int dsym = distPair >> 4, dne = distPair & 0xF;
            int32_t dp = distCode[dsym];
            sk_bits(out, (uint32_t)dp >> 4, dp & 0xF);
            sk_bits(out, tok[k++], dne);
        }
    }
done:
    free(tok);
    return rc;
}

/* Uncompressed.decide/compressTo (D/comp/Uncompressed.java:19-51). */
static void unc_compress(const uint8_t* b, int64_t off, int64_t histLen, int64_t dataLen, int isFinal, sink_t* out) {
    int64_t index = off + histLen;
    const int64_t end = index + dataLen;
    do {
        int64_t n = end - index; if (n > 65535) n = 65535;
        sk_bits(out, (isFinal && n == end - index) ? 1u : 0u, 1);
        sk_bits(out, 0, 2);
        sk_bits(out, 0, (8 - sk_pos(out)) % 8);
        sk_bits(out, (uint32_t)(n ^ 0x0000), 16);
        sk_bits(out, (uint32_t)(n ^ 0xFFFF), 16);
        int64_t e = index + n;
        for (; index < e; index++) sk_bits(out, b[index], 8);
    } while (index < end);
}

/* ------------------------------------------------------------------------------------------ */
/* DeflaterOutputStream chunking (D/DeflaterOutputStream.java:76-137)                           */
/* ------------------------------------------------------------------------------------------ */
static const lz_params PRESETS[6] = {
    {0, 0, 0, 0, 0}, {1, 0, 0, 0, 0},          /* LITERAL_STATIC / LITERAL_DYNAMIC :298-299 */
    {0, 3, 258, 1, 1}, {1, 3, 258, 1, 1},      /* RLE_STATIC / RLE_DYNAMIC :301-302 */
    {0, 3, 258, 1, 32768}, {1, 3, 258, 1, 32768} /* FULL_STATIC / FULL_DYNAMIC :304-305 */
};

/* Drive the whole stream.  Chunk boundaries are exact multiples of chunk_len; the last chunk
 * (1..chunk_len bytes, or 0 for empty input) is final (:79-108).  History = the preceding
 * min(hist_limit, pos) raw bytes (:128-136). */
static int64_t drive(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                     int is_unc, const lz_params* P, int brute, bw_t* w, uint64_t* block_bits, uint64_t bcap) {
    if (chunk_len < 1 || hist_limit > 32768) return OR_ERR_ARG;
    uint64_t pos = 0, nb = 0;
    for (;;) {
        uint64_t dlen = len - pos;
        int fin = 1;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (dlen == chunk_len && pos + dlen < len) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        const uint8_t* base = data + (pos - hlen);
        uint64_t before = w ? (w->n * 8 + (uint64_t)w->len) : 0;
        sink_t s = { w, 0 };
        if (is_unc) unc_compress(base, 0, (int64_t)hlen, (int64_t)dlen, fin, &s);
        else if (lz_compress(base, 0, (int64_t)hlen, (int64_t)dlen, P, fin, &s, brute) != 0) return OR_ERR_ARG;
        if (block_bits && nb < bcap) block_bits[nb] = (w ? (w->n * 8 + (uint64_t)w->len) : 0) - before;
        nb++;
        pos += dlen;
        if (fin) break;
    }
    return (int64_t)nb;
}

int64_t or_deflate_lz(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                      int dynamic, int min_run, int max_run, int min_dist, int max_dist, int brute,
                      uint8_t* out, uint64_t out_cap) {
    /* Lz77Huffman record validation (:20-39) */
    if (!(min_run == 0 && max_run == 0 && min_dist == 0 && max_dist == 0) &&
        !(3 <= min_run && min_run <= max_run && max_run <= 258 && 1 <= min_dist && min_dist <= max_dist && max_dist <= 32768))
        return OR_ERR_ARG;
    lz_params P = {dynamic ? 1 : 0, min_run, max_run, min_dist, max_dist};
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    int64_t r = drive(data, len, chunk_len, hist_limit, 0, &P, brute, &w, NULL, 0);
    if (r < 0) return r;
    bw_finish(&w);
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

int64_t or_deflate(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                   int strategy, int brute, uint8_t* out, uint64_t out_cap) {
    if (strategy < 0 || strategy > 6) return OR_ERR_ARG;
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    int64_t r = drive(data, len, chunk_len, hist_limit, strategy == OR_UNCOMPRESSED,
                      strategy == OR_UNCOMPRESSED ? NULL : &PRESETS[strategy], brute, &w, NULL, 0);
    if (r < 0) return r;
    bw_finish(&w);
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

int64_t or_deflate_chunks(const uint8_t* hist, uint64_t hist_len, const uint8_t* data, uint64_t len,
                          uint32_t chunk_len, uint32_t hist_limit, int strategy, int final_flag,
                          uint8_t* out, uint64_t out_cap, uint64_t* out_bits) {
    if (strategy < 0 || strategy > 6 || chunk_len < 1 || hist_limit > 32768) return OR_ERR_ARG;
    if (!final_flag && (len == 0 || len % chunk_len != 0)) return OR_ERR_ARG;
    if (hist_len > hist_limit) { hist += hist_len - hist_limit; hist_len = hist_limit; }
    uint8_t* buf = (uint8_t*)malloc((size_t)(hist_len + len + 1));
    if (!buf) return OR_ERR_ARG;
    if (hist_len) memcpy(buf, hist, (size_t)hist_len);
    if (len) memcpy(buf + hist_len, data, (size_t)len);
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    uint64_t pos = hist_len, end = hist_len + len;               /* positions in buf */
    for (;;) {                                                   /* writeBuffer per chunk */
        uint64_t dlen = end - pos; int fin = final_flag;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (final_flag && dlen == chunk_len && pos + dlen < end) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        sink_t sk = { &w, 0 };
        if (strategy == OR_UNCOMPRESSED) unc_compress(buf + (pos - hlen), 0, (int64_t)hlen, (int64_t)dlen, fin, &sk);
        else lz_compress(buf + (pos - hlen), 0, (int64_t)hlen, (int64_t)dlen, &PRESETS[strategy], fin, &sk, 0);
        pos += dlen;
        if (fin || pos >= end) break;
    }
    free(buf);
    *out_bits = w.n * 8 + (uint64_t)w.len;
    for (; w.len > 0; w.len -= 8, w.buf >>= 8) bw_put(&w, (uint8_t)w.buf);   /* pending bits, zero-padded */
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

int64_t or_deflate_mixed(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                         const int8_t* strat, uint32_t nstrat, uint8_t* out, uint64_t out_cap) {
    /* Fixture generator: chunk i is encoded with strategy strat[i % nstrat] (a mix of stored,
     * fixed and dynamic blocks, e.g. config 2's "stored + fixed-Huffman" stream). */
    if (chunk_len < 1 || hist_limit > 32768 || nstrat == 0) return OR_ERR_ARG;
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    uint64_t pos = 0, ci = 0;
    for (;;) {
        uint64_t dlen = len - pos; int fin = 1;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (dlen == chunk_len && pos + dlen < len) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        const uint8_t* base = data + (pos - hlen);
        sink_t sk = { &w, 0 };
        int st = strat[ci % nstrat];
        if (st == OR_UNCOMPRESSED) unc_compress(base, 0, (int64_t)hlen, (int64_t)dlen, fin, &sk);
        else if (st >= 0 && st < 6) lz_compress(base, 0, (int64_t)hlen, (int64_t)dlen, &PRESETS[st], fin, &sk, 0);
        else return OR_ERR_ARG;
        pos += dlen; ci++;
        if (fin) break;
    }
    bw_finish(&w);
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

/* MultiStrategy(subs...).decide/compressTo (D/comp/MultiStrategy.java:31-57) over Lz77Huffman /
 * Uncompressed substrategies, driven like DeflaterOutputStream (D/DeflaterOutputStream.java:119-137).
 * desc: n x {kind (0 Lz77Huffman, 1 Uncompressed), dynamic, minRun, maxRun, minDist, maxDist}. */
int64_t or_deflate_multi(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                         const int32_t* desc, uint32_t n, uint8_t* out, uint64_t out_cap) {
    if (chunk_len < 1 || hist_limit > 32768 || n == 0 || n > 64) return OR_ERR_ARG;
    lz_params P[64];
    for (uint32_t k = 0; k < n; k++) {
        const int32_t* d = desc + 6 * k;
        if (d[0] == 1) continue;
        if (d[0] != 0) return OR_ERR_ARG;
        if (!(d[2] == 0 && d[3] == 0 && d[4] == 0 && d[5] == 0) &&
            !(3 <= d[2] && d[2] <= d[3] && d[3] <= 258 && 1 <= d[4] && d[4] <= d[5] && d[5] <= 32768))
            return OR_ERR_ARG;
        lz_params q = {d[1] ? 1 : 0, d[2], d[3], d[4], d[5]};
        P[k] = q;
    }
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    uint64_t pos = 0;
    for (;;) {
        uint64_t dlen = len - pos; int fin = 1;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (dlen == chunk_len && pos + dlen < len) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        const uint8_t* base = data + (pos - hlen);
        /* decide: bitLengths of every substrategy (:35-44) */
        int64_t best[8]; int pick[8];
        for (int i = 0; i < 8; i++) { best[i] = INT64_MAX; pick[i] = -1; }
        for (uint32_t k = 0; k < n; k++) {
            int64_t bl[8];
            if (desc[6 * k] == 1) {                  /* Uncompressed (:22-26) */
                int64_t nblk = ((int64_t)dlen + 65534) / 65535; if (nblk < 1) nblk = 1;
                for (int i = 0; i < 8; i++) bl[i] = (int64_t)dlen * 8 + nblk * 40 + ((13 - i) % 8 - 5);
            } else {                                 /* Lz77Huffman: a counting pass (:45-53) */
                sink_t cnt = { NULL, 0 };
                if (lz_compress(base, 0, (int64_t)hlen, (int64_t)dlen, &P[k], 0, &cnt, 0) != 0) return OR_ERR_ARG;
                for (int i = 0; i < 8; i++) bl[i] = (int64_t)cnt.count;
            }
            for (int i = 0; i < 8; i++) if (bl[i] < best[i]) { best[i] = bl[i]; pick[i] = (int)k; }
        }
        /* compressTo: the decision for the current bit position (:51-53) */
        sink_t sk = { &w, 0 };
        const int k = pick[sk_pos(&sk)];
        if (desc[6 * k] == 1) unc_compress(base, 0, (int64_t)hlen, (int64_t)dlen, fin, &sk);
        else if (lz_compress(base, 0, (int64_t)hlen, (int64_t)dlen, &P[k], fin, &sk, 0) != 0) return OR_ERR_ARG;
        pos += dlen;
        if (fin) break;
    }
    bw_finish(&w);
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

/* BinarySplit(sub, minBlockLen).decide/compressTo (D/comp/BinarySplit.java:21-82), with the
 * reference's loop as written: the split's bit length is accumulated from position 0 whatever the
 * starting position i (:45-50, :56-63).  sub: {kind, dynamic, minRun, maxRun, minDist, maxDist}. */
typedef struct bs_dec {
    int64_t hl, dl;                       /* data = b[hl, hl + dl) relative to the chunk's off */
    int64_t bits[8];
    struct bs_dec* pick[8][2];            /* NULL: the substrategy's own decision for the range */
    struct bs_dec* own[2];                /* children owned by this node */
} bs_dec;

static void bs_leaf_bits(const uint8_t* b, int64_t hl, int64_t dl, const int32_t* d, const lz_params* P, int64_t out[8]) {
    if (d[0] == 1) {
        int64_t nblk = (dl + 65534) / 65535; if (nblk < 1) nblk = 1;
        for (int i = 0; i < 8; i++) out[i] = dl * 8 + nblk * 40 + ((13 - i) % 8 - 5);
    } else {
        sink_t cnt = { NULL, 0 };
        lz_compress(b, 0, hl, dl, P, 0, &cnt, 0);
        for (int i = 0; i < 8; i++) out[i] = (int64_t)cnt.count;
    }
}

static bs_dec* bs_new_leaf(const uint8_t* b, int64_t hl, int64_t dl, const int32_t* d, const lz_params* P) {
    bs_dec* x = (bs_dec*)calloc(1, sizeof(bs_dec));
    x->hl = hl; x->dl = dl;
    bs_leaf_bits(b, hl, dl, d, P, x->bits);
    return x;
}

static void bs_free(bs_dec* x) {
    if (!x) return;
    bs_free(x->own[0]); bs_free(x->own[1]);
    free(x);
}

/* decide(b, off, historyLen, dataLen, curDec) (:33-66); `cur` becomes the returned node. */
static bs_dec* bs_decide(const uint8_t* b, bs_dec* cur, const int32_t* d, const lz_params* P, int64_t M) {
    int64_t first = (cur->dl + 1) / 2, second = cur->dl - first;
    if ((first < second ? first : second) > M) {
        bs_dec* sp[2] = { bs_new_leaf(b, cur->hl, first, d, P), bs_new_leaf(b, cur->hl + first, second, d, P) };
        int improved = 0;
        for (int i = 0; i < 8; i++) {
            int64_t bl = 0;
            for (int k = 0; k < 2; k++) bl += sp[k]->bits[bl % 8];
            improved |= bl < cur->bits[i];
        }
        if (improved) { sp[0] = bs_decide(b, sp[0], d, P, M); sp[1] = bs_decide(b, sp[1], d, P, M); }
        int used = 0;
        for (int i = 0; i < 8; i++) {
            int64_t bl = 0;
            for (int k = 0; k < 2; k++) bl += sp[k]->bits[bl % 8];
            if (bl < cur->bits[i]) { cur->bits[i] = bl; cur->pick[i][0] = sp[0]; cur->pick[i][1] = sp[1]; used = 1; }
        }
        cur->own[0] = sp[0]; cur->own[1] = sp[1];
        (void)used;
    }
    return cur;
}

static void bs_emit(const uint8_t* b, const bs_dec* x, const int32_t* d, const lz_params* P, int isFinal, sink_t* sk) {
    const int pos = sk_pos(sk);
    if (x->pick[pos][0]) {
        bs_emit(b, x->pick[pos][0], d, P, 0, sk);
        bs_emit(b, x->pick[pos][1], d, P, isFinal, sk);
    } else if (d[0] == 1) {
        unc_compress(b, 0, x->hl, x->dl, isFinal, sk);
    } else {
        lz_compress(b, 0, x->hl, x->dl, P, isFinal, sk, 0);
    }
}

int64_t or_deflate_binsplit(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                            const int32_t* desc, int32_t min_block_len, uint8_t* out, uint64_t out_cap) {
    if (chunk_len < 1 || hist_limit > 32768 || min_block_len < 1) return OR_ERR_ARG;
    lz_params P = {0, 0, 0, 0, 0};
    if (desc[0] == 0) {
        if (!(desc[2] == 0 && desc[3] == 0 && desc[4] == 0 && desc[5] == 0) &&
            !(3 <= desc[2] && desc[2] <= desc[3] && desc[3] <= 258 && 1 <= desc[4] && desc[4] <= desc[5] && desc[5] <= 32768))
            return OR_ERR_ARG;
        lz_params q = {desc[1] ? 1 : 0, desc[2], desc[3], desc[4], desc[5]};
        P = q;
    } else if (desc[0] != 1) return OR_ERR_ARG;
    bw_t w = {out, out_cap, 0, 0, 0, 0};
    uint64_t pos = 0;
    for (;;) {
        uint64_t dlen = len - pos; int fin = 1;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (dlen == chunk_len && pos + dlen < len) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        const uint8_t* base = data + (pos - hlen);
        bs_dec* root = bs_decide(base, bs_new_leaf(base, (int64_t)hlen, (int64_t)dlen, desc, &P), desc, &P, min_block_len);
        sink_t sk = { &w, 0 };
        bs_emit(base, root, desc, &P, fin, &sk);
        bs_free(root);
        pos += dlen;
        if (fin) break;
    }
    bw_finish(&w);
    if (w.overflow) return OR_ERR_CAPACITY;
    return (int64_t)w.n;
}

int64_t or_deflate_block_bits(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                              int strategy, uint64_t* bits, uint64_t cap) {
    if (strategy < 0 || strategy > 6) return OR_ERR_ARG;
    /* Count pass only (the CountingBitOutputStream of Lz77Huffman.decide, :45-53). */
    uint64_t pos = 0, nb = 0;
    for (;;) {
        uint64_t dlen = len - pos; int fin = 1;
        if (dlen > chunk_len) { dlen = chunk_len; fin = 0; }
        else if (dlen == chunk_len && pos + dlen < len) fin = 0;
        uint64_t hlen = pos < hist_limit ? pos : hist_limit;
        const uint8_t* base = data + (pos - hlen);
        sink_t s = { NULL, 0 };
        if (strategy == OR_UNCOMPRESSED) unc_compress(base, 0, (int64_t)hlen, (int64_t)dlen, fin, &s);
        else lz_compress(base, 0, (int64_t)hlen, (int64_t)dlen, &PRESETS[strategy], fin, &s, 0);
        if (nb < cap) bits[nb] = s.count;
        nb++; pos += dlen;
        if (fin) break;
    }
    return (int64_t)nb;
}

/* ------------------------------------------------------------------------------------------ */
/* Decoder: restates D/decomp/Open.java as one pass over an in-memory stream.                  */
/* The reference's buffering (two 64-bit bit buffers, 9-bit tables) affects speed only          */
/* (:802-804); its observable semantics are: bits LSB-first, UNEXPECTED_END_OF_STREAM exactly   */
/* when a needed bit lies past the input, and the check order restated below.                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct { const uint8_t* in; uint64_t nbits, pos; } br_t;

static int br_bit(br_t* r, uint32_t* v) {
    if (r->pos >= r->nbits) return OR_UNEXPECTED_END_OF_STREAM;
    *v = (r->in[r->pos >> 3] >> (r->pos & 7)) & 1u;
    r->pos++;
    return 0;
}
static int br_bits(br_t* r, int n, uint32_t* v) {           /* readBits :137-170 */
    if (r->pos + (uint64_t)n > r->nbits) return OR_UNEXPECTED_END_OF_STREAM;
    uint32_t x = 0;
    for (int i = 0; i < n; i++) { x |= (uint32_t)((r->in[r->pos >> 3] >> (r->pos & 7)) & 1u) << i; r->pos++; }
    *v = x;
    return 0;
}

/* codeLengthsToCodeTree (:705-756), including its exact error detection order. */
static int code_tree(const uint8_t* lens, int n, int16_t* tree /* >= 2*(n-1) */, int* tree_len) {
    uint16_t pairs[320];
    for (int i = 0; i < n; i++) pairs[i] = (uint16_t)(lens[i] << 11 | i);
    for (int i = 1; i < n; i++) {                           /* Arrays.sort ascending */
        uint16_t v = pairs[i]; int j = i - 1;
        while (j >= 0 && pairs[j] > v) { pairs[j + 1] = pairs[j]; j--; }
        pairs[j + 1] = v;
    }
    int k = 0;
    while (k < n && (pairs[k] >> 11) == 0) k++;
    int numCodes = n - k;
    if (numCodes < 2) return OR_HUFFMAN_CODE_UNDER_FULL;
    int rlen = (numCodes - 1) * 2;
    int next = 0, rend = 2, cur = 1;
    for (; k < n; k++) {
        int pair = pairs[k];
        for (int cl = pair >> 11; cur < cl; cur++) {
            for (int e = rend; next < e; next++) {
                if (rend >= rlen) return OR_HUFFMAN_CODE_UNDER_FULL;
                tree[next] = (int16_t)rend;
                rend += 2;
            }
        }
        if (next >= rend) return OR_HUFFMAN_CODE_OVER_FULL;
        tree[next] = (int16_t)~(pair & 0x7FF);
        next++;
    }
    if (rend != rlen) return -100;                          /* AssertionError("Unreachable") */
    if (next < rend) return OR_HUFFMAN_CODE_UNDER_FULL;
    *tree_len = rlen;
    return 0;
}

static int decode_sym(br_t* r, const int16_t* tree, int* sym) {   /* decodeSymbol :634-646 */
    int node = 0;
    while (node >= 0) {
        uint32_t b;
        int e = br_bit(r, &b);
        if (e) return e;
        node = tree[node + (int)b];
    }
    *sym = ~node;
    return 0;
}

static const int16_t RUN_BASE[29] = {3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
static const int8_t  RUN_EXTRA[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
static const int32_t DIST_BASE[30] = {1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577};
static const int8_t  DIST_EXTRA[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};

typedef struct { uint8_t* out; uint64_t cap, n; } ob_t;

/* HuffmanBlock(true) (D/decomp/Open.java:336-431): the dynamic header after BFINAL/BTYPE, with its
 * exact check order.  *dt = NULL for the empty distance code (:398-401). */
static int dynamic_header(br_t* r, int16_t* litTree, int16_t* distTree, int16_t* clTree, const int16_t** dt) {
    uint32_t hlit, hdist, hclen, v;
    int err, tl;
#define HCHK(x) do { err = (x); if (err) return err; } while (0)
    HCHK(br_bits(r, 5, &hlit)); HCHK(br_bits(r, 5, &hdist)); HCHK(br_bits(r, 4, &hclen));
    int numLit = (int)hlit + 257, numDist = (int)hdist + 1, numCl = (int)hclen + 4;
    uint8_t clLen[19]; memset(clLen, 0, sizeof clLen);
    for (int i = 0; i < numCl; i++) { HCHK(br_bits(r, 3, &v)); clLen[CLC_ORDER[i]] = (uint8_t)v; }
    HCHK(code_tree(clLen, 19, clTree, &tl));
    uint8_t lens[320];
    int total = numLit + numDist, runVal = -1;
    for (int i = 0; i < total;) {
        int sym;
        HCHK(decode_sym(r, clTree, &sym));
        if (sym < 16) { runVal = sym; lens[i++] = (uint8_t)sym; }
        else {
            int runLen;
            if (sym == 16) {
                if (runVal == -1) HCHK(OR_NO_PREVIOUS_CODE_LENGTH_TO_COPY);
                HCHK(br_bits(r, 2, &v)); runLen = (int)v + 3;
            } else if (sym == 17) { runVal = 0; HCHK(br_bits(r, 3, &v)); runLen = (int)v + 3; }
            else { runVal = 0; HCHK(br_bits(r, 7, &v)); runLen = (int)v + 11; }
            for (; runLen > 0; runLen--, i++) {
                if (i >= total) HCHK(OR_CODE_LENGTH_CODE_OVER_FULL);
                lens[i] = (uint8_t)runVal;
            }
        }
    }
    if (lens[256] == 0) HCHK(OR_END_OF_BLOCK_CODE_ZERO_LENGTH);
    HCHK(code_tree(lens, numLit, litTree, &tl));
    uint8_t dl[32]; int nd = numDist;
    memcpy(dl, lens + numLit, (size_t)numDist);
    if (nd == 1 && dl[0] == 0) { *dt = NULL; return 0; }    /* empty distance code :398-401 */
    int one = 0, other = 0;
    for (int i = 0; i < nd; i++) { if (dl[i] == 1) one++; else if (dl[i] > 1) other++; }
    if (one == 1 && other == 0) {                            /* :411-425 */
        for (int i = nd; i < 32; i++) dl[i] = 0;
        nd = 32; dl[31] = 1;
    }
    HCHK(code_tree(dl, nd, distTree, &tl));
    *dt = distTree;
    return 0;
#undef HCHK
}

/* One raw DEFLATE stream (or a block-aligned range of one): Open.read (:83-124) run to the end.
 * Range form (multi-GPU shards): decoding starts at bit `start_bit` with `dict_len` bytes of
 * preceding output available to copies (the reference's 32 KiB ring, :592-603), and stops at the
 * first block boundary == `end_bit` (UINT64_MAX: after the final block). */
/* the reserved symbol of the calling thread's last RESERVED_*_SYMBOL error (the reference's message
 * appends it: "Reserved run length symbol: " + sym, D/decomp/Open.java:516, 550), else -1 */
static _Thread_local int or_err_sym = -1;
int or_error_symbol(void) { return or_err_sym; }

int or_inflate_range(const uint8_t* in, uint64_t in_len, uint64_t start_bit, uint64_t end_bit,
                     const uint8_t* dict, uint64_t dict_len, uint8_t* out, uint64_t out_cap,
                     uint64_t* out_len, uint64_t* consumed_bits) {
    br_t r = {in, in_len * 8, start_bit};
    uint64_t n = 0;
    if (dict_len > 32768) { dict += dict_len - 32768; dict_len = 32768; }
    int err = 0, last = 0;
    or_err_sym = -1;
    int16_t litTree[2 * 288], distTree[2 * 32], clTree[2 * 19];
    int16_t fixLit[2 * 288], fixDist[2 * 32];
    {
        uint8_t l[288], d[32]; int tl;
        for (int i = 0; i < 288; i++) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;  /* :812-830 */
        for (int i = 0; i < 32; i++) d[i] = 5;
        code_tree(l, 288, fixLit, &tl);
        code_tree(d, 32, fixDist, &tl);
    }
#define CHK(x) do { err = (x); if (err) goto fail; } while (0)
    while (!last) {                                          /* Open.read :83-110 */
        uint32_t bf, bt;
        if (r.pos == end_bit) break;
        CHK(br_bits(&r, 1, &bf));
        last = (int)bf;
        CHK(br_bits(&r, 2, &bt));
        if (bt == 3) CHK(OR_RESERVED_BLOCK_TYPE);
        if (bt == 0) {                                       /* UncompressedBlock :232-297 */
            uint32_t pad, ln, nln;
            CHK(br_bits(&r, (int)((8 - (r.pos & 7)) & 7), &pad));
            CHK(br_bits(&r, 16, &ln));
            CHK(br_bits(&r, 16, &nln));
            if (ln != (nln ^ 0xFFFF)) CHK(OR_UNCOMPRESSED_BLOCK_LENGTH_MISMATCH);
            uint64_t avail = (r.nbits - r.pos) / 8;
            uint64_t take = ln < avail ? ln : avail;
            if (n + take > out_cap) { err = OR_ERR_CAPACITY; goto fail; }
            memcpy(out + n, in + (r.pos >> 3), (size_t)take);
            n += take; r.pos += take * 8;
            if (take < ln) CHK(OR_UNEXPECTED_END_OF_STREAM);
            continue;
        }
        const int16_t* lt; const int16_t* dt;
        if (bt == 1) { lt = fixLit; dt = fixDist; }
        else {
            CHK(dynamic_header(&r, litTree, distTree, clTree, &dt));
            lt = litTree;
        }
        for (;;) {                                           /* HuffmanBlock.read :446-618 */
            int sym;
            CHK(decode_sym(&r, lt, &sym));
            if (sym < 256) {
                if (n >= out_cap) { err = OR_ERR_CAPACITY; goto fail; }
                out[n++] = (uint8_t)sym;
                continue;
            }
            if (sym == 256) break;
            if (sym > 285) { or_err_sym = sym; CHK(OR_RESERVED_LENGTH_SYMBOL); }  /* :513-517, :655-660 */
            uint32_t e;
            CHK(br_bits(&r, RUN_EXTRA[sym - 257], &e));
            int run = RUN_BASE[sym - 257] + (int)e;
            if (!dt) CHK(OR_LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE);
            int dsym;
            CHK(decode_sym(&r, dt, &dsym));
            if (dsym > 29) { or_err_sym = dsym; CHK(OR_RESERVED_DISTANCE_SYMBOL); }   /* :548-551, :673-675 */
            CHK(br_bits(&r, DIST_EXTRA[dsym], &e));
            uint64_t dist = (uint64_t)DIST_BASE[dsym] + e;
            uint64_t dictLen = n + dict_len < 32768 ? n + dict_len : 32768;
            if (dist > dictLen) CHK(OR_COPY_FROM_BEFORE_DICTIONARY_START);   /* :592-593 */
            if (n + (uint64_t)run > out_cap) { err = OR_ERR_CAPACITY; goto fail; }
            for (int i = 0; i < run; i++, n++)                               /* byte-serial copy */
                out[n] = n >= dist ? out[n - dist] : dict[dict_len - (dist - n)];
        }
    }
    *out_len = n;
    *consumed_bits = r.pos;
    return 0;
fail:
    *out_len = n;
    *consumed_bits = r.pos;
    return err;
#undef CHK
}

int or_inflate(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
               uint64_t* out_len, uint64_t* consumed_bits) {
    return or_inflate_range(in, in_len, 0, UINT64_MAX, NULL, 0, out, out_cap, out_len, consumed_bits);
}

/* ------------------------------------------------------------------------------------------ */
/* Checksums (java.util.zip.CRC32 / Adler32).                                                  */
/* ------------------------------------------------------------------------------------------ */
static uint32_t CRC_T[256];
static int crc_ready = 0;
uint32_t or_crc32(uint32_t crc, const uint8_t* p, uint64_t n) {
    if (!crc_ready) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
            CRC_T[i] = c;
        }
        crc_ready = 1;
    }
    crc = ~crc;
    for (uint64_t i = 0; i < n; i++) crc = CRC_T[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}
uint32_t or_adler32(uint32_t adler, const uint8_t* p, uint64_t n) {
    uint32_t a = adler & 0xFFFF, b = adler >> 16;
    for (uint64_t i = 0; i < n; i++) { a = (a + p[i]) % 65521; b = (b + a) % 65521; }
    return b << 16 | a;
}

/* ------------------------------------------------------------------------------------------ */
/* Gzip / zlib containers.                                                                     */
/* ------------------------------------------------------------------------------------------ */
static int put(uint8_t* out, uint64_t cap, uint64_t* n, uint8_t b) {
    if (*n >= cap) return -1;
    out[(*n)++] = b;
    return 0;
}

int64_t or_gzip_compress(const uint8_t* data, uint64_t len, const or_gzip_meta* m,
                         uint8_t* out, uint64_t out_cap) {
    uint64_t n = 0;
    /* GzipMetadata ctor validation (D/GzipMetadata.java:44-67) */
    if ((m->has_mtime && m->mtime == 0) || (m->extra_flags >> 8) != 0 || (m->has_extra && m->extra_len > 0xFFFF))
        return OR_ERR_ARG;
    if (!((m->os >= 0 && m->os < 14) || m->os == 255)) return OR_ERR_ARG;
    uint8_t flg = (uint8_t)((m->is_text ? 1 : 0) | (m->has_header_crc ? 2 : 0) | (m->has_extra ? 4 : 0) |
                            (m->has_name ? 8 : 0) | (m->has_comment ? 16 : 0));    /* :176-187 */
    uint32_t mt = m->has_mtime ? m->mtime : 0;
    uint8_t hdr[10] = {0x1F, 0x8B, 8, flg, (uint8_t)mt, (uint8_t)(mt >> 8), (uint8_t)(mt >> 16), (uint8_t)(mt >> 24),
                       (uint8_t)m->extra_flags, (uint8_t)m->os};
    for (int i = 0; i < 10; i++) if (put(out, out_cap, &n, hdr[i])) return OR_ERR_CAPACITY;
    if (m->has_extra) {
        if (put(out, out_cap, &n, (uint8_t)m->extra_len) || put(out, out_cap, &n, (uint8_t)(m->extra_len >> 8))) return OR_ERR_CAPACITY;
        for (uint32_t i = 0; i < m->extra_len; i++) if (put(out, out_cap, &n, m->extra[i])) return OR_ERR_CAPACITY;
    }
    if (m->has_name) { for (const char* s = m->name;; s++) { if (put(out, out_cap, &n, (uint8_t)*s)) return OR_ERR_CAPACITY; if (!*s) break; } }
    if (m->has_comment) { for (const char* s = m->comment;; s++) { if (put(out, out_cap, &n, (uint8_t)*s)) return OR_ERR_CAPACITY; if (!*s) break; } }
    if (m->has_header_crc) {                                  /* :210-211 */
        uint32_t c = or_crc32(0, out, n);
        if (put(out, out_cap, &n, (uint8_t)c) || put(out, out_cap, &n, (uint8_t)(c >> 8))) return OR_ERR_CAPACITY;
    }
    int64_t d = or_deflate(data, len, 65536, 32768, OR_RLE_DYNAMIC, 0, out + n, out_cap - n);  /* D/GzipOutputStream.java:32-34 */
    if (d < 0) return d;
    n += (uint64_t)d;
    uint32_t crc = or_crc32(0, data, len);                    /* D/GzipOutputStream.java:64-70 */
    uint32_t isz = (uint32_t)len;
    uint8_t tr[8] = {(uint8_t)crc, (uint8_t)(crc >> 8), (uint8_t)(crc >> 16), (uint8_t)(crc >> 24),
                     (uint8_t)isz, (uint8_t)(isz >> 8), (uint8_t)(isz >> 16), (uint8_t)(isz >> 24)};
    for (int i = 0; i < 8; i++) if (put(out, out_cap, &n, tr[i])) return OR_ERR_CAPACITY;
    return (int64_t)n;
}

int or_gunzip(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
              or_gzip_meta* h, uint64_t* member_end) {
    uint64_t p = 0;
    *out_len = 0;
    memset(h, 0, sizeof *h);
#define NEED(k) do { if (p + (k) > in_len) return OR_UNEXPECTED_END_OF_STREAM; } while (0)
    NEED(2);                                                  /* GzipMetadata.read :73-146 */
    if (in[0] != 0x1F || in[1] != 0x8B) return OR_GZIP_INVALID_MAGIC_NUMBER;
    p = 2;
    NEED(1);
    if (in[p] != 8) return OR_UNSUPPORTED_COMPRESSION_METHOD;
    p++;
    NEED(1);
    uint8_t flg = in[p++];
    if (flg & 0xE0) return OR_GZIP_RESERVED_FLAGS_SET;
    NEED(4);
    uint32_t mt = (uint32_t)in[p] | (uint32_t)in[p + 1] << 8 | (uint32_t)in[p + 2] << 16 | (uint32_t)in[p + 3] << 24;
    p += 4;
    h->has_mtime = mt != 0; h->mtime = mt;
    NEED(1); h->extra_flags = in[p++];
    NEED(1);
    int os = in[p++];
    if (!(os < 14 || os == 255)) return OR_GZIP_UNSUPPORTED_OPERATING_SYSTEM;
    h->os = os;
    h->is_text = flg & 1;
    if (flg & 4) {
        NEED(2);
        uint32_t xl = (uint32_t)in[p] | (uint32_t)in[p + 1] << 8;
        p += 2;
        NEED(xl);
        h->has_extra = 1; h->extra_len = xl; h->extra = in + p;
        p += xl;
    }
    if (flg & 8) {
        h->has_name = 1; h->name = (const char*)(in + p);
        for (;;) { NEED(1); if (in[p++] == 0) break; }
    }
    if (flg & 16) {
        h->has_comment = 1; h->comment = (const char*)(in + p);
        for (;;) { NEED(1); if (in[p++] == 0) break; }
    }
    h->has_header_crc = (flg >> 1) & 1;
    if (h->has_header_crc) {
        uint32_t expect = or_crc32(0, in, p) & 0xFFFF;
        NEED(2);
        uint32_t actual = (uint32_t)in[p] | (uint32_t)in[p + 1] << 8;
        p += 2;
        if (actual != expect) return OR_HEADER_CHECKSUM_MISMATCH;
    }
    uint64_t bits = 0;
    int e = or_inflate(in + p, in_len - p, out, out_cap, out_len, &bits);   /* D/GzipInputStream.java:44 */
    if (e) return e;
    p += (bits + 7) / 8;                                      /* endExactly (D/decomp/Open.java:113-124) */
    NEED(8);                                                  /* D/GzipInputStream.java:76-87 */
    uint32_t crc = (uint32_t)in[p] | (uint32_t)in[p + 1] << 8 | (uint32_t)in[p + 2] << 16 | (uint32_t)in[p + 3] << 24;
    uint32_t isz = (uint32_t)in[p + 4] | (uint32_t)in[p + 5] << 8 | (uint32_t)in[p + 6] << 16 | (uint32_t)in[p + 7] << 24;
    p += 8;
    if (or_crc32(0, out, *out_len) != crc) return OR_DECOMPRESSED_CHECKSUM_MISMATCH;
    if ((uint32_t)*out_len != isz) return OR_DECOMPRESSED_SIZE_MISMATCH;
    *member_end = p;
    return 0;
#undef NEED
}

int64_t or_zlib_compress(const uint8_t* data, uint64_t len, int cinfo, int level,
                         uint8_t* out, uint64_t out_cap) {
    if (cinfo < 0 || cinfo > 7 || level < 0 || level > 3) return OR_ERR_ARG;   /* D/ZlibMetadata.java:31-32 */
    uint64_t n = 0;
    int cmf = 8 | cinfo << 4;                                 /* ZlibMetadata.write :86-103 */
    int flg = level << 6;
    flg |= (31 - (cmf << 8 | flg) % 31) % 31;
    if (put(out, out_cap, &n, (uint8_t)cmf) || put(out, out_cap, &n, (uint8_t)flg)) return OR_ERR_CAPACITY;
    int64_t d = or_deflate(data, len, 65536, 32768, OR_RLE_DYNAMIC, 0, out + n, out_cap - n);
    if (d < 0) return d;
    n += (uint64_t)d;
    uint32_t a = or_adler32(1, data, len);                    /* D/ZlibOutputStream.java:60-67 (big-endian) */
    for (int i = 3; i >= 0; i--) if (put(out, out_cap, &n, (uint8_t)(a >> (8 * i)))) return OR_ERR_CAPACITY;
    return (int64_t)n;
}

int or_zlib_decompress(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
    *out_len = 0;
    uint64_t p = 0;
    if (in_len < 2) return OR_UNEXPECTED_END_OF_STREAM;       /* ZlibMetadata.read :47-84 */
    int cmf = in[0], flg = in[1];
    p = 2;
    if ((cmf << 8 | flg) % 31 != 0) return OR_HEADER_CHECKSUM_MISMATCH;
    int cm = cmf & 0xF;
    if (cm != 8 && cm != 15) return OR_UNSUPPORTED_COMPRESSION_METHOD;
    if ((flg >> 5) & 1) {
        if (p + 4 > in_len) return OR_UNEXPECTED_END_OF_STREAM;
        p += 4;
    }
    if (cm == 8 && (cmf >> 4) > 7) return -3;                 /* IllegalArgumentException from the record ctor */
    uint64_t bits = 0;
    int e = or_inflate(in + p, in_len - p, out, out_cap, out_len, &bits);
    if (e) return e;
    p += (bits + 7) / 8;
    if (p + 4 > in_len) return OR_UNEXPECTED_END_OF_STREAM;   /* D/ZlibInputStream.java:70-79 */
    uint32_t expect = (uint32_t)in[p] << 24 | (uint32_t)in[p + 1] << 16 | (uint32_t)in[p + 2] << 8 | in[p + 3];
    if (or_adler32(1, out, *out_len) != expect) return OR_DECOMPRESSED_CHECKSUM_MISMATCH;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Decoder test support: the chain starts of the GPU decoder's header finder.                  */
/* ------------------------------------------------------------------------------------------ */
/* 64 bits from bit p on, LSB first (zeros past the input, as the GPU's zero-padded staging). */
static uint64_t scan_win64(const uint8_t* in, uint64_t in_len, uint64_t p) {
    uint64_t v = 0;
    const uint64_t b = p >> 3;
    for (int k = 7; k >= 0; k--) v = v << 8 | (b + (uint64_t)k < in_len ? in[b + k] : 0u);
    const uint32_t sh = (uint32_t)(p & 7);
    if (sh) v = v >> sh | (uint64_t)(b + 8 < in_len ? in[b + 8] : 0u) << (64 - sh);
    return v;
}

/* The header after a stored block is plausible: not BTYPE 3; stored -> LEN == ~NLEN; dynamic ->
 * a complete code-length code; fixed -> no check (bits past the input read as zeros). */
static int scan_next_plausible(const uint8_t* in, uint64_t in_len, uint64_t q) {
    const uint64_t h = scan_win64(in, in_len, q);
    const uint32_t bt = (uint32_t)(h >> 1) & 3u;
    if (bt == 3) return 0;
    if (bt == 0) {
        const uint64_t x = scan_win64(in, in_len, (q + 3 + 7) & ~7ull);
        return ((uint32_t)x & 0xFFFFu) == (((uint32_t)(x >> 16) & 0xFFFFu) ^ 0xFFFFu);
    }
    if (bt == 2) {
        const uint32_t ncl = (uint32_t)(h >> 13 & 15u) + 4;
        const uint64_t f = scan_win64(in, in_len, q + 17);
        uint32_t kr = 0, nz = 0;
        for (uint32_t i = 0; i < ncl; i++) { uint32_t l = (uint32_t)(f >> (3 * i)) & 7u; if (l) { kr += 128u >> l; nz++; } }
        return kr == 128 && nz >= 2;
    }
    return 1;
}

int64_t or_scan_headers(const uint8_t* in, uint64_t in_len, uint64_t lo, uint64_t hi, uint64_t* out, uint64_t cap) {
    const uint64_t nbits = in_len * 8;
    if (hi > nbits) hi = nbits;
    int16_t litTree[2 * 288], distTree[2 * 32], clTree[2 * 19];
    uint64_t n = 0;
    for (uint64_t p = lo; p + 3 <= hi; p++) {
        const uint64_t h = scan_win64(in, in_len, p);
        if (h & 1u) continue;                                     /* BFINAL = 1: not a chain start */
        const uint32_t bt = (uint32_t)(h >> 1) & 3u;
        int ok = 0;
        if (bt == 0) {                                            /* UncompressedBlock ctor :232-241 */
            const uint64_t al = (p + 3 + 7) & ~7ull;
            if (al - (p + 3) && (uint32_t)(h >> 3) & ((1u << (al - (p + 3))) - 1u)) continue;   /* padding 0 */
            const uint64_t x = scan_win64(in, in_len, al);
            const uint32_t ln = (uint32_t)x & 0xFFFFu, nln = (uint32_t)(x >> 16) & 0xFFFFu;
            if (ln != (nln ^ 0xFFFFu) || al + 32 + 8ull * ln > nbits) continue;
            ok = scan_next_plausible(in, in_len, al + 32 + 8ull * ln);
        } else if (bt == 2) {                                     /* HuffmanBlock(true) :336-431 */
            if (((h >> 3) & 31u) >= 30 || ((h >> 8) & 31u) >= 30) continue;
            /* complete code-length code first (a cheap necessary condition of code_tree's success) */
            const uint32_t ncl = (uint32_t)(h >> 13 & 15u) + 4;
            if (p + 17 + 3 * ncl > nbits) continue;
            const uint64_t f = scan_win64(in, in_len, p + 17);
            uint32_t kr = 0;
            for (uint32_t i = 0; i < ncl; i++) { uint32_t l = (uint32_t)(f >> (3 * i)) & 7u; if (l) kr += 128u >> l; }
            if (kr != 128) continue;
            br_t r = {in, nbits, p + 3};
            const int16_t* dt;
            ok = dynamic_header(&r, litTree, distTree, clTree, &dt) == 0;
        }
        if (ok) { if (n < cap) out[n] = p; n++; }
    }
    return (int64_t)n;
}
