// inflate_kernels.hip -- MI355X (gfx950) parallel DEFLATE decoder.
//
// Replaces InflaterInputStream.read -> Open.read -> {UncompressedBlock,HuffmanBlock}.read run to
// the end of one raw DEFLATE stream (D/InflaterInputStream.java:147-164, D/decomp/Open.java:83-620).
//
// A single DEFLATE stream has no block index, so the decoder speculates:
//   1. finder   every bit position is tested (32 per lane, bit-parallel btype masks); positions
//               that start a header passing the reference's own validity checks (dynamic: complete
//               code-length code, decodable code lengths, EOB present, complete litlen/distance
//               codes; stored: LEN == ~NLEN, zero padding, plausible successor) are candidates;
//   2. count    (one lane per candidate): decode blocks from the candidate until the first block
//               boundary at or past the next candidate, recording end bit, output size, status;
//   3. link     (host): follow end bit == candidate start from bit 0; boundaries that are not
//               candidates (fixed-Huffman blocks) are decoded on in parallel repair rounds;
//   4. emit     (one lane per linked chain): decode again into the final output at the chain's
//               offset.  A copy whose source precedes the chain waits (agent-scope acquire) on the
//               owning chains' completion flags; chains are claimed in order through a ticket, so a
//               lane only ever waits on chains whose lanes already run.  The loop is a per-token
//               step machine (bounded work per step) so a waiting lane never blocks its wave.
// Per-lane decoding is latency-bound, so: the bitstream is read through a double-buffered 16-byte
// prefetch, every Huffman table lives in LDS (lane-interleaved: entry e of lane l at e*64+l, bank
// conflict-free for any per-lane index), and the dynamic header is parsed in two passes over the
// stream bits so that no per-lane array (private scratch memory) is ever needed.
// Errors are the reference's DataFormatException Reasons, checked in the reference's order; the
// first error in stream order wins.
// D/ = /root/reference/src/io/nayuki/deflate/
#pragma once
#include "ndfl_common.hpp"
#include <vector>
#include <algorithm>
#include <unordered_map>
#include <string.h>
#include <stdlib.h>

namespace inf {

constexpr uint32_t SEG_BYTES = 65536;      // finder segment (compressed bytes)
constexpr uint32_t SEG_CAP = 256;          // candidates kept per finder segment
constexpr uint64_t NONE = ~0ull;

// per-lane LDS layout, in u16 entries (each entry is 64 lanes wide)
constexpr uint32_t PL = 8;                 // literal/length primary bits
constexpr uint32_t PD = 7;                 // distance primary bits (also the code-length code table)
constexpr uint32_t O_LIT = 0;
constexpr uint32_t O_DST = O_LIT + (1u << PL);
constexpr uint32_t O_LF = O_DST + (1u << PD);     // lit first[16]
constexpr uint32_t O_LC = O_LF + 16;              // lit count[16]
constexpr uint32_t O_LO = O_LC + 16;              // lit offs[16]
constexpr uint32_t O_DF = O_LO + 16;
constexpr uint32_t O_DC = O_DF + 16;
constexpr uint32_t O_DO = O_DC + 16;
constexpr uint32_t O_NX = O_DO + 16;              // running ranks during table fill
constexpr uint32_t LANE_ENTRIES = O_NX + 16;
constexpr uint32_t LDS_BYTES = LANE_ENTRIES * 64 * 2;
// global per-lane canonical symbol lists (lane-interleaved per wave): lit 288 + dist 32
constexpr uint32_t G_SORT = 320;

enum : uint32_t { ST_BOUNDARY = 0, ST_FINAL = 1, ST_ERROR = 2 };
enum : int { R_UEOS = 1, R_RESERVED_BLOCK_TYPE, R_LEN_MISMATCH, R_UNDER_FULL, R_OVER_FULL, R_NO_PREV,
             R_CL_OVER_FULL, R_EOB_ZERO, R_RESERVED_LEN, R_RESERVED_DIST, R_EMPTY_DIST, R_COPY_BEFORE,
             R_INTERNAL = 100 };

constexpr int CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// RUN_LENGTH_TABLE / DISTANCE_TABLE of D/decomp/Open.java:841-886 in closed form.
__device__ __forceinline__ void run_base(uint32_t i, uint32_t& base, uint32_t& ne) {
    if (i < 8) { base = i + 3; ne = 0; }
    else if (i == 28) { base = 258; ne = 0; }
    else { ne = (i >> 2) - 1; base = ((4u + (i & 3)) << ne) + 3; }
}
__device__ __forceinline__ void dist_base(uint32_t d, uint32_t& base, uint32_t& ne) {
    if (d < 4) { base = d + 1; ne = 0; }
    else { ne = (d >> 1) - 1; base = ((2u + (d & 1)) << ne) + 1; }
}

struct In {
    const uint32_t* w;
    uint64_t nwords;
    uint64_t nbits;
    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return i < nwords ? w[i] : 0u; }
    __device__ __forceinline__ u32x4 ld4(uint64_t g) const {
        if (g * 4 + 3 < nwords) return *(const u32x4*)(w + g * 4);
        u32x4 r;
        r.x = ld(g * 4); r.y = ld(g * 4 + 1); r.z = ld(g * 4 + 2); r.w = ld(g * 4 + 3);
        return r;
    }
};

__device__ __forceinline__ uint32_t rev_bits(uint32_t v, uint32_t n) { return __brev(v) >> (32 - n); }

// Simple bit reader (finder / validation paths).
struct Rd {
    uint64_t pos, bb;
    uint32_t bn;
    uint64_t nextw;
    __device__ __forceinline__ void init(const In& in, uint64_t p) {
        pos = p; nextw = p >> 5;
        bb = (uint64_t)(in.ld(nextw) >> (p & 31));
        bn = 32 - (uint32_t)(p & 31);
        nextw++;
        fill(in);
    }
    __device__ __forceinline__ void fill(const In& in) {
        if (bn <= 32) { bb |= (uint64_t)in.ld(nextw) << bn; bn += 32; nextw++; }
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1u); }
    __device__ __forceinline__ void skip(uint32_t n) { bb >>= n; bn -= n; pos += n; }
    __device__ __forceinline__ uint32_t get(const In& in, uint32_t n) {
        fill(in);
        uint32_t v = n ? peek(n) : 0u;
        skip(n);
        return v;
    }
};

// Decode-lane bit reader: 64-bit active buffer refilled 32 bits at a time from a 4-word group,
// with the next 4-word group already in flight (one 16-byte load per 128 bits consumed).
struct Rp {
    uint64_t bb;
    uint32_t bn;
    uint32_t ci;          // next word of `cur` (0..3)
    uint64_t qw;          // group index of `cur`
    uint64_t pos;
    u32x4 cur, nxt;
    __device__ __forceinline__ static uint32_t pick(const u32x4& v, uint32_t i) {
        uint32_t a = (i & 1) ? v.y : v.x, b = (i & 1) ? v.w : v.z;
        return (i & 2) ? b : a;
    }
    __device__ __forceinline__ void adv(const In& in) {
        if (++ci == 4) { cur = nxt; qw++; nxt = in.ld4(qw + 1); ci = 0; }
    }
    __device__ __forceinline__ void init(const In& in, uint64_t p) {
        pos = p;
        qw = p >> 7;
        cur = in.ld4(qw);
        nxt = in.ld4(qw + 1);
        ci = (uint32_t)(p >> 5) & 3;
        bb = (uint64_t)(pick(cur, ci) >> (p & 31));
        bn = 32 - (uint32_t)(p & 31);
        adv(in);
        fill(in);
    }
    __device__ __forceinline__ void fill(const In& in) {
        if (bn <= 32) { bb |= (uint64_t)pick(cur, ci) << bn; bn += 32; adv(in); }
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1u); }
    __device__ __forceinline__ void skip(uint32_t n) { bb >>= n; bn -= n; pos += n; }
    __device__ __forceinline__ uint32_t get(const In& in, uint32_t n) {
        fill(in);
        uint32_t v = n ? peek(n) : 0u;
        skip(n);
        return v;
    }
};

// codeLengthsToCodeTree's error detection (D/decomp/Open.java:705-756) from per-length counts.
__device__ int tree_check(const uint32_t (&cnt)[16]) {
    uint32_t num = 0, maxL = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) { num += cnt[l]; if (cnt[l]) maxL = (uint32_t)l; }
    if (num < 2) return R_UNDER_FULL;
    const uint64_t R = 2ull * (num - 1);
    uint64_t next = 0, end = 2;
#pragma unroll
    for (uint32_t l = 1; l < 16; l++) {
        if (l > maxL) break;
        if (l > 1) {
            uint64_t open = end - next;
            if (open > 0) {
                if (end + 2 * (open - 1) >= R) return R_UNDER_FULL;
                next = end;
                end += 2 * open;
            }
        }
        uint64_t c = cnt[l];
        if (c > end - next) return R_OVER_FULL;
        next += c;
    }
    if (end != R) return R_INTERNAL;
    if (next < end) return R_UNDER_FULL;
    return 0;
}

// LDS view of one lane's tables.
struct LT {
    uint16_t* b;          // lane base (entry e at b[e*64])
    __device__ __forceinline__ uint16_t& at(uint32_t e) const { return b[e * 64]; }
};

// ---- dynamic block header (D/decomp/Open.java:336-431) ---------------------------------------
// Pass 1 decodes the code lengths into per-length counts (and validates in the reference's
// order); pass 2 re-reads the same bits to fill the LDS primary tables and the canonical symbol
// lists.  `gs` is this lane's canonical-list base in global memory (stride 64).
__device__ int parse_dynamic(Rp& rd, const In& in, LT t, uint16_t* gs, bool& empty_dist) {
    const uint32_t hlit = rd.get(in, 5), hdist = rd.get(in, 5), hclen = rd.get(in, 4);
    if (rd.pos > in.nbits) return R_UEOS;
    const uint32_t numLit = hlit + 257, numDist = hdist + 1, numCl = hclen + 4;
    uint32_t cl[19];
#pragma unroll
    for (int i = 0; i < 19; i++) cl[i] = 0;
#pragma unroll
    for (int i = 0; i < 19; i++)
        if ((uint32_t)i < numCl) cl[CLO[i]] = rd.get(in, 3);
    if (rd.pos > in.nbits) return R_UEOS;
    // code-length code (D/decomp/Open.java:341-344)
    uint32_t cc[16];
#pragma unroll
    for (int l = 0; l < 16; l++) cc[l] = 0;
#pragma unroll
    for (int l = 1; l < 8; l++) {
        uint32_t c = 0;
#pragma unroll
        for (int s = 0; s < 19; s++) c += cl[s] == (uint32_t)l;
        cc[l] = c;
    }
    int e = tree_check(cc);
    if (e) return e;
    {
        uint32_t first[8];
        uint32_t code = 0;
        first[0] = 0;
#pragma unroll
        for (int l = 1; l < 8; l++) { code = (code + (l > 1 ? cc[l - 1] : 0)) << 1; first[l] = code; }
        for (uint32_t k = 0; k < (1u << PD); k++) t.at(O_DST + k) = 0;
#pragma unroll
        for (int s = 0; s < 19; s++) {
            const uint32_t l = cl[s];
            if (l) {
                uint32_t rank = 0;
#pragma unroll
                for (int s2 = 0; s2 < s; s2++) rank += cl[s2] == l;
                uint32_t f = 0;
#pragma unroll
                for (int l2 = 1; l2 < 8; l2++) f = (l == (uint32_t)l2) ? first[l2] : f;
                const uint32_t r = rev_bits(f + rank, l);
                const uint16_t ent = (uint16_t)(s | (l << 9));
                for (uint32_t k = r; k < (1u << PD); k += (1u << l)) t.at(O_DST + k) = ent;
            }
        }
    }
    // pass 1
    const Rp saved = rd;
    for (int l = 0; l < 16; l++) { t.at(O_LC + l) = 0; t.at(O_DC + l) = 0; }
    const uint32_t total = numLit + numDist;
    uint32_t i = 0;
    int runVal = -1;
    uint32_t eob = 0, ones = 0, other = 0, d0 = 0, d31 = 0;
    while (i < total) {
        rd.fill(in);
        const uint32_t ent = t.at(O_DST + rd.peek(PD));
        rd.skip(ent >> 9);
        const uint32_t sym = ent & 0x1FF;
        if (rd.pos > in.nbits) return R_UEOS;
        uint32_t run = 1, v;
        if (sym < 16) { v = sym; runVal = (int)sym; }
        else if (sym == 16) {
            if (runVal == -1) return R_NO_PREV;
            run = rd.get(in, 2) + 3; v = (uint32_t)runVal;
        } else if (sym == 17) { runVal = 0; run = rd.get(in, 3) + 3; v = 0; }
        else { runVal = 0; run = rd.get(in, 7) + 11; v = 0; }
        if (rd.pos > in.nbits) return R_UEOS;
        if (i + run > total) return R_CL_OVER_FULL;
        const uint32_t en = i + run;
        if (i < numLit) {
            const uint32_t c = min(en, numLit) - i;
            if (v) t.at(O_LC + v) += (uint16_t)c;
            if (i <= 256 && 256 < en) eob = v;
        }
        if (en > numLit) {
            const uint32_t a = max(i, numLit) - numLit, b = en - numLit, c = b - a;
            if (v) { t.at(O_DC + v) += (uint16_t)c; if (v == 1) ones += c; else other += c; }
            if (a == 0) d0 = v;
            if (a <= 31 && 31 < b) d31 = v;
        }
        i = en;
    }
    if (eob == 0) return R_EOB_ZERO;
    uint32_t lc[16], dc[16];
#pragma unroll
    for (int l = 0; l < 16; l++) { lc[l] = l ? t.at(O_LC + l) : 0u; dc[l] = l ? t.at(O_DC + l) : 0u; }
    e = tree_check(lc);
    if (e) return e;
    bool pad31 = false;
    empty_dist = (numDist == 1 && d0 == 0);
    if (!empty_dist) {
        if (ones == 1 && other == 0) { pad31 = true; dc[1] += 1; if (numDist == 32 && d31 == 1) dc[1] -= 1; }
        e = tree_check(dc);
        if (e) return e;
    }
    {
        uint32_t code = 0, off = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            code = (code + (l > 1 ? lc[l - 1] : 0)) << 1;
            t.at(O_LF + l) = (uint16_t)code; t.at(O_LO + l) = (uint16_t)off; t.at(O_LC + l) = (uint16_t)lc[l];
            off += lc[l];
        }
        code = 0; off = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            code = (code + (l > 1 ? dc[l - 1] : 0)) << 1;
            t.at(O_DF + l) = (uint16_t)code; t.at(O_DO + l) = (uint16_t)off; t.at(O_DC + l) = (uint16_t)dc[l];
            off += dc[l];
        }
    }
    // pass 2: literal/length table + canonical list; distance lengths packed into 4 registers
    for (uint32_t k = 0; k < (1u << PL); k++) t.at(O_LIT + k) = 0;
    for (int l = 0; l < 16; l++) t.at(O_NX + l) = 0;
    rd = saved;
    i = 0;
    runVal = 0;
    uint32_t dpk[4] = {0, 0, 0, 0};
    while (i < total) {
        rd.fill(in);
        const uint32_t ent = t.at(O_DST + rd.peek(PD));
        rd.skip(ent >> 9);
        const uint32_t sym = ent & 0x1FF;
        uint32_t run = 1, v;
        if (sym < 16) { v = sym; runVal = (int)sym; }
        else if (sym == 16) { run = rd.get(in, 2) + 3; v = (uint32_t)runVal; }
        else if (sym == 17) { runVal = 0; run = rd.get(in, 3) + 3; v = 0; }
        else { runVal = 0; run = rd.get(in, 7) + 11; v = 0; }
        if (v) {
            for (uint32_t k = 0; k < run; k++) {
                const uint32_t idx = i + k;
                if (idx < numLit) {
                    const uint32_t rank = t.at(O_NX + v);
                    t.at(O_NX + v) = (uint16_t)(rank + 1);
                    gs[(t.at(O_LO + v) + rank) * 64] = (uint16_t)idx;
                    if (v <= PL) {
                        const uint32_t r = rev_bits(t.at(O_LF + v) + rank, v);
                        const uint16_t en2 = (uint16_t)(idx | (v << 9));
                        for (uint32_t q = r; q < (1u << PL); q += (1u << v)) t.at(O_LIT + q) = en2;
                    }
                } else {
                    const uint32_t j = idx - numLit;
                    const uint32_t sh = (j & 7) * 4, w = j >> 3;
                    dpk[0] |= (w == 0) ? (v << sh) : 0u;
                    dpk[1] |= (w == 1) ? (v << sh) : 0u;
                    dpk[2] |= (w == 2) ? (v << sh) : 0u;
                    dpk[3] |= (w == 3) ? (v << sh) : 0u;
                }
            }
        }
        i += run;
    }
    if (empty_dist) return 0;
    if (pad31) dpk[3] |= 1u << 28;      // dummy code at index 31 (D/decomp/Open.java:411-425)
    for (uint32_t k = 0; k < (1u << PD); k++) t.at(O_DST + k) = 0;
    for (int l = 0; l < 16; l++) t.at(O_NX + l) = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
        const uint32_t v = (dpk[j >> 3] >> ((j & 7) * 4)) & 15u;
        if (v) {
            const uint32_t rank = t.at(O_NX + v);
            t.at(O_NX + v) = (uint16_t)(rank + 1);
            gs[(288 + t.at(O_DO + v) + rank) * 64] = (uint16_t)j;
            if (v <= PD) {
                const uint32_t r = rev_bits(t.at(O_DF + v) + rank, v);
                const uint16_t en2 = (uint16_t)(j | (v << 9));
                for (uint32_t q = r; q < (1u << PD); q += (1u << v)) t.at(O_DST + q) = en2;
            }
        }
    }
    return 0;
}

// Literal/length symbol: LDS primary, canonical slow path for longer codes.
__device__ __forceinline__ uint32_t dec_lit(Rp& rd, const In& in, LT t, const uint16_t* gs) {
    rd.fill(in);
    const uint32_t e = t.at(O_LIT + rd.peek(PL));
    if (e >> 9) { rd.skip(e >> 9); return e & 0x1FF; }
    const uint32_t r15 = rev_bits(rd.peek(15), 15);
    for (uint32_t l = PL + 1; l < 16; l++) {
        const uint32_t idx = (r15 >> (15 - l)) - t.at(O_LF + l);
        if (idx < t.at(O_LC + l)) { rd.skip(l); return gs[(t.at(O_LO + l) + idx) * 64]; }
    }
    rd.skip(15);
    return 0xFFFF;
}
__device__ __forceinline__ uint32_t dec_dist(Rp& rd, const In& in, LT t, const uint16_t* gs) {
    rd.fill(in);
    const uint32_t e = t.at(O_DST + rd.peek(PD));
    if (e >> 9) { rd.skip(e >> 9); return e & 0x1FF; }
    const uint32_t r15 = rev_bits(rd.peek(15), 15);
    for (uint32_t l = PD + 1; l < 16; l++) {
        const uint32_t idx = (r15 >> (15 - l)) - t.at(O_DF + l);
        if (idx < t.at(O_DC + l)) { rd.skip(l); return gs[(288 + t.at(O_DO + l) + idx) * 64]; }
    }
    rd.skip(15);
    return 0xFFFF;
}

// Fixed-Huffman tables (D/decomp/Open.java:812-830): 9-bit literal/length and 5-bit distance
// primaries, shared by all lanes (global, cache-resident).
struct FixedTabs { uint16_t lit[512]; uint16_t dist[32]; };

// ---- finder ---------------------------------------------------------------------------------
// Strict check of a dynamic block header at bit p with running Kraft sums (no arrays): accepts
// exactly the headers the reference accepts.
__device__ bool strict_dynamic(const In& in, uint64_t p) {
    Rd rd; rd.init(in, p + 3);
    const uint32_t hlit = rd.get(in, 5), hdist = rd.get(in, 5), hclen = rd.get(in, 4);
    const uint32_t numLit = hlit + 257, numDist = hdist + 1, numCl = hclen + 4;
    uint32_t cl[19];
#pragma unroll
    for (int i = 0; i < 19; i++) cl[i] = 0;
#pragma unroll
    for (int i = 0; i < 19; i++)
        if ((uint32_t)i < numCl) cl[CLO[i]] = rd.get(in, 3);
    uint32_t cc[8];
#pragma unroll
    for (int l = 0; l < 8; l++) cc[l] = 0;
#pragma unroll
    for (int l = 1; l < 8; l++) {
        uint32_t c = 0;
#pragma unroll
        for (int s = 0; s < 19; s++) c += cl[s] == (uint32_t)l;
        cc[l] = c;
    }
    uint32_t kr = 0;
#pragma unroll
    for (int l = 1; l < 8; l++) kr += cc[l] << (7 - l);
    if (kr != 128) return false;
    uint32_t first[8], offs[8];
    {
        uint32_t code = 0, off = 0;
        first[0] = 0; offs[0] = 0;
#pragma unroll
        for (int l = 1; l < 8; l++) { code = (code + (l > 1 ? cc[l - 1] : 0)) << 1; first[l] = code; offs[l] = off; off += cc[l]; }
    }
    // canonical symbol list packed 6 x 5 bits per register
    uint32_t pk[4] = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 19; s++) {
        const uint32_t l = cl[s];
        if (l) {
            uint32_t rank = 0, o = 0;
#pragma unroll
            for (int s2 = 0; s2 < s; s2++) rank += cl[s2] == l;
#pragma unroll
            for (int l2 = 1; l2 < 8; l2++) o = (l == (uint32_t)l2) ? offs[l2] : o;
            const uint32_t pos = o + rank, wd = pos / 6, sh = (pos % 6) * 5;
#pragma unroll
            for (int q = 0; q < 4; q++) pk[q] |= (wd == (uint32_t)q) ? ((uint32_t)s << sh) : 0u;
        }
    }
    const uint32_t total = numLit + numDist;
    uint32_t i = 0;
    int runVal = -1;
    uint32_t litK = 0, distK = 0, ones = 0, other = 0, eob = 0, d0 = 0, d31 = 0;
    while (i < total) {
        rd.fill(in);
        const uint32_t r7 = rev_bits(rd.peek(7), 7);
        uint32_t sym = 0, len = 0, gi = 0;
#pragma unroll
        for (int l = 1; l < 8; l++) {
            const uint32_t idx = (r7 >> (7 - l)) - first[l];
            if (len == 0 && idx < cc[l]) { len = (uint32_t)l; gi = offs[l] + idx; }
        }
        {
            const uint32_t wd = gi / 6, sh = (gi % 6) * 5;
            uint32_t x = pk[0];
            x = wd == 1 ? pk[1] : x; x = wd == 2 ? pk[2] : x; x = wd == 3 ? pk[3] : x;
            sym = (x >> sh) & 31u;
        }
        rd.skip(len);
        uint32_t run = 1;
        if (sym < 16) runVal = (int)sym;
        else if (sym == 16) { if (runVal < 0) return false; run = rd.get(in, 2) + 3; }
        else if (sym == 17) { runVal = 0; run = rd.get(in, 3) + 3; }
        else { runVal = 0; run = rd.get(in, 7) + 11; }
        if (i + run > total || rd.pos > in.nbits) return false;
        const uint32_t v = (uint32_t)runVal;
        const uint32_t en = i + run;
        if (i < numLit) {
            const uint32_t c = min(en, numLit) - i;
            if (v) { litK += c * (32768u >> v); if (litK > 32768u) return false; }
            if (i <= 256 && 256 < en) eob = v;
        }
        if (en > numLit) {
            const uint32_t a = max(i, numLit) - numLit, b2 = en - numLit, c = b2 - a;
            if (v) { distK += c * (32768u >> v); if (distK > 32768u) return false; if (v == 1) ones += c; else other += c; }
            if (a == 0) d0 = v;
            if (a <= 31 && 31 < b2) d31 = v;
        }
        i = en;
    }
    if (eob == 0 || litK != 32768u) return false;
    if (numDist == 1 && d0 == 0) return true;
    if (ones == 1 && other == 0) return !(numDist == 32 && d31 == 1);
    return distK == 32768u;
}

// A stored block at p (LEN == ~NLEN already checked) must be final or be followed by a plausible
// header: not btype 3; stored -> LEN == ~NLEN; dynamic -> complete code-length code.
__device__ bool strict_stored(const In& in, uint64_t p) {
    Rd rd; rd.init(in, p);
    const uint32_t bf = rd.get(in, 1);
    const uint64_t al = (p + 3 + 7) & ~7ull;
    rd.init(in, al);
    const uint32_t ln = rd.get(in, 16);
    const uint64_t q = al + 32 + 8ull * ln;
    if (bf) return true;
    if (q + 3 > in.nbits) return false;
    rd.init(in, q);
    rd.get(in, 1);
    const uint32_t bt2 = rd.get(in, 2);
    if (bt2 == 3) return false;
    if (bt2 == 0) {
        const uint64_t al2 = (q + 3 + 7) & ~7ull;
        rd.init(in, al2);
        const uint32_t l2 = rd.get(in, 16), n2 = rd.get(in, 16);
        return l2 == (n2 ^ 0xFFFFu);
    }
    if (bt2 == 2) {
        rd.get(in, 10);
        const uint32_t ncl = rd.get(in, 4) + 4;
        uint32_t kr = 0, nz = 0;
        for (uint32_t i = 0; i < ncl; i++) { uint32_t l = rd.get(in, 3); if (l) { kr += 128u >> l; nz++; } }
        return kr == 128 && nz >= 2;
    }
    return true;   // fixed block: no cheap check
}

}  // namespace inf

// Header finder over every bit position.  Each thread tests 32 consecutive positions: btype masks
// for all 32 come from two shifts of a 64-bit window; the per-position tests read a 128-bit
// funnel-shifted window with compile-time offsets only (no private arrays).  Survivors are
// gathered per workgroup in LDS and strictly validated one per lane, then appended to their
// 64 KiB segment's list.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_find_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, uint32_t* seg_cnt, uint64_t* seg_list) {
    using namespace inf;
    __shared__ uint64_t cand[1024];
    __shared__ uint32_t ncand;
    if (threadIdx.x == 0) ncand = 0;
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p0 = t * 32;
    In in{w, nwords, nbits};
    if (p0 < nbits) {
        const uint32_t w0 = in.ld(t), w1 = in.ld(t + 1), w2 = in.ld(t + 2), w3 = in.ld(t + 3), w4 = in.ld(t + 4);
        const uint64_t W = (uint64_t)w0 | ((uint64_t)w1 << 32);
        const uint32_t b1 = (uint32_t)(W >> 1), b2 = (uint32_t)(W >> 2);
        uint32_t valid = 0xFFFFFFFFu;
        if (p0 + 35 > nbits) valid = (nbits >= p0 + 3) ? (uint32_t)((1ull << (nbits - p0 - 2)) - 1) : 0u;
        uint32_t m2 = ~b1 & b2 & valid;
        uint32_t m0 = ~b1 & ~b2 & valid;
        const uint64_t lo = W, hi = (uint64_t)w2 | ((uint64_t)w3 << 32);
        while (m2) {
            const uint32_t o = __builtin_ctz(m2);
            m2 &= m2 - 1;
            // 96 bits starting at position o: x0 = bits [o, o+64), x1 = bits [o+64, o+96)
            const uint64_t x0 = o ? (lo >> o) | (hi << (64 - o)) : lo;
            const uint64_t hw = (uint64_t)w3 | ((uint64_t)w4 << 32);
            const uint32_t x1 = (uint32_t)((o ? (hi >> o) | (hw << (64 - o)) : hi));
            const uint32_t ncl = (uint32_t)(x0 >> 13) & 15u;
            // 19 x 3-bit lengths at offsets 17..73 (relative to o)
            uint32_t kr = 0, nz = 0;
#pragma unroll
            for (int i = 0; i < 19; i++) {
                const int off = 17 + 3 * i;
                uint32_t l;
                if (off + 3 <= 64) l = (uint32_t)(x0 >> off) & 7u;
                else if (off >= 64) l = (x1 >> (off - 64)) & 7u;
                else l = (uint32_t)((x0 >> off) | ((uint64_t)x1 << (64 - off))) & 7u;
                const bool in_range = (uint32_t)i < ncl + 4;
                kr += (in_range && l) ? (128u >> l) : 0u;
                nz += in_range && l;
            }
            if (kr == 128 && nz >= 2 && p0 + o + 17 + 3 * (ncl + 4) <= nbits) {
                uint32_t k = atomicAdd(&ncand, 1u);
                if (k < 1024) cand[k] = (p0 + o) | (1ull << 63);
            }
        }
        while (m0) {
            const uint32_t o = __builtin_ctz(m0);
            m0 &= m0 - 1;
            const uint32_t q = o + 3, al = (q + 7) & ~7u;            // al <= 40
            const uint64_t x = al ? (lo >> al) | (hi << (64 - al)) : lo;
            const uint32_t pad = al > q ? (uint32_t)(lo >> q) & ((1u << (al - q)) - 1u) : 0u;
            if (pad) continue;
            const uint32_t ln = (uint32_t)x & 0xFFFFu, nln = (uint32_t)(x >> 16) & 0xFFFFu;
            if (ln == (nln ^ 0xFFFFu) && p0 + al + 32 + 8ull * ln <= nbits) {
                uint32_t k = atomicAdd(&ncand, 1u);
                if (k < 1024) cand[k] = p0 + o;
            }
        }
    }
    __syncthreads();
    const uint32_t nc = min(ncand, 1024u);
    for (uint32_t k = threadIdx.x; k < nc; k += blockDim.x) {
        const uint64_t e = cand[k];
        const uint64_t p = e & ~(1ull << 63);
        const bool ok = (e >> 63) ? strict_dynamic(in, p) : strict_stored(in, p);
        if (ok) {
            const uint32_t seg = (uint32_t)(p / ((uint64_t)SEG_BYTES * 8));
            uint32_t idx = atomicAdd(&seg_cnt[seg], 1u);
            if (idx < SEG_CAP) seg_list[(uint64_t)seg * SEG_CAP + idx] = p;
        }
    }
}

// Sort each segment's candidates (arrival order is arbitrary) and compact them into one sorted
// list at the offsets of an exclusive scan of the segment counts.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_compact_kernel(const uint32_t* seg_cnt, const uint64_t* seg_list, const uint64_t* seg_off,
                            uint32_t nseg, uint64_t* out) {
    using namespace inf;
    const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= nseg) return;
    const uint32_t c = min(seg_cnt[seg], SEG_CAP);
    uint64_t* o = out + seg_off[seg];
    for (uint32_t i = 0; i < c; i++) {
        uint64_t v = seg_list[(uint64_t)seg * SEG_CAP + i];
        uint32_t j = i;
        while (j > 0 && o[j - 1] > v) { o[j] = o[j - 1]; j--; }
        o[j] = v;
    }
}

struct ChainRes {
    uint64_t end_bit;     // boundary reached / final block end / error position
    uint64_t out_count;   // output bytes (before the error, if any)
    uint32_t status;      // ST_*
    uint32_t reason;      // for ST_ERROR
};

struct EmitChain {
    uint64_t start_bit;
    uint64_t end_bit;     // stop at this boundary (or final / error)
    uint64_t out_off;
    uint64_t out_count;
};

namespace inf {

// Huffman-block symbol decoders shared by both passes.
__device__ __forceinline__ uint32_t lit_sym(bool fixed, Rp& rd, const In& in, LT t, const uint16_t* gs,
                                            const FixedTabs* fx) {
    if (fixed) {
        rd.fill(in);
        const uint32_t e = fx->lit[rd.peek(9)];
        rd.skip(e >> 9);
        return e & 0x1FF;
    }
    return dec_lit(rd, in, t, gs);
}
__device__ __forceinline__ uint32_t dist_sym(bool fixed, Rp& rd, const In& in, LT t, const uint16_t* gs,
                                             const FixedTabs* fx) {
    if (fixed) {
        rd.fill(in);
        const uint32_t e = fx->dist[rd.peek(5)];
        rd.skip(5);
        return e & 0x1FF;
    }
    return dec_dist(rd, in, t, gs);
}

// Count pass for one chain: straight-line decode, no output.  Stops at the first block boundary at
// or past `stop`, after a final block, or at the first error (reference check order).
__device__ void count_chain(uint64_t start, uint64_t stop, uint64_t lim, const In& in, LT t, uint16_t* gs,
                            const FixedTabs* fx, ChainRes& res) {
    Rp rd;
    rd.init(in, start);
    uint64_t n = 0;
    uint32_t status = ST_BOUNDARY, reason = 0;
#define CFAIL(r) do { status = ST_ERROR; reason = (r); goto out; } while (0)
    for (;;) {
        if (rd.pos >= stop) break;                       // (start < stop: first block always decoded)
        const uint32_t bf = rd.get(in, 1), bt = rd.get(in, 2);
        if (rd.pos > in.nbits) CFAIL(R_UEOS);
        if (bt == 3) CFAIL(R_RESERVED_BLOCK_TYPE);
        if (bt == 0) {
            const uint32_t pad = (uint32_t)((8 - (rd.pos & 7)) & 7);
            rd.get(in, pad);
            const uint32_t ln = rd.get(in, 16), nln = rd.get(in, 16);
            if (rd.pos > in.nbits) CFAIL(R_UEOS);
            if (ln != (nln ^ 0xFFFFu)) CFAIL(R_LEN_MISMATCH);
            const uint64_t avail = (in.nbits - rd.pos) / 8;
            const uint64_t take = min((uint64_t)ln, avail);
            n += take;
            rd.init(in, rd.pos + 8 * take);
            if (take < ln) CFAIL(R_UEOS);
            if (bf) { status = ST_FINAL; break; }
            continue;
        }
        const bool fixed = bt == 1;
        bool empty_dist = false;
        if (!fixed) {
            const int e = parse_dynamic(rd, in, t, gs, empty_dist);
            if (e) CFAIL((uint32_t)e);
        }
        for (;;) {
            const uint32_t sym = lit_sym(fixed, rd, in, t, gs, fx);
            if (rd.pos > in.nbits) CFAIL(R_UEOS);
            if (sym < 256) { n++; continue; }
            if (sym == 256) break;
            if (sym > 285) CFAIL(R_RESERVED_LEN);
            uint32_t base, ne;
            run_base(sym - 257, base, ne);
            const uint32_t run = base + rd.get(in, ne);
            if (rd.pos > in.nbits) CFAIL(R_UEOS);
            if (empty_dist) CFAIL(R_EMPTY_DIST);
            const uint32_t dsym = dist_sym(fixed, rd, in, t, gs, fx);
            if (rd.pos > in.nbits) CFAIL(R_UEOS);
            if (dsym > 29) CFAIL(R_RESERVED_DIST);
            dist_base(dsym, base, ne);
            const uint32_t dist = base + rd.get(in, ne);
            if (rd.pos > in.nbits) CFAIL(R_UEOS);
            // the dictionary bound needs the absolute position: decidable here only for the chain
            // at the range start (lim = dictionary bytes before it; others pass lim = 2^62)
            if ((uint64_t)dist > n + lim) CFAIL(R_COPY_BEFORE);
            n += run;
        }
        if (bf) { status = ST_FINAL; break; }
    }
out:
#undef CFAIL
    res.end_bit = rd.pos;
    res.out_count = n;
    res.status = status;
    res.reason = reason;
}

// Emit pass: per-lane state machine with a token budget per step, so a lane waiting on an earlier
// chain never blocks its wave.  Output bytes are write-combined into aligned 32-bit stores.
struct Lane {
    Rp rd;
    uint64_t n;                 // bytes produced by this chain so far
    uint64_t stop_bit;          // stop at the block boundary == stop_bit
    uint32_t state;             // 0 header, 1 stored, 2 huffman, 3 done
    uint32_t stored_left;
    bool last, fixed, empty_dist;
    uint32_t status, reason;
    uint32_t cp_len, cp_dist;   // copy waiting for its source
    uint32_t lastb;             // last output byte (dist-1 copies need no load)
    uint32_t wc, wcn;           // write-combining word and its byte count
};

__device__ __forceinline__ void putb(Lane& L, uint8_t* out, uint64_t P, uint32_t b) {
    if (L.wcn == 0 && (P & 3)) { out[P] = (uint8_t)b; return; }
    L.wc |= b << (8 * (uint32_t)(P & 3));
    L.wcn++;
    if ((P & 3) == 3) { *(uint32_t*)(out + P - 3) = L.wc; L.wc = 0; L.wcn = 0; }
}
__device__ __forceinline__ void flushb(Lane& L, uint8_t* out, uint64_t Pnext) {
    for (uint32_t k = 0; k < L.wcn; k++) out[Pnext - L.wcn + k] = (uint8_t)(L.wc >> (8 * k));
    L.wc = 0; L.wcn = 0;
}

// Copy `len` bytes from src to dst (= out_off + L.n), reference byte-serial semantics.
__device__ __forceinline__ void do_copy(Lane& L, uint8_t* out, uint64_t dst, uint64_t src, uint32_t len, uint32_t dist,
                                        uint64_t out_off) {
    if (dist == 1) {
        const uint32_t v = (L.n > 0) ? L.lastb : (uint32_t)out[src];
        uint32_t k = 0;
        for (; k < len && (L.wcn > 0 || ((dst + k) & 3)); k++) putb(L, out, dst + k, v);
        const uint32_t v4 = v * 0x01010101u;
        for (; k + 4 <= len; k += 4) *(uint32_t*)(out + dst + k) = v4;
        for (; k < len; k++) putb(L, out, dst + k, v);
        L.lastb = v;
        return;
    }
    uint32_t b = L.lastb;
    if (dist < 4) {
        // sources may lie in the pending word: no write-combining for short periods
        flushb(L, out, dst);
        for (uint32_t k = 0; k < len; k++) { b = out[src + k]; out[dst + k] = (uint8_t)b; }
    } else {
        // every source byte lies at least 4 bytes back, i.e. before the pending word
        for (uint32_t k = 0; k < len; k++) { b = out[src + k]; putb(L, out, dst + k, b); }
    }
    L.lastb = b;
}

}  // namespace inf

template <bool DUMMY = true>
__device__ bool emit_step(inf::Lane& L, const inf::In& in, inf::LT t, uint16_t* gs, const inf::FixedTabs* fx,
                          uint8_t* out, uint64_t out_off, const uint64_t* chain_off, const uint32_t* done,
                          uint32_t my_chain, bool& waiting, uint64_t dict_len, const uint32_t* taint,
                          bool& tainted) {
    using namespace inf;
    waiting = false;
#define FAIL(r) do { flushb(L, out, out_off + L.n); L.status = ST_ERROR; L.reason = (r); L.state = 3; return false; } while (0)
    if (L.state == 0) {
        if (L.rd.pos == L.stop_bit) { flushb(L, out, out_off + L.n); L.status = ST_BOUNDARY; L.state = 3; return false; }
        const uint32_t bf = L.rd.get(in, 1), bt = L.rd.get(in, 2);
        if (L.rd.pos > in.nbits) FAIL(R_UEOS);
        L.last = bf != 0;
        if (bt == 3) FAIL(R_RESERVED_BLOCK_TYPE);
        if (bt == 0) {
            const uint32_t pad = (uint32_t)((8 - (L.rd.pos & 7)) & 7);
            L.rd.get(in, pad);
            const uint32_t ln = L.rd.get(in, 16), nln = L.rd.get(in, 16);
            if (L.rd.pos > in.nbits) FAIL(R_UEOS);
            if (ln != (nln ^ 0xFFFFu)) FAIL(R_LEN_MISMATCH);
            L.stored_left = ln;
            L.state = 1;
            return true;
        }
        if (bt == 1) { L.fixed = true; L.empty_dist = false; L.state = 2; return true; }
        bool ed = false;
        const int e = parse_dynamic(L.rd, in, t, gs, ed);
        if (e) FAIL((uint32_t)e);
        L.fixed = false; L.empty_dist = ed; L.state = 2;
        return true;
    }
    if (L.state == 1) {
        const uint64_t avail = (in.nbits - min(L.rd.pos, in.nbits)) / 8;
        const uint32_t want = min(L.stored_left, 64u);
        const uint32_t take = (uint32_t)min((uint64_t)want, avail);
        for (uint32_t k = 0; k < take; k++) {
            const uint32_t b = L.rd.get(in, 8);
            putb(L, out, out_off + L.n + k, b);
            L.lastb = b;
        }
        L.n += take;
        L.stored_left -= take;
        if (take < want) FAIL(R_UEOS);
        if (L.stored_left == 0) {
            if (L.last) { flushb(L, out, out_off + L.n); L.status = ST_FINAL; L.state = 3; return false; }
            L.state = 0;
        }
        return true;
    }
    // state 2: up to 32 tokens per step
    for (int budget = 0; budget < 32; budget++) {
        if (L.cp_len == 0) {
            const uint32_t sym = lit_sym(L.fixed, L.rd, in, t, gs, fx);
            if (L.rd.pos > in.nbits) FAIL(R_UEOS);
            if (sym < 256) {
                putb(L, out, out_off + L.n, sym);
                L.lastb = sym;
                L.n++;
                continue;
            }
            if (sym == 256) {
                if (L.last) { flushb(L, out, out_off + L.n); L.status = ST_FINAL; L.state = 3; return false; }
                L.state = 0;
                return true;
            }
            if (sym > 285) FAIL(R_RESERVED_LEN);
            uint32_t base, ne;
            run_base(sym - 257, base, ne);
            const uint32_t run = base + L.rd.get(in, ne);
            if (L.rd.pos > in.nbits) FAIL(R_UEOS);
            if (L.empty_dist) FAIL(R_EMPTY_DIST);
            const uint32_t dsym = dist_sym(L.fixed, L.rd, in, t, gs, fx);
            if (L.rd.pos > in.nbits) FAIL(R_UEOS);
            if (dsym > 29) FAIL(R_RESERVED_DIST);
            dist_base(dsym, base, ne);
            const uint32_t dist = base + L.rd.get(in, ne);
            if (L.rd.pos > in.nbits) FAIL(R_UEOS);
            if ((uint64_t)dist > out_off + L.n) FAIL(R_COPY_BEFORE);
            L.cp_len = run;
            L.cp_dist = dist;
        }
        const uint64_t dst = out_off + L.n;
        const uint64_t src = dst - L.cp_dist;
        if (src < out_off && !(L.cp_dist == 1 && L.n > 0)) {
            // source precedes this chain.  Bytes below dict_len are the caller's window (in deferred
            // mode its content arrives later: the chain is tainted and re-emitted by the resolve
            // pass); bytes in [dict_len, out_off) wait for the chains owning them.
            const uint64_t src_end = min(dst, src + L.cp_len);
            if (src < dict_len) tainted = true;
            if (src_end > dict_len) {
                const uint64_t s0 = max(src, dict_len);
                uint32_t lo = 0, hi = my_chain;
                while (lo + 1 < hi) { const uint32_t mid = (lo + hi) >> 1; if (chain_off[mid] <= s0) lo = mid; else hi = mid; }
                uint32_t need_hi = lo;
                while (need_hi + 1 < my_chain && chain_off[need_hi + 1] < src_end) need_hi++;
                for (uint32_t j = lo; j <= need_hi; j++)
                    if (__hip_atomic_load(&done[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) { waiting = true; return true; }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (taint)
                    for (uint32_t j = lo; j <= need_hi; j++) tainted |= taint[j] != 0;
            }
        }
        do_copy(L, out, dst, src, L.cp_len, L.cp_dist, out_off);
        L.n += L.cp_len;
        L.cp_len = 0;
    }
    return true;
#undef FAIL
}

// One lane per candidate: count output bytes until the first boundary >= stop.
extern "C" __global__ void __launch_bounds__(64)
ndfl_inflate_count_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* starts,
                          const uint64_t* stops, uint32_t nchains, ChainRes* res, uint16_t* gsort,
                          const inf::FixedTabs* fx, uint64_t base_bit, uint64_t dict_len) {
    using namespace inf;
    extern __shared__ uint16_t lds_tab[];
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const LT t{lds_tab + threadIdx.x};
    uint16_t* gs = gsort + (uint64_t)blockIdx.x * G_SORT * 64 + threadIdx.x;
    if (i >= nchains) return;
    In in{w, nwords, nbits};
    ChainRes r;
    count_chain(starts[i], stops[i], starts[i] == base_bit ? dict_len : (1ull << 62), in, t, gs, fx, r);
    res[i] = r;
}

// One lane per linked chain, in stream order.  Each wave claims its 64 chains through `ticket`,
// so every chain a lane may wait on already belongs to a running wave.
extern "C" __global__ void __launch_bounds__(64)
ndfl_inflate_emit_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const EmitChain* chains,
                         const uint64_t* chain_off, uint32_t nlist, uint32_t* done, uint32_t* ticket,
                         uint8_t* out, ChainRes* res, uint16_t* gsort, const inf::FixedTabs* fx,
                         uint64_t dict_len, uint32_t* taint, const uint32_t* sel) {
    using namespace inf;
    extern __shared__ uint16_t lds_tab[];
    const int lane = threadIdx.x & 63;
    const LT t{lds_tab + lane};
    uint16_t* gs = gsort + (uint64_t)blockIdx.x * G_SORT * 64 + lane;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(ticket, 64u);
    base = __shfl(base, 0, 64);
    // `sel` (resolve pass): the listed chains only, in stream order; the others are already done
    const uint32_t k = base + (uint32_t)lane;
    const bool valid = k < nlist;
    const uint32_t i = valid ? (sel ? sel[k] : k) : 0;
    In in{w, nwords, nbits};
    Lane L;
    EmitChain ch;
    if (valid) ch = chains[i];
    else { ch.start_bit = 0; ch.end_bit = 0; ch.out_off = 0; ch.out_count = 0; }
    L.rd.init(in, ch.start_bit);
    L.n = 0; L.stop_bit = ch.end_bit; L.state = 0; L.stored_left = 0; L.last = false; L.fixed = false;
    L.empty_dist = false; L.status = 0; L.reason = 0; L.cp_len = 0; L.cp_dist = 0; L.lastb = 0;
    L.wc = 0; L.wcn = 0;
    bool active = valid;
    bool tainted = false;
    int idle = 0;
    uint32_t waits = 0;
    while (__any(active)) {
        bool waiting = false;
        if (active) {
            bool more = emit_step(L, in, t, gs, fx, out, ch.out_off, chain_off, done, i, waiting, dict_len,
                                  taint, tainted);
            if (waiting && ++waits > (1u << 26)) {          // safety net: never hang the device
                more = false; L.status = ST_ERROR; L.reason = R_INTERNAL;
            }
            if (!more) {
                active = false;
                if (taint) taint[i] = tainted ? 1u : 0u;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&done[i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ChainRes r;
                r.end_bit = L.rd.pos; r.out_count = L.n; r.status = L.status; r.reason = L.reason;
                res[i] = r;
            }
        }
        if (__all(!active || waiting)) { if (++idle > 2) __builtin_amdgcn_s_sleep(2); }
        else idle = 0;
    }
}

// ---- host orchestration ---------------------------------------------------------------------

struct InflateScratch {
    void* d_in = nullptr; size_t d_in_cap = 0;
    void* d_cand = nullptr; size_t d_cand_cap = 0;
    void* d_starts = nullptr; size_t d_starts_cap = 0;
    void* d_stops = nullptr; size_t d_stops_cap = 0;
    void* d_res = nullptr; size_t d_res_cap = 0;
    void* d_tabs = nullptr; size_t d_tabs_cap = 0;
    void* d_fixed = nullptr;
    void* d_chains = nullptr; size_t d_chains_cap = 0;
    void* d_off = nullptr; size_t d_off_cap = 0;
    void* d_done = nullptr; size_t d_done_cap = 0;
    void* d_taint = nullptr; size_t d_taint_cap = 0;
    void* d_sel = nullptr; size_t d_sel_cap = 0;
    void* d_ticket = nullptr;
    void* d_out = nullptr; size_t d_out_cap = 0;
    double last_ms_find = 0, last_ms_count = 0, last_ms_emit = 0, last_ms_wall = 0;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    uint64_t repairs = 0, chains = 0, candidates = 0;
    bool count_first = false;
    // state kept for ndfl_inflate_resolve after a deferred-window range decode
    bool pending = false;
    const uint32_t* p_w = nullptr;
    uint64_t p_nwords = 0, p_nbits = 0, p_dict_len = 0;
    uint8_t* p_out = nullptr;
    uint32_t p_nch = 0;
    void release() {
        void** ps[] = {&d_in, &d_cand, &d_starts, &d_stops, &d_res, &d_tabs, &d_fixed, &d_chains, &d_off,
                       &d_done, &d_taint, &d_sel, &d_ticket, &d_out};
        for (void** p : ps) { if (*p) hipFree(*p); *p = nullptr; }
        for (auto& e : ev) { if (e) hipEventDestroy(e); e = nullptr; }
        d_in_cap = d_cand_cap = d_starts_cap = d_stops_cap = d_res_cap = d_tabs_cap = d_chains_cap = 0;
        d_off_cap = d_done_cap = d_taint_cap = d_sel_cap = d_out_cap = 0;
        pending = false;
    }
};

static hipError_t inf_ensure(void** p, size_t* cap, size_t n) {
    if (n <= *cap && *p) return hipSuccess;
    if (*p) { hipFree(*p); *p = nullptr; *cap = 0; }
    size_t want = n < 4096 ? 4096 : n;
    hipError_t e = hipMalloc(p, want);
    if (e == hipSuccess) *cap = want;
    return e;
}

// Host-side construction of the fixed-Huffman decode tables (D/decomp/Open.java:812-830).
static void host_build_fixed(inf::FixedTabs* t) {
    memset(t, 0, sizeof(*t));
    auto build = [](const uint8_t* lens, int n, uint16_t* prim, int pbits) {
        uint16_t cnt[16] = {0};
        for (int s = 0; s < n; s++) cnt[lens[s]]++;
        cnt[0] = 0;
        uint16_t first[16] = {0};
        uint32_t code = 0;
        for (int l = 1; l < 16; l++) { code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1; first[l] = (uint16_t)code; }
        uint16_t nxt[16] = {0};
        for (int s = 0; s < n; s++) {
            uint32_t l = lens[s];
            if (!l) continue;
            uint32_t c = first[l] + nxt[l]++, r = 0;
            for (uint32_t b = 0; b < l; b++) r |= ((c >> b) & 1u) << (l - 1 - b);
            for (uint32_t k = r; k < (1u << pbits); k += (1u << l)) prim[k] = (uint16_t)(s | (l << 9));
        }
    };
    uint8_t ll[288], dl[32];
    for (int i = 0; i < 288; i++) ll[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
    for (int i = 0; i < 32; i++) dl[i] = 5;
    build(ll, 288, t->lit, 9);
    build(dl, 32, t->dist, 5);
}

static constexpr uint32_t LDS_TAB_BYTES = inf::LDS_BYTES;

#define INF_CHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return -4; } while (0)

// Decode one raw DEFLATE stream, or the block-aligned range [start_bit, end_bit) of one.
//   out       the window start: out[0, dict_len) holds the dict_len bytes of output preceding the
//             range (0 for a whole stream); decoded bytes go to out[dict_len, dict_len + n)
//   deferred  the window content is not valid yet: chains that read it (directly or through other
//             chains) are recorded and re-emitted by inflate_resolve once it is written
static int inflate_run(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint64_t start_bit,
                       uint64_t end_bit, uint8_t* out, uint64_t dict_len, uint64_t out_cap, uint64_t* out_len,
                       uint64_t* consumed_bits, uint32_t flags, bool deferred, double* last_ms) {
    using namespace inf;
    *out_len = 0;
    *consumed_bits = 0;
    S.pending = false;
    const uint64_t nbits = in_len * 8;
    const uint64_t nwords = (in_len + 3) / 4;
    if (start_bit > nbits) return -1;
    // input words (padded copy when the caller's buffer is host memory or unaligned)
    const uint32_t* d_w;
    if ((flags & 1u) && (((uintptr_t)in) & 3) == 0 && (in_len % 4 == 0)) {
        d_w = (const uint32_t*)in;
    } else {
        INF_CHK(inf_ensure(&S.d_in, &S.d_in_cap, nwords * 4 + 16));
        INF_CHK(hipMemsetAsync(S.d_in, 0, nwords * 4 + 16, s));
        if (in_len)
            INF_CHK(hipMemcpyAsync(S.d_in, in, in_len, (flags & 1u) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
        d_w = (const uint32_t*)S.d_in;
    }
    if (!S.d_fixed) {
        INF_CHK(hipFuncSetAttribute((const void*)ndfl_inflate_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)LDS_TAB_BYTES));
        INF_CHK(hipFuncSetAttribute((const void*)ndfl_inflate_emit_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)LDS_TAB_BYTES));
        INF_CHK(hipMalloc(&S.d_fixed, sizeof(FixedTabs)));
        FixedTabs* h = (FixedTabs*)malloc(sizeof(FixedTabs));
        host_build_fixed(h);
        INF_CHK(hipMemcpy(S.d_fixed, h, sizeof(FixedTabs), hipMemcpyHostToDevice));
        free(h);
    }
    if (!S.ev[0]) for (auto& e : S.ev) INF_CHK(hipEventCreate(&e));
    const uint32_t nseg = (uint32_t)std::max<uint64_t>(1, (in_len + SEG_BYTES - 1) / SEG_BYTES);
    INF_CHK(inf_ensure(&S.d_cand, &S.d_cand_cap, (uint64_t)nseg * SEG_CAP * 8ull + (uint64_t)nseg * 4 + 64));
    uint64_t* d_list = (uint64_t*)S.d_cand;
    uint32_t* d_cnt = (uint32_t*)((char*)S.d_cand + (uint64_t)nseg * SEG_CAP * 8ull);
    INF_CHK(hipMemsetAsync(d_cnt, 0, (uint64_t)nseg * 4, s));
    INF_CHK(hipEventRecord(S.ev[0], s));
    {
        const uint64_t nthr = (nbits + 31) / 32;
        INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, 64));
        if (nthr)
            hipLaunchKernelGGL(ndfl_inflate_find_kernel, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, s, d_w,
                               nwords, nbits, d_cnt, d_list);
        INF_CHK(hipGetLastError());
    }
    INF_CHK(hipEventRecord(S.ev[1], s));
    std::vector<uint32_t> hcnt(nseg);
    INF_CHK(hipMemcpyAsync(hcnt.data(), d_cnt, nseg * 4ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    std::vector<uint64_t> hoff(nseg + 1);
    hoff[0] = 1;                                   // slot 0 is the range start
    for (uint32_t k = 0; k < nseg; k++) hoff[k + 1] = hoff[k] + std::min(hcnt[k], SEG_CAP);
    const uint64_t ncand_all = hoff[nseg];
    INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, (ncand_all + nseg + 2) * 8));
    uint64_t* d_sorted = (uint64_t*)S.d_starts;
    uint64_t* d_segoff = d_sorted + ncand_all;
    INF_CHK(hipMemcpyAsync(d_segoff, hoff.data(), nseg * 8ull, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(ndfl_inflate_compact_kernel, dim3((nseg + 255) / 256), dim3(256), 0, s, (const uint32_t*)d_cnt,
                       (const uint64_t*)d_list, (const uint64_t*)d_segoff, nseg, d_sorted);
    INF_CHK(hipGetLastError());
    std::vector<uint64_t> starts(ncand_all);
    INF_CHK(hipMemcpyAsync(starts.data() + 1, d_sorted + 1, (ncand_all - 1) * 8, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    starts[0] = start_bit;
    // keep candidates inside the range; drop a duplicate of the start (a header found there)
    {
        size_t m = 1;
        for (size_t k = 1; k < starts.size(); k++)
            if (starts[k] > start_bit && starts[k] < end_bit) starts[m++] = starts[k];
        starts.resize(m);
    }
    const std::vector<uint64_t> sorted_cand(starts);

    auto next_after = [&](uint64_t b) -> uint64_t {
        auto ub = std::upper_bound(sorted_cand.begin(), sorted_cand.end(), b);
        const uint64_t nx = ub != sorted_cand.end() ? *ub : NONE;
        return std::min(nx, end_bit);
    };
    std::vector<ChainRes> res;
    auto run_count = [&](const std::vector<uint64_t>& st, std::vector<ChainRes>& r) -> int {
        const size_t n = st.size();
        std::vector<uint64_t> sp(n);
        for (size_t k = 0; k < n; k++) sp[k] = next_after(st[k]);
        INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, n * 8));
        INF_CHK(inf_ensure(&S.d_stops, &S.d_stops_cap, n * 8));
        INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, n * sizeof(ChainRes)));
        INF_CHK(inf_ensure(&S.d_tabs, &S.d_tabs_cap, ((n + 63) / 64) * (uint64_t)G_SORT * 64 * 2));
        INF_CHK(hipMemcpyAsync(S.d_starts, st.data(), n * 8, hipMemcpyHostToDevice, s));
        INF_CHK(hipMemcpyAsync(S.d_stops, sp.data(), n * 8, hipMemcpyHostToDevice, s));
        if (S.count_first) INF_CHK(hipEventRecord(S.ev[2], s));
        hipLaunchKernelGGL(ndfl_inflate_count_kernel, dim3((uint32_t)((n + 63) / 64)), dim3(64), LDS_TAB_BYTES, s, d_w,
                           nwords, nbits, (const uint64_t*)S.d_starts, (const uint64_t*)S.d_stops, (uint32_t)n,
                           (ChainRes*)S.d_res, (uint16_t*)S.d_tabs, (const FixedTabs*)S.d_fixed, start_bit, dict_len);
        INF_CHK(hipGetLastError());
        if (S.count_first) { INF_CHK(hipEventRecord(S.ev[3], s)); S.count_first = false; }
        r.resize(n);
        INF_CHK(hipMemcpyAsync(r.data(), S.d_res, n * sizeof(ChainRes), hipMemcpyDeviceToHost, s));
        INF_CHK(hipStreamSynchronize(s));
        return 0;
    };
    S.repairs = 0;
    S.count_first = true;
    int rc = run_count(starts, res);
    if (rc) return rc;
    {
        float a = 0, b = 0;
        hipEventElapsedTime(&a, S.ev[0], S.ev[1]);
        hipEventElapsedTime(&b, S.ev[2], S.ev[3]);
        S.last_ms_find = a; S.last_ms_count = b;
    }

    // link from the range start.  A boundary that is no candidate (fixed-Huffman block, header
    // rejected by the finder) is repaired: every such boundary of every chain is decoded on in
    // parallel rounds; a final serial fallback guarantees progress.
    std::unordered_map<uint64_t, size_t> at;
    at.reserve(starts.size() * 2);
    for (size_t k = 0; k < starts.size(); k++) at[starts[k]] = k;
    for (int round = 0; round < 8; round++) {
        std::vector<uint64_t> todo;
        for (size_t k = 0; k < res.size(); k++)
            if (res[k].status == ST_BOUNDARY && res[k].end_bit < end_bit && !at.count(res[k].end_bit)) {
                at[res[k].end_bit] = NONE;          // placeholder, filled below
                todo.push_back(res[k].end_bit);
            }
        if (todo.empty()) break;
        std::vector<ChainRes> r2;
        rc = run_count(todo, r2);
        if (rc) return rc;
        for (size_t k = 0; k < todo.size(); k++) {
            starts.push_back(todo[k]);
            res.push_back(r2[k]);
            at[todo[k]] = starts.size() - 1;
        }
        S.repairs += todo.size();
    }
    std::vector<EmitChain> chains;
    std::vector<uint64_t> offs;
    uint64_t off = dict_len;
    size_t cur = 0;
    uint64_t stop_bit = 0;
    for (;;) {
        const ChainRes& r = res[cur];
        EmitChain ec;
        ec.start_bit = starts[cur];
        ec.end_bit = r.end_bit;
        ec.out_off = off;
        ec.out_count = r.out_count;
        chains.push_back(ec);
        offs.push_back(off);
        off += r.out_count;
        if (r.status == ST_FINAL) { stop_bit = r.end_bit; break; }
        if (r.status == ST_ERROR) break;
        if (r.end_bit == end_bit) { stop_bit = end_bit; break; }
        if (r.end_bit > end_bit) return -1;          // the range end is no block boundary
        auto it = at.find(r.end_bit);
        if (it != at.end() && it->second != (size_t)NONE) { cur = it->second; continue; }
        // serial fallback (beyond the parallel rounds)
        std::vector<uint64_t> st1{r.end_bit};
        std::vector<ChainRes> r1;
        rc = run_count(st1, r1);
        if (rc) return rc;
        starts.push_back(r.end_bit);
        res.push_back(r1[0]);
        at[r.end_bit] = starts.size() - 1;
        cur = starts.size() - 1;
        S.repairs++;
    }
    S.chains = chains.size();
    S.candidates = sorted_cand.size();
    const uint64_t total = off - dict_len;
    if (total > out_cap) { *out_len = total; return -3; }

    // emit pass
    const uint32_t nch = (uint32_t)chains.size();
    INF_CHK(inf_ensure(&S.d_chains, &S.d_chains_cap, nch * sizeof(EmitChain)));
    INF_CHK(inf_ensure(&S.d_off, &S.d_off_cap, (nch + 1) * 8ull));
    INF_CHK(inf_ensure(&S.d_done, &S.d_done_cap, nch * 4ull));
    INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, nch * sizeof(ChainRes)));
    INF_CHK(inf_ensure(&S.d_tabs, &S.d_tabs_cap, ((nch + 63) / 64) * (uint64_t)G_SORT * 64 * 2));
    if (deferred) INF_CHK(inf_ensure(&S.d_taint, &S.d_taint_cap, nch * 4ull));
    if (!S.d_ticket) INF_CHK(hipMalloc(&S.d_ticket, 64));
    INF_CHK(hipMemcpyAsync(S.d_chains, chains.data(), nch * sizeof(EmitChain), hipMemcpyHostToDevice, s));
    offs.push_back(off);
    INF_CHK(hipMemcpyAsync(S.d_off, offs.data(), (nch + 1) * 8ull, hipMemcpyHostToDevice, s));
    INF_CHK(hipMemsetAsync(S.d_done, 0, nch * 4ull, s));
    INF_CHK(hipMemsetAsync(S.d_ticket, 0, 64, s));
    uint8_t* d_out;
    const bool direct = (flags & 2u) != 0;
    if (direct) d_out = out;
    else {
        INF_CHK(inf_ensure(&S.d_out, &S.d_out_cap, dict_len + total + 64));
        d_out = (uint8_t*)S.d_out;
        if (dict_len) INF_CHK(hipMemcpyAsync(d_out, out, dict_len, hipMemcpyHostToDevice, s));
    }
    hipEvent_t e2 = S.ev[4], e3 = S.ev[5];
    INF_CHK(hipEventRecord(e2, s));
    const uint32_t waves = (nch + 63) / 64;
    hipLaunchKernelGGL(ndfl_inflate_emit_kernel, dim3(waves), dim3(64), LDS_TAB_BYTES, s, d_w, nwords, nbits,
                       (const EmitChain*)S.d_chains, (const uint64_t*)S.d_off, nch, (uint32_t*)S.d_done,
                       (uint32_t*)S.d_ticket, d_out, (ChainRes*)S.d_res, (uint16_t*)S.d_tabs,
                       (const FixedTabs*)S.d_fixed, dict_len, deferred ? (uint32_t*)S.d_taint : (uint32_t*)nullptr,
                       (const uint32_t*)nullptr);
    INF_CHK(hipGetLastError());
    INF_CHK(hipEventRecord(e3, s));
    std::vector<ChainRes> er(nch);
    INF_CHK(hipMemcpyAsync(er.data(), S.d_res, nch * sizeof(ChainRes), hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    float ms = 0;
    hipEventElapsedTime(&ms, e2, e3);
    S.last_ms_emit = ms;
    float ms2 = 0;
    hipEventElapsedTime(&ms2, S.ev[0], e3);
    S.last_ms_wall = ms2;
    *last_ms = ms;
    if (deferred) {
        S.pending = true;
        S.p_w = d_w; S.p_nwords = nwords; S.p_nbits = nbits; S.p_dict_len = dict_len; S.p_out = d_out; S.p_nch = nch;
    }
    // first error in stream order (the emit pass also checks the dictionary bound exactly)
    for (uint32_t k = 0; k < nch; k++) {
        if (er[k].status == ST_ERROR) {
            const uint64_t produced = chains[k].out_off - dict_len + er[k].out_count;
            if (!direct && produced) INF_CHK(hipMemcpy(out + dict_len, d_out + dict_len, produced, hipMemcpyDeviceToHost));
            *out_len = produced;
            *consumed_bits = er[k].end_bit;
            return (int)er[k].reason;
        }
    }
    if (!direct && total) INF_CHK(hipMemcpy(out + dict_len, d_out + dict_len, total, hipMemcpyDeviceToHost));
    *out_len = total;
    *consumed_bits = stop_bit;
    return 0;
}

// Second half of a deferred-window range decode: the caller has written the window
// (out[0, dict_len)); re-emit, in stream order, exactly the chains that read it.
static int inflate_resolve(InflateScratch& S, hipStream_t s, uint64_t* n_reemitted) {
    using namespace inf;
    *n_reemitted = 0;
    if (!S.pending) return -5;
    S.pending = false;
    const uint32_t nch = S.p_nch;
    std::vector<uint32_t> taint(nch);
    INF_CHK(hipMemcpyAsync(taint.data(), S.d_taint, nch * 4ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    std::vector<uint32_t> sel, done(nch);
    for (uint32_t k = 0; k < nch; k++) {
        done[k] = taint[k] ? 0u : 1u;
        if (taint[k]) sel.push_back(k);
    }
    *n_reemitted = sel.size();
    if (sel.empty()) return 0;
    const uint32_t nsel = (uint32_t)sel.size();
    INF_CHK(inf_ensure(&S.d_sel, &S.d_sel_cap, nsel * 4ull));
    INF_CHK(hipMemcpyAsync(S.d_sel, sel.data(), nsel * 4ull, hipMemcpyHostToDevice, s));
    INF_CHK(hipMemcpyAsync(S.d_done, done.data(), nch * 4ull, hipMemcpyHostToDevice, s));
    INF_CHK(hipMemsetAsync(S.d_ticket, 0, 64, s));
    hipLaunchKernelGGL(ndfl_inflate_emit_kernel, dim3((nsel + 63) / 64), dim3(64), LDS_TAB_BYTES, s, S.p_w, S.p_nwords,
                       S.p_nbits, (const EmitChain*)S.d_chains, (const uint64_t*)S.d_off, nsel, (uint32_t*)S.d_done,
                       (uint32_t*)S.d_ticket, S.p_out, (ChainRes*)S.d_res, (uint16_t*)S.d_tabs,
                       (const FixedTabs*)S.d_fixed, S.p_dict_len, (uint32_t*)nullptr, (const uint32_t*)S.d_sel);
    INF_CHK(hipGetLastError());
    INF_CHK(hipStreamSynchronize(s));
    return 0;
}
