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
#include "../../../include/ndfl.h"
#include <vector>
#include <algorithm>
#include <unordered_map>
#include <chrono>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

namespace inf {

constexpr uint32_t SEG_BYTES = 65536;      // finder segment (compressed bytes)
constexpr uint32_t SEG_CAP = 256;          // candidates kept per finder segment
constexpr uint64_t NONE = ~0ull;

enum : uint32_t { ST_BOUNDARY = 0, ST_FINAL = 1, ST_ERROR = 2 };
constexpr int NEED_INPUT = 64;             // NDFL_NEED_INPUT (include/ndfl.h): partial-input decode stopped
enum : int { R_UEOS = 1, R_RESERVED_BLOCK_TYPE, R_LEN_MISMATCH, R_UNDER_FULL, R_OVER_FULL, R_NO_PREV,
             R_CL_OVER_FULL, R_EOB_ZERO, R_RESERVED_LEN, R_RESERVED_DIST, R_EMPTY_DIST, R_COPY_BEFORE,
             // internal: the second reserved symbol of each alphabet (287, distance 31); the C ABI
             // returns R_RESERVED_LEN / R_RESERVED_DIST and keeps the symbol (ndfl_ctx_error_symbol),
             // which the reference puts in its message (D/decomp/Open.java:516, 550)
             R_RESERVED_LEN_HI = 20, R_RESERVED_DIST_HI = 21,
             R_INTERNAL = 100 };

constexpr int CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
// position of code-length symbol sy in CLO (its 3-bit length's index in the header)
constexpr int CLO_INV[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};

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

constexpr uint64_t IN_PAD = 256;           // zero bytes after the staged input
static_assert(IN_PAD == NDFL_IN_PAD_BYTES, "kernel pad and the NDFL_IN_PADDED contract must agree");
// the furthest unchecked reads: In::ld4 clamps 16-byte group indices at (nwords + 3) / 4 + 1, so a
// lane reads at most ((nwords + 3) / 4 + 2) * 16 <= nwords * 4 + 44 bytes; the decode passes' round
// staging (wv::stage_round) clamps word indices at nwords + 60, i.e. nwords * 4 + 244 bytes
static_assert(3 * 4 + 2 * 16 + 16 <= IN_PAD, "16-byte prefetch clamp must stay inside the zero padding");
static_assert((60 + 1) * 4 <= IN_PAD, "round staging clamp must stay inside the zero padding");
#ifndef NDFL_FIND_WPT
#define NDFL_FIND_WPT 16
#endif
constexpr uint32_t FIND_WPT = NDFL_FIND_WPT;     // finder: input words per thread
#ifndef NDFL_STRICT_SLICE
#define NDFL_STRICT_SLICE 128
#endif
#ifndef NDFL_STRICT_REFILL
#define NDFL_STRICT_REFILL 32     // strict stage: refill a wave once this many lanes are idle
#endif
constexpr uint32_t STRICT_SLICE = NDFL_STRICT_SLICE;  // strict stage: survivors per ticket
#ifndef NDFL_COUNT_W_DEFAULT
#define NDFL_COUNT_W_DEFAULT 1
#endif
constexpr uint32_t COUNT_WAVES = 256 * 16;       // count / emit passes: persistent waves at most (the
constexpr uint32_t EMIT_WAVES = 256 * 16;        // grids are sized by occupancy, wave_grid below)

struct In {
    const uint32_t* w;
    uint64_t nwords;
    uint64_t nbits;
    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return i < nwords ? w[i] : 0u; }
    // the input from bit p on (at least 32 bits; zeros past the end)
    __device__ __forceinline__ uint64_t win64(uint64_t p) const {
        const uint64_t i = p >> 5;
        return (((uint64_t)ld(i + 1) << 32) | ld(i)) >> (p & 31);
    }
    // unchecked 16-byte group load; positions past the end are clamped into the zero padding
    __device__ __forceinline__ u32x4 ld4(uint64_t g) const {
        const uint64_t gmax = (nwords + 3) / 4 + 1;
        return *(const u32x4*)(w + min(g, gmax) * 4);
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
// with the next two 4-word groups already in flight (one 16-byte load per 128 bits consumed,
// issued 256 bits ahead of use).  The loads are unconditional (zero-padded input), so nothing
// forces an early wait on them.
struct Rp {
    uint64_t bb;
    uint32_t bn;
    uint32_t ci;          // next word of `cur` (0..3)
    uint64_t qw;          // group index of `cur`
    uint64_t pos;
    u32x4 cur, nxt, nx2;
    __device__ __forceinline__ static uint32_t pick(const u32x4& v, uint32_t i) {
        uint32_t a = (i & 1) ? v.y : v.x, b = (i & 1) ? v.w : v.z;
        return (i & 2) ? b : a;
    }
    __device__ __forceinline__ void adv(const In& in) {
        if (++ci == 4) { cur = nxt; nxt = nx2; qw++; nx2 = in.ld4(qw + 2); ci = 0; }
    }
    __device__ __forceinline__ void init(const In& in, uint64_t p) {
        pos = p;
        qw = p >> 7;
        cur = in.ld4(qw);
        nxt = in.ld4(qw + 1);
        nx2 = in.ld4(qw + 2);
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
// Straight-line (no early exit inside the loop): fully unrolled with constant indices, so the
// counts stay in registers -- a loop with a break left them in scratch memory (round 6).
__device__ __forceinline__ int tree_check(const uint32_t (&cnt)[16]) {
    uint32_t num = 0, maxL = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) { num += cnt[l]; maxL = cnt[l] ? (uint32_t)l : maxL; }
    if (num < 2) return R_UNDER_FULL;
    // (32-bit: end stays below R + 2 <= 2 * 320, or the under-full test has fired -- 64-bit
    // compares of wave-uniform values went through the vector unit)
    const uint32_t R = 2u * (num - 1);
    uint32_t next = 0, end = 2;
    int res = 0;
#pragma unroll
    for (uint32_t l = 1; l < 16; l++) {
        const bool on = l <= maxL && res == 0;
        if (l > 1) {
            const uint32_t open = end - next;
            const bool op = on && open > 0;
            const bool uf = op && end + 2 * (open - 1) >= R;
            res = uf ? (int)R_UNDER_FULL : res;
            const bool adv = op && !uf;
            next = adv ? end : next;
            end = adv ? end + 2 * open : end;
        }
        const bool on2 = on && res == 0;
        const uint32_t c = cnt[l];
        const bool of = on2 && c > end - next;
        res = of ? (int)R_OVER_FULL : res;
        next = (on2 && !of) ? next + c : next;
    }
    if (res) return res;
    if (end != R) return R_INTERNAL;
    if (next < end) return R_UNDER_FULL;
    return 0;
}

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
// header: not btype 3; stored -> LEN == ~NLEN; dynamic -> complete code-length code.  (Inlined: the
// strict stage must not use scratch memory, see there.)
__device__ __forceinline__ bool strict_stored(const In& in, uint64_t p) {
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

// Header finder over every bit position, stage 1 (quick filter): BTYPE from two shifts of the
// input; dynamic headers need a complete code-length code (Kraft sum exactly 1 over the HCLEN+4
// 3-bit lengths); stored headers need LEN == ~NLEN at the next byte boundary and zero padding.
// Survivors (about 1 in 1000 positions) go to a global list for the strict stage.
#ifndef NDFL_FIND_WPE
#define NDFL_FIND_WPE 3
#endif
#ifndef NDFL_FIND_LASTBLK
#define NDFL_FIND_LASTBLK 0
#endif
#ifndef NDFL_STRICT_WPE
#define NDFL_STRICT_WPE 5
#endif
namespace inf {
// The 32 positions of each input word, for the 64 words of a wave at once.  The cheap masks
// (BTYPE, BFINAL, HLIT/HDIST, stored LEN/NLEN) are bit-sliced per lane (bit i = position p0 + i);
// the positions they leave for the code-length code's Kraft test -- about 1 in 9 -- are compacted
// into a wave list and tested one per lane: the HCLEN + 4 three-bit lengths as one 57-bit field,
// summed by five lookups of a 4,096-entry table of the Kraft sums of four lengths (kr4).  About 30
// operations per such position (round 4; a bit-sliced Kraft test at every position took 451 per
// 32 positions).  A pass takes at most FIND_TAKE positions per lane (a dense pattern takes more
// passes).
constexpr uint32_t FIND_TAKE = 8;
constexpr uint32_t FIND_CLIST = 64 * FIND_TAKE;
constexpr uint32_t FIND_CCAP = 1024;               // survivors listed in LDS per workgroup (131,072 positions; ~65 on average)
struct FindWaveScratch {
    uint32_t w[64 + 4];                            // the wave's words and the three after them
    uint16_t list[FIND_CLIST];                     // lane << 5 | bit of each position to test
};
// (survivors go to the workgroup's LDS list as 32-bit offsets from bit `pb`, bit 31 set: dynamic)
// (a workgroup's survivors past the LDS list's FIND_CCAP go straight to the global list, one global
// atomic each -- periodic bit patterns can pass the filters every few bits, and a dropped survivor
// would be a real header lost at random)
__device__ __forceinline__ void find_spill(uint64_t v, uint64_t* qlist, uint32_t* qcount, uint32_t qcap) {
    const uint32_t g = atomicAdd(qcount, 1u);
    if (g < qcap) qlist[g] = v;
}
__device__ __forceinline__ void find_word_wave(const In& in, uint64_t t, uint64_t scan_end, uint32_t* cand,
                                               uint32_t* ncand, FindWaveScratch& fw, const uint16_t* kr4, uint64_t pb,
                                               uint64_t* qlist, uint32_t* qcount, uint32_t qcap) {
    const uint64_t nbits = in.nbits;
    const int lane = threadIdx.x & 63;
    const uint64_t p0 = t * 32;
    const uint32_t w0 = in.ld(t), w1 = in.ld(t + 1), w2 = in.ld(t + 2), w3 = in.ld(t + 3);
    const uint64_t W = (uint64_t)w0 | ((uint64_t)w1 << 32);
    const uint32_t b1 = (uint32_t)(W >> 1), b2 = (uint32_t)(W >> 2);
    uint32_t valid = 0xFFFFFFFFu;
    if (p0 + 35 > nbits) valid = (nbits >= p0 + 3) ? (uint32_t)((1ull << (nbits - p0 - 2)) - 1) : 0u;
    if (p0 + 32 > scan_end) valid &= p0 < scan_end ? (uint32_t)((1ull << (scan_end - p0)) - 1) : 0u;
#if NDFL_FIND_LASTBLK
    const uint32_t notfinal = ~0u;
#else
    const uint32_t notfinal = ~w0;
#endif
    const uint32_t h4 = (uint32_t)(W >> 4), h5 = (uint32_t)(W >> 5), h6 = (uint32_t)(W >> 6),
                   h7 = (uint32_t)(W >> 7), d9 = (uint32_t)(W >> 9), d10 = (uint32_t)(W >> 10),
                   d11 = (uint32_t)(W >> 11), d12 = (uint32_t)(W >> 12);
    const uint32_t big = (h4 & h5 & h6 & h7) | (d9 & d10 & d11 & d12);     // HLIT or HDIST >= 30
    const uint32_t pm = ~b1 & b2 & valid & notfinal & ~big;         // before the Kraft test
    // stored headers: LEN == ~NLEN (as find_word)
    const uint64_t W12 = (uint64_t)w1 | ((uint64_t)w2 << 32);
    const uint32_t x1 = (uint32_t)(W >> 8), x2 = (uint32_t)(W >> 16), x3 = (uint32_t)(W >> 24), x4 = w1,
                   x5 = (uint32_t)(W12 >> 8);
#define NDFL_LENOK(x) ((((x) ^ ((x) >> 16)) & 0xFFFFu) == 0xFFFFu)
    const uint32_t okm = (NDFL_LENOK(x1) ? 0x0000003Fu : 0u) | (NDFL_LENOK(x2) ? 0x00003FC0u : 0u) |
                         (NDFL_LENOK(x3) ? 0x003FC000u : 0u) | (NDFL_LENOK(x4) ? 0x3FC00000u : 0u) |
                         (NDFL_LENOK(x5) ? 0xC0000000u : 0u);
#undef NDFL_LENOK
    uint32_t m0 = ~b1 & ~b2 & valid & notfinal & okm;
    while (m0) {
        const uint32_t o = __builtin_ctz(m0);
        m0 &= m0 - 1;
        const uint32_t q = o + 3, al = (q + 7) & ~7u;
        const uint32_t pad = al > q ? (uint32_t)(W >> q) & ((1u << (al - q)) - 1u) : 0u;
        if (pad) continue;
        const uint32_t ln = (al < 32 ? (uint32_t)(W >> al) : (uint32_t)(W12 >> (al - 32))) & 0xFFFFu;
        if (p0 + al + 32 + 8ull * ln <= nbits) {
            uint32_t k = atomicAdd(ncand, 1u);
            if (k < FIND_CCAP) cand[k] = (uint32_t)(p0 + o - pb);
            else find_spill(p0 + o, qlist, qcount, qcap);
        }
    }
    // dynamic headers
    fw.w[lane] = w0;
    {
        const uint32_t e1 = __shfl(w1, 63, 64), e2 = __shfl(w2, 63, 64), e3 = __shfl(w3, 63, 64);
        if (lane < 3) fw.w[64 + lane] = lane == 0 ? e1 : lane == 1 ? e2 : e3;
    }
    const uint64_t tw0 = t - (uint64_t)lane;                        // the wave's first word
    uint32_t rem = pm;
    while (__any(rem != 0)) {                                        // (uniform; no empty scan pass)
        const uint32_t cnt = min((uint32_t)__popc(rem), FIND_TAKE);
        // inclusive wave scan by DPP (row shifts, then the row totals broadcast across rows)
        uint32_t incl = cnt;
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xF, 0xF, false);   // row_shr:1
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xF, 0xF, false);   // row_shr:2
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xF, 0xF, false);   // row_shr:4
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xF, 0xF, false);   // row_shr:8
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x142, 0xA, 0xF, false);   // row_bcast:15
        incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x143, 0xC, 0xF, false);   // row_bcast:31
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        {
            uint32_t k = incl - cnt;
            for (uint32_t i = 0; i < cnt; i++) {
                fw.list[k++] = (uint16_t)((lane << 5) | __builtin_ctz(rem));
                rem &= rem - 1;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j = (uint32_t)lane; j < total; j += 64) {
            const uint32_t c = fw.list[j];
            const uint32_t lw = c >> 5, o = c & 31;
            const uint64_t A = (uint64_t)fw.w[lw] | ((uint64_t)fw.w[lw + 1] << 32);
            const uint64_t B = (uint64_t)fw.w[lw + 2] | ((uint64_t)fw.w[lw + 3] << 32);
            const uint32_t ncl = (uint32_t)((A >> (o + 13)) & 15u) + 4;
            const uint32_t sh = o + 17;                              // 17..48
            uint64_t F = (A >> sh) | (B << (64 - sh));
            F &= (1ull << (3 * ncl)) - 1;                            // the HCLEN + 4 lengths (<= 57 bits)
            const uint32_t ks = (uint32_t)kr4[F & 4095] + kr4[(F >> 12) & 4095] + kr4[(F >> 24) & 4095] +
                                kr4[(F >> 36) & 4095] + kr4[(F >> 48) & 4095];
            const uint64_t p = (tw0 + lw) * 32 + o;
            if (ks == 128 && p + 17 + 3 * ncl <= nbits) {
                uint32_t k = atomicAdd(ncand, 1u);
                if (k < FIND_CCAP) cand[k] = (uint32_t)(p - pb) | (1u << 31);
                else find_spill(p | (1ull << 63), qlist, qcount, qcap);
            }
        }
        __builtin_amdgcn_wave_barrier();                             // (the list is rewritten next)
    }
}
// Kraft sums of four 3-bit lengths (index: four fields, the first in the low bits), x 1/128.  (Ten
// lookups of a 64-entry two-length table -- one entry per LDS bank, no bank conflicts -- measured
// slower: finder phase 6.12 -> 6.50 ms, round 5.)
__device__ __forceinline__ void kr4_fill(uint16_t* kr4) {
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) {
        uint32_t s = 0;
#pragma unroll
        for (int f = 0; f < 4; f++) { const uint32_t l = (i >> (3 * f)) & 7u; s += l ? 128u >> l : 0u; }
        kr4[i] = (uint16_t)s;
    }
}

}  // namespace inf

// The dense scan with the compacted Kraft test (find_word_wave): every position of [w_lo * 32, scan_end).
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NDFL_FIND_WPE)))
ndfl_inflate_find_compact_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, uint64_t* qlist, uint32_t* qcount,
                                 uint32_t qcap, uint64_t w_lo, uint64_t scan_end) {
    using namespace inf;
    __shared__ uint32_t cand[FIND_CCAP];
    __shared__ uint32_t ncand, gbase;
    __shared__ uint16_t kr4[4096];
    __shared__ FindWaveScratch fws[4];
    kr4_fill(kr4);
    if (threadIdx.x == 0) ncand = 0;
    __syncthreads();
    In in{w, nwords, nbits};
    const uint64_t pb = (w_lo + (uint64_t)blockIdx.x * FIND_WPT * 256) * 32;    // the workgroup's first bit
    for (uint32_t kk = 0; kk < FIND_WPT; kk++) {
        const uint64_t tt = ((uint64_t)blockIdx.x * FIND_WPT + kk) * blockDim.x + threadIdx.x;
        find_word_wave(in, w_lo + tt, scan_end, cand, &ncand, fws[threadIdx.x >> 6], kr4, pb, qlist, qcount, qcap);
    }
    // the workgroup's LDS survivors -> the global survivor list (one global atomic)
    __syncthreads();
    const uint32_t nc = min(ncand, FIND_CCAP);
    if (threadIdx.x == 0) gbase = nc ? atomicAdd(qcount, nc) : 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nc; k += blockDim.x) {
        const uint32_t c = cand[k];
        if (gbase + k < qcap) qlist[gbase + k] = (pb + (c & 0x7FFFFFFFu)) | ((uint64_t)(c >> 31) << 63);
    }
}

namespace inf {
// strict-stage reader: a 256-bit window of the input (two 16-byte groups) in registers and a 64-bit
// bit buffer filled from it.  The window moves wave-wide: when an active lane has used its window
// up, every lane past its first group loads the next two groups, so one memory wait serves the
// wave.  (A per-lane rolling prefetch -- load the next group whenever a lane crosses one -- put a
// load wait into almost every step: with ~40 lanes active some lane crosses a group nearly every
// step, and the compiler waits for the new group where it copies it into the loop's registers.)
struct SRd {
    uint64_t bb, pos, qw;    // bit buffer; the stream position of its bit 0; the window's first group
    uint32_t bn, fi;         // valid bits in bb; the next window word to add to it (8: used up)
    u32x4 cur, nxt;
    __device__ __forceinline__ static uint32_t pick(const u32x4& v, uint32_t i) {
        uint32_t a = (i & 1) ? v.y : v.x, b = (i & 1) ? v.w : v.z;
        return (i & 2) ? b : a;
    }
    __device__ __forceinline__ uint32_t pick8(uint32_t i) const {
        const uint32_t a = pick(cur, i), b = pick(nxt, i);
        return (i & 4) ? b : a;
    }
    __device__ __forceinline__ void load(const In& in, uint64_t g) {
        qw = g;
        cur = in.ld4(g);
        nxt = in.ld4(g + 1);
    }
    // 64 bits from window bit o (o < 160)
    __device__ __forceinline__ uint64_t bits64(uint32_t o) const {
        const uint32_t i = o >> 5, sh = o & 31;
        const uint64_t x = (uint64_t)pick8(i) | ((uint64_t)pick8(i + 1) << 32);
        return sh ? (x >> sh) | ((uint64_t)pick8(i + 2) << (64 - sh)) : x;
    }
    __device__ __forceinline__ void fill() {
        if (bn <= 32 && fi < 8) { bb |= (uint64_t)pick8(fi) << bn; bn += 32; fi++; }
    }
    // the buffer from stream bit p on (p - 128 qw < 224)
    __device__ __forceinline__ void seek(uint64_t p) {
        pos = p;
        const uint32_t o = (uint32_t)(p - qw * 128);
        fi = o >> 5;
        bb = (uint64_t)(pick8(fi) >> (o & 31));
        bn = 32 - (o & 31);
        fi++;
        fill();
    }
    __device__ __forceinline__ bool starved() const { return bn <= 32 && fi >= 8; }
    // move the window to the group holding the next word to add (bb and bn stay)
    __device__ __forceinline__ void reload(const In& in) {
        const uint64_t wn = qw * 4 + fi;
        load(in, wn >> 2);
        fi = (uint32_t)wn & 3u;
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1u); }
    __device__ __forceinline__ void skip(uint32_t n) { bb >>= n; bn -= n; pos += n; }
};
}  // namespace inf

// Stage 2: the reference's own header checks (as strict_dynamic / strict_stored) on every
// survivor.  Each wave takes a contiguous slice of the survivor list; a lane that finishes its
// header takes the next one (refills are batched: at least 16 idle lanes), so short and long
// headers do not hold each other.  Dynamic headers decode the code lengths one symbol per step
// through a per-lane 128-entry table of the code-length code (LDS, indexed by the next 7 bits
// MSB first: canonical codes fill it in (length, symbol) order).  Accepted headers go to their
// 64 KiB segment's list.
// No scratch memory (tests/test_kernel_resources.py checks it): builds that used scratch here -- a
// call to a non-inlined strict_stored (its stack), or register spills at 5 waves/SIMD -- rejected
// 2-4 % of the real headers at full load, a different set on every run, while the same builds
// without scratch accepted exactly the oracle's set in every run.  Hence
// strict_stored is inlined, the code-length code's lengths travel as one 57-bit field, and the
// table build is a rolled loop: 94 VGPRs, no spills, 5 waves/SIMD.
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NDFL_STRICT_WPE)))
ndfl_inflate_strict_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* qlist,
                           const uint32_t* qcount, uint32_t qcap, uint32_t* seg_cnt, uint64_t* seg_list,
                           uint32_t* ticket, unsigned long long* sst) {
    using namespace inf;
    __shared__ uint4 tabs[256 * 8];                          // 128 bytes per lane
    uint8_t* tab = (uint8_t*)&tabs[threadIdx.x * 8];
    const uint32_t n = min(*qcount, qcap);
    In in{w, nwords, nbits};
    const uint32_t lane = threadIdx.x & 63u;
    // survivors are claimed STRICT_SLICE at a time from a global ticket, so the grid is sized to
    // what fits on the chip and waves that draw short headers take more slices
    uint32_t next = 0, end = 0;
    bool drained = false;
    const uint64_t below = (1ull << lane) - 1ull;
    auto record = [&](uint64_t p) {
        const uint32_t seg = (uint32_t)(p / ((uint64_t)SEG_BYTES * 8));
        const uint32_t idx = atomicAdd(&seg_cnt[seg], 1u);
        if (idx < SEG_CAP) seg_list[(uint64_t)seg * SEG_CAP + idx] = p;
    };
    bool active = false;
    uint64_t p = 0;
    SRd rd;
    rd.bb = 0; rd.pos = 0; rd.qw = 0; rd.bn = 0; rd.fi = 8;
    uint32_t i = 0, total = 0, numLit = 0, numDist = 0, litK = 0, distK = 0, nz = 0, eob = 0;
    int runVal = -1;
    uint64_t n_iter = 0, n_refill = 0, n_steps = 0;      // NDFL_STATS (sst != nullptr)
    for (;;) {
        const uint64_t idle = __ballot(!active);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        n_iter++;
        if (next >= end && !drained && nidle >= NDFL_STRICT_REFILL) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(ticket, STRICT_SLICE);
            t = __shfl(t, 0);
            if (t >= n) drained = true;
            else { next = t; end = min(n, t + STRICT_SLICE); }
        }
        if (next < end && nidle >= NDFL_STRICT_REFILL) {
            n_refill++;
            if (!active) {
                const uint32_t k = next + (uint32_t)__popcll(idle & below);
                if (k < end) {
                    const uint64_t e = qlist[k];
                    p = e & ~(1ull << 63);
                    if (!(e >> 63)) {
                        if (strict_stored(in, p)) record(p);
                    } else {
                        // the header's fields straight from the window (p + 74 < 128 qw + 256)
                        rd.load(in, p >> 7);
                        const uint32_t o = (uint32_t)p & 127u;
                        const uint32_t h = (uint32_t)rd.bits64(o + 3);
                        const uint32_t hlit = h & 31u, hdist = (h >> 5) & 31u, hclen = (h >> 10) & 15u;
                        numLit = hlit + 257; numDist = hdist + 1; total = numLit + numDist;
                        const uint32_t numCl = hclen + 4;
                        // the numCl 3-bit code-length code lengths in stream (CLO) order as one field
                        // (two registers where a per-symbol array held 19 at the refill's peak)
                        const uint64_t F = rd.bits64(o + 17) & ((1ull << (3 * numCl)) - 1ull);
                        rd.seek(p + 17 + 3 * numCl);
                        // the stage-1 test guarantees a complete code: the runs fill all 128 entries
                        // canonical (length, symbol) order without a pass per length: each length's
                        // first entry is the byte-wise exclusive prefix sum of count x run, all seven
                        // held in one u64 (byte l = entries taken by lengths < l, at most 128)
                        uint64_t wp = 0;
                        uint32_t kraft = 0;
#pragma unroll
                        for (int sy = 0; sy < 19; sy++) {
                            const uint32_t l = (uint32_t)(F >> (3 * CLO_INV[sy])) & 7u;
                            wp += l ? ((uint64_t)(128u >> l) << (8 * l)) : 0ull;
                            kraft += l ? (128u >> l) : 0u;
                        }
                        // the byte-wise sums only hold for a complete code (every prefix <= 128): a
                        // stage-1 regression must not let an incomplete code scribble over the
                        // neighbouring lanes' tables, so such a survivor is dropped here
                        const bool complete = kraft == 128u;
                        uint64_t off = (wp * 0x0101010101010101ull) << 8;
#pragma unroll 1
                        for (int sy = 0; sy < 19; sy++) {
                            const uint32_t l = (uint32_t)(F >> (3 * CLO_INV[sy])) & 7u;
                            if (l && complete) {
                                const uint32_t sh = 8 * l, run = 128u >> l;
                                const uint32_t pos = (uint32_t)(off >> sh) & 255u;
                                off += (uint64_t)run << sh;
                                const uint32_t v = ((uint32_t)sy | (l << 5)) * 0x01010101u;
                                if (run >= 16) {
                                    for (uint32_t r = 0; r < run; r += 16) *(uint4*)(tab + pos + r) = make_uint4(v, v, v, v);
                                } else if (run == 8) {
                                    *(uint2*)(tab + pos) = make_uint2(v, v);
                                } else if (run == 4) {
                                    *(uint32_t*)(tab + pos) = v;
                                } else if (run == 2) {
                                    *(uint16_t*)(tab + pos) = (uint16_t)v;
                                } else {
                                    tab[pos] = (uint8_t)v;
                                }
                            }
                        }
                        i = 0; runVal = -1; litK = 0; distK = 0; nz = 0; eob = 0;
                        active = complete;
                    }
                }
            }
            next = min(end, next + nidle);
            continue;
        }
        if (!__any(active)) {
            if (next >= end && drained) break;
            continue;
        }
        // steps until enough lanes are idle for a refill (or none is active): a loop of its own, so
        // the step's state stays in place across iterations (the refill above is cold code)
        const bool more = next < end || !drained;
        for (uint32_t ni = nidle;;) {
        n_steps += 64 - ni;
        if (__any(active && rd.starved())) {            // (rare: once per ~20 steps, not per step)
            if (active && rd.fi >= 4) rd.reload(in);
        }
        if (active) {
            // one code-length symbol (D/decomp/Open.java's dynamic header loop, same checks)
            // one refill covers the code (<= 7 bits) and its extra bits (<= 7): no branch per symbol kind
            rd.fill();
            const uint32_t b = (uint32_t)rd.bb;
            const uint32_t te = tab[__builtin_bitreverse32(b) >> 25];
            const uint32_t sym = te & 31u, cl = te >> 5;
            const bool s16 = sym == 16, s17 = sym == 17, s18 = sym == 18;
            const uint32_t nx = s16 ? 2u : s17 ? 3u : s18 ? 7u : 0u;
            const uint32_t ex = (b >> cl) & ((1u << nx) - 1u);
            const uint32_t run = sym < 16 ? 1u : ex + (s18 ? 11u : 3u);
            const bool bad = s16 && runVal < 0;
            runVal = sym < 16 ? (int)sym : s16 ? runVal : 0;
            rd.skip(cl + nx);
            // running Kraft sums of the literal/length part [i, min(en, numLit)) and the distance part
            // (branch-free: the lane's state is only read again if it stays active)
            const uint32_t en = i + run;
            const uint32_t v = (uint32_t)runVal;
            const uint32_t wt = v ? (32768u >> v) : 0u;
            litK += (min(en, numLit) - min(i, numLit)) * wt;
            const uint32_t da = max(i, numLit) - numLit, db = max(en, numLit) - numLit, cd = db - da;
            distK += cd * wt;
            nz += v ? cd : 0u;                  // distance codes of nonzero length
            eob = (i <= 256 && 256 < en) ? v : eob;
            i = en;
            // (past the input end the window reads zeros, which only end the loop: the end test
            // below rejects such a header, as the reference's first read past the end would)
            const bool go = !(bad || en > total) && litK <= 32768u && distK <= 32768u;
            active = go && i < total;
            if (go && i >= total) {
                // the reference's end checks (as strict_dynamic): numDist <= 30 here (stage 1 drops
                // HDIST >= 30), so the single distance code's dummy-31 case cannot arise; one
                // distance code of length 1 is distK == 1/2 with one nonzero length; numDist == 1
                // with a zero length is distK == 0
                bool ok;
                if (eob == 0 || litK != 32768u || rd.pos > in.nbits) ok = false;
                else if (numDist == 1 && distK == 0) ok = true;
                else if (nz == 1 && distK == 16384u) ok = true;
                else ok = distK == 32768u;
                if (ok) record(p);
            }
        }
        const uint64_t am = __ballot(active);
        ni = 64u - (uint32_t)__popcll(am);
        if (!am || (more && ni >= NDFL_STRICT_REFILL)) break;
        n_iter++;
        }
    }
    if (sst && lane == 0) {
        atomicAdd(&sst[0], (unsigned long long)n_iter);
        atomicAdd(&sst[1], (unsigned long long)n_refill);
        atomicAdd(&sst[2], (unsigned long long)n_steps);
        atomicAdd(&sst[3], 1ull);
    }
}
// Sort each segment's candidates (arrival order is arbitrary) and compact them into one sorted
// list at the offsets of an exclusive scan of the segment counts: one wave per segment, each
// candidate placed at its rank among the segment's (positions are distinct), counted against the
// segment's list in LDS.  (One thread per segment with an insertion sort through global memory took
// 0.17 ms, its dense segments' quadratic chains of dependent reads.)
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_compact_kernel(const uint32_t* seg_cnt, const uint64_t* seg_list, const uint64_t* seg_off,
                            uint32_t nseg, uint64_t* out) {
    using namespace inf;
    __shared__ uint64_t sv[4][SEG_CAP];
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t seg = blockIdx.x * 4 + wid;
    if (seg >= nseg) return;                    // (no workgroup barrier below)
    const uint32_t c = min(seg_cnt[seg], SEG_CAP);
    const uint64_t* src = seg_list + (uint64_t)seg * SEG_CAP;
    uint64_t* o = out + seg_off[seg];
    static_assert(SEG_CAP == 256, "four candidates per lane");
    uint64_t v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t i = lane + 64u * q;
        v[q] = i < c ? src[i] : ~0ull;
        if (i < c) sv[wid][i] = v[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t r[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < c; j++) {
        const uint64_t u = sv[wid][j];
#pragma unroll
        for (int q = 0; q < 4; q++) r[q] += u < v[q] ? 1u : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (lane + 64u * q < c) o[r[q]] = v[q];
}

struct ChainRes {
    uint64_t end_bit;     // boundary reached / final block end / error position
    uint64_t out_count;   // output bytes (before the error, if any)
    uint32_t status;      // ST_*
    uint32_t reason;      // for ST_ERROR
    uint32_t next;        // count pass, ST_BOUNDARY at a candidate: its index in the candidate list
    uint32_t pad;
    uint64_t bnd_bit;     // emit pass, ST_ERROR: start bit of the block the error is in
    uint64_t bnd_cnt;     //   and the chain's output bytes before that block (partial-input decodes)
};

struct EmitChain {
    uint64_t start_bit;
    uint64_t end_bit;     // stop at this boundary (or final / error)
    uint64_t out_off;
    uint64_t out_count;
    uint64_t slot;        // count-pass segment record of this chain (>= slot capacity: none)
};

// ---- device-side candidate list and chain linking (one host synchronization per decode) ----------
// Link summary (DevLink::info, u64): the decode's results the host reads once at the end.
enum : uint32_t { LI_NCAND = 0, LI_NCH, LI_TOTAL, LI_FLAGS, LI_STOP, LI_CODE, LI_OUTLEN, LI_CONSUMED, LI_NCAND_ALL,
                  LI_LO, LI_NREP, LI_NFLAT, LI_WORDS = 16 };
enum : uint64_t { LF_REPAIR = 1, LF_RANGE = 2, LF_CAPACITY = 4 };
constexpr uint32_t NOLINK = 0xFFFFFFFFu;

// Exclusive scan of the finder segments' candidate counts (capped at SEG_CAP) from 1 (slot 0 is
// the range start): the compact kernel's offsets; info[LI_NCAND_ALL] = the list length.  Two
// launches (ndfl_common.hpp scan_tile_*); grid = tiles.
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_segsum_kernel(const uint32_t* cnt, uint32_t nseg, uint64_t* part) {
    using namespace inf;
    scan_tile_sum([&](uint32_t i) { return (uint64_t)min(cnt[i], SEG_CAP); }, nseg, part);
}
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_segscan_kernel(const uint32_t* cnt, uint32_t nseg, uint64_t* segoff, uint64_t* info, const uint64_t* part) {
    using namespace inf;
    scan_tile_apply([&](uint32_t i) { return (uint64_t)min(cnt[i], SEG_CAP); },
                    [&](uint32_t i, uint64_t v) { segoff[i] = v; }, nseg, part, 1, info + LI_NCAND_ALL);
}

extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_cand_slice_kernel(const uint64_t* sorted, uint64_t* info, uint64_t start_bit, uint64_t end_bit,
                               uint64_t* cands) {
    __shared__ uint64_t s_lo, s_hi;
    const uint64_t na = info[LI_NCAND_ALL];
    if (threadIdx.x == 0) {
        uint64_t lo = 1, hi = na;                           // first index with value > start_bit
        while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (sorted[m] <= start_bit) lo = m + 1; else hi = m; }
        uint64_t lo2 = lo, hi2 = na;                        // first index with value >= end_bit
        while (lo2 < hi2) { const uint64_t m = (lo2 + hi2) >> 1; if (sorted[m] < end_bit) lo2 = m + 1; else hi2 = m; }
        s_lo = lo; s_hi = lo2;
        if (blockIdx.x == 0) { info[LI_NCAND] = 1 + (lo2 - lo); info[LI_LO] = lo; cands[0] = start_bit; }
    }
    __syncthreads();
    const uint64_t lo = s_lo, n = s_hi - s_lo;
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256)
        cands[1 + k] = sorted[lo + k];
}

// Stored-header aliases: a stored block's header can be read at up to 8 bit positions before its
// byte-aligned LEN (the padding between the 3 header bits and the byte boundary is not checked, so
// a header with zero bits before it is also found one, two, ... bits earlier).  Candidates with the
// same BFINAL bit and the same LEN position decode identically from there on, so the count pass
// counts one of them (the first) and the others take its result (ndfl_inflate_alias_copy_kernel).
// Config 2's sync-flush empty stored blocks have ~6 aliases each, each of which otherwise counts
// the whole next piece again.
__device__ __forceinline__ uint64_t stored_key(const inf::In& in, uint64_t p) {
    const uint32_t h = (uint32_t)in.win64(p) & 7u;
    if ((h >> 1) != 0 || p + 3 > in.nbits) return ~0ull;                 // (not a stored header)
    return (((p + 3 + 7) & ~7ull) << 1) | (h & 1u);
}

// rep[k] = the candidate counted for candidate k (the first of its aliases, else k) over the
// info[LI_NCAND] candidates; info[LI_NREP] += the candidates counted (the host reads it with the
// candidate count and picks the count pass's width from it).
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_alias_mark_kernel(const uint64_t* cands, uint64_t* info, const uint32_t* w, uint64_t nwords, uint64_t nbits,
                               uint32_t* rep) {
    const inf::In in{w, nwords, nbits};
    const uint32_t n = (uint32_t)min<uint64_t>(info[LI_NCAND], 0xFFFFFFFFull);
    for (uint32_t k0 = blockIdx.x * 256; k0 < n; k0 += gridDim.x * 256) {
        const uint32_t k = k0 + threadIdx.x;
        bool own = false;
        if (k < n) {
            const uint64_t p = cands[k], key = stored_key(in, p);
            uint32_t r = k;
            if (key != ~0ull)
                for (uint32_t j = k; j > 0 && cands[j - 1] + 10 >= p; j--)
                    if (stored_key(in, cands[j - 1]) == key) r = j - 1;
            rep[k] = r;
            own = r == k;
        }
        const uint32_t c = (uint32_t)__popcll(__ballot(own));
        if ((threadIdx.x & 63) == 0 && c) atomicAdd((unsigned long long*)&info[LI_NREP], (unsigned long long)c);
    }
}

// Bucket orders (the count and emit passes' claim orders) in two launches over tiles of SCAN_TILE
// items, like the scans: the first adds each block's bucket counts into tot[OB_NB]; the second
// places the block's items -- bucket b's slots start at the sum of tot[0..b) plus what the blocks
// before it in arrival order took of bucket b (cursor[b]).  tot and cursor start at zero.  (One
// workgroup over the whole list ran at one CU's bandwidth from other XCDs' data: ~80 us each.)
constexpr uint32_t OB_NB = 24;
constexpr uint32_t OB_WORDS = 2 * OB_NB;      // tot, cursor
constexpr size_t CTK_BYTES = 512;             // chain ticket, nord, two bucket orders, first error
static_assert((16 + 2 * OB_WORDS + 1) * 4 <= CTK_BYTES, "ticket buffer layout");
template <class Bk>
__device__ __forceinline__ void border_count(Bk bk, uint32_t n, uint32_t* ob) {
    __shared__ uint32_t h[OB_NB];
    const uint32_t t = threadIdx.x;
    if (t < OB_NB) h[t] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * SCAN_TILE + t * SCAN_PER;
    if (i0 < n) {
        uint32_t b[SCAN_PER];
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; k++) b[k] = bk(min(i0 + k, n - 1));
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; k++) if (i0 + k < n && b[k] < OB_NB) atomicAdd(&h[b[k]], 1u);
    }
    __syncthreads();
    if (t < OB_NB && h[t]) atomicAdd(&ob[t], h[t]);
}
template <class Bk>
__device__ __forceinline__ void border_place(Bk bk, uint32_t n, uint32_t* ob, uint32_t* order, uint32_t* ntot) {
    __shared__ uint32_t h[OB_NB], base[OB_NB];
    const uint32_t t = threadIdx.x;
    if (t < OB_NB) h[t] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * SCAN_TILE + t * SCAN_PER;
    uint32_t b[SCAN_PER];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) b[k] = OB_NB;
    if (i0 < n) {
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; k++) b[k] = bk(min(i0 + k, n - 1));
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; k++) {
            if (i0 + k >= n) b[k] = OB_NB;
            if (b[k] < OB_NB) atomicAdd(&h[b[k]], 1u);
        }
    }
    __syncthreads();
    if (t < OB_NB) {
        uint32_t p = 0;
        for (uint32_t q = 0; q < t; q++) p += ob[q];
        base[t] = p + (h[t] ? atomicAdd(&ob[OB_NB + t], h[t]) : 0u);
        h[t] = 0;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++)
        if (b[k] < OB_NB) order[base[b[k]] + atomicAdd(&h[b[k]], 1u)] = i0 + k;
    if (ntot && blockIdx.x == 0 && t == 0) {
        uint32_t p = 0;
        for (uint32_t q = 0; q < OB_NB; q++) p += ob[q];
        *ntot = p;
    }
}

// Claim order of the count pass: longest first by the bits to the next start (24 buckets of 32
// Kibit), so that no long chain is left for the end of the launch.  With `rep`
// (ndfl_inflate_alias_mark_kernel), stored-header aliases are left out of the order (*nord = the
// chains to count).  grid = tiles of n.
struct OrderBucket {
    const uint64_t* cands; uint32_t n; uint64_t end_bit; const uint32_t* rep; const uint32_t* flat;
    __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
        const uint64_t c0 = cands[k], c1 = cands[min(k + 1, n - 1)];
        const uint32_t r = rep ? rep[k] : k;
        const uint64_t nx = k + 1 < n ? c1 : end_bit;
        const uint64_t len = nx > c0 ? nx - c0 : 0;
        if (flat && flat[k]) return OB_NB;      // (counted in flat groups)
        return r == k ? OB_NB - 1 - (uint32_t)min<uint64_t>(OB_NB - 1, len >> 15) : OB_NB;
    }
};
// flat: per candidate, nonzero for a chain counted in a flat group (ndfl_inflate_hdr_kernel), or null
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_order_count_kernel(const uint64_t* cands, uint32_t n, uint64_t end_bit, const uint32_t* rep, uint32_t* ob,
                                const uint32_t* flat) {
    border_count(OrderBucket{cands, n, end_bit, rep, flat}, n, ob);
}
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_order_kernel(const uint64_t* cands, uint32_t n, uint64_t end_bit, uint32_t* order, const uint32_t* rep,
                          uint32_t* nord, uint32_t* ob, const uint32_t* flat) {
    border_place(OrderBucket{cands, n, end_bit, rep, flat}, n, ob, order, nord);
}

// The emit pass's claim order over the linked chain list (info[LI_NCH] chains): costliest first, by
// a cost key of input bits and output bytes (32 Kbit or 16 KiB per unit), so that no long chain --
// a stream's last blocks, which share one chain -- starts at the end of the pass.  grid = tiles of
// an upper bound of the chains (the candidates).
struct EmitBucket {
    const EmitChain* chains;
    __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
        const EmitChain& e = chains[k];
        const uint64_t key = ((e.end_bit - e.start_bit) >> 15) + (e.out_count >> 14);
        return OB_NB - 1 - (uint32_t)min<uint64_t>(OB_NB - 1, key);
    }
};
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_emit_order_count_kernel(const EmitChain* chains, const uint64_t* info, uint32_t* ob) {
    if (info[LI_FLAGS]) return;                 // (the emit pass does not run)
    border_count(EmitBucket{chains}, (uint32_t)info[LI_NCH], ob);
}
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_emit_order_kernel(const EmitChain* chains, const uint64_t* info, uint32_t* order, uint32_t* ob) {
    if (info[LI_FLAGS]) return;
    border_place(EmitBucket{chains}, (uint32_t)info[LI_NCH], ob, order, (uint32_t*)nullptr);
}

// Linking by pointer jumping.  Chain k links to the chain starting where it stopped when it stopped
// at a block boundary that is the next candidate (res[k].next), before the range end; the links form
// a forest (a false candidate's chain may end on a real boundary too).  Init: J0 = the link, S = the
// chain's output bytes, D = 1 if linked.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_link_init_kernel(const ChainRes* res, uint32_t n, const uint64_t* cands, uint64_t end_bit, uint32_t* J0,
                              uint64_t* S, uint32_t* D) {
    using namespace inf;
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const ChainRes r = res[k];
        const bool lk = r.status == ST_BOUNDARY && r.end_bit < end_bit && r.next < n && cands[r.next] == r.end_bit;
        J0[k] = lk ? r.next : NOLINK;
        S[k] = r.out_count;
        D[k] = lk ? 1u : 0u;
    }
}
// One doubling round: J_{r+1} = J_r o J_r, S and D summed along (double-buffered).
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_link_jump_kernel(const uint32_t* J, uint32_t* J2, const uint64_t* S, uint64_t* S2, const uint32_t* D,
                              uint32_t* D2, uint32_t n) {
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t j = J[k];
        if (j != NOLINK) { J2[k] = J[j]; S2[k] = S[k] + S[j]; D2[k] = D[k] + D[j]; }
        else { J2[k] = NOLINK; S2[k] = S[k]; D2[k] = D[k]; }
    }
}
// The chain list from the range start: position t is the chain t links away from chain 0
// (binary lifting over the J levels), its output offset dict_len + S[0] - S[node].  The terminal
// chain sets the summary: chains, total bytes, the stop bit, flags (a boundary that is no
// candidate: repair on the host; the range end inside a block; output beyond out_cap).
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_link_path_kernel(const uint32_t* Jall, uint32_t nlev, const uint64_t* S, const uint32_t* D,
                              const ChainRes* res, const uint64_t* cands, uint32_t n, uint64_t dict_len, uint64_t end_bit,
                              uint64_t out_cap, EmitChain* chains, uint64_t* info) {
    using namespace inf;
    const uint32_t len = D[0] + 1;
    for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < len; t += gridDim.x * 256) {
        uint32_t node = 0;
        for (uint32_t r = 0; r < nlev; r++)
            if ((t >> r) & 1u) node = Jall[(uint64_t)r * n + node];
        const ChainRes c = res[node];
        EmitChain e;
        e.start_bit = cands[node];
        e.end_bit = c.end_bit;
        e.out_off = dict_len + S[0] - S[node];
        e.out_count = c.out_count;
        e.slot = node;
        chains[t] = e;
        if (t + 1 == len) {
            uint64_t flags = 0, stop = 0;
            if (c.status == ST_FINAL) stop = c.end_bit;
            else if (c.status == ST_BOUNDARY) {
                if (c.end_bit == end_bit) stop = end_bit;
                else if (c.end_bit > end_bit) flags |= LF_RANGE;
                else flags |= LF_REPAIR;
            }
            if (S[0] > out_cap) flags |= LF_CAPACITY;
            info[LI_NCH] = len; info[LI_TOTAL] = S[0]; info[LI_FLAGS] = flags; info[LI_STOP] = stop;
        }
    }
}
// The decode's result from the emit pass's chain results: the first error in stream order (a
// partial-input decode that ran out of input inside a block stops at that block's start instead).
// ndfl_inflate_first_error_kernel (grid = tiles of an upper bound of the chains) leaves the first
// erring chain in *first (set to ~0 before); the summary kernel (one thread) writes the result.
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_inflate_first_error_kernel(const ChainRes* er, const uint64_t* info, uint32_t* first) {
    using namespace inf;
    const uint32_t nch = (uint32_t)info[LI_NCH];
    const uint32_t i0 = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
    if (i0 >= nch) return;
    uint32_t st[SCAN_PER];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) st[k] = er[min(i0 + k, nch - 1)].status;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++)
        if (i0 + k < nch && st[k] == ST_ERROR) { atomicMin(first, i0 + k); break; }
}
extern "C" __global__ void __launch_bounds__(64)
ndfl_inflate_summary_kernel(const ChainRes* er, const EmitChain* chains, uint64_t* info, uint64_t dict_len,
                            uint32_t partial, const uint32_t* firstp) {
    using namespace inf;
    if (threadIdx.x != 0) return;
    const uint32_t first = *firstp;
    if (first == NOLINK) {
        info[LI_CODE] = 0; info[LI_OUTLEN] = info[LI_TOTAL]; info[LI_CONSUMED] = info[LI_STOP];
        return;
    }
    const ChainRes r = er[first];
    if (partial && r.reason == R_UEOS) {
        info[LI_CODE] = NEED_INPUT;
        info[LI_OUTLEN] = chains[first].out_off - dict_len + r.bnd_cnt;
        info[LI_CONSUMED] = r.bnd_bit;
    } else {
        info[LI_CODE] = r.reason;
        info[LI_OUTLEN] = chains[first].out_off - dict_len + r.out_count;
        info[LI_CONSUMED] = r.end_bit;
    }
}

// Count-pass records of every round of a chain: each lane's exact segment, so the emit pass
// decodes each segment once instead of re-running the speculation.  Records come from a pool and
// are linked per chain in decode order (chain slot -> head record -> next ...).
constexpr uint32_t NOREC = 0xFFFFFFFFu;
struct SegMeta {
    uint32_t ft, kind_ft, reason_ft, next;
    uint64_t end_ft, exit63;
    uint32_t pw, pad;     // the round's words per lane segment (staging geometry)
    uint64_t rs;          // staging origin: the record's lane 0 segment start (absolute bit)
};
struct SegPool {
    uint64_t* start;      // [nrec][64]
    uint32_t* cnt;        // [nrec][64]
    SegMeta* meta;        // [nrec]
    uint32_t* head;       // [nslot] first record of the chain counted at that slot (NOREC: none)
    uint32_t* ctr;        // records handed out
    uint32_t nrec;
    uint64_t nslot;
    // per Huffman block: the count pass's decode tables and header fields (BT_BYTES each), so the
    // emit pass loads them instead of parsing the header and building the tables again; a block's
    // first round record names its table record in SegMeta::pad (NOREC: none)
    char* bt;
    uint32_t* bctr;       // table records handed out
    uint32_t nbt;
};
constexpr uint32_t BT_BYTES = 6720;   // wv::Tabs (6656) + hdr bit, data bit (u64 each), bfinal, btype, ed, pad

#include "inflate_wave.hpp"
#include "inflate_wg.hpp"

// Aliases take the result (and the segment records) of the candidate counted for them.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_alias_copy_kernel(const uint32_t* rep, uint32_t n, ChainRes* res, SegPool pool) {
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t r = rep[k];
        if (r == k) continue;
        res[k] = res[r];
        if (k < pool.nslot) pool.head[k] = r < pool.nslot ? pool.head[r] : NOREC;
    }
}

// ---- host orchestration ---------------------------------------------------------------------

struct InflateScratch {
    void* d_in = nullptr; size_t d_in_cap = 0;
    void* d_cand = nullptr; size_t d_cand_cap = 0;
    void* d_starts = nullptr; size_t d_starts_cap = 0;
    void* d_stops = nullptr; size_t d_stops_cap = 0;
    void* d_res = nullptr; size_t d_res_cap = 0;
    void* d_cands = nullptr; size_t d_cands_cap = 0;
    void* d_stats = nullptr;
    void* d_q = nullptr; size_t d_q_cap = 0;           // finder survivors (stage 1 -> stage 2)
    void* d_seg = nullptr; size_t d_seg_cap = 0;      // segment record pool (SegPool)
    SegPool pool{};
    void* d_chains = nullptr; size_t d_chains_cap = 0;
    void* d_off = nullptr; size_t d_off_cap = 0;
    void* d_ref = nullptr; size_t d_ref_cap = 0;      // emit: back-reference per output byte (deferred copies)
    void* d_pend = nullptr; size_t d_pend_cap = 0;    // emit: pending bit per output byte
    void* d_rl = nullptr; size_t d_rl_cap = 0;        // resolve: two group lists + round bits
    void* d_ticket = nullptr;
    void* d_slow = nullptr; size_t d_slow_cap = 0;    // emit: chains the fast emit pass leaves to the full one
    void* d_rep = nullptr; size_t d_rep_cap = 0;      // count: the candidate counted for each (stored-header aliases)
    void* d_ph = nullptr;                             // count pass: phase-fallback slot per wave
    void* d_hrec = nullptr;                           // count pass: header records, one per candidate
    size_t d_hrec_cap = 0;
    void* d_cticket = nullptr;                        // count pass: chain tickets (one per launch)
    void* d_out = nullptr; size_t d_out_cap = 0;
    Knobs knobs;                                       // the context's switches (ndfl_common.hpp)
    uint32_t q_cap = 0, q_min = 0;                    // finder survivor list: capacity of the last scan / asked minimum
    bool q_full = false;                              //   the last scan's list could not grow (budget, allocation)
    double last_ms_find = 0, last_ms_count = 0, last_ms_emit = 0, last_ms_wall = 0;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    uint64_t repairs = 0, chains = 0, candidates = 0, resolved_groups = 0, flat_chains = 0;
    void* h_cnt = nullptr;                            // pinned: resolve list size
    void* d_info = nullptr;                           // device-side linking: summary (LI_*)
    void* h_info = nullptr;                           //   and its pinned host copy
    void* d_link = nullptr; size_t d_link_cap = 0;    //   pointer-jumping levels and sums
    bool count_first = false;
    // state kept for ndfl_inflate_resolve after a deferred-window range decode
    bool pending = false;
    uint8_t* p_out = nullptr;
    uint64_t p_nbytes = 0, p_dict_len = 0;
    void release() {
        void** ps[] = {&d_in, &d_cand, &d_starts, &d_stops, &d_res, &d_cands, &d_stats, &d_q, &d_seg, &d_chains, &d_off,
                       &d_ref, &d_pend, &d_rl, &d_ticket, &d_ph, &d_cticket, &d_out, &d_hrec, &d_slow, &d_rep};
        for (void** p : ps) { if (*p) hipFree(*p); *p = nullptr; }
        for (auto& e : ev) { if (e) hipEventDestroy(e); e = nullptr; }
        if (h_cnt) hipHostFree(h_cnt);
        h_cnt = nullptr;
        if (h_info) hipHostFree(h_info);
        h_info = nullptr;
        if (d_info) hipFree(d_info);
        d_info = nullptr;
        if (d_link) hipFree(d_link);
        d_link = nullptr; d_link_cap = 0;
        d_in_cap = d_cand_cap = d_starts_cap = d_stops_cap = d_res_cap = d_cands_cap = d_seg_cap = d_q_cap = d_chains_cap = 0;
        d_off_cap = d_ref_cap = d_pend_cap = d_rl_cap = d_out_cap = d_hrec_cap = 0;
        pending = false;
    }
};

// Persistent-wave grid of a one-wave-workgroup kernel: what fits on the chip at once (occupancy),
// at most `cap` waves.
template <typename K>
static uint32_t wave_grid(K kernel, uint32_t cap, const char* env = nullptr) {
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64, 0) != hipSuccess || ncu <= 0 || per <= 0)
        return cap;
    if (env && getenv(env)) per = std::max(1, atoi(getenv(env)));     // waves per CU override (tuning)
    return std::min<uint32_t>(cap, (uint32_t)(ncu * per));
}

// The count pass: one wave per chain (W = 1) or W waves per chain (workgroup rounds,
// inflate_wg.hpp); NDFL_COUNT_W selects W (1, 2, 4, 8).  Persistent grid sized by occupancy; the
// phase-fallback slots (d_ph) cover COUNT_WAVES waves.
static uint32_t count_w(const Knobs& k) {
    const uint32_t v = k.count_w ? k.count_w : (uint32_t)NDFL_COUNT_W_DEFAULT;
    return (v == 2 || v == 4 || v == 8) ? v : 1u;
}
template <typename K>
static uint32_t wg_grid(K kernel, uint32_t threads, uint32_t cap) {
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, (int)threads, 0) != hipSuccess || ncu <= 0 || per <= 0)
        return cap;
    return std::min<uint32_t>(cap, (uint32_t)(ncu * per));
}
template <typename... A>
static void launch_count(hipStream_t s, uint32_t W, uint32_t nchains, A... args) {
    if (W == 1) {
        static const uint32_t g1 = wave_grid(ndfl_inflate_count_wave_kernel, inf::COUNT_WAVES, "NDFL_COUNT_WPC");
        hipLaunchKernelGGL(ndfl_inflate_count_wave_kernel, dim3(std::min(nchains, g1)), dim3(64), 0, s, args...);
    } else if (W == 2) {
        static const uint32_t g = wg_grid(ndfl_inflate_count_wg_kernel<2>, 128, inf::COUNT_WAVES / 2);
        hipLaunchKernelGGL(ndfl_inflate_count_wg_kernel<2>, dim3(std::min(nchains, g)), dim3(128), 0, s, args...);
    } else if (W == 4) {
        static const uint32_t g = wg_grid(ndfl_inflate_count_wg_kernel<4>, 256, inf::COUNT_WAVES / 4);
        hipLaunchKernelGGL(ndfl_inflate_count_wg_kernel<4>, dim3(std::min(nchains, g)), dim3(256), 0, s, args...);
    } else {
        static const uint32_t g = wg_grid(ndfl_inflate_count_wg_kernel<8>, 512, inf::COUNT_WAVES / 8);
        hipLaunchKernelGGL(ndfl_inflate_count_wg_kernel<8>, dim3(std::min(nchains, g)), dim3(512), 0, s, args...);
    }
}

static hipError_t inf_ensure(void** p, size_t* cap, size_t n) {
    if (n <= *cap && *p) return hipSuccess;
    if (*p) { hipFree(*p); *p = nullptr; *cap = 0; }
    size_t want = n < 4096 ? 4096 : n;
    hipError_t e = hipMalloc(p, want);
    if (e == hipSuccess) *cap = want;
    return e;
}


static bool inf_debug() { static const bool d = getenv("NDFL_DEBUG") != nullptr; return d; }
#define INF_CHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) {                                             \
        if (inf_debug()) fprintf(stderr, "[ndfl] HIP error %d (%s) at inflate_kernels.hip:%d\n", (int)_e,     \
                                 hipGetErrorString(_e), __LINE__);                                              \
        return -4; } } while (0)
#define INF_RC(x) do { const int _r = (x); if (_r) return _r; } while (0)

// Resolve the deferred copies of an emit pass: pointer-jumping rounds over the pending 32-byte
// groups of out[0, nbytes) until none is left.  *groups = pending groups at the start.
static int resolve_rounds(InflateScratch& S, hipStream_t s, uint8_t* d_out, uint64_t nbytes, uint64_t* groups) {
    using namespace inf;
    *groups = 0;
    const uint64_t npw = (nbytes + 31) / 32;
    if (npw == 0) return 0;
    if (npw > 0xFFFFFFFFull) return -2;
    INF_CHK(inf_ensure(&S.d_rl, &S.d_rl_cap, npw * 12 + 64));
    uint32_t* cnt = (uint32_t*)S.d_rl;                       // [0], [1]: list sizes
    uint32_t* lst[2] = {(uint32_t*)((char*)S.d_rl + 64), (uint32_t*)((char*)S.d_rl + 64) + npw};
    uint32_t* nb = lst[1] + npw;
    uint32_t* pend = (uint32_t*)S.d_pend;
    uint32_t* ref = (uint32_t*)S.d_ref;
    INF_CHK(hipMemsetAsync(cnt, 0, 8, s));
    hipLaunchKernelGGL(ndfl_inflate_pending_list_kernel, dim3((uint32_t)((npw + 4095) / 4096)), dim3(256), 0, s,
                       (const uint32_t*)pend, (uint64_t)0, npw, lst[0], cnt);
    INF_CHK(hipGetLastError());
    if (!S.h_cnt) INF_CHK(hipHostMalloc(&S.h_cnt, 64, 0));
    uint32_t* h = (uint32_t*)S.h_cnt;
    // rounds are queued four at a time on grid-stride kernels; the host reads the list size between
    // batches only (pointer jumping needs ~log2(reference depth) rounds)
    int cur = 0;
    uint32_t n = 0;
    for (int round = 0;; round++) {
        const bool rstats = S.knobs.stats;
        if ((round & 3) == 0 || rstats) {
            INF_CHK(hipMemcpyAsync(h, cnt + cur, 4, hipMemcpyDeviceToHost, s));
            if (rstats) INF_CHK(hipMemcpyAsync(h + 1, cnt + 2 + cur, 4, hipMemcpyDeviceToHost, s));
            INF_CHK(hipStreamSynchronize(s));
            n = *h;
            if (rstats) fprintf(stderr, "[ndfl] resolve round %d: %u pending groups, %u bytes\n", round, n, h[1]);
            if (round == 0) *groups = n;
            if (n == 0) return 0;
            if (round >= 96) return R_INTERNAL;              // distances double each round: unreachable
        }
        INF_CHK(hipMemsetAsync(cnt + (cur ^ 1), 0, 4, s));
        if (rstats) INF_CHK(hipMemsetAsync(cnt + 2 + (cur ^ 1), 0, 4, s));
        const uint32_t gb = (uint32_t)std::min<uint64_t>(4096, ((uint64_t)n * 32 + 255) / 256);
        hipLaunchKernelGGL(ndfl_inflate_resolve_kernel, dim3(gb), dim3(256), 0, s,
                           (const uint32_t*)lst[cur], (const uint32_t*)(cnt + cur), (const uint32_t*)pend, ref, d_out, nb);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_resolve_apply_kernel, dim3((uint32_t)std::min<uint64_t>(1024, (n + 255) / 256)),
                           dim3(256), 0, s, (const uint32_t*)lst[cur], (const uint32_t*)(cnt + cur), pend,
                           (const uint32_t*)nb, lst[cur ^ 1], cnt + (cur ^ 1), rstats ? cnt + 2 + (cur ^ 1) : (uint32_t*)nullptr);
        INF_CHK(hipGetLastError());
        cur ^= 1;
    }
}

// Segment-record pool for `nstarts` chain starts (SegPool): the rounds of all chains, one head per
// counted chain start, with room for repairs, and the per-block table records.
static int setup_pool(InflateScratch& S, hipStream_t s, uint64_t nstarts, uint64_t nbits) {
    using namespace inf;
    const uint64_t nslot = nstarts + std::max<uint64_t>(4096, nstarts / 2);
    const uint64_t nrec = std::min<uint64_t>(0xFFFFFFF0ull, 2 * nstarts + nbits / (wv::MAX_SPAN / 2) + 65536);
    // table records: at most one per block; bounded (a stream of tiny blocks parses the rest again)
    const uint64_t nbt = std::min<uint64_t>(nrec, S.knobs.no_bt ? 0 : (1u << 18));
    const uint64_t seg_bytes = nrec * (64 * 8 + 64 * 4 + sizeof(SegMeta)) + nslot * 4 + 64 + nbt * BT_BYTES;
    INF_CHK(inf_ensure(&S.d_seg, &S.d_seg_cap, seg_bytes));
    SegPool pool;
    pool.start = (uint64_t*)S.d_seg;
    pool.cnt = (uint32_t*)(pool.start + nrec * 64);
    pool.meta = (SegMeta*)(pool.cnt + nrec * 64);
    pool.head = (uint32_t*)(pool.meta + nrec);
    pool.ctr = (uint32_t*)S.d_stats + 12;
    pool.bctr = (uint32_t*)S.d_stats + 13;
    pool.nbt = (uint32_t)nbt;
    pool.bt = (char*)(((uintptr_t)(pool.head + nslot) + 63) & ~(uintptr_t)63);
    pool.nrec = (uint32_t)nrec;
    pool.nslot = nslot;
    S.pool = pool;
    INF_CHK(hipMemsetAsync(pool.head, 0xFF, nslot * 4, s));
    return 0;
}

// Queue `rounds` resolve rounds without reading anything back (the kernels read the list sizes on
// the device; a round with nothing pending costs two empty launches).  *cnt_slot = where the size of
// the list left after them is (cnt + cur).
static int resolve_rounds_dev(InflateScratch& S, hipStream_t s, uint8_t* d_out, uint64_t nbytes, int rounds,
                              uint32_t** left, uint64_t* first_count_dst) {
    using namespace inf;
    const uint64_t npw = (nbytes + 31) / 32;
    *left = nullptr;
    if (npw == 0) return 0;
    if (npw > 0xFFFFFFFFull) return -2;
    INF_CHK(inf_ensure(&S.d_rl, &S.d_rl_cap, npw * 12 + 64));
    uint32_t* cnt = (uint32_t*)S.d_rl;
    uint32_t* lst[2] = {(uint32_t*)((char*)S.d_rl + 64), (uint32_t*)((char*)S.d_rl + 64) + npw};
    uint32_t* nb = lst[1] + npw;
    uint32_t* pend = (uint32_t*)S.d_pend;
    uint32_t* ref = (uint32_t*)S.d_ref;
    INF_CHK(hipMemsetAsync(cnt, 0, 8, s));
    hipLaunchKernelGGL(ndfl_inflate_pending_list_kernel, dim3((uint32_t)((npw + 4095) / 4096)), dim3(256), 0, s,
                       (const uint32_t*)pend, (uint64_t)0, npw, lst[0], cnt);
    INF_CHK(hipGetLastError());
    if (first_count_dst) INF_CHK(hipMemcpyAsync(first_count_dst, cnt, 4, hipMemcpyDeviceToDevice, s));
    int cur = 0;
    for (int round = 0; round < rounds; round++) {
        INF_CHK(hipMemsetAsync(cnt + (cur ^ 1), 0, 4, s));
        hipLaunchKernelGGL(ndfl_inflate_resolve_kernel, dim3(4096), dim3(256), 0, s, (const uint32_t*)lst[cur],
                           (const uint32_t*)(cnt + cur), (const uint32_t*)pend, ref, d_out, nb);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_resolve_apply_kernel, dim3(1024), dim3(256), 0, s, (const uint32_t*)lst[cur],
                           (const uint32_t*)(cnt + cur), pend, (const uint32_t*)nb, lst[cur ^ 1], cnt + (cur ^ 1),
                           (uint32_t*)nullptr);
        INF_CHK(hipGetLastError());
        cur ^= 1;
    }
    *left = cnt + cur;
    return 0;
}

constexpr int LINK_FALLBACK = 1000;      // the device-side path hands over to the host path
constexpr int FIND_OVERFLOW = 1001;      // more finder survivors than the list held: scan again
constexpr uint32_t LI_QCOUNT = 14;       // (host copy only: the finder's survivor count)

// The decode after the header finder with everything on the device and ONE host synchronization
// in the middle (the number of chain starts, which sizes the record pool and the grids) and one at
// the end (the summary): candidate list (segment scan, compaction, the range's slice), the count
// pass in longest-first order, chain linking by pointer jumping, the emit pass, the first error,
// the resolve rounds.  Returns LINK_FALLBACK when the host's linking has to step in (a chain that
// stopped at a boundary that is no candidate) -- the host path then starts over from the finder's
// candidates -- or when the list of chain starts is too long for the jump tables.
static int inflate_devlink(InflateScratch& S, hipStream_t s, const uint32_t* d_w, uint64_t nwords, uint64_t nbits,
                           uint32_t nseg, const uint32_t* d_cnt, const uint64_t* d_list, uint64_t start_bit,
                           uint64_t end_bit, uint8_t* out, uint64_t dict_len, uint64_t out_cap, uint64_t* out_len,
                           uint64_t* consumed_bits, uint32_t flags, bool deferred, bool partial, double* last_ms) {
    using namespace inf;
    if (!S.d_info) INF_CHK(hipMalloc(&S.d_info, LI_WORDS * 8));
    if (!S.h_info) INF_CHK(hipHostMalloc(&S.h_info, LI_WORDS * 8, 0));
    uint64_t* info = (uint64_t*)S.d_info;
    volatile uint64_t* hinfo = (volatile uint64_t*)S.h_info;
    INF_CHK(hipMemsetAsync(info, 0, LI_WORDS * 8, s));
    const uint64_t cap_all = (uint64_t)nseg * SEG_CAP + 1;      // the sorted list's length at most
    const uint32_t ntile = (nseg + SCAN_TILE - 1) / SCAN_TILE;
    INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, (cap_all + nseg + 2 + ntile) * 8));
    uint64_t* d_sorted = (uint64_t*)S.d_starts;
    uint64_t* d_segoff = d_sorted + cap_all;
    uint64_t* d_part = d_segoff + nseg + 2;
    hipLaunchKernelGGL(ndfl_inflate_segsum_kernel, dim3(ntile), dim3(SCAN_T), 0, s, d_cnt, nseg, d_part);
    INF_CHK(hipGetLastError());
    hipLaunchKernelGGL(ndfl_inflate_segscan_kernel, dim3(ntile), dim3(SCAN_T), 0, s, d_cnt, nseg, d_segoff, info,
                       (const uint64_t*)d_part);
    INF_CHK(hipGetLastError());
    hipLaunchKernelGGL(ndfl_inflate_compact_kernel, dim3((nseg + 3) / 4), dim3(256), 0, s, d_cnt, d_list,
                       (const uint64_t*)d_segoff, nseg, d_sorted);
    INF_CHK(hipGetLastError());
    INF_CHK(inf_ensure(&S.d_cands, &S.d_cands_cap, (cap_all + 1) * 8ull));
    hipLaunchKernelGGL(ndfl_inflate_cand_slice_kernel, dim3((uint32_t)std::min<uint64_t>(4096, (cap_all + 255) / 256)),
                       dim3(256), 0, s, (const uint64_t*)d_sorted, info, start_bit, end_bit, (uint64_t*)S.d_cands);
    INF_CHK(hipGetLastError());
    // stored-header aliases counted once (NDFL_NO_ALIAS: every candidate counted)
    const bool alias_on = !S.knobs.no_alias;
    uint32_t* d_rep = nullptr;
    if (alias_on) {
        INF_CHK(inf_ensure(&S.d_rep, &S.d_rep_cap, (size_t)cap_all * 4 + 64));
        d_rep = (uint32_t*)S.d_rep;
        hipLaunchKernelGGL(ndfl_inflate_alias_mark_kernel, dim3((uint32_t)std::min<uint64_t>(1024, (cap_all + 255) / 256)),
                           dim3(256), 0, s, (const uint64_t*)S.d_cands, info, d_w, nwords, nbits, d_rep);
        INF_CHK(hipGetLastError());
    }
    INF_CHK(hipMemcpyAsync((void*)hinfo, info, (LI_NREP + 1) * 8, hipMemcpyDeviceToHost, s));
    hinfo[LI_QCOUNT] = 0;
    INF_CHK(hipMemcpyAsync((void*)(hinfo + LI_QCOUNT), (const uint32_t*)S.d_stats + 8, 4, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));                          // (1) the number of chain starts
    if ((uint32_t)hinfo[LI_QCOUNT] > S.q_cap && !S.q_full) { S.q_min = (uint32_t)hinfo[LI_QCOUNT] + 65536; return FIND_OVERFLOW; }
    const uint64_t n = hinfo[LI_NCAND];
    // the count pass's width: one wave per chain, unless the chains to count are few against the
    // count waves (fewer than 2 per wave), where a chain's rounds in sequence bound the pass (config
    // 2: 3,286 chains, ~1.1 per wave: 4 waves per chain count it in 2.0 ms instead of 4.0; one rank's
    // 512 MiB share of the bench at 8 GPUs: 8,191 chains, ~2.7 per wave: one wave each, 2.1 ms
    // instead of 3.1 -- profiles/r05_shard_count_width.txt; the bench's 66,770 chains: one wave
    // each) -- NDFL_COUNT_W overrides
    const uint64_t nrep = alias_on ? hinfo[LI_NREP] : n;
    static const uint32_t count_waves = wave_grid(ndfl_inflate_count_wave_kernel, COUNT_WAVES, "NDFL_COUNT_WPC");
    const uint32_t W = S.knobs.count_w ? count_w(S.knobs) : (nrep < 2ull * count_waves && nbits >= (1ull << 24)) ? 4u : 1u;
    if (S.knobs.stats) fprintf(stderr, "[ndfl] count pass: %llu candidates, %llu counted, width %u\n",
                                      (unsigned long long)n, (unsigned long long)nrep, W);
    if (n == 0 || n > (1ull << 24)) return LINK_FALLBACK;
    const uint32_t ncand = (uint32_t)n;
    int rc = setup_pool(S, s, n, nbits);
    if (rc) return rc;
    // count pass, longest chains first
    INF_CHK(inf_ensure(&S.d_stops, &S.d_stops_cap, n * 12));
    INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, n * sizeof(ChainRes)));
    uint32_t* d_order = (uint32_t*)((char*)S.d_stops + n * 8);
    if (!S.d_cticket) INF_CHK(hipMalloc(&S.d_cticket, CTK_BYTES));
    INF_CHK(hipMemsetAsync(S.d_cticket, 0, CTK_BYTES, s));
    uint32_t* d_nord = (uint32_t*)S.d_cticket + 8;
    uint32_t* d_nflat = (uint32_t*)S.d_cticket + 4;
    uint32_t* d_ob = (uint32_t*)S.d_cticket + 16;                      // count order: tot, cursor
    const uint32_t otiles = (ncand + SCAN_TILE - 1) / SCAN_TILE;
    if (!S.d_ph) INF_CHK(hipMalloc(&S.d_ph, (size_t)std::max(COUNT_WAVES, EMIT_WAVES) * sizeof(wv::PhArr)));
    const bool stats_on = S.knobs.stats;
    const uint64_t limit = std::min(end_bit, nbits);
    INF_CHK(hipEventRecord(S.ev[2], s));
    // header records, and the chains whose first block is counted by one lane (flat groups: the
    // one-wave count kernel only); those leave the count order
    const bool hrec_on = !S.knobs.no_hdrrec;
    // (a flat group decodes its 64 blocks one lane each: ~7 ms of latency however few the chains, so
    // only a pass long enough to hide it takes them -- the bench's 66,770 chains; one rank's 8,191 at
    // 8 GPUs counts its incompressible blocks in wave form, by escape scans)
    const bool flat_on = hrec_on && W == 1 && S.knobs.flat && nrep >= S.knobs.flat_min;
    uint32_t* d_flist = nullptr;
    uint32_t* d_fflag = nullptr;
    if (hrec_on) {
        INF_CHK(inf_ensure(&S.d_hrec, &S.d_hrec_cap, (size_t)ncand * (sizeof(wv::HdrRec) + 8) + 64));
        d_flist = (uint32_t*)((char*)S.d_hrec + (size_t)ncand * sizeof(wv::HdrRec));
        d_fflag = d_flist + ncand;
        hipLaunchKernelGGL(ndfl_inflate_hdr_kernel, dim3((ncand + 63) / 64), dim3(64), 0, s, d_w, nwords, nbits,
                           (const uint64_t*)S.d_cands, ncand, (wv::HdrRec*)S.d_hrec, flat_on ? d_flist : nullptr,
                           d_nflat, flat_on ? d_fflag : nullptr);
        INF_CHK(hipGetLastError());
    }
    hipLaunchKernelGGL(ndfl_inflate_order_count_kernel, dim3(otiles), dim3(SCAN_T), 0, s, (const uint64_t*)S.d_cands,
                       ncand, end_bit, (const uint32_t*)d_rep, d_ob, flat_on ? (const uint32_t*)d_fflag : nullptr);
    INF_CHK(hipGetLastError());
    hipLaunchKernelGGL(ndfl_inflate_order_kernel, dim3(otiles), dim3(SCAN_T), 0, s, (const uint64_t*)S.d_cands, ncand,
                       end_bit, d_order, (const uint32_t*)d_rep, (alias_on || flat_on) ? d_nord : (uint32_t*)nullptr, d_ob,
                       flat_on ? (const uint32_t*)d_fflag : nullptr);
    INF_CHK(hipGetLastError());
    if (flat_on) INF_CHK(hipMemcpyAsync(info + LI_NFLAT, d_nflat, 4, hipMemcpyDeviceToDevice, s));
    launch_count(s, W, ncand,
                       d_w, nwords, nbits, (const uint64_t*)S.d_cands, (const uint64_t*)nullptr, ncand,
                       (const uint64_t*)S.d_cands, ncand, limit, (ChainRes*)S.d_res,
                       stats_on ? (uint32_t*)S.d_stats : nullptr, (uint64_t)0, S.pool, (uint32_t*)S.d_cticket,
                       (wv::PhArr*)S.d_ph, (const uint32_t*)d_order, end_bit,
                       hrec_on ? (const wv::HdrRec*)S.d_hrec : nullptr,
                       (alias_on || flat_on) ? (const uint32_t*)d_nord : nullptr, flat_on ? (const uint32_t*)d_flist : nullptr,
                       flat_on ? (const uint32_t*)d_nflat : nullptr);
    INF_CHK(hipGetLastError());
    if (alias_on) {
        hipLaunchKernelGGL(ndfl_inflate_alias_copy_kernel, dim3(std::min<uint32_t>(1024, (ncand + 255) / 256)), dim3(256), 0, s,
                           (const uint32_t*)d_rep, ncand, (ChainRes*)S.d_res, S.pool);
        INF_CHK(hipGetLastError());
    }
    INF_CHK(hipEventRecord(S.ev[3], s));
    if (stats_on) {                             // the count pass's chains by outcome (wave time in 10 us units)
        std::vector<ChainRes> cr(ncand);
        INF_CHK(hipMemcpyAsync(cr.data(), S.d_res, ncand * sizeof(ChainRes), hipMemcpyDeviceToHost, s));
        INF_CHK(hipStreamSynchronize(s));
        uint64_t cnt[3] = {0, 0, 0}, tsum[3] = {0, 0, 0}, tmax[3] = {0, 0, 0}, blk[3] = {0, 0, 0};
        for (uint32_t k = 0; k < ncand; k++) {
            const uint32_t st = std::min<uint32_t>(cr[k].status, 2u), t = cr[k].pad >> 16;
            cnt[st]++; tsum[st] += t; tmax[st] = std::max<uint64_t>(tmax[st], t); blk[st] += cr[k].pad & 0xFFFFu;
        }
        if (flat_on) {
            uint32_t fw[12] = {0};
            INF_CHK(hipMemcpy(fw, (uint32_t*)S.d_cticket + 4, 48, hipMemcpyDeviceToHost));
            fprintf(stderr, "[ndfl] count flat groups sent back: (unused) %u, full-table tokens %u, "
                    "error %u, chain goes on %u, table %u\n", fw[7], fw[8], fw[9], fw[10], fw[11]);
            const unsigned long long gt = (unsigned long long)fw[2] | ((unsigned long long)fw[3] << 32);
            fprintf(stderr, "[ndfl] count flat groups: %u chains in %u groups, %u sent back to the wave decode, "
                    "group wave time %.3f ms mean\n", fw[0], (fw[0] + 63) / 64, fw[1], fw[0] ? gt * 1e-5 / ((fw[0] + 63) / 64) : 0.0);
#ifdef NDFL_FLAT_PROF
            unsigned long long fpv[4] = {0, 0, 0, 0}, z[4] = {0, 0, 0, 0};
            INF_CHK(hipMemcpyFromSymbol(fpv, HIP_SYMBOL(wv::g_flat_prof), 32));
            INF_CHK(hipMemcpyToSymbol(HIP_SYMBOL(wv::g_flat_prof), z, 32));
            fprintf(stderr, "[ndfl] flat decode loops (lane 0, clock64): %llu cycles, %llu at %llu phase points\n", fpv[0], fpv[1], fpv[2]);
#endif
        }
        const char* nm[3] = {"boundary", "final", "error"};
        for (int k = 0; k < 3; k++)
            fprintf(stderr, "[ndfl] count chains %s: %llu, wave time %.2f ms (max %.3f ms), blocks %llu\n", nm[k],
                    (unsigned long long)cnt[k], tsum[k] * 1e-2, tmax[k] * 1e-2, (unsigned long long)blk[k]);
        // wave time against the chain's bits (the count order's key): per 32-Kibit bucket, and the
        // longest chains
        std::vector<uint64_t> cb(ncand);
        INF_CHK(hipMemcpy(cb.data(), S.d_cands, ncand * 8, hipMemcpyDeviceToHost));
        uint64_t bn[OB_NB] = {}, bt[OB_NB] = {}, bm[OB_NB] = {};
        uint32_t bk[OB_NB] = {};
        std::vector<uint32_t> top;
        for (uint32_t k = 0; k < ncand; k++) {
            const uint64_t nx = k + 1 < ncand ? cb[k + 1] : end_bit, len = nx > cb[k] ? nx - cb[k] : 0;
            const uint32_t b = (uint32_t)std::min<uint64_t>(OB_NB - 1, len >> 15), t = cr[k].pad >> 16;
            bn[b]++; bt[b] += t;
            if (t >= bm[b]) { bm[b] = t; bk[b] = k; }
            top.push_back(k);
        }
        for (uint32_t b = 0; b < OB_NB; b++)
            if (bn[b]) fprintf(stderr, "[ndfl] count bits %2u x 32Ki: %6llu chains, mean %.3f ms, max %.3f ms "
                               "(chain %u at bit %llu: blocks %u, status %u, out %llu)\n", b,
                               (unsigned long long)bn[b], bt[b] * 1e-2 / bn[b], bm[b] * 1e-2, bk[b],
                               (unsigned long long)cb[bk[b]], cr[bk[b]].pad & 0xFFFFu, cr[bk[b]].status,
                               (unsigned long long)cr[bk[b]].out_count);
        const size_t nt = std::min<size_t>(8, top.size());
        std::partial_sort(top.begin(), top.begin() + nt, top.end(),
                          [&](uint32_t a, uint32_t b) { return (cr[a].pad >> 16) > (cr[b].pad >> 16); });
        for (size_t i = 0; i < nt; i++) {
            const uint32_t k = top[i];
            const uint64_t nx = k + 1 < ncand ? cb[k + 1] : end_bit;
            fprintf(stderr, "[ndfl] count longest: chain %u at bit %llu, %llu bits, %.3f ms, blocks %u, status %u, out %llu\n",
                    k, (unsigned long long)cb[k], (unsigned long long)(nx - cb[k]), (cr[k].pad >> 16) * 1e-2,
                    cr[k].pad & 0xFFFFu, cr[k].status, (unsigned long long)cr[k].out_count);
        }
    }
    // linking: J levels (u32), S and D double-buffered
    uint32_t nlev = 1;
    while ((1ull << nlev) < n) nlev++;
    const size_t link_bytes = (size_t)(nlev + 1) * n * 4 + 2 * n * 8 + 2 * n * 4 + 64;
    INF_CHK(inf_ensure(&S.d_link, &S.d_link_cap, link_bytes));
    uint32_t* J = (uint32_t*)S.d_link;
    uint64_t* Ssum[2] = {(uint64_t*)(((uintptr_t)(J + (size_t)(nlev + 1) * n) + 7) & ~(uintptr_t)7), nullptr};
    Ssum[1] = Ssum[0] + n;
    uint32_t* Dd[2] = {(uint32_t*)(Ssum[1] + n), nullptr};
    Dd[1] = Dd[0] + n;
    const uint32_t lg = (uint32_t)std::min<uint64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(ndfl_inflate_link_init_kernel, dim3(lg), dim3(256), 0, s, (const ChainRes*)S.d_res, ncand,
                       (const uint64_t*)S.d_cands, end_bit, J, Ssum[0], Dd[0]);
    INF_CHK(hipGetLastError());
    int cur = 0;
    for (uint32_t r = 0; r < nlev; r++) {
        hipLaunchKernelGGL(ndfl_inflate_link_jump_kernel, dim3(lg), dim3(256), 0, s, (const uint32_t*)(J + (size_t)r * n),
                           J + (size_t)(r + 1) * n, (const uint64_t*)Ssum[cur], Ssum[cur ^ 1], (const uint32_t*)Dd[cur],
                           Dd[cur ^ 1], ncand);
        INF_CHK(hipGetLastError());
        cur ^= 1;
    }
    INF_CHK(inf_ensure(&S.d_chains, &S.d_chains_cap, n * sizeof(EmitChain)));
    hipLaunchKernelGGL(ndfl_inflate_link_path_kernel, dim3(lg), dim3(256), 0, s, (const uint32_t*)J, nlev,
                       (const uint64_t*)Ssum[cur], (const uint32_t*)Dd[cur], (const ChainRes*)S.d_res,
                       (const uint64_t*)S.d_cands, ncand, dict_len, end_bit, out_cap, (EmitChain*)S.d_chains, info);
    INF_CHK(hipGetLastError());
    // the emit pass claims the linked chains costliest first (the count pass's order buffer is free)
    {
        uint32_t* d_eob = (uint32_t*)S.d_cticket + 16 + OB_WORDS;      // emit order: tot, cursor (zeroed above)
        const uint32_t etiles = (ncand + SCAN_TILE - 1) / SCAN_TILE;    // (chains <= candidates)
        hipLaunchKernelGGL(ndfl_inflate_emit_order_count_kernel, dim3(etiles), dim3(SCAN_T), 0, s,
                           (const EmitChain*)S.d_chains, (const uint64_t*)info, d_eob);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_emit_order_kernel, dim3(etiles), dim3(SCAN_T), 0, s, (const EmitChain*)S.d_chains,
                           (const uint64_t*)info, d_order, d_eob);
        INF_CHK(hipGetLastError());
    }
    // emit into the output (or a device staging buffer sized by the bound out_cap)
    uint8_t* d_out;
    const bool direct = (flags & 2u) != 0;
    // the output's size is known on the device only: the scratch (back-references, pending bits,
    // a staging copy) is sized by out_cap, capped at DEFLATE's largest expansion (258 bytes per 2 bits)
    const uint64_t obytes = dict_len + std::min<uint64_t>(out_cap, 129 * nbits + 65536);
    if (obytes > (40ull << 30)) return LINK_FALLBACK;          // (the host path sizes it exactly)
    if (direct) d_out = out;
    else {
        INF_CHK(inf_ensure(&S.d_out, &S.d_out_cap, obytes + 64));
        d_out = (uint8_t*)S.d_out;
        if (dict_len) INF_CHK(hipMemcpyAsync(d_out, out, dict_len, hipMemcpyHostToDevice, s));
    }
    const uint64_t nbytes = obytes;
    if ((nbytes + 31) / 32 > 0xFFFFFFFFull) return LINK_FALLBACK;
    const uint64_t npw = (nbytes + 31) / 32;
    INF_CHK(inf_ensure(&S.d_ref, &S.d_ref_cap, nbytes * 4 + 64));
    INF_CHK(inf_ensure(&S.d_pend, &S.d_pend_cap, npw * 4 + 64));
    INF_CHK(hipMemsetAsync(S.d_pend, 0, npw * 4 + 64, s));
    if (!S.d_ticket) INF_CHK(hipMalloc(&S.d_ticket, 64));
    INF_CHK(hipMemsetAsync(S.d_ticket, 0, 64, s));
    if (S.knobs.test_segflip && S.pool.cnt) {         // (test: record 0, lane 0 counts one byte more)
        uint32_t c0 = 0;
        INF_CHK(hipMemcpyAsync(&c0, S.pool.cnt, 4, hipMemcpyDeviceToHost, s));
        INF_CHK(hipStreamSynchronize(s));
        c0++;
        INF_CHK(hipMemcpyAsync(S.pool.cnt, &c0, 4, hipMemcpyHostToDevice, s));
        INF_CHK(hipStreamSynchronize(s));
    }
    INF_CHK(hipEventRecord(S.ev[4], s));
    static const uint32_t emit_grid = wave_grid(ndfl_inflate_emit_wave_kernel, EMIT_WAVES, "NDFL_EMIT_WPC");
    // the record-replay emit kernel first, the full one over what it leaves (NDFL_EMIT_FAST=0: the
    // full one alone)
    if (S.knobs.emit_fast) {
        INF_CHK(inf_ensure(&S.d_slow, &S.d_slow_cap, (size_t)ncand * 4 + 64));
        uint32_t* tk = (uint32_t*)S.d_ticket;             // [0] fast tickets, [4] full tickets, [8] slow count
        static const uint32_t fast_grid = wave_grid(ndfl_inflate_emit_fast_kernel, EMIT_WAVES, "NDFL_EMITF_WPC");
        hipLaunchKernelGGL(ndfl_inflate_emit_fast_kernel, dim3(std::min<uint32_t>(ncand, fast_grid)), dim3(64), 0, s, d_w,
                           nwords, nbits, (const EmitChain*)S.d_chains, tk, d_out, (ChainRes*)S.d_res,
                           (uint32_t*)S.d_ref, (uint32_t*)S.d_pend, S.pool, (const uint64_t*)info, (const uint32_t*)d_order,
                           (uint32_t*)S.d_slow, tk + 8);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_emit_wave_kernel, dim3(std::min<uint32_t>(ncand, emit_grid)), dim3(64), 0, s, d_w,
                           nwords, nbits, (const EmitChain*)S.d_chains, ncand, tk + 4, d_out,
                           (ChainRes*)S.d_res, (const uint64_t*)S.d_cands, ncand, (uint32_t*)S.d_ref, (uint32_t*)S.d_pend,
                           S.pool, (wv::PhArr*)S.d_ph, stats_on ? (uint32_t*)S.d_stats : nullptr, (const uint64_t*)info,
                           (const uint32_t*)S.d_slow, (const uint32_t*)(tk + 8));
        INF_CHK(hipGetLastError());
        if (stats_on) {
            uint32_t nsl = 0;
            INF_CHK(hipMemcpyAsync(&nsl, tk + 8, 4, hipMemcpyDeviceToHost, s));
            INF_CHK(hipStreamSynchronize(s));
            fprintf(stderr, "[ndfl] fast emit pass left %u chains to the full emit pass\n", nsl);
        }
    } else {
        hipLaunchKernelGGL(ndfl_inflate_emit_wave_kernel, dim3(std::min<uint32_t>(ncand, emit_grid)), dim3(64), 0, s, d_w,
                           nwords, nbits, (const EmitChain*)S.d_chains, ncand, (uint32_t*)S.d_ticket, d_out,
                           (ChainRes*)S.d_res, (const uint64_t*)S.d_cands, ncand, (uint32_t*)S.d_ref, (uint32_t*)S.d_pend,
                           S.pool, (wv::PhArr*)S.d_ph, stats_on ? (uint32_t*)S.d_stats : nullptr, (const uint64_t*)info,
                           (const uint32_t*)d_order, (const uint32_t*)nullptr);
        INF_CHK(hipGetLastError());
    }
    INF_CHK(hipEventRecord(S.ev[5], s));
    {
        uint32_t* d_first = (uint32_t*)S.d_cticket + 16 + 2 * OB_WORDS;
        INF_CHK(hipMemsetAsync(d_first, 0xFF, 4, s));
        hipLaunchKernelGGL(ndfl_inflate_first_error_kernel, dim3((ncand + SCAN_TILE - 1) / SCAN_TILE), dim3(SCAN_T), 0, s,
                           (const ChainRes*)S.d_res, (const uint64_t*)info, d_first);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_summary_kernel, dim3(1), dim3(64), 0, s, (const ChainRes*)S.d_res,
                           (const EmitChain*)S.d_chains, info, dict_len, partial ? 1u : 0u, (const uint32_t*)d_first);
        INF_CHK(hipGetLastError());
    }
    // the resolve rounds, as far as they usually go, without a host read in between
    uint32_t* left = nullptr;
    if (!deferred) {
        rc = resolve_rounds_dev(S, s, d_out, nbytes, 6, &left, stats_on ? info + LI_WORDS - 3 : (uint64_t*)nullptr);
        if (rc) return rc;
        if (left) INF_CHK(hipMemcpyAsync(info + LI_WORDS - 1, left, 4, hipMemcpyDeviceToDevice, s));
    }
    INF_CHK(hipMemcpyAsync((void*)hinfo, info, LI_WORDS * 8, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));                          // (2) the summary
    if (stats_on) {
        uint32_t st[64] = {0};
        INF_CHK(hipMemcpy(st, S.d_stats, 256, hipMemcpyDeviceToHost));
        const uint64_t* t64 = (const uint64_t*)(st + 32);
        fprintf(stderr, "[ndfl] device link: chains %llu of %u candidates; count pass: slow-verify lanes %u fixups %u "
                "rounds %u\n", (unsigned long long)hinfo[LI_NCH], ncand, st[0], st[1], st[2]);
        const unsigned long long* ss = (const unsigned long long*)(st + 16);
        fprintf(stderr, "[ndfl] strict stage: %llu waves, %llu loop trips (%llu refills), %llu lane-symbol steps\n",
                ss[3], ss[0], ss[1], ss[2]);
        fprintf(stderr, "[ndfl] emit: %u pending 32-byte groups before the resolve rounds, %u after six\n",
                (uint32_t)(hinfo[LI_WORDS - 3] & 0xFFFFFFFFu), (uint32_t)(hinfo[LI_WORDS - 1] & 0xFFFFFFFFu));
        fprintf(stderr, "[ndfl] count wave-time (ms x waves, 100 MHz clock; -DNDFL_PHASE_CLOCK builds): header %.1f spec %.1f "
                "verify %.1f phases %.1f serial %.1f record %.1f build %.1f phase-mapped %.1f\n", t64[0] * 1e-5,
                t64[1] * 1e-5, t64[2] * 1e-5, t64[3] * 1e-5, t64[4] * 1e-5, t64[5] * 1e-5, t64[6] * 1e-5, t64[7] * 1e-5);
        const double span = (double)(t64[9] - ~t64[10]);
        fprintf(stderr, "[ndfl] count waves %llu: busy %.1f ms x waves, span %.3f ms, occupancy %.3f, longest chain %.3f ms\n",
                (unsigned long long)t64[11], t64[8] * 1e-5, span * 1e-5, t64[11] ? t64[8] / (span * t64[11]) : 0.0,
                t64[12] * 1e-5);
    }
    const uint64_t lflags = hinfo[LI_FLAGS];
    if (lflags & LF_REPAIR) return LINK_FALLBACK;
    if (lflags & LF_RANGE) return -1;                          // the range end is no block boundary
    S.chains = hinfo[LI_NCH];
    S.candidates = ncand;
    S.flat_chains = hinfo[LI_NFLAT];
    S.repairs = 0;
    if (lflags & LF_CAPACITY) { *out_len = hinfo[LI_TOTAL]; return -3; }
    const uint32_t pending_left = (uint32_t)(hinfo[LI_WORDS - 1] & 0xFFFFFFFFu);
    if (!deferred && pending_left) {
        uint64_t groups = 0;
        rc = resolve_rounds(S, s, d_out, nbytes, &groups);     // (the rest, with the host's checks)
        if (rc) return rc;
    }
    {
        float a = 0, b = 0, c = 0;
        hipEventElapsedTime(&a, S.ev[0], S.ev[1]);
        hipEventElapsedTime(&b, S.ev[2], S.ev[3]);
        hipEventElapsedTime(&c, S.ev[4], S.ev[5]);
        S.last_ms_find = a; S.last_ms_count = b; S.last_ms_emit = c;
    }
    if (deferred) { S.pending = true; S.p_out = d_out; S.p_nbytes = dict_len + hinfo[LI_TOTAL]; S.p_dict_len = dict_len; }
    INF_CHK(hipEventRecord(S.ev[5], s));
    INF_CHK(hipStreamSynchronize(s));
    float w = 0;
    hipEventElapsedTime(&w, S.ev[0], S.ev[5]);
    S.last_ms_wall = w;
    *last_ms = w;
    const int code = (int)hinfo[LI_CODE];
    const uint64_t produced = hinfo[LI_OUTLEN];
    if (!direct && produced) INF_CHK(hipMemcpy(out + dict_len, d_out + dict_len, produced, hipMemcpyDeviceToHost));
    *out_len = produced;
    *consumed_bits = hinfo[LI_CONSUMED];
    return code;
}

// The decoder's input words: staged into a zero-padded scratch copy, so the decode lanes' 16-byte
// prefetches (up to IN_PAD bytes past the end) need no bounds checks -- unless the caller says its
// device buffer already is one (NDFL_IN_PADDED: 16-byte aligned, IN_PAD zero bytes after the data),
// in which case it is read in place.
static int stage_input(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint32_t flags,
                       const uint32_t** d_w) {
    using namespace inf;
    const uint64_t nwords = (in_len + 3) / 4;
    const bool in_place = in_len && (flags & 1u) && (flags & 8u) && ((uintptr_t)in & 15u) == 0;
    *d_w = (const uint32_t*)in;
    if (!in_place) {
        INF_CHK(inf_ensure(&S.d_in, &S.d_in_cap, nwords * 4 + IN_PAD));
        if (in_len) INF_CHK(hipMemcpyAsync(S.d_in, in, in_len, (flags & 1u) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
        INF_CHK(hipMemsetAsync((char*)S.d_in + in_len, 0, nwords * 4 + IN_PAD - in_len, s));
        *d_w = (const uint32_t*)S.d_in;
    }
    return 0;
}

// The header finder phase: every bit position of [start_bit, min(end_bit, nbits)) tested for a
// block header (finder: cheap masks + the code-length code's Kraft test), the survivors checked by
// the reference's own header rules (strict stage), the accepted ones into the per-segment lists
// d_list / d_cnt (SEG_BYTES of input each).  S.d_stats and d_cnt must be zeroed.
static int find_headers(InflateScratch& S, hipStream_t s, const uint32_t* d_w, uint64_t nwords, uint64_t nbits,
                        uint64_t start_bit, uint64_t end_bit, uint32_t* d_cnt, uint64_t* d_list) {
    using namespace inf;
    // only the range's own bits are scanned: candidates outside [start_bit, end_bit) are dropped
    // later anyway (a range decode of one stream shard, or a sync probe)
    const uint64_t scan_end = std::min(end_bit, nbits);
    const uint64_t w_lo = start_bit >> 5;
    const uint64_t nw32 = scan_end > w_lo * 32 ? (scan_end + 31) / 32 - w_lo : 0;
    // The survivor list: nbits / 256 + 64 K entries (about one survivor per 1,000 positions on real
    // streams).  A scan whose survivors overflowed it is run again with room for all of them
    // (FIND_OVERFLOW, q_min), up to Q_BUDGET entries (1 GiB of list): periodic stored data can pass
    // the filters every ~32 bits, and a 4 GiB stream of it would ask for 8 GiB.  Past the budget, or
    // when the allocation fails, the decode goes on with the list it has (q_full): a survivor past
    // the list is a chain start not taken -- the chain before it decodes through that block -- so it
    // costs parallelism, never a result.
    constexpr uint64_t Q_BUDGET = (1ull << 30) / 8;
    const uint64_t qbase = std::min<uint64_t>(0x7FFFFFFFull, nbits / 256 + 65536);
    const uint64_t qtop = std::min<uint64_t>(0x7FFFFFFFull, std::max(qbase, Q_BUDGET));
    uint32_t qcap = (uint32_t)std::max(qbase, std::min<uint64_t>(S.q_min, qtop));
    S.q_full = qcap >= qtop;
    if (inf_ensure(&S.d_q, &S.d_q_cap, (uint64_t)qcap * 8 + 64) != hipSuccess) {
        (void)hipGetLastError();                     // (an out-of-memory result is not a sticky error)
        qcap = (uint32_t)qbase;
        S.q_full = true;
        S.q_min = 0;
        INF_CHK(inf_ensure(&S.d_q, &S.d_q_cap, (uint64_t)qcap * 8 + 64));
    }
    S.q_cap = qcap;
    uint32_t* d_qcount = (uint32_t*)S.d_stats + 8;
    uint64_t* d_qlist = (uint64_t*)((char*)S.d_q + 64);
    static const uint32_t strict_grid = [] {
        int dev = 0, ncu = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ndfl_inflate_strict_kernel, 256, 0) != hipSuccess ||
            ncu <= 0 || per <= 0)
            return 1280u;
        return (uint32_t)(ncu * per);
    }();
    unsigned long long* sst = S.knobs.stats ? (unsigned long long*)((uint32_t*)S.d_stats + 16) : nullptr;
    if (nw32) {
        const uint32_t fgrid = (uint32_t)((nw32 + 256 * FIND_WPT - 1) / (256 * FIND_WPT));
        hipLaunchKernelGGL(ndfl_inflate_find_compact_kernel, dim3(fgrid), dim3(256), 0, s, d_w, nwords, nbits, d_qlist,
                           d_qcount, qcap, w_lo, scan_end);
        INF_CHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_inflate_strict_kernel, dim3(strict_grid), dim3(256), 0, s, d_w, nwords, nbits,
                           (const uint64_t*)d_qlist, (const uint32_t*)d_qcount, qcap, d_cnt, d_list,
                           (uint32_t*)S.d_stats + 10, sst);
        INF_CHK(hipGetLastError());
    }
    return 0;
}

// Diagnostics (ndfl_inflate_headers): the finder phase alone over a whole stream.  out = the accepted
// headers in ascending order (the per-segment lists, each capped at SEG_CAP, as the decode sees
// them); surv = the finder's survivors (unsorted, bit 63 = dynamic); stats[0] survivors found,
// [1] headers accepted before the cap, [2] segments over SEG_CAP, [3] survivors past the list's
// capacity (dropped).
static int inflate_headers(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint32_t flags,
                           uint64_t* out, uint64_t cap, uint64_t* n_out, uint64_t* surv, uint64_t surv_cap,
                           uint64_t* stats) {
    using namespace inf;
    const uint64_t nbits = in_len * 8, nwords = (in_len + 3) / 4;
    const uint32_t* d_w = nullptr;
    INF_RC(stage_input(S, s, in, in_len, flags, &d_w));
    if (!S.d_stats) INF_CHK(hipMalloc(&S.d_stats, 512));
    const uint32_t nseg = (uint32_t)std::max<uint64_t>(1, (in_len + SEG_BYTES - 1) / SEG_BYTES);
    INF_CHK(inf_ensure(&S.d_cand, &S.d_cand_cap, (uint64_t)nseg * SEG_CAP * 8ull + (uint64_t)nseg * 4 + 64));
    uint64_t* d_list = (uint64_t*)S.d_cand;
    uint32_t* d_cnt = (uint32_t*)((char*)S.d_cand + (uint64_t)nseg * SEG_CAP * 8ull);
    std::vector<uint32_t> cnt(nseg);
    std::vector<uint64_t> lists((uint64_t)nseg * SEG_CAP);
    uint32_t qc = 0;
    for (int finds = 0; finds < 2; finds++) {                   // (as inflate_run: FIND_OVERFLOW scans again)
        INF_CHK(hipMemsetAsync(S.d_stats, 0, 512, s));
        INF_CHK(hipMemsetAsync(d_cnt, 0, (uint64_t)nseg * 4, s));
        INF_RC(find_headers(S, s, d_w, nwords, nbits, 0, NONE, d_cnt, d_list));
        INF_CHK(hipMemcpyAsync(&qc, (uint32_t*)S.d_stats + 8, 4, hipMemcpyDeviceToHost, s));
        INF_CHK(hipStreamSynchronize(s));
        if (qc <= S.q_cap || S.q_full) break;
        S.q_min = qc + 65536;
    }
    INF_CHK(hipMemcpyAsync(cnt.data(), d_cnt, nseg * 4ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipMemcpyAsync(lists.data(), d_list, lists.size() * 8, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    const uint32_t qcap = S.q_cap;
    std::vector<uint64_t> acc;
    uint64_t total = 0, over = 0;
    for (uint32_t k = 0; k < nseg; k++) {
        total += cnt[k];
        over += cnt[k] > SEG_CAP;
        for (uint32_t i = 0; i < std::min(cnt[k], SEG_CAP); i++) acc.push_back(lists[(uint64_t)k * SEG_CAP + i]);
    }
    std::sort(acc.begin(), acc.end());
    *n_out = acc.size();
    if (out) memcpy(out, acc.data(), std::min<uint64_t>(cap, acc.size()) * 8);
    if (surv && surv_cap) {
        const uint64_t ns = std::min<uint64_t>(std::min<uint64_t>(qc, qcap), surv_cap);
        if (ns) INF_CHK(hipMemcpy(surv, (const char*)S.d_q + 64, ns * 8, hipMemcpyDeviceToHost));
    }
    if (stats) { stats[0] = qc; stats[1] = total; stats[2] = over; stats[3] = qc > qcap ? qc - qcap : 0; }
    return 0;
}

// Decode one raw DEFLATE stream, or the block-aligned range [start_bit, end_bit) of one.
//   out       the window start: out[0, dict_len) holds the dict_len bytes of output preceding the
//             range (0 for a whole stream); decoded bytes go to out[dict_len, dict_len + n)
//   deferred  the window content is not valid yet: chains that read it (directly or through other
//             chains) are recorded and re-emitted by inflate_resolve once it is written
static int inflate_run(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint64_t start_bit,
                       uint64_t end_bit, uint8_t* out, uint64_t dict_len, uint64_t out_cap, uint64_t* out_len,
                       uint64_t* consumed_bits, uint32_t flags, bool deferred, double* last_ms, bool partial = false,
                       uint64_t* probe_sync = nullptr) {
    using namespace inf;
    *out_len = 0;
    *consumed_bits = 0;
    S.pending = false;
    const bool htime = S.knobs.host_times;
    auto hnow = []() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double ht[8] = {hnow(), 0, 0, 0, 0, 0, 0, 0};
    const uint64_t nbits = in_len * 8;
    const uint64_t nwords = (in_len + 3) / 4;
    if (start_bit > nbits) return -1;
    const uint32_t* d_w = nullptr;
    INF_RC(stage_input(S, s, in, in_len, flags, &d_w));
    if (!S.d_stats) INF_CHK(hipMalloc(&S.d_stats, 512));
    if (!S.ev[0]) for (auto& e : S.ev) INF_CHK(hipEventCreate(&e));
    int finds = 0;
refind:
    INF_CHK(hipMemsetAsync(S.d_stats, 0, 512, s));
    const uint32_t nseg = (uint32_t)std::max<uint64_t>(1, (in_len + SEG_BYTES - 1) / SEG_BYTES);
    INF_CHK(inf_ensure(&S.d_cand, &S.d_cand_cap, (uint64_t)nseg * SEG_CAP * 8ull + (uint64_t)nseg * 4 + 64));
    uint64_t* d_list = (uint64_t*)S.d_cand;
    uint32_t* d_cnt = (uint32_t*)((char*)S.d_cand + (uint64_t)nseg * SEG_CAP * 8ull);
    INF_CHK(hipMemsetAsync(d_cnt, 0, (uint64_t)nseg * 4, s));
    INF_CHK(hipEventRecord(S.ev[0], s));
    INF_RC(find_headers(S, s, d_w, nwords, nbits, start_bit, end_bit, d_cnt, d_list));
    INF_CHK(hipEventRecord(S.ev[1], s));
    // the device-side path (NDFL_HOST_LINK selects the host's linking); sync probes keep the host's
    {
        const bool host_link = S.knobs.host_link;
        if (!probe_sync && !host_link) {
            const int rc = inflate_devlink(S, s, d_w, nwords, nbits, nseg, d_cnt, d_list, start_bit, end_bit, out,
                                           dict_len, out_cap, out_len, consumed_bits, flags, deferred, partial, last_ms);
            if (rc == FIND_OVERFLOW && finds++ == 0) goto refind;
            if (rc != LINK_FALLBACK && rc != FIND_OVERFLOW) return rc;
        }
    }
    std::vector<uint32_t> hcnt(nseg);
    uint32_t hqc = 0;
    INF_CHK(hipMemcpyAsync(hcnt.data(), d_cnt, nseg * 4ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipMemcpyAsync(&hqc, (const uint32_t*)S.d_stats + 8, 4, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    if (hqc > S.q_cap && !S.q_full && finds++ == 0) { S.q_min = hqc + 65536; goto refind; }
    std::vector<uint64_t> hoff(nseg + 1);
    hoff[0] = 1;                                   // slot 0 is the range start
    for (uint32_t k = 0; k < nseg; k++) hoff[k + 1] = hoff[k] + std::min(hcnt[k], SEG_CAP);
    const uint64_t ncand_all = hoff[nseg];
    INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, (ncand_all + nseg + 2) * 8));
    uint64_t* d_sorted = (uint64_t*)S.d_starts;
    uint64_t* d_segoff = d_sorted + ncand_all;
    INF_CHK(hipMemcpyAsync(d_segoff, hoff.data(), nseg * 8ull, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(ndfl_inflate_compact_kernel, dim3((nseg + 3) / 4), dim3(256), 0, s, (const uint32_t*)d_cnt,
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
    // the sorted candidate list on the device: the wave passes split block data at the next one
    const uint32_t ncand = (uint32_t)sorted_cand.size();
    INF_CHK(inf_ensure(&S.d_cands, &S.d_cands_cap, (ncand + 1) * 8ull));
    INF_CHK(hipMemcpyAsync(S.d_cands, sorted_cand.data(), ncand * 8ull, hipMemcpyHostToDevice, s));
    const uint64_t limit = std::min(end_bit, nbits);
    // segment records: a pool for the rounds of all chains, one head per counted chain start (index
    // in `starts`), with room for repairs
    const uint64_t nslot = starts.size() + std::max<uint64_t>(4096, starts.size() / 2);
    const uint64_t nrec = std::min<uint64_t>(0xFFFFFFF0ull, 2 * starts.size() + nbits / (wv::MAX_SPAN / 2) + 65536);
    // table records: at most one per block; bounded (a stream of tiny blocks parses the rest again)
    const uint64_t nbt = std::min<uint64_t>(nrec, S.knobs.no_bt ? 0 : (1u << 18));
    const uint64_t seg_bytes = nrec * (64 * 8 + 64 * 4 + sizeof(SegMeta)) + nslot * 4 + 64 + nbt * BT_BYTES;
    INF_CHK(inf_ensure(&S.d_seg, &S.d_seg_cap, seg_bytes));
    SegPool pool;
    pool.start = (uint64_t*)S.d_seg;
    pool.cnt = (uint32_t*)(pool.start + nrec * 64);
    pool.meta = (SegMeta*)(pool.cnt + nrec * 64);
    pool.head = (uint32_t*)(pool.meta + nrec);
    pool.ctr = (uint32_t*)S.d_stats + 12;
    pool.bctr = (uint32_t*)S.d_stats + 13;
    pool.nbt = (uint32_t)nbt;
    pool.bt = (char*)(((uintptr_t)(pool.head + nslot) + 63) & ~(uintptr_t)63);
    pool.nrec = (uint32_t)nrec;
    pool.nslot = nslot;
    S.pool = pool;
    INF_CHK(hipMemsetAsync(pool.head, 0xFF, nslot * 4, s));

    const bool stats_on = S.knobs.stats;
    std::vector<ChainRes> res;
    auto run_count = [&](const std::vector<uint64_t>& st, std::vector<ChainRes>& r) -> int {
        const uint64_t slot_base = starts.size() - (&st == &starts ? st.size() : 0);
        const size_t n = st.size();
        std::vector<uint64_t> sp(n);
        for (size_t k = 0; k < n; k++) sp[k] = end_bit;     // chains stop at exact candidates (kernel)
        // claim order: longest first (by the bits to the next start), so that no long chain is
        // left for the end of the launch; bucketed by 32 Kibit
        std::vector<uint32_t> order(n);
        {
            constexpr int NB = 24;
            uint32_t bc[NB + 1] = {0};
            auto bucket = [&](size_t k) {
                const uint64_t nx = k + 1 < n ? st[k + 1] : end_bit;
                const uint64_t len = nx > st[k] ? nx - st[k] : 0;
                return NB - 1 - (int)std::min<uint64_t>(NB - 1, len >> 15);
            };
            const bool sorted_st = std::is_sorted(st.begin(), st.end());
            if (sorted_st) {
                for (size_t k = 0; k < n; k++) bc[bucket(k) + 1]++;
                for (int b = 0; b < NB; b++) bc[b + 1] += bc[b];
                for (size_t k = 0; k < n; k++) order[bc[bucket(k)]++] = (uint32_t)k;
            } else {
                for (size_t k = 0; k < n; k++) order[k] = (uint32_t)k;
            }
        }
        INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, n * 8));
        INF_CHK(inf_ensure(&S.d_stops, &S.d_stops_cap, n * 12));
        INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, n * sizeof(ChainRes)));
        INF_CHK(hipMemcpyAsync(S.d_starts, st.data(), n * 8, hipMemcpyHostToDevice, s));
        INF_CHK(hipMemcpyAsync(S.d_stops, sp.data(), n * 8, hipMemcpyHostToDevice, s));
        uint32_t* d_order = (uint32_t*)((char*)S.d_stops + n * 8);
        INF_CHK(hipMemcpyAsync(d_order, order.data(), n * 4, hipMemcpyHostToDevice, s));
        if (!S.d_ph) INF_CHK(hipMalloc(&S.d_ph, (size_t)std::max(COUNT_WAVES, EMIT_WAVES) * sizeof(wv::PhArr)));
        if (!S.d_cticket) INF_CHK(hipMalloc(&S.d_cticket, CTK_BYTES));
        INF_CHK(hipMemsetAsync(S.d_cticket, 0, 4, s));
        if (S.count_first) INF_CHK(hipEventRecord(S.ev[2], s));
        launch_count(s, count_w(S.knobs), (uint32_t)n,
                           d_w, nwords, nbits,
                           (const uint64_t*)S.d_starts, (const uint64_t*)S.d_stops, (uint32_t)n,
                           (const uint64_t*)S.d_cands, ncand, limit, (ChainRes*)S.d_res, stats_on ? (uint32_t*)S.d_stats : nullptr,
                           slot_base, pool, (uint32_t*)S.d_cticket, (wv::PhArr*)S.d_ph, (const uint32_t*)d_order,
                           end_bit, (const wv::HdrRec*)nullptr, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                           (const uint32_t*)nullptr);
        INF_CHK(hipGetLastError());
        if (S.count_first) { INF_CHK(hipEventRecord(S.ev[3], s)); S.count_first = false; }
        r.resize(n);
        INF_CHK(hipMemcpyAsync(r.data(), S.d_res, n * sizeof(ChainRes), hipMemcpyDeviceToHost, s));
        INF_CHK(hipStreamSynchronize(s));
        return 0;
    };
    ht[1] = hnow();
    S.repairs = 0;
    S.count_first = true;
    int rc = run_count(starts, res);
    if (rc) return rc;
    if (probe_sync) {
        // sync probe: a chain of blocks from a header candidate that ends exactly at another
        // candidate y has decoded up to y in step with the stream (a decode that starts off a block
        // boundary re-synchronises inside the block and then ends at its real end-of-block), so y
        // is a block boundary; y is taken when its own chain links on in turn (or is final)
        *probe_sync = NONE;
        auto linked = [&](size_t k) {
            return res[k].status == ST_BOUNDARY && res[k].next < starts.size() && starts[res[k].next] == res[k].end_bit;
        };
        for (size_t k = 1; k < res.size(); k++) {
            if (!linked(k)) continue;
            const size_t j = res[k].next;
            if (j >= 1 && (linked(j) || res[j].status == ST_FINAL)) { *probe_sync = starts[j]; break; }
        }
        return 0;
    }
    if (S.knobs.stats && !probe_sync) {
        // the most expensive chains (wave time, blocks, bits, output bytes)
        std::vector<size_t> idx(res.size());
        for (size_t k = 0; k < idx.size(); k++) idx[k] = k;
        const size_t top = std::min<size_t>(8, idx.size());
        std::partial_sort(idx.begin(), idx.begin() + top, idx.end(),
                          [&](size_t a, size_t b) { return (res[a].pad >> 16) > (res[b].pad >> 16); });
        for (size_t t = 0; t < top; t++) {
            const ChainRes& r = res[idx[t]];
            fprintf(stderr, "[ndfl] count chain %zu: %.2f ms, %u blocks, start %llu, %llu bits, %llu bytes, status %u\n",
                    idx[t], (r.pad >> 16) * 0.01, r.pad & 0xFFFFu, (unsigned long long)starts[idx[t]],
                    (unsigned long long)(r.end_bit - starts[idx[t]]), (unsigned long long)r.out_count, r.status);
        }
    }
    {
        float a = 0, b = 0;
        hipEventElapsedTime(&a, S.ev[0], S.ev[1]);
        hipEventElapsedTime(&b, S.ev[2], S.ev[3]);
        S.last_ms_find = a; S.last_ms_count = b;
    }

    // link from the range start.  A boundary that is no candidate (fixed-Huffman block, header
    // rejected by the finder) is repaired: every such boundary of every chain is decoded on in
    // parallel rounds; a final serial fallback guarantees progress.
    // chain starts: the sorted candidate prefix (binary search) plus repaired boundaries
    const size_t n0 = starts.size();
    std::unordered_map<uint64_t, size_t> extra;
    auto find_at = [&](uint64_t b, size_t& idx) -> bool {
        auto it = std::lower_bound(starts.begin(), starts.begin() + n0, b);
        if (it != starts.begin() + n0 && *it == b) { idx = (size_t)(it - starts.begin()); return true; }
        auto e = extra.find(b);
        if (e != extra.end()) { idx = e->second; return true; }
        return false;
    };
    for (int round = 0; round < 8; round++) {
        std::vector<uint64_t> todo;
        size_t dummy;
        for (size_t k = 0; k < res.size(); k++)
            if (res[k].status == ST_BOUNDARY && res[k].end_bit < end_bit &&
                !(res[k].next < n0 && starts[res[k].next] == res[k].end_bit) && !find_at(res[k].end_bit, dummy)) {
                extra[res[k].end_bit] = NONE;       // placeholder, filled below
                todo.push_back(res[k].end_bit);
            }
        if (todo.empty()) break;
        std::vector<ChainRes> r2;
        rc = run_count(todo, r2);
        if (rc) return rc;
        for (size_t k = 0; k < todo.size(); k++) {
            starts.push_back(todo[k]);
            res.push_back(r2[k]);
            extra[todo[k]] = starts.size() - 1;
        }
        S.repairs += todo.size();
    }
    ht[2] = hnow();
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
        ec.slot = cur;
        chains.push_back(ec);
        offs.push_back(off);
        off += r.out_count;
        if (r.status == ST_FINAL) { stop_bit = r.end_bit; break; }
        if (r.status == ST_ERROR) break;
        if (r.end_bit == end_bit) { stop_bit = end_bit; break; }
        if (r.end_bit > end_bit) return -1;          // the range end is no block boundary
        size_t nxt;
        if (r.next < n0 && starts[r.next] == r.end_bit) { cur = r.next; continue; }
        if (find_at(r.end_bit, nxt) && nxt != (size_t)NONE) { cur = nxt; continue; }
        // serial fallback (beyond the parallel rounds)
        std::vector<uint64_t> st1{r.end_bit};
        std::vector<ChainRes> r1;
        rc = run_count(st1, r1);
        if (rc) return rc;
        starts.push_back(r.end_bit);
        res.push_back(r1[0]);
        extra[r.end_bit] = starts.size() - 1;
        cur = starts.size() - 1;
        S.repairs++;
    }
    S.chains = chains.size();
    S.flat_chains = 0;
    S.candidates = sorted_cand.size();
    if (S.knobs.stats) {
        uint32_t st[64] = {0};
        INF_CHK(hipMemcpy(st, S.d_stats, 256, hipMemcpyDeviceToHost));
        st[4] = st[8];
        fprintf(stderr, "[ndfl] finder quick survivors %u; count pass: chains %zu candidates %zu repairs %llu "
                "slow-verify lanes %u fixups %u rounds %u\n", st[4], chains.size(), sorted_cand.size(),
                (unsigned long long)S.repairs, st[0], st[1], st[2]);
        const uint64_t* t64 = (const uint64_t*)(st + 32);
        const unsigned long long* ss = (const unsigned long long*)(st + 16);
        fprintf(stderr, "[ndfl] strict stage: %llu waves, %llu loop trips (%llu refills), %llu lane-symbol steps\n",
                ss[3], ss[0], ss[1], ss[2]);
        fprintf(stderr, "[ndfl] count wave-time (ms x waves, 100 MHz clock): header %.1f spec %.1f verify %.1f phases %.1f "
                "serial %.1f record %.1f build %.1f phase-mapped %.1f\n", t64[0] * 1e-5, t64[1] * 1e-5, t64[2] * 1e-5, t64[3] * 1e-5,
                t64[4] * 1e-5, t64[5] * 1e-5, t64[6] * 1e-5, t64[7] * 1e-5);
        const double span = (double)(t64[9] - ~t64[10]);
        fprintf(stderr, "[ndfl] count waves %llu: busy %.1f ms x waves, span %.3f ms, occupancy %.3f, longest chain %.3f ms\n",
                (unsigned long long)t64[11], t64[8] * 1e-5, span * 1e-5, t64[11] ? t64[8] / (span * t64[11]) : 0.0,
                t64[12] * 1e-5);
    }
    const uint64_t total = off - dict_len;
    ht[3] = hnow();
    if (total > out_cap) { *out_len = total; return -3; }

    // emit pass
    const uint32_t nch = (uint32_t)chains.size();
    INF_CHK(inf_ensure(&S.d_chains, &S.d_chains_cap, nch * sizeof(EmitChain)));
    INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, nch * sizeof(ChainRes)));
    if (!S.d_ticket) INF_CHK(hipMalloc(&S.d_ticket, 64));
    INF_CHK(hipMemcpyAsync(S.d_chains, chains.data(), nch * sizeof(EmitChain), hipMemcpyHostToDevice, s));
    INF_CHK(hipMemsetAsync(S.d_ticket, 0, 64, s));
    uint8_t* d_out;
    const bool direct = (flags & 2u) != 0;
    if (direct) d_out = out;
    else {
        INF_CHK(inf_ensure(&S.d_out, &S.d_out_cap, dict_len + total + 64));
        d_out = (uint8_t*)S.d_out;
        if (dict_len) INF_CHK(hipMemcpyAsync(d_out, out, dict_len, hipMemcpyHostToDevice, s));
    }
    const uint64_t nbytes = dict_len + total;
    if ((nbytes + 31) / 32 > 0xFFFFFFFFull) return -2;       // u32 group indices in the resolve lists
    const uint64_t npw = (nbytes + 31) / 32;
    INF_CHK(inf_ensure(&S.d_ref, &S.d_ref_cap, nbytes * 4 + 64));
    INF_CHK(inf_ensure(&S.d_pend, &S.d_pend_cap, npw * 4 + 64));
    INF_CHK(hipMemsetAsync(S.d_pend, 0, npw * 4 + 64, s));
    if (!S.h_cnt) INF_CHK(hipHostMalloc(&S.h_cnt, 64, 0));
    hipEvent_t e2 = S.ev[4], e3 = S.ev[5];
    INF_CHK(hipEventRecord(e2, s));
    if (!S.d_ph) INF_CHK(hipMalloc(&S.d_ph, (size_t)std::max(COUNT_WAVES, EMIT_WAVES) * sizeof(wv::PhArr)));
    static const uint32_t emit_grid = wave_grid(ndfl_inflate_emit_wave_kernel, EMIT_WAVES, "NDFL_EMIT_WPC");
    hipLaunchKernelGGL(ndfl_inflate_emit_wave_kernel, dim3(std::min<uint32_t>(nch, emit_grid)), dim3(64), 0, s, d_w,
                       nwords, nbits, (const EmitChain*)S.d_chains, nch, (uint32_t*)S.d_ticket, d_out,
                       (ChainRes*)S.d_res, (const uint64_t*)S.d_cands, ncand, (uint32_t*)S.d_ref, (uint32_t*)S.d_pend,
                       pool, (wv::PhArr*)S.d_ph, stats_on ? (uint32_t*)S.d_stats : nullptr, (const uint64_t*)nullptr,
                       (const uint32_t*)nullptr, (const uint32_t*)nullptr);
    INF_CHK(hipGetLastError());
    INF_CHK(hipEventRecord(e3, s));
    std::vector<ChainRes> er(nch);
    INF_CHK(hipMemcpyAsync(er.data(), S.d_res, nch * sizeof(ChainRes), hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    ht[4] = hnow();
    float ms = 0;
    hipEventElapsedTime(&ms, e2, e3);
    S.last_ms_emit = ms;
    if (stats_on) {
        uint64_t t64[48];
        INF_CHK(hipMemcpy(t64, (const char*)S.d_stats + 128, sizeof(t64), hipMemcpyDeviceToHost));
        const double span = (double)(t64[17] - ~t64[18]);
        fprintf(stderr, "[ndfl] emit waves %llu: busy %.1f ms x waves, span %.3f ms, occupancy %.3f, longest chain %.3f ms\n",
                (unsigned long long)t64[19], t64[16] * 1e-5, span * 1e-5, t64[19] ? t64[16] / (span * t64[19]) : 0.0,
                t64[20] * 1e-5);
    }
    if (deferred) {
        S.pending = true;
        S.p_out = d_out; S.p_nbytes = nbytes; S.p_dict_len = dict_len;
    } else {
        uint64_t groups = 0;
        const int rr = resolve_rounds(S, s, d_out, nbytes, &groups);
        if (rr) return rr;
        S.resolved_groups = groups;
    }
    INF_CHK(hipEventRecord(e3, s));
    INF_CHK(hipStreamSynchronize(s));
    float ms2 = 0;
    hipEventElapsedTime(&ms2, S.ev[0], e3);
    S.last_ms_wall = ms2;
    hipEventElapsedTime(&ms2, e2, e3);
    *last_ms = ms2;
    ht[5] = hnow();
    if (htime) fprintf(stderr, "[ndfl] inflate host ms: finder+starts %.2f count+repairs %.2f link %.2f emit %.2f resolve %.2f\n",
                       ht[1] - ht[0], ht[2] - ht[1], ht[3] - ht[2], ht[4] - ht[3], ht[5] - ht[4]);
    // first error in stream order (the emit pass also checks the dictionary bound exactly)
    for (uint32_t k = 0; k < nch; k++) {
        if (er[k].status == ST_ERROR) {
            if (partial && er[k].reason == R_UEOS) {
                // the input is a prefix of the stream: stop at the last block boundary reached
                const uint64_t produced = chains[k].out_off - dict_len + er[k].bnd_cnt;
                if (!direct && produced) INF_CHK(hipMemcpy(out + dict_len, d_out + dict_len, produced, hipMemcpyDeviceToHost));
                *out_len = produced;
                *consumed_bits = er[k].bnd_bit;
                return NEED_INPUT;
            }
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

// First confirmed block boundary at or past from_bit, looking at most window_bits ahead (NONE if
// none): the finder and count passes of inflate_run on that window, without the emit.
static int inflate_sync(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint64_t from_bit,
                        uint64_t window_bits, uint32_t flags, uint64_t* sync_bit, double* last_ms) {
    uint64_t olen = 0, bits = 0;
    const uint64_t end = std::min(in_len * 8, from_bit + window_bits);
    if (from_bit >= end) { *sync_bit = inf::NONE; return 0; }
    return inflate_run(S, s, in, in_len, from_bit, end, nullptr, 0, 0, &olen, &bits, flags, false, last_ms, false,
                       sync_bit);
}

// The last n bytes of a deferred-window range decode's output once the caller has written the
// window, without resolving the rest: each byte follows its back-references (pending bytes only;
// window bytes are never pending) to a final byte.  A chain longer than TAIL_STEPS sets *fail.
constexpr uint32_t TAIL_STEPS = 4096;
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_tail_kernel(const uint32_t* pend, const uint32_t* ref, const uint8_t* out, uint64_t t0, uint64_t n,
                         uint8_t* dst, uint32_t* fail) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    uint64_t p = t0 + k;
    uint32_t steps = 0;
    while ((pend[p >> 5] >> (p & 31)) & 1) {
        p -= ref[p];
        if (++steps > TAIL_STEPS) { atomicOr(fail, 1u); return; }
    }
    dst[k] = out[p];
}

// The same bytes as a map of the window: entry k = the window byte index its value comes from
// (< dict_len), or TAIL_LITERAL | value for a byte that does not depend on the window.  Needs no
// window content: GPU r's map composed with the maps of GPUs 0..r-1 gives its window directly.
constexpr uint32_t TAIL_LITERAL = 0x80000000u;
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_tail_map_kernel(const uint32_t* pend, const uint32_t* ref, const uint8_t* out, uint64_t t0, uint64_t n,
                             uint64_t dict_len, uint32_t* dst, uint32_t* fail) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    uint64_t p = t0 + k;
    uint32_t steps = 0;
    while ((pend[p >> 5] >> (p & 31)) & 1) {
        p -= ref[p];
        if (++steps > TAIL_STEPS) { atomicOr(fail, 1u); return; }
    }
    dst[k] = p < dict_len ? (uint32_t)p : TAIL_LITERAL | out[p];
}

static int inflate_tail_map(InflateScratch& S, hipStream_t s, uint64_t n, uint32_t* dst) {
    if (!S.pending) return -5;
    if (n > S.p_nbytes) return -1;
    if (n == 0) return 0;
    if (!S.h_cnt) INF_CHK(hipHostMalloc(&S.h_cnt, 64, 0));
    uint32_t* d_fail = (uint32_t*)S.d_stats + 14;
    INF_CHK(hipMemsetAsync(d_fail, 0, 4, s));
    hipLaunchKernelGGL(ndfl_inflate_tail_map_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       (const uint32_t*)S.d_pend, (const uint32_t*)S.d_ref, (const uint8_t*)S.p_out, S.p_nbytes - n, n,
                       S.p_dict_len, dst, d_fail);
    INF_CHK(hipGetLastError());
    uint32_t* h = (uint32_t*)S.h_cnt;
    INF_CHK(hipMemcpyAsync(h + 8, d_fail, 4, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    return h[8] ? -6 : 0;
}

static int inflate_tail(InflateScratch& S, hipStream_t s, uint64_t n, uint8_t* dst) {
    if (!S.pending) return -5;
    if (n > S.p_nbytes) return -1;
    if (n == 0) return 0;
    if (!S.h_cnt) INF_CHK(hipHostMalloc(&S.h_cnt, 64, 0));
    uint32_t* d_fail = (uint32_t*)S.d_stats + 14;
    INF_CHK(hipMemsetAsync(d_fail, 0, 4, s));
    hipLaunchKernelGGL(ndfl_inflate_tail_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       (const uint32_t*)S.d_pend, (const uint32_t*)S.d_ref, (const uint8_t*)S.p_out, S.p_nbytes - n, n,
                       dst, d_fail);
    INF_CHK(hipGetLastError());
    uint32_t* h = (uint32_t*)S.h_cnt;
    INF_CHK(hipMemcpyAsync(h + 8, d_fail, 4, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    return h[8] ? -6 : 0;
}

// Second half of a deferred-window range decode: the caller has written the window
// (out[0, dict_len)); resolve every deferred copy (those that read the window directly or through
// other copies included).  *n_resolved = pending 32-byte groups at the start.
static int inflate_resolve(InflateScratch& S, hipStream_t s, uint64_t* n_resolved) {
    using namespace inf;
    *n_resolved = 0;
    if (!S.pending) return -5;
    S.pending = false;
    const int rr = resolve_rounds(S, s, S.p_out, S.p_nbytes, n_resolved);
    if (rr) return rr;
    S.resolved_groups = *n_resolved;
    return 0;
}
