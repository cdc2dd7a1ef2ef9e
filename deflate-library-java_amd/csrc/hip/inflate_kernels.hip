// inflate_kernels.hip -- MI355X (gfx950) parallel DEFLATE decoder.
//
// Replaces InflaterInputStream.read -> Open.read -> {UncompressedBlock,HuffmanBlock}.read run to
// the end of one raw DEFLATE stream (D/InflaterInputStream.java:147-164, D/decomp/Open.java:83-620).
//
// A single DEFLATE stream has no block index, so the decoder speculates:
//   1. finder   (one wave per 64 KiB of compressed input): the first bit position in the segment
//               that starts a block header which passes the reference's own validity checks
//               (dynamic: complete code-length code, decodable code lengths, EOB present, complete
//               litlen/distance codes; stored: LEN == ~NLEN with zero padding) is a candidate;
//   2. count    (one lane per candidate): decode blocks from the candidate until the first block
//               boundary at or past the next candidate, recording end bit, output size, status;
//   3. link     (host): follow end bit == candidate start from bit 0; a boundary that is not a
//               candidate (fixed-Huffman block, shadowed header) is repaired by decoding on from it;
//   4. emit     (one lane per linked chain): decode again into the final output at the chain's
//               offset.  A copy whose source precedes the chain waits (agent-scope acquire) on the
//               owning chain's completion flag; chains are claimed in order through a ticket, so a
//               lane only ever waits on chains whose lanes already run.  The loop is a per-token
//               step machine so a waiting lane never blocks the other lanes of its wave.
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
constexpr int PRIM = 10;                   // primary table bits
constexpr uint64_t NONE = ~0ull;

enum : uint32_t { ST_BOUNDARY = 0, ST_FINAL = 1, ST_ERROR = 2 };
enum : int { R_UEOS = 1, R_RESERVED_BLOCK_TYPE, R_LEN_MISMATCH, R_UNDER_FULL, R_OVER_FULL, R_NO_PREV,
             R_CL_OVER_FULL, R_EOB_ZERO, R_RESERVED_LEN, R_RESERVED_DIST, R_EMPTY_DIST, R_COPY_BEFORE,
             R_INTERNAL = 100 };

__constant__ uint16_t RUN_BASE[29] = {3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
__constant__ uint8_t RUN_EXTRA[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
__constant__ uint16_t DIST_BASE[30] = {1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577};
__constant__ uint8_t DIST_EXTRA[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
__constant__ uint8_t CL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Decode table for one Huffman code: primary 2^PRIM entries (sym | len << 9; len 0 = longer
// code), plus canonical first-code/count/offset per length and the symbols in canonical order.
struct Tab {
    uint16_t prim[1 << PRIM];
    uint16_t sorted[288];
    uint16_t first[16];
    uint16_t count[16];
    uint16_t offs[16];
};
struct LaneTabs { Tab lit, dist; };

struct In {
    const uint32_t* w;
    uint64_t nwords;
    uint64_t nbits;
    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return i < nwords ? w[i] : 0u; }
};

struct Rd {
    uint64_t pos;     // absolute position of the next unread bit
    uint64_t bb;      // buffered bits (LSB = next)
    uint32_t bn;      // valid bits in bb
    uint64_t nextw;   // next word to load
    __device__ __forceinline__ void init(const In& in, uint64_t p) {
        pos = p;
        nextw = p >> 5;
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

__device__ __forceinline__ uint32_t rev_bits(uint32_t v, uint32_t n) { return __brev(v) >> (32 - n); }

// codeLengthsToCodeTree's error detection (D/decomp/Open.java:705-756) from per-length counts.
__device__ int tree_check(const uint16_t* cnt /*[16]*/) {
    uint32_t num = 0, maxL = 0;
    for (int l = 1; l < 16; l++) { num += cnt[l]; if (cnt[l]) maxL = (uint32_t)l; }
    if (num < 2) return R_UNDER_FULL;
    const uint64_t R = 2ull * (num - 1);
    uint64_t next = 0, end = 2;
    for (uint32_t l = 1; l <= maxL; l++) {
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

// Build canonical decoding structure for lens[0..n).  Returns tree_check's verdict.
template <bool PRIMARY>
__device__ int build_tab(const uint8_t* lens, int n, Tab* t) {
    uint16_t cnt[16];
    for (int l = 0; l < 16; l++) cnt[l] = 0;
    for (int s = 0; s < n; s++) cnt[lens[s]]++;
    cnt[0] = 0;
    int e = tree_check(cnt);
    if (e) return e;
    uint16_t offs[16], first[16];
    uint32_t code = 0, off = 0;
    for (int l = 1; l < 16; l++) {
        code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1;
        first[l] = (uint16_t)code;
        offs[l] = (uint16_t)off;
        off += cnt[l];
        t->first[l] = (uint16_t)code;
        t->count[l] = cnt[l];
        t->offs[l] = (uint16_t)offs[l];
    }
    if (PRIMARY) {
        uint64_t* p64 = (uint64_t*)t->prim;
        for (int i = 0; i < (1 << PRIM) / 4; i++) p64[i] = 0;
    }
    uint16_t nxt[16];
    for (int l = 0; l < 16; l++) nxt[l] = 0;
    for (int s = 0; s < n; s++) {
        uint32_t l = lens[s];
        if (!l) continue;
        uint32_t rank = nxt[l]++;
        t->sorted[offs[l] + rank] = (uint16_t)s;
        if (PRIMARY && l <= (uint32_t)PRIM) {
            uint32_t r = rev_bits(first[l] + rank, l);
            uint16_t ent = (uint16_t)(s | (l << 9));
            for (uint32_t k = r; k < (1u << PRIM); k += (1u << l)) t->prim[k] = ent;
        }
    }
    return 0;
}

// Canonical decode starting at length `from` (slow path).  Codes are complete, so it terminates.
__device__ __forceinline__ uint32_t slow_decode(const Tab* t, uint32_t bits15, uint32_t from, uint32_t& len) {
    uint32_t r15 = rev_bits(bits15, 15);
    for (uint32_t l = from; l < 16; l++) {
        uint32_t c = r15 >> (15 - l);
        uint32_t idx = c - t->first[l];
        if (idx < t->count[l]) { len = l; return t->sorted[t->offs[l] + idx]; }
    }
    len = 15;
    return 0xFFFF;   // unreachable for complete codes
}

__device__ __forceinline__ uint32_t decode_sym(const Tab* t, Rd& rd, const In& in) {
    rd.fill(in);
    uint32_t e = t->prim[rd.peek(PRIM)];
    uint32_t len = e >> 9;
    uint32_t sym;
    if (len) sym = e & 0x1FF;
    else sym = slow_decode(t, rd.peek(15), PRIM + 1, len);
    rd.skip(len);
    return sym;
}

// Dynamic block header (D/decomp/Open.java:336-431).  On success fills the lane's tables and
// sets empty_dist.  Returns 0 or a Reason.
__device__ int read_dynamic_header(Rd& rd, const In& in, LaneTabs* tabs, bool& empty_dist) {
    uint32_t hlit = rd.get(in, 5), hdist = rd.get(in, 5), hclen = rd.get(in, 4);
    if (rd.pos > in.nbits) return R_UEOS;
    const int numLit = (int)hlit + 257, numDist = (int)hdist + 1, numCl = (int)hclen + 4;
    uint8_t cl[19];
    for (int i = 0; i < 19; i++) cl[i] = 0;
    for (int i = 0; i < numCl; i++) {
        cl[CL_ORDER[i]] = (uint8_t)rd.get(in, 3);
        if (rd.pos > in.nbits) return R_UEOS;
    }
    // code-length code: canonical arrays only (max 7 bits), kept in the dist slot temporarily
    Tab* ct = &tabs->dist;
    int e = build_tab<false>(cl, 19, ct);
    if (e) return e;
    uint8_t lens[320];
    const int total = numLit + numDist;
    int runVal = -1;
    for (int i = 0; i < total;) {
        rd.fill(in);
        uint32_t len;
        uint32_t sym = slow_decode(ct, rd.peek(15), 1, len);
        rd.skip(len);
        if (rd.pos > in.nbits) return R_UEOS;
        if (sym < 16) { runVal = (int)sym; lens[i++] = (uint8_t)sym; continue; }
        int runLen;
        if (sym == 16) {
            if (runVal == -1) return R_NO_PREV;
            runLen = (int)rd.get(in, 2) + 3;
        } else if (sym == 17) { runVal = 0; runLen = (int)rd.get(in, 3) + 3; }
        else { runVal = 0; runLen = (int)rd.get(in, 7) + 11; }
        if (rd.pos > in.nbits) return R_UEOS;
        for (; runLen > 0; runLen--, i++) {
            if (i >= total) return R_CL_OVER_FULL;
            lens[i] = (uint8_t)runVal;
        }
    }
    if (lens[256] == 0) return R_EOB_ZERO;
    e = build_tab<true>(lens, numLit, &tabs->lit);
    if (e) return e;
    uint8_t* dl = lens + numLit;
    int nd = numDist;
    if (nd == 1 && dl[0] == 0) { empty_dist = true; return 0; }
    empty_dist = false;
    int one = 0, other = 0;
    for (int i = 0; i < nd; i++) { if (dl[i] == 1) one++; else if (dl[i] > 1) other++; }
    uint8_t d32[32];
    for (int i = 0; i < 32; i++) d32[i] = i < nd ? dl[i] : 0;
    if (one == 1 && other == 0) { nd = 32; d32[31] = 1; }
    return build_tab<true>(d32, nd, &tabs->dist);
}

// ---- header finder -------------------------------------------------------------------------
// Strict check of a dynamic block header at bit p, without storing the code lengths: running
// Kraft sums give exactly the reference's acceptance (complete litlen code with EOB present;
// empty / single-code-padded / complete distance code), D/decomp/Open.java:336-431.
__device__ bool strict_dynamic(const In& in, uint64_t p) {
    Rd rd; rd.init(in, p + 3);
    uint32_t hlit = rd.get(in, 5), hdist = rd.get(in, 5), hclen = rd.get(in, 4);
    const uint32_t numLit = hlit + 257, numDist = hdist + 1, numCl = hclen + 4;
    uint32_t cnt[8], first[8], offs[8];
    uint8_t cl[19];
    for (int i = 0; i < 19; i++) cl[i] = 0;
    for (uint32_t i = 0; i < numCl; i++) cl[CL_ORDER[i]] = (uint8_t)rd.get(in, 3);
    for (int l = 0; l < 8; l++) cnt[l] = 0;
    for (int s2 = 0; s2 < 19; s2++) cnt[cl[s2]]++;
    cnt[0] = 0;
    uint32_t kr = 0;
    for (int l = 1; l < 8; l++) kr += cnt[l] << (7 - l);
    if (kr != 128) return false;
    uint8_t sorted[19];
    {
        uint32_t code = 0, off = 0, nxt[8];
        for (int l = 1; l < 8; l++) { code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1; first[l] = code; offs[l] = off; off += cnt[l]; nxt[l] = 0; }
        for (int s2 = 0; s2 < 19; s2++) if (cl[s2]) sorted[offs[cl[s2]] + nxt[cl[s2]]++] = (uint8_t)s2;
    }
    const uint32_t total = numLit + numDist;
    uint32_t i = 0;
    int runVal = -1;
    uint32_t litK = 0, distK = 0, ones = 0, other = 0, eob = 0, d0 = 0, d31 = 0;
    while (i < total) {
        rd.fill(in);
        uint32_t r7 = rev_bits(rd.peek(7), 7);
        uint32_t sym = 0, len = 0;
        for (uint32_t l = 1; l < 8; l++) {
            uint32_t idx = (r7 >> (7 - l)) - first[l];
            if (idx < cnt[l]) { sym = sorted[offs[l] + idx]; len = l; break; }
        }
        rd.skip(len);
        uint32_t run = 1;
        if (sym < 16) runVal = (int)sym;
        else if (sym == 16) { if (runVal < 0) return false; run = rd.get(in, 2) + 3; }
        else if (sym == 17) { runVal = 0; run = rd.get(in, 3) + 3; }
        else { runVal = 0; run = rd.get(in, 7) + 11; }
        if (i + run > total || rd.pos > in.nbits) return false;
        const uint32_t v = (uint32_t)runVal;
        const uint32_t e = i + run;
        if (i < numLit) {
            uint32_t c = min(e, numLit) - i;
            if (v) { litK += c * (32768u >> v); if (litK > 32768u) return false; }
            if (i <= 256 && 256 < e) eob = v;
        }
        if (e > numLit) {
            uint32_t a = max(i, numLit) - numLit, b2 = e - numLit;
            uint32_t c = b2 - a;
            if (v) { distK += c * (32768u >> v); if (distK > 32768u) return false; if (v == 1) ones += c; else other += c; }
            if (a == 0) d0 = v;
            if (a <= 31 && 31 < b2) d31 = v;
        }
        i = e;
    }
    if (eob == 0 || litK != 32768u) return false;
    if (numDist == 1 && d0 == 0) return true;
    if (ones == 1 && other == 0) return !(numDist == 32 && d31 == 1);
    return distK == 32768u;
}

// Window helper: n (<= 32) bits at bit offset o of a 5-word window.
__device__ __forceinline__ uint32_t wbits(const uint32_t (&w)[5], uint32_t o, uint32_t n) {
    uint32_t k = o >> 5;
    uint64_t x = (uint64_t)w[k] | ((uint64_t)w[k + 1] << 32);
    return (uint32_t)(x >> (o & 31)) & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
}

constexpr uint32_t SEG_CAP = 64;   // candidates kept per finder segment

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

// Quick filter over every bit position: each thread tests 32 consecutive positions from a
// 160-bit register window.  Dynamic: btype 2 and a complete code-length code (Kraft == 1, >= 2
// codes).  Stored: btype 0, zero padding, LEN == ~NLEN, data inside the stream.  Survivors are
// appended to their segment's list.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_find_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, uint32_t* seg_cnt, uint64_t* seg_list) {
    using namespace inf;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p0 = t * 32;
    if (p0 >= nbits) return;
    In in{w, nwords, nbits};
    uint32_t win[5];
#pragma unroll
    for (int k = 0; k < 5; k++) win[k] = in.ld(t + (uint64_t)k);
    const uint32_t seg = (uint32_t)(p0 / ((uint64_t)SEG_BYTES * 8));
    for (uint32_t o = 0; o < 32; o++) {
        const uint64_t p = p0 + o;
        if (p + 3 > nbits) break;
        const uint32_t bt = wbits(win, o + 1, 2);
        bool ok = false;
        if (bt == 2) {
            if (p + 17 > nbits) continue;
            const uint32_t ncl = wbits(win, o + 13, 4) + 4;
            uint32_t kr = 0, nz = 0;
            for (uint32_t i = 0; i < ncl; i++) {
                uint32_t l = wbits(win, o + 17 + 3 * i, 3);
                if (l) { kr += 128u >> l; nz++; }
            }
            ok = kr == 128 && nz >= 2 && p + 17 + 3 * ncl <= nbits;
        } else if (bt == 0) {
            const uint32_t q = o + 3, al = (q + 7) & ~7u;
            if (al > q && wbits(win, q, al - q) != 0) continue;
            const uint32_t ln = wbits(win, al, 16), nln = wbits(win, al + 16, 16);
            ok = ln == (nln ^ 0xFFFFu) && (p0 + al + 32 + 8ull * ln <= nbits);
        }
        if (ok) ok = bt == 2 ? strict_dynamic(in, p) : strict_stored(in, p);
        if (ok) {
            uint32_t idx = atomicAdd(&seg_cnt[seg], 1u);
            if (idx < SEG_CAP) seg_list[(uint64_t)seg * SEG_CAP + idx] = p;
        }
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

// Per-lane decode state machine.  MODE 0 = count, 1 = emit.
struct Lane {
    Rd rd;
    uint64_t n;           // bytes produced by this chain so far
    uint64_t stop_bit;    // count: stop at first boundary >= stop_bit; emit: stop at boundary == stop_bit
    uint32_t state;       // 0 header, 1 stored, 2 huffman, 3 done
    uint32_t stored_left;
    bool last;            // current block is final
    bool fixed;
    bool empty_dist;
    uint32_t status, reason;
    // pending copy (emit)
    uint32_t cp_len, cp_dist;
    uint32_t lastb;       // last output byte (for dist-1 copies without a load)
};

}  // namespace inf


// Common per-token step.  Returns false when the lane finished (status set).
template <int MODE>
__device__ __forceinline__ bool lane_step(inf::Lane& L, const inf::In& in, inf::LaneTabs* mytabs,
                                          const inf::LaneTabs* fixedTabs, uint8_t* out, uint64_t out_off,
                                          const uint64_t* chain_off, const uint32_t* done, uint32_t nchains,
                                          uint32_t my_chain, bool& waiting) {
    using namespace inf;
    waiting = false;
    if (L.state == 0) {
        // block boundary
        if (MODE == 0) {
            if (L.rd.pos >= L.stop_bit && L.n >= 0) { L.status = ST_BOUNDARY; L.state = 3; return false; }
        } else {
            if (L.rd.pos == L.stop_bit) { L.status = ST_BOUNDARY; L.state = 3; return false; }
        }
        uint32_t bf = L.rd.get(in, 1), bt = L.rd.get(in, 2);
        if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        L.last = bf != 0;
        if (bt == 3) { L.status = ST_ERROR; L.reason = R_RESERVED_BLOCK_TYPE; L.state = 3; return false; }
        if (bt == 0) {
            uint32_t pad = (uint32_t)((8 - (L.rd.pos & 7)) & 7);
            L.rd.get(in, pad);
            uint32_t ln = L.rd.get(in, 16);
            uint32_t nln = L.rd.get(in, 16);
            if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
            if (ln != (nln ^ 0xFFFFu)) { L.status = ST_ERROR; L.reason = R_LEN_MISMATCH; L.state = 3; return false; }
            L.stored_left = ln;
            L.state = 1;
            return true;
        }
        if (bt == 1) { L.fixed = true; L.empty_dist = false; L.state = 2; return true; }
        bool ed = false;
        int e = read_dynamic_header(L.rd, in, mytabs, ed);
        if (e) { L.status = ST_ERROR; L.reason = (uint32_t)e; L.state = 3; return false; }
        L.fixed = false; L.empty_dist = ed; L.state = 2;
        return true;
    }
    if (L.state == 1) {
        // stored bytes: the stream is byte aligned here
        uint64_t avail = (in.nbits - min(L.rd.pos, in.nbits)) / 8;
        const uint32_t lim = MODE == 1 ? 32u : 0xFFFFu;
        uint32_t take = (uint32_t)min((uint64_t)min(L.stored_left, lim), avail);
        if (MODE == 1) {
            for (uint32_t k = 0; k < take; k++) {
                uint32_t b = L.rd.get(in, 8);
                out[out_off + L.n + k] = (uint8_t)b;
                L.lastb = b;
            }
        } else {
            // skip whole bytes quickly
            uint64_t np = L.rd.pos + 8ull * take;
            L.rd.init(in, np);
        }
        L.n += take;
        L.stored_left -= take;
        if (take < min(L.stored_left + take, lim)) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        if (L.stored_left == 0) {
            if (L.last) { L.status = ST_FINAL; L.state = 3; return false; }
            L.state = 0;
        }
        return true;
    }
    // state 2: one Huffman token
    if (MODE == 1 && L.cp_len) {
        // a copy that was waiting for its source
        goto do_copy;
    }
    {
        const Tab* lt = L.fixed ? &fixedTabs->lit : &mytabs->lit;
        uint32_t sym = decode_sym(lt, L.rd, in);
        if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        if (sym < 256) {
            if (MODE == 1) out[out_off + L.n] = (uint8_t)sym;
            L.lastb = sym;
            L.n++;
            return true;
        }
        if (sym == 256) {
            if (L.last) { L.status = ST_FINAL; L.state = 3; return false; }
            L.state = 0;
            return true;
        }
        if (sym > 285) { L.status = ST_ERROR; L.reason = R_RESERVED_LEN; L.state = 3; return false; }
        uint32_t run = RUN_BASE[sym - 257] + L.rd.get(in, RUN_EXTRA[sym - 257]);
        if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        if (L.empty_dist) { L.status = ST_ERROR; L.reason = R_EMPTY_DIST; L.state = 3; return false; }
        const Tab* dt = L.fixed ? &fixedTabs->dist : &mytabs->dist;
        uint32_t dsym = decode_sym(dt, L.rd, in);
        if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        if (dsym > 29) { L.status = ST_ERROR; L.reason = R_RESERVED_DIST; L.state = 3; return false; }
        uint32_t dist = DIST_BASE[dsym] + L.rd.get(in, DIST_EXTRA[dsym]);
        if (L.rd.pos > in.nbits) { L.status = ST_ERROR; L.reason = R_UEOS; L.state = 3; return false; }
        if (MODE == 0) {
            // dictionary check needs the absolute position: only decidable here for chain offset 0
            if (out_off == 0 && (uint64_t)dist > L.n) { L.status = ST_ERROR; L.reason = R_COPY_BEFORE; L.state = 3; return false; }
            L.n += run;
            return true;
        }
        if ((uint64_t)dist > out_off + L.n) { L.status = ST_ERROR; L.reason = R_COPY_BEFORE; L.state = 3; return false; }
        L.cp_len = run;
        L.cp_dist = dist;
    }
do_copy:
    if (MODE == 1) {
        const uint64_t dst = out_off + L.n;
        const uint64_t src = dst - L.cp_dist;
        if (src < out_off && !(L.cp_dist == 1 && L.n > 0)) {
            // source precedes this chain: wait for the chains that own bytes [src, min(dst, src+len))
            uint32_t lo = 0, hi = my_chain;
            while (lo + 1 < hi) { uint32_t mid = (lo + hi) >> 1; if (chain_off[mid] <= src) lo = mid; else hi = mid; }
            const uint64_t src_end = min(dst, src + L.cp_len);
            uint32_t need_hi = lo;
            while (need_hi + 1 < my_chain && chain_off[need_hi + 1] < src_end) need_hi++;
            for (uint32_t j = lo; j <= need_hi; j++) {
                if (__hip_atomic_load(&done[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) { waiting = true; return true; }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        // bounded work per step (<= 32 bytes) keeps the lanes of a wave in step
        const uint32_t take = min(L.cp_len, 32u);
        if (L.cp_dist == 1) {
            const uint32_t v = (L.n > 0) ? L.lastb : (uint32_t)out[src];
            for (uint32_t k = 0; k < take; k++) out[dst + k] = (uint8_t)v;
            L.lastb = v;
        } else {
            uint32_t b = L.lastb;
            for (uint32_t k = 0; k < take; k++) {
                b = out[src + k];
                out[dst + k] = (uint8_t)b;
            }
            L.lastb = b;
        }
        L.n += take;
        L.cp_len -= take;
    }
    return true;
}

// One lane per candidate: count output bytes until the first boundary >= stop.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_count_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* starts,
                          const uint64_t* stops, uint32_t nchains, ChainRes* res, inf::LaneTabs* tabs,
                          const inf::LaneTabs* fixedTabs) {
    using namespace inf;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nchains) return;
    In in{w, nwords, nbits};
    Lane L;
    L.rd.init(in, starts[i]);
    L.n = 0; L.stop_bit = stops[i]; L.state = 0; L.stored_left = 0; L.last = false; L.fixed = false;
    L.empty_dist = false; L.status = 0; L.reason = 0; L.cp_len = 0; L.cp_dist = 0; L.lastb = 0;
    // starts[i] < stops[i], so the first block is always decoded
    bool waiting;
    while (lane_step<0>(L, in, &tabs[i], fixedTabs, nullptr, starts[i] == 0 ? 0 : 1, nullptr, nullptr, 0, 0, waiting)) {}
    ChainRes r;
    r.end_bit = L.rd.pos;
    r.out_count = L.n;
    r.status = L.status;
    r.reason = L.reason;
    res[i] = r;
}

// One lane per linked chain, in stream order.  Lanes claim chains through `ticket` in groups of
// 64 (one wave), so every chain a lane may wait on already belongs to a running wave.
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_emit_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const EmitChain* chains,
                         const uint64_t* chain_off, uint32_t nchains, uint32_t* done, uint32_t* ticket,
                         uint8_t* out, ChainRes* res, inf::LaneTabs* tabs, const inf::LaneTabs* fixedTabs) {
    using namespace inf;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(ticket, 64u);
    base = __shfl(base, 0, 64);
    const uint32_t i = base + (uint32_t)lane;
    const bool valid = i < nchains;
    In in{w, nwords, nbits};
    Lane L;
    EmitChain ch;
    if (valid) ch = chains[i];
    else { ch.start_bit = 0; ch.end_bit = 0; ch.out_off = 0; ch.out_count = 0; }
    L.rd.init(in, ch.start_bit);
    L.n = 0; L.stop_bit = ch.end_bit; L.state = 0; L.stored_left = 0; L.last = false; L.fixed = false;
    L.empty_dist = false; L.status = 0; L.reason = 0; L.cp_len = 0; L.cp_dist = 0; L.lastb = 0;
    bool active = valid;
    int idle = 0;
    uint32_t waits = 0;
    while (__any(active)) {
        bool waiting = false;
        if (active) {
            bool more = lane_step<1>(L, in, &tabs[i], fixedTabs, out, ch.out_off, chain_off, done, nchains, i, waiting);
            if (waiting && ++waits > (1u << 26)) {          // safety net: never hang the device
                more = false; L.status = ST_ERROR; L.reason = R_INTERNAL;
            }
            if (!more) {
                active = false;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&done[i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ChainRes r;
                r.end_bit = L.rd.pos; r.out_count = L.n; r.status = L.status; r.reason = L.reason;
                res[i] = r;
            }
        }
        // back off only when every active lane is waiting
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
    void* d_ticket = nullptr;
    void* d_out = nullptr; size_t d_out_cap = 0;
    double last_ms_find = 0, last_ms_count = 0, last_ms_emit = 0, last_ms_wall = 0;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    uint64_t repairs = 0, chains = 0, candidates = 0;
    bool count_first = false;
    void release() {
        void** ps[] = {&d_in, &d_cand, &d_starts, &d_stops, &d_res, &d_tabs, &d_fixed, &d_chains, &d_off,
                       &d_done, &d_ticket, &d_out};
        for (void** p : ps) { if (*p) hipFree(*p); *p = nullptr; }
        for (auto& e : ev) { if (e) hipEventDestroy(e); e = nullptr; }
        d_in_cap = d_cand_cap = d_starts_cap = d_stops_cap = d_res_cap = d_tabs_cap = d_chains_cap = 0;
        d_off_cap = d_done_cap = d_out_cap = 0;
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
static void host_build_fixed(inf::LaneTabs* t) {
    memset(t, 0, sizeof(*t));
    auto build = [](const uint8_t* lens, int n, inf::Tab* tab) {
        uint16_t cnt[16] = {0};
        for (int s = 0; s < n; s++) cnt[lens[s]]++;
        cnt[0] = 0;
        uint16_t first[16] = {0}, offs[16] = {0};
        uint32_t code = 0, off = 0;
        for (int l = 1; l < 16; l++) {
            code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1;
            first[l] = (uint16_t)code; offs[l] = (uint16_t)off; off += cnt[l];
            tab->first[l] = first[l]; tab->count[l] = cnt[l]; tab->offs[l] = offs[l];
        }
        uint16_t nxt[16] = {0};
        for (int s = 0; s < n; s++) {
            uint32_t l = lens[s];
            if (!l) continue;
            uint32_t rank = nxt[l]++;
            tab->sorted[offs[l] + rank] = (uint16_t)s;
            uint32_t c = first[l] + rank, r = 0;
            for (uint32_t b = 0; b < l; b++) r |= ((c >> b) & 1u) << (l - 1 - b);
            for (uint32_t k = r; k < (1u << inf::PRIM); k += (1u << l)) tab->prim[k] = (uint16_t)(s | (l << 9));
        }
    };
    uint8_t ll[288], dl[32];
    for (int i = 0; i < 288; i++) ll[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
    for (int i = 0; i < 32; i++) dl[i] = 5;
    build(ll, 288, &t->lit);
    build(dl, 32, &t->dist);
}

#define INF_CHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return -4; } while (0)

static int inflate_run(InflateScratch& S, hipStream_t s, const uint8_t* in, uint64_t in_len, uint8_t* out,
                       uint64_t out_cap, uint64_t* out_len, uint64_t* consumed_bits, uint32_t flags,
                       hipEvent_t ev0, hipEvent_t ev1, double* last_ms) {
    using namespace inf;
    *out_len = 0;
    *consumed_bits = 0;
    const uint64_t nbits = in_len * 8;
    const uint64_t nwords = (in_len + 3) / 4;
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
        INF_CHK(hipMalloc(&S.d_fixed, sizeof(LaneTabs)));
        LaneTabs* h = (LaneTabs*)malloc(sizeof(LaneTabs));
        host_build_fixed(h);
        INF_CHK(hipMemcpy(S.d_fixed, h, sizeof(LaneTabs), hipMemcpyHostToDevice));
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
        if (nthr)
            hipLaunchKernelGGL(ndfl_inflate_find_kernel, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, s, d_w,
                               nwords, nbits, d_cnt, d_list);
        INF_CHK(hipGetLastError());
    }
    INF_CHK(hipEventRecord(S.ev[1], s));
    std::vector<uint32_t> hcnt(nseg);
    std::vector<uint64_t> hlist((uint64_t)nseg * SEG_CAP);
    INF_CHK(hipMemcpyAsync(hcnt.data(), d_cnt, nseg * 4ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipMemcpyAsync(hlist.data(), d_list, (uint64_t)nseg * SEG_CAP * 8ull, hipMemcpyDeviceToHost, s));
    INF_CHK(hipStreamSynchronize(s));
    std::vector<uint64_t> starts;
    starts.reserve((size_t)nseg * 4);
    starts.push_back(0);
    for (uint32_t k = 0; k < nseg; k++) {
        const uint32_t c = std::min(hcnt[k], SEG_CAP);
        const size_t b0 = starts.size();
        for (uint32_t j = 0; j < c; j++) {
            const uint64_t v = hlist[(uint64_t)k * SEG_CAP + j];
            if (v != NONE && v != 0) starts.push_back(v);
        }
        std::sort(starts.begin() + b0, starts.end());
    }
    const std::vector<uint64_t> sorted_cand(starts);

    auto next_after = [&](uint64_t b) -> uint64_t {
        auto ub = std::upper_bound(sorted_cand.begin(), sorted_cand.end(), b);
        return ub != sorted_cand.end() ? *ub : NONE;
    };
    std::vector<ChainRes> res;
    auto run_count = [&](const std::vector<uint64_t>& st, std::vector<ChainRes>& r) -> int {
        const size_t n = st.size();
        std::vector<uint64_t> sp(n);
        for (size_t k = 0; k < n; k++) sp[k] = next_after(st[k]);
        INF_CHK(inf_ensure(&S.d_starts, &S.d_starts_cap, n * 8));
        INF_CHK(inf_ensure(&S.d_stops, &S.d_stops_cap, n * 8));
        INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, n * sizeof(ChainRes)));
        INF_CHK(inf_ensure(&S.d_tabs, &S.d_tabs_cap, n * sizeof(LaneTabs)));
        INF_CHK(hipMemcpyAsync(S.d_starts, st.data(), n * 8, hipMemcpyHostToDevice, s));
        INF_CHK(hipMemcpyAsync(S.d_stops, sp.data(), n * 8, hipMemcpyHostToDevice, s));
        if (S.count_first) INF_CHK(hipEventRecord(S.ev[2], s));
        hipLaunchKernelGGL(ndfl_inflate_count_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d_w, nwords,
                           nbits, (const uint64_t*)S.d_starts, (const uint64_t*)S.d_stops, (uint32_t)n,
                           (ChainRes*)S.d_res, (LaneTabs*)S.d_tabs, (const LaneTabs*)S.d_fixed);
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

    // link from bit 0.  A boundary that is no candidate (fixed-Huffman block, header rejected by
    // the finder) is repaired: every such boundary of every chain is decoded on in parallel
    // rounds; a final serial fallback guarantees progress.
    std::unordered_map<uint64_t, size_t> at;
    at.reserve(starts.size() * 2);
    for (size_t k = 0; k < starts.size(); k++) at[starts[k]] = k;
    for (int round = 0; round < 8; round++) {
        std::vector<uint64_t> todo;
        for (size_t k = 0; k < res.size(); k++)
            if (res[k].status == ST_BOUNDARY && !at.count(res[k].end_bit)) {
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
    uint64_t off = 0;
    size_t cur = 0;
    uint64_t end_bit = 0;
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
        if (r.status == ST_FINAL) { end_bit = r.end_bit; break; }
        if (r.status == ST_ERROR) break;
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
    const uint64_t total = off;
    if (total > out_cap) { *out_len = total; return -3; }

    // emit pass
    const uint32_t nch = (uint32_t)chains.size();
    INF_CHK(inf_ensure(&S.d_chains, &S.d_chains_cap, nch * sizeof(EmitChain)));
    INF_CHK(inf_ensure(&S.d_off, &S.d_off_cap, (nch + 1) * 8ull));
    INF_CHK(inf_ensure(&S.d_done, &S.d_done_cap, nch * 4ull));
    INF_CHK(inf_ensure(&S.d_res, &S.d_res_cap, nch * sizeof(ChainRes)));
    INF_CHK(inf_ensure(&S.d_tabs, &S.d_tabs_cap, nch * sizeof(LaneTabs)));
    if (!S.d_ticket) INF_CHK(hipMalloc(&S.d_ticket, 64));
    INF_CHK(hipMemcpyAsync(S.d_chains, chains.data(), nch * sizeof(EmitChain), hipMemcpyHostToDevice, s));
    offs.push_back(total);
    INF_CHK(hipMemcpyAsync(S.d_off, offs.data(), (nch + 1) * 8ull, hipMemcpyHostToDevice, s));
    INF_CHK(hipMemsetAsync(S.d_done, 0, nch * 4ull, s));
    INF_CHK(hipMemsetAsync(S.d_ticket, 0, 64, s));
    uint8_t* d_out;
    bool direct = (flags & 2u) != 0;
    if (direct) d_out = out;
    else { INF_CHK(inf_ensure(&S.d_out, &S.d_out_cap, total + 64)); d_out = (uint8_t*)S.d_out; }
    hipEvent_t e2 = S.ev[4], e3 = S.ev[5];
    INF_CHK(hipEventRecord(e2, s));
    const uint32_t waves = (nch + 63) / 64;
    hipLaunchKernelGGL(ndfl_inflate_emit_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, d_w, nwords, nbits,
                       (const EmitChain*)S.d_chains, (const uint64_t*)S.d_off, nch, (uint32_t*)S.d_done,
                       (uint32_t*)S.d_ticket, d_out, (ChainRes*)S.d_res, (LaneTabs*)S.d_tabs,
                       (const LaneTabs*)S.d_fixed);
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
    (void)ev0; (void)ev1;
    // first error in stream order (the emit pass also checks the dictionary bound exactly)
    uint64_t produced = 0;
    for (uint32_t k = 0; k < nch; k++) {
        if (er[k].status == ST_ERROR) {
            produced = chains[k].out_off + er[k].out_count;
            if (!direct && produced) INF_CHK(hipMemcpy(out, d_out, produced, hipMemcpyDeviceToHost));
            *out_len = produced;
            *consumed_bits = er[k].end_bit;
            return (int)er[k].reason;
        }
    }
    if (!direct && total) INF_CHK(hipMemcpy(out, d_out, total, hipMemcpyDeviceToHost));
    *out_len = total;
    *consumed_bits = end_bit;
    return 0;
}
