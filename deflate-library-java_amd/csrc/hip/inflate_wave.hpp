// inflate_wave.hpp -- wave-per-chain decode passes (count + emit) of the MI355X DEFLATE decoder.
//
// One wave64 per chain of blocks (a chain starts at a header candidate).  Per block:
//   * lane 0 parses the header (D/decomp/Open.java:232-431, the reference's check order) into
//     code lengths in LDS; the wave builds ONE set of decode tables in LDS for the block
//     (canonical codes by ballot ranks, D/decomp/Open.java:705-789): a 10-bit literal/length and an
//     8-bit distance primary whose entries carry the run/distance base and extra-bit count, with a
//     canonical slow path for longer codes;
//   * the block's data bits are split into 64 segments, one per lane.  Lane j decodes from its
//     segment start s_j (usually inside a codeword: speculative), recording its first token
//     starts, up to the first token boundary >= s_{j+1}.  Then every lane re-decodes from the TRUE
//     start (the previous lane's exit) until it reaches one of its own recorded token starts --
//     from there its speculative decode is exact (Huffman decoding self-synchronises, usually
//     within a few tokens) -- or decodes its whole segment if it never meets one.  A fix-up loop
//     re-runs lanes whose predecessor's exit moved.  The first lane that sees the end-of-block
//     symbol or an error ends the block; when no lane does (the segment end was a false header
//     candidate), the next round continues from lane 63's exit.
//   * count pass: output bytes, end bit, status per chain (the host links chains);
//     emit pass: a third decode per segment writes the output at its offset.  No lane or chain
//     waits on another: copies whose source is not yet known there are deferred (back-references
//     + pending bits) and resolved afterwards by pointer-jumping rounds.
// Many waves per CU (small LDS footprint) hide the per-token latency chain.
#pragma once

namespace wv {
using namespace inf;

constexpr uint32_t LB = 10;                 // literal/length primary bits
constexpr uint32_t DB = 8;                  // distance primary bits
// table entry: [4:0] code length (0: longer than the primary), [8:5] extra bits, [10:9] kind,
// [31:16] literal byte / run base / distance base
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3 };
enum : uint32_t { T_EXIT = 0, T_EOB = 1, T_ERR = 2 };

// Codes longer than the primary: a second-level table per primary prefix when they fit in the
// extension area (the primary entry then points at it: length 0, [8:5] index bits, [31:16] offset),
// otherwise the canonical slow path, whose arrays take the extension area instead (primary entry 0).
constexpr uint32_t LX = 320;                // literal/length extension words
constexpr uint32_t DX = 64;                 // distance extension words
struct Tabs {
    uint32_t lit[1u << LB];
    uint32_t dst[1u << DB];
    // sub-tables, or (fallback) the entry of every symbol in canonical order [0, n), the
    // left-justified 15-bit upper limit of each length [n, n + 16), first code and rank offset per
    // length (u16) [n + 16, n + 32)
    uint32_t lx[LX];
    uint32_t dx[DX];
};

// The same tables split over two memories (the fast emit pass): the primary tables in LDS, the
// extension areas -- read only for codes longer than the primary -- in the count pass's table
// record in global memory.
struct TabsG {
    const uint32_t* lit;
    const uint32_t* dst;
    const uint32_t* lx;
    const uint32_t* dx;
};

struct Shared {
    Tabs t;
    uint8_t lens[320];                       // literal/length 0..287, distance at 288..319
    uint16_t cl_tab[128];                    // code-length code, full 7-bit table: sym | len << 9
    uint32_t exit_[64];                      // round-relative lane exits
    uint8_t kind_[64];
    // header broadcast (lane 0 -> wave)
    uint64_t h_pos, h_d0;
    uint32_t h_err, h_bfinal, h_btype, h_len, h_numlit, h_numdist;
};

// phase-fallback results (phases 1..7) of one wave: per lane, written and read by that lane only,
// so they may live in LDS (emit) or in a per-wave global slot (count)
struct PhArr {
    uint32_t cp[7][64];                      // checkpoint offset | bytes before it << 16
    uint32_t end[7][64];                     // end offset
    uint32_t cnt[7][64];                     // bytes
    uint8_t kr[7][64];                       // kind << 5 | reason
};

__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t len) {
    if (sym < 256) return len | (K_LIT << 9) | (sym << 16);
    if (sym == 256) return len | (K_EOB << 9);
    if (sym <= 285) {
        uint32_t base, ne;
        run_base(sym - 257, base, ne);
        return len | (ne << 5) | (K_LEN << 9) | (base << 16);
    }
    return len | (K_BAD << 9) | ((sym & 1u) << 16);     // 286 / 287 (bit 16: which, for the Reason)
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t sym, uint32_t len) {
    if (sym <= 29) {
        uint32_t base, ne;
        dist_base(sym, base, ne);
        return len | (ne << 5) | (base << 16);
    }
    return len | (K_BAD << 9) | ((sym & 1u) << 16);     // 30 / 31
}
// the Reason of a reserved symbol's table entry (K_BAD): its second symbol has an internal code
__device__ __forceinline__ uint32_t rsv_len(uint32_t e) { return (e >> 16) & 1u ? (uint32_t)R_RESERVED_LEN_HI : (uint32_t)R_RESERVED_LEN; }
__device__ __forceinline__ uint32_t rsv_dist(uint32_t d) { return (d >> 16) & 1u ? (uint32_t)R_RESERVED_DIST_HI : (uint32_t)R_RESERVED_DIST; }

// Length of a code longer than the primary: the smallest l with code < lim[l] (limits are
// non-decreasing for a canonical code); branch-free over the five candidate lengths.
template <uint32_t PB>
__device__ __forceinline__ uint32_t slow_entry(uint32_t p15, const uint32_t* lim, const uint16_t* first,
                                               const uint16_t* off, const uint32_t* ent) {
    const uint32_t c = rev_bits(p15, 15);
    uint32_t l = PB + 1;
#pragma unroll
    for (uint32_t k = PB + 1; k < 15; k++) l += c >= lim[k] ? 1u : 0u;
    const uint32_t idx = (c >> (15 - l)) - first[l];
    return ent[off[l] + idx];
}
template <class TT>
__device__ __forceinline__ uint32_t slow_lit(uint32_t p15, const TT& t) {
    return slow_entry<LB>(p15, t.lx + 288, (const uint16_t*)(t.lx + 304), (const uint16_t*)(t.lx + 312), t.lx);
}
template <class TT>
__device__ __forceinline__ uint32_t slow_dist(uint32_t p15, const TT& t) {
    return slow_entry<DB>(p15, t.dx + 32, (const uint16_t*)(t.dx + 48), (const uint16_t*)(t.dx + 56), t.dx);
}
// entry of a code longer than the primary (e: its primary entry; bits: the window from the code's start)
template <class TT>
__device__ __forceinline__ uint32_t long_lit(uint32_t e, uint32_t bits, const TT& t) {
    const uint32_t sd = (e >> 5) & 15;
    if (sd) return t.lx[(e >> 16) + ((bits >> LB) & ((1u << sd) - 1u))];
    return slow_lit(bits & 0x7FFFu, t);
}
template <class TT>
__device__ __forceinline__ uint32_t long_dist(uint32_t d, uint32_t bits, const TT& t) {
    const uint32_t sd = (d >> 5) & 15;
    if (sd) return t.dx[(d >> 16) + ((bits >> DB) & ((1u << sd) - 1u))];
    return slow_dist(bits & 0x7FFFu, t);
}

struct Tok {
    uint32_t kind;      // K_LIT (n bytes in val), K_LEN (n = run, dist), K_EOB, K_BAD (val = reason)
    uint32_t val, dist, n;
};

// ---- staged round input -------------------------------------------------------------------------
// A round is decoded by the wave's 64 lanes over consecutive segments of pw words each.  Its input
// is staged in LDS transposed: word i of lane j's region (the segment plus the words a token that
// starts inside it can still read) at w[i * 64 + j], so every lane's window read is bank-conflict
// free whatever its position.  The loads are LDS-DMA (global_load_lds_dword, one 256-byte row of
// the image per instruction), so the decode loop carries no prefetch state at all: a token is read
// from its absolute position with one ds_read2st64 + one ds_read and two funnel shifts.
#ifndef NDFL_LPW
#define NDFL_LPW 14
#endif
constexpr uint32_t LPW = NDFL_LPW;             // words per lane segment at most (448 bits by default)
constexpr uint32_t SW = LPW + 4;               // staged words per lane region (+ the tail window)
constexpr uint64_t RSPAN = 64ull * LPW * 32;   // round span cap (bits)
// Words per lane segment at least: a short round (a small block, a block's last round) is split
// over fewer lanes rather than into segments too short for a speculative decode to meet its true
// token boundaries before the segment ends (every such lane otherwise costs a fix-up decode).
#ifndef NDFL_PW_MIN
#define NDFL_PW_MIN 4
#endif
static_assert(NDFL_PW_MIN >= 1 && NDFL_PW_MIN <= NDFL_LPW, "NDFL_PW_MIN");

struct Stage {
    uint32_t w[SW * 64];
};

struct Geo {            // wave-uniform geometry of one round
    uint64_t base;      // absolute bit of the round's word 0 (word-aligned)
    uint32_t r0, re;    // round start / end relative to base
    uint32_t pw;        // words per lane segment
    uint32_t nb;        // input bits relative to base (saturated)
};
__device__ __forceinline__ Geo make_geo(const In& in, uint64_t rs, uint64_t E, uint32_t pw = 0) {
    Geo g;
    g.base = rs & ~31ull;
    g.r0 = (uint32_t)(rs - g.base);
    g.re = (uint32_t)(E - g.base);
    const uint32_t span = g.re - g.r0;
    g.pw = pw ? pw : max((uint32_t)NDFL_PW_MIN, ((span + 63) / 64 + 31) / 32);
    g.nb = (uint32_t)min(in.nbits - min(in.nbits, g.base), (uint64_t)0xFFFFFFFFu);
    return g;
}
// lane j's segment [s, e) (relative bits); lane 63 ends at the round end
__device__ __forceinline__ void lane_seg(const Geo& g, int lane, uint32_t& s, uint32_t& e) {
    const uint32_t per = g.pw * 32;
    s = min(g.r0 + (uint32_t)lane * per, g.re);
    e = lane == 63 ? g.re : min(g.r0 + (uint32_t)(lane + 1) * per, g.re);
}

// Stage the round's input (all lanes call).  Words past the input end read the zero padding.
// NDFL_STAGE_CPOL: cache policy of the staging loads (2 = non-temporal: the input is read once and
// should not push the emit pass's partly written output lines out of L2; measured: 2 is ~1 ms
// slower and leaves the emit write traffic unchanged, 20.0 vs 21.5 GB).  Touching the next round's
// input into L2 after each staging (one LDS-DMA dword per 128-byte line, round 5) made count and
// emit slower too (+0.3 / +0.4 ms, profiles/r05_ab_stage_touch.txt).
#ifndef NDFL_STAGE_CPOL
#define NDFL_STAGE_CPOL 0
#endif
__device__ __forceinline__ void stage_round(const In& in, const Geo& g, Stage& st, int lane) {
    const uint64_t w0 = (g.base >> 5) + (uint64_t)lane * g.pw;
    const uint64_t wmax = in.nwords + 60;          // inside the IN_PAD zero bytes after the input
    __syncthreads();                               // the previous round's reads are done
#pragma unroll 4
    for (uint32_t i = 0; i < SW; i++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(in.w + min(w0 + i, wmax)),
                                         (__attribute__((address_space(3))) void*)&st.w[i * 64], 4, 0, NDFL_STAGE_CPOL);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// The lane's view of the staged round: 64 bits of input from relative bit `pos`.  (A cached 128-bit
// window re-read every two words was measured slower: the selects cost more than the LDS read.)
struct Lv {
    const uint32_t* p;     // &st.w[lane]
    uint32_t rw;           // region's first word (relative to base)
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return p[i * 64]; }   // region word i
    __device__ __forceinline__ void win(uint32_t pos, uint32_t& lo, uint32_t& hi) const {
        const uint32_t* q = p + ((pos >> 5) - rw) * 64;
        const uint32_t a = q[0], b = q[64], c = q[128];
        lo = __builtin_amdgcn_alignbit(b, a, pos & 31);
        hi = __builtin_amdgcn_alignbit(c, b, pos & 31);
    }
};
// The lane's view of a round read straight from the input in global memory (the fast emit pass):
// the same region-relative words as Lv, through L1/L2 instead of an LDS stage.  Reads up to the
// region's end plus the tail words, inside the IN_PAD zero bytes after the input (as the stage).
struct Gv {
    const uint32_t* q;     // the lane's region word 0 in the input
    uint32_t rw;           // region's first word (relative to base)
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return q[i]; }
    __device__ __forceinline__ void win(uint32_t pos, uint32_t& lo, uint32_t& hi) const {
        const uint32_t i = (pos >> 5) - rw;
        const uint32_t a = q[i], b = q[i + 1], c = q[i + 2];
        lo = __builtin_amdgcn_alignbit(b, a, pos & 31);
        hi = __builtin_amdgcn_alignbit(c, b, pos & 31);
    }
};
__device__ __forceinline__ Lv make_lv(const Stage& st, const Geo& g, int lane) {
    Lv v;
    v.p = st.w + lane;
    v.rw = (uint32_t)lane * g.pw;
    return v;
}

// One token at `pos` with the reference's check order (D/decomp/Open.java:446-618).  A literal
// pair (two literal codes fitting the primary table together) comes as one step (tk.n = 2), except
// when its first literal already reaches `stop` (a checkpoint or the segment end): every decode then
// stands on the first token boundary at or past each stop, whatever its grouping before it.
// CAREFUL = false: the caller guarantees pos + 48 < stop <= nb (no token can reach the stop or the
// input end), so those checks are dropped.
template <bool CAREFUL, class TT>
__device__ __forceinline__ void tok_e(uint32_t lo, uint32_t hi, uint32_t e, uint32_t& pos, const TT& t,
                                      bool empty_dist, uint32_t stop, uint32_t nb, Tok& tk);
template <bool CAREFUL, class V, class TT>
__device__ __forceinline__ void tok(const V& v, uint32_t& pos, const TT& t, bool empty_dist, uint32_t stop,
                                    uint32_t nb, Tok& tk) {
    // (the result goes through scalars and is stored into tk once: stores of different fields on
    // different paths made the compiler keep tk in scratch memory)
    uint32_t lo, hi;
    v.win(pos, lo, hi);
    tok_e<CAREFUL>(lo, hi, t.lit[lo & ((1u << LB) - 1u)], pos, t, empty_dist, stop, nb, tk);
}
// the rest of a token step once its window (lo, hi) and primary entry e are loaded
template <bool CAREFUL, class TT>
__device__ __forceinline__ void tok_e(uint32_t lo, uint32_t hi, uint32_t e, uint32_t& pos, const TT& t,
                                      bool empty_dist, uint32_t stop, uint32_t nb, Tok& tk) {
    uint32_t kind, val, n = 1, dist = 0;
    do {
        if (e >> 31) {
            // [3:0] the entry's advance (both codes of a pair), [7:4] the first code's length
            const uint32_t adv = e & 15;
            bool two = (e >> 8) & 1;
            if (CAREFUL) {
                const uint32_t l1 = (e >> 4) & 15;
                two = two && pos + l1 < stop && pos + adv <= nb;
                pos += two ? adv : l1;
            } else {
                pos += adv;
            }
            kind = K_LIT; n = 1u + (uint32_t)two; val = (e >> 9) & (two ? 0xFFFFu : 0xFFu);
            if (CAREFUL && pos > nb) { kind = K_BAD; val = R_UEOS; n = 1; }
            break;
        }
        if (!(e & 31)) e = long_lit(e, lo, t);
        const uint32_t cl = e & 31, k = (e >> 9) & 3;
        if (k != K_LEN) {
            pos += cl;
            kind = k; val = k == K_LIT ? e >> 16 : rsv_len(e);
            if (CAREFUL && pos > nb) { kind = K_BAD; val = R_UEOS; }
            break;
        }
        kind = K_BAD; val = R_UEOS;
        const uint32_t xb = (e >> 5) & 15;
        if (CAREFUL && pos + cl > nb) { pos += cl; break; }
        const uint32_t run = (e >> 16) + ((lo >> cl) & ((1u << xb) - 1u));
        const uint32_t sh = cl + xb;
        if (CAREFUL && pos + sh > nb) { pos += sh; break; }
        if (empty_dist) { pos += sh; val = R_EMPTY_DIST; break; }
        const uint32_t dw = __builtin_amdgcn_alignbit(hi, lo, sh);      // 32 bits from the distance code
        uint32_t d = t.dst[dw & ((1u << DB) - 1u)];
        if (!(d & 31)) d = long_dist(d, dw, t);
        const uint32_t dl = d & 31, dxb = (d >> 5) & 15;
        if (CAREFUL && pos + sh + dl > nb) { pos += sh + dl; break; }
        if (((d >> 9) & 3) == K_BAD) { pos += sh + dl; val = rsv_dist(d); break; }
        dist = (d >> 16) + ((dw >> dl) & ((1u << dxb) - 1u));
        pos += sh + dl + dxb;
        if (CAREFUL && pos > nb) break;
        kind = K_LEN; n = run; val = 0;
    } while (false);
    tk.kind = kind; tk.val = val; tk.n = n; tk.dist = dist;
}

// ---- register bit buffer (the unchecked token steps) ----------------------------------------------
// A token's dependency chain through tok<false> is two LDS round trips: the window at pos (three
// staged words), then the table entry.  Bb keeps the lane's next 32..64 bits in a 64-bit register
// and the word after them loaded ahead, so the table read is the only LDS access on the chain; the
// refill (one word when fewer than 32 bits are left, after the length part of a copy token too)
// only consumes a word loaded a step earlier.  Same steps, same results as tok<false>.
#ifndef NDFL_BITBUF
#define NDFL_BITBUF 1
#endif
struct Bb {
    uint64_t buf;      // the bits from pos on (nb of them valid)
    uint32_t nb;       // 32..64 at a token's start
    uint32_t wi;       // region word index of the next word to append
    uint32_t nxt;      // that word
    uint32_t pos;      // round-relative bit position
};
// (V: the staged round in LDS (Lv) or the input in global memory (Gv): region word i = v.ld(i))
template <class V>
__device__ __forceinline__ void bb_init(Bb& b, const V& v, uint32_t pos) {
    const uint32_t i = (pos >> 5) - v.rw, s = pos & 31;
    b.buf = ((uint64_t)v.ld(i) | ((uint64_t)v.ld(i + 1) << 32)) >> s;
    b.nb = 64 - s;
    b.wi = i + 2;
    b.nxt = v.ld(i + 2);
    b.pos = pos;
}
template <class V>
__device__ __forceinline__ void bb_refill(Bb& b, const V& v) {
    if (b.nb < 32) {
        b.buf |= (uint64_t)b.nxt << b.nb;
        b.nb += 32;
        b.wi++;
        b.nxt = v.ld(b.wi);
    }
}
__device__ __forceinline__ void bb_skip(Bb& b, uint32_t n) {
    b.buf >>= n; b.nb -= n; b.pos += n;
}
// A token step on the bit buffer: the caller guarantees pos + 48 < nb (no token reaches the input
// end, so none of its checks are needed).  STOP = false: also pos + 48 < stop (tok<false>);
// STOP = true: any pos < stop -- a literal pair whose first literal reaches `stop` is split, as in
// tok<true>, so the buffer carries a decode right up to a checkpoint or the segment end.
template <bool STOP = false, class V, class TT>
__device__ __forceinline__ void tok_bb(Bb& b, const V& v, const TT& t, bool empty_dist, Tok& tk, uint32_t stop = 0) {
    uint32_t lo = (uint32_t)b.buf;
    uint32_t e = t.lit[lo & ((1u << LB) - 1u)];
    uint32_t kind, val, n = 1, dist = 0;
    do {
        if (e >> 31) {
            if (STOP) {
                const uint32_t l1 = (e >> 4) & 15;
                const bool two = ((e >> 8) & 1) && b.pos + l1 < stop;
                bb_skip(b, two ? e & 15 : l1);
                n = 1u + (uint32_t)two;
            } else {
                bb_skip(b, e & 15);
                n = 1u + ((e >> 8) & 1u);
            }
            kind = K_LIT; val = (e >> 9) & (n == 2 ? 0xFFFFu : 0xFFu);
            break;
        }
        if (!(e & 31)) e = long_lit(e, lo, t);
        const uint32_t cl = e & 31, k = (e >> 9) & 3;
        if (k != K_LEN) {
            bb_skip(b, cl);
            kind = k; val = k == K_LIT ? e >> 16 : rsv_len(e);
            break;
        }
        const uint32_t xb = (e >> 5) & 15;
        const uint32_t run = (e >> 16) + ((lo >> cl) & ((1u << xb) - 1u));
        bb_skip(b, cl + xb);
        if (empty_dist) { kind = K_BAD; val = R_EMPTY_DIST; break; }
        bb_refill(b, v);
        const uint32_t dw = (uint32_t)b.buf;
        uint32_t d = t.dst[dw & ((1u << DB) - 1u)];
        if (!(d & 31)) d = long_dist(d, dw, t);
        const uint32_t dl = d & 31, dxb = (d >> 5) & 15;
        if (((d >> 9) & 3) == K_BAD) { bb_skip(b, dl); kind = K_BAD; val = rsv_dist(d); break; }
        dist = (d >> 16) + ((dw >> dl) & ((1u << dxb) - 1u));
        bb_skip(b, dl + dxb);
        kind = K_LEN; n = run; val = 0;
    } while (false);
    bb_refill(b, v);
    tk.kind = kind; tk.val = val; tk.n = n; tk.dist = dist;
}

// Count tokens from pos to the first token boundary at or past `stop` (<= input end) or to a
// terminal token (true: end of block or an error, in tk).
__device__ __forceinline__ bool run_to(const Lv& v, uint32_t& pos, const Tabs& t, bool ed, uint32_t stop, uint32_t nb,
                                       uint32_t& cnt, Tok& tk) {
#if NDFL_BITBUF
    // the bit buffer up to the stop itself (pairs split there); only the input's last 48 bits go
    // through the checked decoder
    const uint32_t lim = min(stop, nb - min(nb, 48u));
    if (pos < lim) {
        Bb b;
        bb_init(b, v, pos);
        do {
            tok_bb<true>(b, v, t, ed, tk, stop);
            if (tk.kind > K_LEN) { pos = b.pos; return true; }
            cnt += tk.n;
        } while (b.pos < lim);
        pos = b.pos;
    }
#else
    while (pos + 48 < stop) {
        tok<false>(v, pos, t, ed, stop, nb, tk);
        if (tk.kind > K_LEN) return true;
        cnt += tk.n;
    }
#endif
    while (pos < stop) {
        tok<true>(v, pos, t, ed, stop, nb, tk);
        if (tk.kind > K_LEN) return true;
        cnt += tk.n;
    }
    return false;
}

// ---- block header (lane 0) ----------------------------------------------------------------------
// Parses the header at p into h and (dynamic) lens[0, numLit) and lens[288, 288 + numDist) (the
// caller zeroes lens); validation in the reference's order up to END_OF_BLOCK_CODE_ZERO_LENGTH; the
// tree checks of the two codes follow in build_code.  cl_tab: 128 u16 of scratch (LDS).
struct Hdr {
    uint64_t pos, d0;
    uint32_t err, bfinal, btype, len, numlit, numdist;
};
// Lane reader over a lane-private LDS window of 8 words (word i of lane j at win[i * 64 + j]: no
// bank conflicts), refilled by two 16-byte loads in flight together: one load wait per 256 bits
// where Rd waits one per 32 (a header of ~1,000 bits: 4 waits instead of 30).  (8 words keep the
// header kernel at 4 workgroups per CU.)
struct RdWin {
    uint32_t* win;        // &lds[lane]
    uint64_t pos, bb, wq;
    uint32_t bn, wi;
    __device__ __forceinline__ void load(const In& in) {
        u32x4 g[2];
#pragma unroll
        for (int k = 0; k < 2; k++) g[k] = in.ld4(wq + k);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            win[(4 * k) * 64] = g[k].x; win[(4 * k + 1) * 64] = g[k].y;
            win[(4 * k + 2) * 64] = g[k].z; win[(4 * k + 3) * 64] = g[k].w;
        }
        wq += 2;
        wi = 0;
    }
    __device__ __forceinline__ void init(const In& in, uint64_t p) {
        pos = p;
        wq = p >> 7;
        load(in);
        wi = (uint32_t)(p >> 5) & 3u;
        bb = (uint64_t)(win[wi * 64] >> (p & 31));
        bn = 32 - (uint32_t)(p & 31);
        wi++;
        fill(in);
    }
    __device__ __forceinline__ void fill(const In& in) {
        if (bn <= 32) {
            if (wi == 8) load(in);
            bb |= (uint64_t)win[wi * 64] << bn; bn += 32; wi++;
        }
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
template <class R = Rd>
__device__ __forceinline__ void parse_hdr_core(const In& in, uint64_t p, uint8_t* lens, uint16_t* cl_tab, Hdr& h,
                                               uint32_t* win = nullptr) {
    R rd;
    if constexpr (std::is_same<R, RdWin>::value) rd.win = win;
    rd.init(in, p);
    h.err = 0; h.len = 0; h.numlit = 0; h.numdist = 0; h.pos = 0; h.d0 = 0;
    const uint32_t bf = rd.get(in, 1), bt = rd.get(in, 2);
    h.bfinal = bf; h.btype = bt;
#define HFAIL(r) do { h.err = (r); h.pos = rd.pos; return; } while (0)
    if (rd.pos > in.nbits) HFAIL(R_UEOS);
    if (bt == 3) HFAIL(R_RESERVED_BLOCK_TYPE);
    if (bt == 0) {
        rd.get(in, (uint32_t)((8 - (rd.pos & 7)) & 7));
        const uint32_t ln = rd.get(in, 16), nln = rd.get(in, 16);
        if (rd.pos > in.nbits) HFAIL(R_UEOS);
        if (ln != (nln ^ 0xFFFFu)) HFAIL(R_LEN_MISMATCH);
        h.len = ln; h.d0 = rd.pos; h.pos = rd.pos;
        return;
    }
    if (bt == 1) { h.d0 = rd.pos; h.pos = rd.pos; return; }
    const uint32_t hlit = rd.get(in, 5), hdist = rd.get(in, 5), hclen = rd.get(in, 4);
    if (rd.pos > in.nbits) HFAIL(R_UEOS);
    const uint32_t numLit = hlit + 257, numDist = hdist + 1, numCl = hclen + 4;
    uint32_t cl[19];
#pragma unroll
    for (int i = 0; i < 19; i++) cl[i] = 0;
#pragma unroll
    for (int i = 0; i < 19; i++)
        if ((uint32_t)i < numCl) cl[CLO[i]] = rd.get(in, 3);
    if (rd.pos > in.nbits) HFAIL(R_UEOS);
    uint32_t cc[16];
#pragma unroll
    for (int l = 0; l < 16; l++) cc[l] = 0;
#pragma unroll
    for (int s = 0; s < 19; s++) cc[cl[s]] += 1;
    cc[0] = 0;
    int e = tree_check(cc);
    if (e) HFAIL(e);
    {
        uint32_t first[8], nx[8];
        uint32_t code = 0;
        first[0] = 0;
        for (int l = 1; l < 8; l++) { code = (code + (l > 1 ? cc[l - 1] : 0)) << 1; first[l] = code; nx[l] = 0; }
        for (int s = 0; s < 19; s++) {
            const uint32_t l = cl[s];
            if (!l) continue;
            const uint32_t r = rev_bits(first[l] + nx[l]++, l);
            for (uint32_t k = r; k < 128; k += (1u << l)) cl_tab[k] = (uint16_t)(s | (l << 9));
        }
    }
    const uint32_t total = numLit + numDist;
    uint32_t i = 0;
    int runVal = -1;
    while (i < total) {
        rd.fill(in);
        const uint32_t ent = cl_tab[rd.peek(7)];
        rd.skip(ent >> 9);
        const uint32_t sym = ent & 0x1FF;
        if (rd.pos > in.nbits) HFAIL(R_UEOS);
        uint32_t run = 1, v;
        if (sym < 16) { v = sym; runVal = (int)sym; }
        else if (sym == 16) {
            if (runVal == -1) HFAIL(R_NO_PREV);
            run = rd.get(in, 2) + 3; v = (uint32_t)runVal;
        } else if (sym == 17) { runVal = 0; run = rd.get(in, 3) + 3; v = 0; }
        else { runVal = 0; run = rd.get(in, 7) + 11; v = 0; }
        if (rd.pos > in.nbits) HFAIL(R_UEOS);
        if (i + run > total) HFAIL(R_CL_OVER_FULL);
        if (v) for (uint32_t k = 0; k < run; k++, i++) lens[i < numLit ? i : 288 + (i - numLit)] = (uint8_t)v;
        else i += run;                          // (lens are zeroed by the caller)
    }
    if (lens[256] == 0) HFAIL(R_EOB_ZERO);
    h.numlit = numLit; h.numdist = numDist;
    h.d0 = rd.pos; h.pos = rd.pos;
#undef HFAIL
}
__device__ __forceinline__ void hdr_to_shared(const Hdr& h, Shared& S) {
    S.h_pos = h.pos; S.h_d0 = h.d0; S.h_err = h.err; S.h_bfinal = h.bfinal; S.h_btype = h.btype;
    S.h_len = h.len; S.h_numlit = h.numlit; S.h_numdist = h.numdist;
}
__device__ void parse_hdr(const In& in, uint64_t p, Shared& S) {
    Hdr h;
    parse_hdr_core(in, p, S.lens, S.cl_tab, h);
    hdr_to_shared(h, S);
}

// Header records (ndfl_inflate_hdr_kernel): every header candidate's parse, one lane each, so the
// count pass's first block of a chain loads it instead of parsing on one lane of its wave.
struct HdrRec {
    uint32_t lens[80];                       // S.lens as words
    Hdr h;
    uint64_t at;                             // the candidate's bit position
    uint32_t flat;                           // escape-prefix literal code (count_flat_group): k + 1, else 0
    uint32_t pad;
};

// Synchronisation of the table build: the whole workgroup (WS = false: the one-wave kernels), or
// one wave of a multi-wave workgroup building the tables alone (WS = true: its own LDS accesses in
// order, no workgroup barrier, which the other waves do not reach).
__device__ __forceinline__ void wsync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
template <bool WS>
__device__ __forceinline__ void bsync() {
    if (WS) wsync(); else __syncthreads();
}

// Canonical code from S.lens[base .. base+n) into the primary table `prim` (pbits) and the
// extension area `x` (cap words): second-level tables for the codes longer than the primary when
// they fit, else the canonical slow-path arrays (wave).  Returns the tree check result of
// codeLengthsToCodeTree (D/decomp/Open.java:705-756) (uniform).
template <bool WS = false>
__device__ int build_code(Shared& S, uint32_t base, uint32_t n, uint32_t* prim, uint32_t pbits, uint32_t* x,
                          uint32_t cap, bool is_lit, int lane) {
    for (uint32_t k = (uint32_t)lane; k < (1u << pbits); k += 64) prim[k] = 0;
    uint32_t c[16];
#pragma unroll
    for (int l = 0; l < 16; l++) c[l] = 0;
    uint32_t mylen[5], rank[5];
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint32_t s = (uint32_t)q * 64 + (uint32_t)lane;
        const uint32_t l = (s < n) ? S.lens[base + s] : 0u;
        mylen[q] = l;
        rank[q] = 0;
        if ((uint32_t)q * 64 < n) {
#pragma unroll
            for (int L = 1; L < 16; L++) {
                const uint64_t m = __ballot(l == (uint32_t)L);
                if (l == (uint32_t)L) rank[q] = c[L] + (uint32_t)__popcll(m & lt);
                c[L] += (uint32_t)__popcll(m);
            }
        }
    }
    const int err = tree_check(c);
    if (err) return err;
    uint32_t fst[16], off[16];
    {
        uint32_t code = 0, o = 0;
        fst[0] = 0; off[0] = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            code = (code + (l > 1 ? c[l - 1] : 0)) << 1;
            fst[l] = code; off[l] = o; o += c[l];
        }
    }
    bsync<WS>();                            // prim zeroed
    // the longest code under each primary prefix of the long codes (a canonical code's prefix set
    // is prefix-free with the short codes, so these entries are free)
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint32_t l = mylen[q];
        if (l <= pbits) continue;
        uint32_t f = 0;
#pragma unroll
        for (int L = 1; L < 16; L++) if (l == (uint32_t)L) f = fst[L];
        atomicMax(&prim[rev_bits((f + rank[q]) >> (l - pbits), pbits)], l);
    }
    bsync<WS>();
    // second-level table offsets: exclusive scan of 2^(longest - pbits) over the primary entries
    const uint32_t per = (1u << pbits) / 64;
    uint32_t loc = 0;
    for (uint32_t i = 0; i < per; i++) {
        const uint32_t m = prim[(uint32_t)lane * per + i];
        loc += m ? 1u << (m - pbits) : 0u;
    }
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const bool two = __shfl(incl, 63, 64) <= cap;
    {
        uint32_t o = incl - loc;
        for (uint32_t i = 0; i < per; i++) {
            const uint32_t k = (uint32_t)lane * per + i;
            const uint32_t m = prim[k];
            if (m) {
                prim[k] = two ? ((o << 16) | ((m - pbits) << 5)) : 0u;
                o += 1u << (m - pbits);
            }
        }
    }
    if (!two && lane < 16) {
        uint16_t* first = (uint16_t*)(x + n + 16);
        uint16_t* offv = first + 16;
        first[lane] = (uint16_t)fst[lane];
        offv[lane] = (uint16_t)off[lane];
        uint32_t ll = 0;
#pragma unroll
        for (int L = 1; L < 16; L++) if (lane == L) ll = fst[L] + c[L];
        x[n + lane] = lane ? (ll << (15 - lane)) : 0u;
    }
    bsync<WS>();
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint32_t l = mylen[q];
        if (!l) continue;
        const uint32_t s = (uint32_t)q * 64 + (uint32_t)lane;
        uint32_t f = 0, o = 0;
#pragma unroll
        for (int L = 1; L < 16; L++) if (l == (uint32_t)L) { f = fst[L]; o = off[L]; }
        const uint32_t ent = is_lit ? lit_entry(s, l) : dist_entry(s, l);
        const uint32_t code = f + rank[q];
        if (l <= pbits) {
            if (l + 4 >= pbits)                 // (<= 16 entries; shorter codes: all lanes, below)
                for (uint32_t k = rev_bits(code, l); k < (1u << pbits); k += (1u << l)) prim[k] = ent;
        } else if (two) {
            const uint32_t pe = prim[rev_bits(code >> (l - pbits), pbits)];
            const uint32_t sb = pe >> 16, sd = (pe >> 5) & 15, r = l - pbits;
            for (uint32_t k = rev_bits(code & ((1u << r) - 1u), r); k < (1u << sd); k += (1u << r)) x[sb + k] = ent;
        }
        if (!two) x[o + rank[q]] = ent;
    }
    // the codes shorter than pbits - 4 (more than 16 entries each, up to 2^(pbits-1)): one symbol at a
    // time over all lanes, where a lane filling its own would hold the wave for its longest run
#pragma unroll
    for (int q = 0; q < 5; q++) {
        if ((uint32_t)q * 64 >= n) continue;    // (uniform)
        uint64_t sm = __ballot(mylen[q] != 0 && mylen[q] + 4 < pbits);
        while (sm) {
            const int src = (int)__builtin_ctzll(sm);
            sm &= sm - 1;
            const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)mylen[q], src);
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rank[q], src);
            uint32_t f = 0;
#pragma unroll
            for (int L = 1; L < 16; L++) if (l == (uint32_t)L) f = fst[L];
            const uint32_t sy = (uint32_t)q * 64 + (uint32_t)src;
            const uint32_t ent = is_lit ? lit_entry(sy, l) : dist_entry(sy, l);
            for (uint32_t k = rev_bits(f + r, l) + ((uint32_t)lane << l); k < (1u << pbits); k += 64u << l) prim[k] = ent;
        }
    }
    bsync<WS>();
    return 0;
}

// Literal pairs in the primary table: an entry whose code is a literal becomes
// 1 << 31 | adv | l1 << 4 | pair << 8 | b1 << 9 | b2 << 17, with pair set when the next LB - l1 bits
// start with a second literal code (its length l2 <= LB - l1) and adv = l1 + l2 for a pair, l1
// otherwise -- an unchecked step adds adv with no select.
template <bool WS = false>
__device__ void group_lits(Tabs& t, int lane) {
    uint32_t nv[(1u << LB) / 64];
#pragma unroll
    for (uint32_t q = 0; q < (1u << LB) / 64; q++) {
        const uint32_t k = q * 64 + (uint32_t)lane;
        const uint32_t e1 = t.lit[k];
        const uint32_t l1 = e1 & 31;
        uint32_t v = e1;
        if (l1 && ((e1 >> 9) & 3) == K_LIT) {
            const uint32_t b1 = (e1 >> 16) & 0xFFu;
            v = (1u << 31) | l1 | (l1 << 4) | (b1 << 9);
            const uint32_t e2 = t.lit[k >> l1];
            const uint32_t l2 = e2 & 31;
            if (l1 < LB && l2 && l1 + l2 <= LB && ((e2 >> 9) & 3) == K_LIT)
                v = (1u << 31) | (l1 + l2) | (l1 << 4) | (1u << 8) | (b1 << 9) | (((e2 >> 16) & 0xFFu) << 17);
        }
        nv[q] = v;
    }
    bsync<WS>();
#pragma unroll
    for (uint32_t q = 0; q < (1u << LB) / 64; q++) t.lit[q * 64 + (uint32_t)lane] = nv[q];
    bsync<WS>();
}

// Fixed code lengths (D/decomp/Open.java:812-830) into S.lens.
__device__ void fixed_lens(Shared& S, int lane) {
    for (uint32_t s = (uint32_t)lane; s < 320; s += 64) {
        uint32_t l;
        if (s < 288) l = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        else l = 5;
        S.lens[s] = (uint8_t)l;
    }
}

// ---- table build, round 6 ---------------------------------------------------------------------
// The same tables (word for word where a decoder reads them: scripts/r06/build_bench.hip compares
// every header of a config-4 stream), built with a fraction of the instructions.  The build above
// runs as a call from the decode passes and took ~33 K cycles for a literal/length code at one wave
// per SIMD: its per-length arrays (counts, first codes, rank offsets) sat in scratch memory, indexed
// by each lane's code length; its tree check compared 64-bit values in the vector unit; 15-way
// select chains picked a lane's per-length values; codes were written one symbol at a time; and
// every LDS access went through a generic pointer (a null check and a conversion per access, the
// callee not knowing its arguments were LDS).  A single wave issues about one instruction per few
// cycles, so the instruction count -- scalar ones included -- sets the time.  Here:
//   * LDS-typed pointers (address space 3) and the primary bits as a template parameter;
//   * ranks bit-sliced: four ballots give each lane the mask of lanes whose length equals its own;
//   * per-length values (rank offset O, first code F, O - F) in LDS, read by length (`scr`: 64 words
//     of the round stage, which holds nothing while a block's tables are built);
//   * complete codes decided by their Kraft sum in a few scalar adds (the level-wise check of the
//     reference's error order only runs for the others: corrupt streams);
//   * the primary table PULLED, all of a lane's entries at once: lane j computes the entries
//     k = i * 64 + j -- the code length from the left-justified limits (codes of length <= L occupy
//     [0, LJ[L]) of the MSB-first prefix space), the symbol from the code's rank, through the
//     canonical entry array every symbol wrote into the extension area (x[O[l] + rank]: the slow
//     path's array anyway);
//   * the long codes' prefixes and second-level tables as before (the second level then overwrites
//     that entry order in x).
#ifndef NDFL_BUILD_V2
#define NDFL_BUILD_V2 1
#endif
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef __attribute__((address_space(3))) uint16_t lu16;
typedef __attribute__((address_space(3))) uint8_t lu8;
typedef __attribute__((address_space(3))) u32x4 lu128;
typedef __attribute__((address_space(3))) Shared LShared;
#ifdef NDFL_BUILD_PROF                          // (A/B builds: per-section clocks of the build)
__device__ unsigned long long g_bprof[8192 * 8];      // per wave (block) and section, no contention
#define BPROF(i) do { const unsigned long long _t = clock64(); if (lane == 0) g_bprof[blockIdx.x * 8 + (i)] += _t - bp_t; bp_t = clock64(); } while (0)
#else
#define BPROF(i) do { } while (0)
#endif
// GROUP (a dynamic literal/length code): literal pairs joined into the primary entries as group_lits
// does, from the pulled entries still in registers
template <bool WS, uint32_t PB, bool GROUP = false>
__device__ __forceinline__ int build_code_l(LShared* S, uint32_t base, uint32_t n, lu32* prim, lu32* x, uint32_t cap,
                                            bool is_lit, int lane, lu32* scr) {
#ifdef NDFL_BUILD_PROF
    unsigned long long bp_t = clock64();
#endif
    constexpr uint32_t PER = (1u << PB) / 64;
    lu32* CUM = scr;                            // [16] symbols of each length so far (then totals)
    lu32* O = scr + 16;                         // [16] rank offset per length
    lu32* F = scr + 32;                         // [16] first code per length
    lu32* DD = scr + 48;                        // [16] O - F
    uint32_t mylen[5], rank[5];
    if (lane < 16) CUM[lane] = 0;
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint32_t s = (uint32_t)q * 64 + (uint32_t)lane;
        const uint32_t l = (s < n) ? S->lens[base + s] : 0u;
        mylen[q] = l;
        uint32_t r = 0;
        if ((uint32_t)q * 64 < n) {
            uint64_t same = ~0ull;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint64_t bj = __ballot((l >> j) & 1u);
                same &= ((l >> j) & 1u) ? bj : ~bj;
            }
            const uint32_t before = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32),
                                    __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
            if (l) {
                const uint32_t cb = CUM[l];
                r = cb + before;
                if (before == 0) CUM[l] = cb + (uint32_t)__popcll(same);
            }
        }
        rank[q] = r;
    }
    wsync();
    const uint32_t cnt_l = lane < 16 && lane > 0 ? CUM[lane] : 0u;
    uint32_t c[16];
    c[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) c[l] = (uint32_t)__builtin_amdgcn_readlane((int)cnt_l, l);
    BPROF(0);
    {
        uint32_t num = 0, kraft = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) { num += c[l]; kraft += c[l] << (15 - l); }
        if (!(num >= 2 && kraft == 32768u)) {   // (complete codes pass without the level-wise check)
            const int err = tree_check(c);
            if (err) return err;
        }
    }
    // first code and rank offset of each length (lane l writes length l's), left-justified limits
    uint32_t lj[PB + 1];
    uint32_t maxl = 0;
    {
        uint32_t code = 0, o = 0, myF = 0, myO = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            code = (code + (l > 1 ? c[l - 1] : 0)) << 1;
            myF = lane == l ? code : myF;
            myO = lane == l ? o : myO;
            o += c[l];
            if ((uint32_t)l <= PB) lj[l] = (code + c[l]) << (PB - (uint32_t)l);
            maxl = c[l] ? (uint32_t)l : maxl;
        }
        if (lane < 16) { F[lane] = myF; O[lane] = myO; DD[lane] = myO - myF; }
    }
    wsync();
    BPROF(1);
    // every symbol's entry at its canonical position (the slow path's array; the pull's source)
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint32_t l = mylen[q];
        if (l) {
            const uint32_t s = (uint32_t)q * 64 + (uint32_t)lane;
            x[O[l] + rank[q]] = is_lit ? lit_entry(s, l) : dist_entry(s, l);
        }
    }
    BPROF(2);
    bool two = true;
    if (maxl > PB) {
        // the longest code under each primary prefix of the long codes (prefix-free with the short
        // codes, so these entries are free), then the second-level offsets (as build_code)
#pragma unroll
        for (uint32_t k = (uint32_t)lane * 4; k < (1u << PB); k += 256) *(lu128*)&prim[k] = u32x4{0u, 0u, 0u, 0u};
        bsync<WS>();
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t l = mylen[q];
            if (l > PB)
                __hip_atomic_fetch_max(&prim[rev_bits((F[l] + rank[q]) >> (l - PB), PB)], l, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        bsync<WS>();
        uint32_t m[PER];
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) m[i] = prim[(uint32_t)lane * PER + i];
        uint32_t loc = 0;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) loc += m[i] ? 1u << (m[i] - PB) : 0u;
        uint32_t incl = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        two = __shfl(incl, 63, 64) <= cap;
        uint32_t o = incl - loc;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            if (m[i]) {
                prim[(uint32_t)lane * PER + i] = two ? ((o << 16) | ((m[i] - PB) << 5)) : 0u;
                o += 1u << (m[i] - PB);
            }
        }
    }
    bsync<WS>();                                // x's canonical entries, the long prefixes
    BPROF(3);
    // pull: every primary entry of a code of at most PB bits, all of the lane's at once
    {
        uint32_t cv[PER], l[PER], d[PER];
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            cv[i] = rev_bits(i * 64 + (uint32_t)lane, PB);
            uint32_t li = 1;
#pragma unroll
            for (uint32_t L = 1; L < PB; L++) li += cv[i] >= lj[L] ? 1u : 0u;
            l[i] = li;
        }
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) d[i] = DD[l[i]];
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) d[i] = x[d[i] + (cv[i] >> (PB - l[i]))];
#pragma unroll
        for (uint32_t i = 0; i < PER; i++)
            if (cv[i] < lj[PB]) prim[i * 64 + (uint32_t)lane] = d[i];
        if (GROUP) {
            // literal pairs (group_lits): an entry whose code is a literal becomes
            // 1 << 31 | adv | l1 << 4 | pair << 8 | b1 << 9 | b2 << 17 (see there); a long prefix's
            // entry (length field 0) stays
            bsync<WS>();
            uint32_t v[PER];
#pragma unroll
            for (uint32_t i = 0; i < PER; i++) {
                const uint32_t k = i * 64 + (uint32_t)lane, e1 = d[i], l1 = e1 & 31;
                const bool lit1 = cv[i] < lj[PB] && ((e1 >> 9) & 3) == K_LIT;
                const uint32_t e2 = lit1 ? prim[k >> l1] : 0u;
                const uint32_t l2 = e2 & 31, b1 = (e1 >> 16) & 0xFFu;
                const bool pair = lit1 && l1 < PB && l2 && l1 + l2 <= PB && ((e2 >> 9) & 3) == K_LIT;
                v[i] = pair ? (1u << 31) | (l1 + l2) | (l1 << 4) | (1u << 8) | (b1 << 9) | (((e2 >> 16) & 0xFFu) << 17)
                            : (1u << 31) | l1 | (l1 << 4) | (b1 << 9);
                d[i] = lit1 ? 1u : 0u;
            }
            bsync<WS>();
#pragma unroll
            for (uint32_t i = 0; i < PER; i++)
                if (d[i]) prim[i * 64 + (uint32_t)lane] = v[i];
        }
    }
    BPROF(4);
    if (!two && lane < 16) {
        // the canonical slow path's limits and per-length first code / offset (u16)
        lu16* first = (lu16*)(x + n + 16);
        lu16* offv = first + 16;
        const uint32_t f = lane ? F[lane] : 0u, o = lane ? O[lane] : 0u;
        first[lane] = (uint16_t)f;
        offv[lane] = (uint16_t)o;
        x[n + lane] = lane ? ((f + cnt_l) << (15 - lane)) : 0u;
    }
    if (maxl > PB && two) {
        bsync<WS>();                            // the pull has read x's canonical entries
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t l = mylen[q];
            if (l <= PB) continue;
            const uint32_t s = (uint32_t)q * 64 + (uint32_t)lane;
            const uint32_t ent = is_lit ? lit_entry(s, l) : dist_entry(s, l);
            const uint32_t code = F[l] + rank[q];
            const uint32_t pe = prim[rev_bits(code >> (l - PB), PB)];
            const uint32_t sb = pe >> 16, sd = (pe >> 5) & 15, r = l - PB;
            for (uint32_t k = rev_bits(code & ((1u << r) - 1u), r); k < (1u << sd); k += (1u << r)) x[sb + k] = ent;
        }
    }
    bsync<WS>();
    BPROF(5);
    return 0;
}
// The whole build (one call from the decode passes): error or 0 in bits 0..7, empty distance code
// in bit 8 -- no reference argument, which would put the caller's flag in scratch memory.
template <bool WS>
__device__ __noinline__ int build_tables_l(LShared* S, int lane, lu32* scr) {
    // (one literal/length build for both block types: fixed codes of 7..9 bits form no pairs in a
    // 10-bit primary, and the function's code stays one build long)
    if (S->h_btype == 1) {
        for (uint32_t s = (uint32_t)lane; s < 320; s += 64) {
            uint32_t l;
            if (s < 288) l = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
            else l = 5;
            S->lens[s] = (uint8_t)l;
        }
        bsync<WS>();
    }
    const int e = build_code_l<WS, LB, true>(S, 0, 288, S->t.lit, S->t.lx, LX, true, lane, scr);
    if (e) return e;
    // distance code: empty (one zero length) or one used code padded at index 31 (:398-425); fixed
    // blocks' 32 lengths of 5 take neither branch
    const uint32_t numDist = S->h_numdist;
    const uint32_t dl = (lane < 32) ? S->lens[288 + lane] : 0u;
    if (S->h_btype != 1 && numDist == 1 && S->lens[288] == 0) return 0x100;
    const uint32_t ones = (uint32_t)__popcll(__ballot(dl == 1)), other = (uint32_t)__popcll(__ballot(dl > 1));
    bsync<WS>();
    if (ones == 1 && other == 0 && lane == 0) S->lens[288 + 31] = 1;
    bsync<WS>();
    return build_code_l<WS, DB>(S, 288, 32, S->t.dst, S->t.dx, DX, false, lane, scr);
}

// Tables for the block whose header S.h_* describes.  Returns a Reason (uniform) or 0.  scr: >= 64
// words of LDS the build may use (the round stage: nothing is staged while a block's tables are built).
template <bool WS = false>
__device__ __forceinline__ int build_tables(Shared& S, int lane, bool& empty_dist, uint32_t* scr) {
#if NDFL_BUILD_V2
    const int r = build_tables_l<WS>((LShared*)&S, lane, (lu32*)scr);
    empty_dist = (r & 0x100) != 0;
    return r & 0xFF;
#else
    (void)scr;
    empty_dist = false;
    if (S.h_btype == 1) {
        fixed_lens(S, lane);
        bsync<WS>();
        build_code<WS>(S, 0, 288, S.t.lit, LB, S.t.lx, LX, true, lane);
        build_code<WS>(S, 288, 32, S.t.dst, DB, S.t.dx, DX, false, lane);
        return 0;
    }
    const uint32_t numDist = S.h_numdist;
    int e = build_code<WS>(S, 0, 288, S.t.lit, LB, S.t.lx, LX, true, lane);
    if (e) return e;
    group_lits<WS>(S.t, lane);
    // distance code: empty (one zero length) or one used code padded at index 31 (:398-425)
    const uint32_t dl = (lane < 32) ? S.lens[288 + lane] : 0u;
    empty_dist = numDist == 1 && S.lens[288] == 0;
    if (empty_dist) return 0;
    const uint32_t ones = (uint32_t)__popcll(__ballot(dl == 1)), other = (uint32_t)__popcll(__ballot(dl > 1));
    bsync<WS>();
    if (ones == 1 && other == 0 && lane == 0) S.lens[288 + 31] = 1;
    bsync<WS>();
    return build_code<WS>(S, 288, 32, S.t.dst, DB, S.t.dx, DX, false, lane);
#endif
}

// ---- segmented speculative decode of one round ------------------------------------------------
// Lane j owns [s_j, e_j) (round-relative bits) and checkpoints C1_j = s_j + min(XCP1, len) and
// C2_j = s_j + min(XCP2, len) (64 and 192 bits; round 4: XCP1 128 -> 64, count 11.1 -> 10.8 ms), and
// the segment end is a third: a verify that decoded to the end is synchronised when it ends where
// its speculation ended.  A wave's verify lasts as long as its slowest lane, and one lane missing C1
// used to decode its whole segment.  A speculative run from a start records, per checkpoint, its first
// token boundary at or past it (offset from s_j) and the output bytes before it, plus its end
// state.  Two decodes that stand on the same boundary at a checkpoint agree from there on, so a
// verify run from the TRUE start only decodes up to the first checkpoint where it meets its own
// speculation and then takes the speculative end state.  Codes whose lengths are (nearly) all
// multiples of 8 resynchronise slowly or never from a wrong bit phase; when several lanes fail the
// fallback adds runs from s_j+1 .. s_j+7 (one per phase) compared at C1.
#ifndef NDFL_XCP1
#define NDFL_XCP1 64
#endif
// The fallback phases 1..7 are decoded only when more than this many lanes of a round failed to
// synchronise (a sign of phase-locked codes), or when the frontier lane of NDFL_PH_FRONTIER fix-up
// sweeps re-ran from its exact start and still missed its speculation; fewer, isolated failures are
// resolved by the fix-up sweeps alone (round 5: frontier trigger 1 -> 4, count 10.8 -> 10.2 ms: the
// 4-byte-periodic binary tables miss ~20 % of their lanes, which two or three sweeps fix for less
// than 7 phase runs cost).  NDFL_FIX_SERIAL=1 restores the in-order fix-up loop (A/B).
#ifndef NDFL_PH_FALLBACK
#define NDFL_PH_FALLBACK 8
#endif
#ifndef NDFL_PH_FRONTIER
#define NDFL_PH_FRONTIER 4      // frontier misses (one per sweep) before the phase runs are decoded
#endif
#ifndef NDFL_FIX_SERIAL
#define NDFL_FIX_SERIAL 0
#endif
#ifndef NDFL_XCP2
#define NDFL_XCP2 192           // (round 5: 1024, i.e. the segment end -> 192 with the end compared as a
#endif                          // third checkpoint: count 10.3 -> 9.9 ms, profiles/r05_ab_count_sync.txt)
constexpr uint32_t XCP1 = NDFL_XCP1, XCP2 = NDFL_XCP2;
constexpr uint32_t NPH = 8;
constexpr uint32_t NOCP = 0xFFFFFFFFu;
constexpr uint64_t MAX_SPAN = RSPAN;         // round span cap

struct Seg {
    uint64_t start, end, cnt;                // absolute bits
    uint32_t kind, reason;
};
struct SegR {
    uint32_t start, end, cnt, kind, reason;  // round-relative
};
struct Spec {
    uint32_t end, cnt, kind, reason;
    uint32_t cp1, cpc1, cp2, cpc2;
};

__device__ __forceinline__ void spec_run(const Lv& v0, const Tabs& t, bool ed, uint32_t nb, uint32_t st, uint32_t s,
                                         uint32_t C1, uint32_t C2, uint32_t e, Spec& o) {
    const Lv& v = v0;
    uint32_t pos = st, cnt = 0, kind = T_EXIT, reason = 0;
    o.cp1 = NOCP; o.cp2 = NOCP; o.cpc1 = 0; o.cpc2 = 0;
    Tok tk;
    // three legs -- to C1, to C2, to e -- each recording its stop's checkpoint
    uint32_t stop = C1, leg = 0;
    for (;;) {
        if (run_to(v, pos, t, ed, stop, nb, cnt, tk)) {
            kind = tk.kind == K_EOB ? T_EOB : T_ERR;
            reason = tk.kind == K_EOB ? 0u : tk.val;
            break;
        }
        if (leg == 0) {
            o.cp1 = pos - s; o.cpc1 = cnt;
            if (pos >= C2) { o.cp2 = pos - s; o.cpc2 = cnt; leg = 2; stop = e; }
            else { leg = 1; stop = C2; }
        } else if (leg == 1) {
            o.cp2 = pos - s; o.cpc2 = cnt; leg = 2; stop = e;
        } else {
            break;
        }
    }
    o.end = pos; o.cnt = cnt; o.kind = kind; o.reason = reason;
}

// Decode from the true start t0; at C1 compare with phase 0 (registers) and, when nph > 1, phases
// 1..nph-1 (per-wave slot); at C2 with phase 0 again; on a match take that run's end state,
// otherwise decode the rest of the segment (authoritative).  Returns true when it synchronised.
__device__ __forceinline__ bool verify_run(const Lv& v0, const Tabs& t, bool ed, uint32_t nb, uint32_t t0, uint32_t s,
                                           uint32_t C1, uint32_t C2, uint32_t e, const Spec& p0, const PhArr* ph,
                                           int lane, uint32_t nph, SegR& r) {
    const Lv& v = v0;
    uint32_t pos = t0, c = 0, stage = 0;
    Tok tk;
    r.start = t0;
    for (;;) {
        const uint32_t stop = stage == 0 ? C1 : stage == 1 ? C2 : e;
        if (run_to(v, pos, t, ed, stop, nb, c, tk)) {
            r.end = pos; r.cnt = c;
            r.kind = tk.kind == K_EOB ? T_EOB : T_ERR;
            r.reason = tk.kind == K_EOB ? 0u : tk.val;
            return false;
        }
        if (stage == 0) {
            stage = 1;
            const uint32_t off = pos - s;
            if (p0.cp1 == off) {
                r.end = p0.end; r.cnt = c + (p0.cnt - p0.cpc1); r.kind = p0.kind; r.reason = p0.reason;
                return true;
            }
            for (uint32_t f = 1; f < nph; f++) {
                const uint32_t pc = ph->cp[f - 1][lane];
                if ((pc & 0xFFFFu) == off) {
                    r.end = s + ph->end[f - 1][lane];
                    r.cnt = c + (ph->cnt[f - 1][lane] - (pc >> 16));
                    const uint32_t kr = ph->kr[f - 1][lane];
                    r.kind = kr >> 5; r.reason = kr & 31;
                    return true;
                }
            }
            if (pos < C2) continue;
        }
        if (stage == 1) {
            stage = 2;
            if (p0.cp2 == pos - s) {
                r.end = p0.end; r.cnt = c + (p0.cnt - p0.cpc2); r.kind = p0.kind; r.reason = p0.reason;
                return true;
            }
            continue;
        }
        // decoded to the segment end: exact either way; synchronised when it ends where the
        // speculation ended (the next lane's verify started there)
        r.end = pos; r.cnt = c; r.kind = T_EXIT; r.reason = 0;
        return pos == p0.end && p0.kind == T_EXIT;
    }
}

// One round over [rs, E) (E - rs <= MAX_SPAN): stage its input, then exact per-lane segments;
// first_term = first lane ending the block (64: none).  All lanes call.
struct PhaseClock {                            // count-pass phase times (wall clock ticks), wave-uniform
    uint64_t hdr, spec, verify, phases, serial, rec, build, phmap;
};
__device__ void round_decode(const In& in, const Tabs& t, bool ed, uint64_t rs, uint64_t E, Shared& S, Stage& stg,
                             int lane, Seg& out, uint32_t& first_term, uint32_t& nslow, uint32_t& nfix, PhArr* ph,
                             Geo& g, PhaseClock* pc = nullptr) {
    uint64_t tk0 = pc ? wall_clock64() : 0;
    g = make_geo(in, rs, E);
    stage_round(in, g, stg, lane);
    const Lv v = make_lv(stg, g, lane);
    const uint32_t nb = g.nb;
    uint32_t s, e;
    lane_seg(g, lane, s, e);
    const uint32_t C1 = s + min(XCP1, e - s), C2 = s + min(XCP2, e - s);
    Spec p0;
    spec_run(v, t, ed, nb, s, s, C1, C2, e, p0);
    S.exit_[lane] = p0.end;
    // lanes up to the first whose speculative run ended the block: the lanes past the end of a block
    // decode the next block's bits with this block's tables (a round spans past the block end when
    // no header candidate marks it) and never synchronise, which must not count as a phase-locked code
    const uint64_t tsp = __ballot(p0.kind != T_EXIT);
    const uint64_t inblk = tsp ? (2ull << __builtin_ctzll(tsp)) - 1ull : ~0ull;
    __syncthreads();
    if (pc) { const uint64_t x = wall_clock64(); pc->spec += x - tk0; tk0 = x; }
    SegR r;
    bool fin;                                   // r is this lane's exact result
    if (lane == 0) {
        r.start = s; r.end = p0.end; r.cnt = p0.cnt; r.kind = p0.kind; r.reason = p0.reason;
        fin = true;
    } else {
        fin = verify_run(v, t, ed, nb, (uint32_t)S.exit_[lane - 1], s, C1, C2, e, p0, ph, lane, 1, r);
    }
    // exact prefix: lanes before the first unsynchronised lane
    const uint64_t um = __ballot(!fin);
    if (pc) { const uint64_t x = wall_clock64(); pc->verify += x - tk0; tk0 = x; }
    const uint32_t j0 = um ? (uint32_t)__builtin_ctzll(um) : 64u;
    const uint64_t tm = __ballot(fin && r.kind != T_EXIT);
    const uint32_t t0 = tm ? (uint32_t)__builtin_ctzll(tm) : 64u;
    if (j0 >= t0) {
        first_term = t0;
    } else {
        // lane j0 started right (its predecessor is exact) but did not meet its own speculation:
        // its verify run already decoded the segment.  Lanes after it resolve in order.
        const uint32_t nun = (uint32_t)__popcll(um & inblk);
        nslow += nun;
        uint32_t nph = nun > NDFL_PH_FALLBACK ? NPH : 1u;
        // the lanes after `from` decode their segments from the phases s+1 .. s+7 as well
        auto phase_runs = [&](uint32_t from) {
            if ((uint32_t)lane > from) {
                for (uint32_t f = 1; f < NPH; f++) {
                    Spec q;
                    spec_run(v, t, ed, nb, min(s + f, e), s, C1, C1, e, q);
                    // (offsets and byte counts at the first checkpoint fit 16 bits; otherwise no match)
                    ph->cp[f - 1][lane] = (q.cp1 < 0xFFFFu && q.cpc1 <= 0xFFFFu) ? (q.cp1 | (q.cpc1 << 16)) : 0xFFFFu;
                    ph->end[f - 1][lane] = q.end - s;
                    ph->cnt[f - 1][lane] = q.cnt;
                    ph->kr[f - 1][lane] = (uint8_t)((q.kind << 5) | q.reason);
                }
            }
        };
        if (nph > 1) phase_runs(j0);
        S.exit_[lane] = r.end;
        if (pc) { const uint64_t x = wall_clock64(); pc->phases += x - tk0; tk0 = x; }
#if NDFL_FIX_SERIAL
        S.kind_[lane] = r.kind;
        __syncthreads();
        first_term = (r.kind != T_EXIT && (uint32_t)lane == j0) ? j0 : 64u;
        first_term = __shfl(first_term, (int)j0, 64);
        for (uint32_t j = j0 + 1; j < 64 && first_term == 64; j++) {
            nfix++;
            if ((uint32_t)lane == j) {
                const uint32_t st = (uint32_t)S.exit_[j - 1];
                if (!(fin && st == r.start)) {
                    verify_run(v, t, ed, nb, st, s, C1, C2, e, p0, ph, lane, nph, r);
                    S.exit_[lane] = r.end;
                    S.kind_[lane] = r.kind;
                }
            }
            __syncthreads();
            if (S.kind_[j] != T_EXIT) first_term = j;
        }
#else
        // Fix-up sweeps: every lane after j0 whose start is not its predecessor's current exit
        // re-runs its verify from that exit, all such lanes at once.  A lane whose start equals its
        // predecessor's exit holds the exact result for that start (a synchronised run ends in its
        // speculation's end state, an unsynchronised one decoded the whole segment), so the lanes
        // before the first one that re-runs are exact, and each sweep makes at least one more lane
        // exact (the first re-run starts from an exact exit).  Failures are usually isolated --
        // the lane after a failing one meets its own speculation from the corrected start -- so a
        // round needs two or three sweeps where the in-order loop took one step per lane.
        // In a cascade (phase-locked stretches: each corrected lane misses its speculation again) a
        // sweep only moves the exact prefix by one lane, and lanes re-running from starts that are
        // about to change again only lengthen the sweep; so after the first sweep a lane re-runs only
        // when it is the first inconsistent lane or its predecessor's exit held still last sweep.
        first_term = 64u;
        uint64_t chgm = 0;                      // lanes whose exit moved in the last sweep
        uint32_t fmiss = 0;                     // sweeps whose frontier lane missed its speculation
        for (;;) {
            __syncthreads();
            const uint32_t st = lane ? (uint32_t)S.exit_[lane - 1] : r.start;
            const bool inc = (uint32_t)lane > j0 && st != r.start;
            const uint64_t cm = __ballot(inc);
            const uint32_t fc = cm ? (uint32_t)__builtin_ctzll(cm) : 64u;
            const uint64_t tx = __ballot((uint32_t)lane < fc && r.kind != T_EXIT);
            if (tx) { first_term = (uint32_t)__builtin_ctzll(tx); break; }
            if (!cm) break;
            nfix++;
            const bool pchg = lane > 0 && ((chgm >> (lane - 1)) & 1ull);
            const bool redo = inc && ((uint32_t)lane == fc || !pchg);
            const uint32_t old_end = r.end;
            bool met = true;
            if (redo) met = verify_run(v, t, ed, nb, st, s, C1, C2, e, p0, ph, lane, nph, r);
            // the frontier lane re-ran from an exact start and still missed its own speculation: a
            // phase-locked stretch (e.g. fixed-Huffman text), where every later lane would miss too
            // -- decode the phase runs now, once, so that the next re-runs meet one of them
            if (nph == 1 && __any((uint32_t)lane == fc && !met) && ++fmiss >= NDFL_PH_FRONTIER) { phase_runs(fc); nph = NPH; }
            chgm = __ballot(redo && r.end != old_end);
            __syncthreads();                    // every lane has read its predecessor's exit
            if (redo) S.exit_[lane] = r.end;
        }
#endif
        if (pc) { const uint64_t x = wall_clock64(); pc->serial += x - tk0; tk0 = x; }
    }
    out.start = g.base + r.start; out.end = g.base + r.end; out.cnt = r.cnt;
    out.kind = r.kind; out.reason = r.reason;
}

// ---- phase-mapped rounds (codes of (nearly) all-equal length, which never resynchronise) -------
// Every lane decodes its segment from all 8 bit phases s..s+7.  Where the true decode enters lane j
// decides which phase run it follows: an entry x with x - s < 8 is phase x - s; a later entry is the
// phase whose first token ends at x.  Lane j turns lane j-1's 8 phase ends into a map (phase of
// lane j-1 -> phase of lane j); a wave prefix scan composes the maps, lane 0 being phase 0.  Only
// lanes whose entry matches no phase fall back to an in-order decode.
#ifndef NDFL_PHASE_SWITCH
#define NDFL_PHASE_SWITCH 48   // lanes of a round that failed to synchronise before the block's next
#endif                         // rounds are phase-mapped (measured: 4-16 much slower; 32 -> 48: config 2
                               // count 16.9 -> 9.5 ms, fixed-Huffman text resyncs through the 8-phase verify)
#ifndef NDFL_PHASE_JUMP
#define NDFL_PHASE_JUMP 1      // phase runs step four 8-bit literals at once where they can
#endif
#ifndef NDFL_PHASE_ESC
#define NDFL_PHASE_ESC 1       // escape-prefix literal blocks: phase runs step to the next escape byte
#endif
#ifndef NDFL_PHASE_GROUP
#define NDFL_PHASE_GROUP 2     // phase runs decoded together (1, 2, 4 or 8; round 3, one token a step:
#endif                         // 1: 14.6, 2: 13.9, 4: 12.9, 8: 12.8 ms count pass; round 5, four 8-bit
                               // literals a step: 8 / 4 / 2: 10.35 / 9.57 / 9.46 against 10.0 ms without
                               // the four-literal step, random-data count pass 7.5 -> 6.5 ms per GiB,
                               // profiles/r05_ab_phase_jump.txt)

// count run from st to the first token boundary at or past e (or the block end); the first step is
// a single token whose end and bytes are returned in fb / fbc (fb = NOCP: none)
__device__ __forceinline__ void phase_run(const Lv& v0, const Tabs& t, bool ed, uint32_t nb, uint32_t st, uint32_t e,
                                          uint32_t& end, uint32_t& cnt, uint32_t& kr, uint32_t& fb, uint32_t& fbc) {
    const Lv& v = v0;
    uint32_t pos = st, c = 0;
    kr = T_EXIT << 5; fb = NOCP; fbc = 0;
    Tok tk;
    if (pos < e) {
        tok<true>(v, pos, t, ed, pos + 1, nb, tk);      // a single token (no pair)
        if (tk.kind > K_LEN) kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val);
        else { c = tk.n; fb = pos; fbc = tk.n; }
        if (tk.kind <= K_LEN && run_to(v, pos, t, ed, e, nb, c, tk))
            kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val);
    }
    end = pos; cnt = c;
}

// Several phase runs at once (same results as phase_run on each).  After each run's first token,
// the runs step together: all windows and all primary lookups are issued before any position
// moves, so the dependent LDS chains of the runs overlap; a step that is not a plain literal (or
// pair) goes through the full token decoder with the window and entry already loaded.  Phase-locked
// codes are literal-dominated.
struct PhOut { uint32_t end, cnt, kr, fb, fbc; };
__device__ __forceinline__ void phase_first(const Lv& v, const Tabs& t, bool ed, uint32_t nb, uint32_t st, uint32_t e,
                                            uint32_t& pos, uint32_t& c, PhOut& o, bool& live) {
    pos = st; c = 0;
    o.kr = T_EXIT << 5; o.fb = NOCP; o.fbc = 0;
    live = false;
    if (pos < e) {
        Tok tk;
        tok<true>(v, pos, t, ed, pos + 1, nb, tk);      // a single token (no pair)
        if (tk.kind > K_LEN) o.kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val);
        else { c = tk.n; o.fb = pos; o.fbc = tk.n; live = true; }
    }
}

template <int N>
__device__ __forceinline__ void phase_multi(const Lv& v, const Tabs& t, bool ed, uint32_t nb, uint32_t s0, uint32_t e,
                                            PhOut (&O)[N]) {
    uint32_t p[N], c[N];
    bool l[N];
#pragma unroll
    for (int k = 0; k < N; k++) phase_first(v, t, ed, nb, s0 + k, e, p[k], c[k], O[k], l[k]);
    for (;;) {
        bool f[N], any = false;
#pragma unroll
        for (int k = 0; k < N; k++) { f[k] = l[k] && p[k] + 48 < e; any = any || f[k]; }
        if (!any) break;
#if NDFL_PHASE_JUMP
        // a run's next four tokens are looked up at once, at p, p+8, p+16, p+24 (independent reads):
        // when all four are literal entries of 8 bits (one 8-bit code, or a pair of 8 bits), the run
        // moves 32 bits in one step -- phase-locked codes are mostly 8-bit literals (random data:
        // ~94 % of its tokens, so ~3/4 of its steps take four)
        uint32_t lo[N], hi[N], en[N], ex[N];
#pragma unroll
        for (int k = 0; k < N; k++) {
            const uint32_t pp = f[k] ? p[k] : p[0];
            const uint32_t* qk = v.p + ((pp >> 5) - v.rw) * 64;
            const uint32_t a = qk[0], wb = qk[64], cw = qk[128];
            lo[k] = __builtin_amdgcn_alignbit(wb, a, pp & 31);
            hi[k] = __builtin_amdgcn_alignbit(cw, wb, pp & 31);
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
            en[k] = t.lit[lo[k] & ((1u << LB) - 1u)];
            const uint32_t e1 = t.lit[(lo[k] >> 8) & ((1u << LB) - 1u)];
            const uint32_t e2 = t.lit[(lo[k] >> 16) & ((1u << LB) - 1u)];
            const uint32_t e3 = t.lit[__builtin_amdgcn_alignbit(hi[k], lo[k], 24) & ((1u << LB) - 1u)];
            // bit 31 | advance 8 in every entry: (x & 0x8000000F) == 0x80000008; pairs add a token each
            const bool all8 = ((en[k] & 0x8000000Fu) == 0x80000008u) && ((e1 & 0x8000000Fu) == 0x80000008u) &&
                              ((e2 & 0x8000000Fu) == 0x80000008u) && ((e3 & 0x8000000Fu) == 0x80000008u);
            ex[k] = all8 ? 4u + ((en[k] >> 8) & 1u) + ((e1 >> 8) & 1u) + ((e2 >> 8) & 1u) + ((e3 >> 8) & 1u) : 0u;
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
            if (f[k] && ex[k]) { p[k] += 32; c[k] += ex[k]; continue; }
            const bool q = f[k] && (en[k] >> 31);
            if (q) { p[k] += en[k] & 15; c[k] += 1u + ((en[k] >> 8) & 1u); }
            if (f[k] && !q) {
                Tok tk;
                tok_e<false>(lo[k], hi[k], en[k], p[k], t, ed, e, nb, tk);
                if (tk.kind > K_LEN) { l[k] = false; O[k].kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val); }
                else c[k] += tk.n;
            }
        }
#else
        // each run's window is its low word pair only; the third word (for a length/distance token's
        // distance bits) is read in the rare non-literal branch -- phase-locked codes are literals
        uint32_t lo[N], wb[N], en[N];
#pragma unroll
        for (int k = 0; k < N; k++) {
            const uint32_t pp = f[k] ? p[k] : p[0];
            const uint32_t* qk = v.p + ((pp >> 5) - v.rw) * 64;
            const uint32_t a = qk[0];
            wb[k] = qk[64];
            lo[k] = __builtin_amdgcn_alignbit(wb[k], a, pp & 31);
        }
#pragma unroll
        for (int k = 0; k < N; k++) en[k] = t.lit[lo[k] & ((1u << LB) - 1u)];
#pragma unroll
        for (int k = 0; k < N; k++) {
            const bool q = f[k] && (en[k] >> 31);
            if (q) { p[k] += en[k] & 15; c[k] += 1u + ((en[k] >> 8) & 1u); }
            if (f[k] && !q) {
                Tok tk;
                const uint32_t cw = v.p[((p[k] >> 5) - v.rw) * 64 + 128];
                const uint32_t hi = __builtin_amdgcn_alignbit(cw, wb[k], p[k] & 31);
                tok_e<false>(lo[k], hi, en[k], p[k], t, ed, e, nb, tk);
                if (tk.kind > K_LEN) { l[k] = false; O[k].kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val); }
                else c[k] += tk.n;
            }
        }
#endif
    }
#pragma unroll
    for (int k = 0; k < N; k++) {
        Tok tk;
        if (l[k] && run_to(v, p[k], t, ed, e, nb, c[k], tk)) O[k].kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val);
        O[k].end = p[k]; O[k].cnt = c[k];
    }
}

// Escape-prefix literal blocks (what encoders make of incompressible data: 255 literals of 8 bits --
// or 254, 252 -- with every longer code under the remaining all-ones (8 - k)-bit prefix): a run
// steps up to 8 tokens at once, to the first byte at its alignment that starts with the prefix
// (a byte-wise zero test on the 64-bit window), and decodes that one through the full token decoder.
// Same results as phase_run.  esc4: the prefix mask repeated in the 4 bytes (flat8_mask).
__device__ __forceinline__ uint32_t esc_index(uint32_t lo, uint32_t hi, uint32_t esc4) {
    const uint32_t tl = (lo & esc4) ^ esc4, th = (hi & esc4) ^ esc4;
    const uint32_t zl = (tl - 0x01010101u) & ~tl & 0x80808080u, zh = (th - 0x01010101u) & ~th & 0x80808080u;
    return zl ? (uint32_t)__builtin_ctz(zl) >> 3 : zh ? 4u + ((uint32_t)__builtin_ctz(zh) >> 3) : 8u;
}
template <int N>
__device__ __forceinline__ void phase_multi_esc(const Lv& v, const Tabs& t, bool ed, uint32_t nb, uint32_t s0, uint32_t e,
                                                uint32_t esc4, PhOut (&O)[N]) {
    uint32_t p[N], c[N];
    bool l[N];
#pragma unroll
    for (int k = 0; k < N; k++) phase_first(v, t, ed, nb, s0 + k, e, p[k], c[k], O[k], l[k]);
    for (;;) {
        bool f[N], any = false;
#pragma unroll
        for (int k = 0; k < N; k++) { f[k] = l[k] && p[k] < e; any = any || f[k]; }
        if (!any) break;
        uint32_t lo[N], hi[N];
#pragma unroll
        for (int k = 0; k < N; k++) {
            const uint32_t pp = f[k] ? p[k] : p[0];
            const uint32_t* qk = v.p + ((pp >> 5) - v.rw) * 64;
            const uint32_t a = qk[0], wb = qk[64], cw = qk[128];
            lo[k] = __builtin_amdgcn_alignbit(wb, a, pp & 31);
            hi[k] = __builtin_amdgcn_alignbit(cw, wb, pp & 31);
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
            if (!f[k]) continue;
            // the literals before the first escape byte, the stop (tokens starting before e) and
            // the input's end
            const uint32_t q = (e - p[k] + 7) >> 3, qi = (nb - min(nb, p[k])) >> 3;
            const uint32_t tt = min(min(esc_index(lo[k], hi[k], esc4), q), qi);
            if (tt) { p[k] += 8 * tt; c[k] += tt; continue; }
            Tok tk;
            tok_e<true>(lo[k], hi[k], t.lit[lo[k] & ((1u << LB) - 1u)], p[k], t, ed, e, nb, tk);
            if (tk.kind > K_LEN) { l[k] = false; O[k].kr = tk.kind == K_EOB ? (T_EOB << 5) : ((T_ERR << 5) | tk.val); }
            else c[k] += tk.n;
        }
    }
#pragma unroll
    for (int k = 0; k < N; k++) { O[k].end = p[k]; O[k].cnt = c[k]; }
}
// The prefix mask of an escape-prefix literal block, repeated in the 4 bytes, or 0: every stream
// byte x with (x & M) != M (M = 2^(8-k) - 1, k <= 2) is a single 8-bit literal's primary entry and
// no other byte is.  All lanes call (the tables in LDS, built).
__device__ __forceinline__ uint32_t flat8_mask(const Tabs& t, int lane) {
    uint64_t L[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) L[i] = __ballot((t.lit[(uint32_t)lane + 64 * i] & 0x800001FFu) == 0x80000088u);
    uint32_t m4 = 0;
#pragma unroll
    for (uint32_t kk = 0; kk < 3; kk++) {
        const uint32_t M = (1u << (8 - kk)) - 1u;
        bool same = true;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) same = same && __ballot((((uint32_t)lane + 64 * i) & M) != M) == L[i];
        if (same && !m4) m4 = M * 0x01010101u;
    }
    return m4;
}

__device__ __forceinline__ uint32_t sel8(const uint32_t (&v)[8], uint32_t i) {
    uint32_t r = v[0];
#pragma unroll
    for (uint32_t k = 1; k < 8; k++) r = i == k ? v[k] : r;
    return r;
}
// phase of an entry at offset d from s: bits 0..3 phase (8 = none), bit 4 entered at its first boundary
__device__ __forceinline__ uint32_t phase_of(uint32_t d, uint32_t fbl, uint32_t fbh) {
    if (d < 8) return d;
    uint32_t r = 8;
#pragma unroll
    for (uint32_t f = 0; f < 8; f++) {
        const uint32_t fo = ((f < 4 ? fbl : fbh) >> (8 * (f & 3))) & 0xFFu;
        if (r == 8 && fo == d) r = f | 16u;
    }
    return r;
}
// (A after B): entry f = A[B[f]], 8 stays 8
__device__ __forceinline__ uint32_t map_compose(uint32_t A, uint32_t B) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t f = 0; f < 8; f++) {
        const uint32_t bf = (B >> (4 * f)) & 15u;
        const uint32_t v = bf < 8 ? (A >> (4 * bf)) & 15u : 8u;
        r |= v << (4 * f);
    }
    return r;
}

__device__ __noinline__ void round_decode_phased(const In& in, const Tabs& t, bool ed, uint64_t rs, uint64_t E,
                                                 Shared& S, Stage& stg, int lane, Seg& out, uint32_t& first_term,
                                                 uint32_t& nfix, Geo& g, uint32_t esc4) {
    g = make_geo(in, rs, E);
    stage_round(in, g, stg, lane);
    const Lv v = make_lv(stg, g, lane);
    const uint32_t nb = g.nb;
    uint32_t s, e;
    lane_seg(g, lane, s, e);
    // the 8 runs' results stay in registers (a lane reads back only its own, through sel8)
    uint32_t endv[8], cntv[8], fbcv[8], krv[8];
    uint32_t fbl = 0, fbh = 0;
#if NDFL_PHASE_GROUP > 1
    constexpr uint32_t G = NDFL_PHASE_GROUP >= 8 ? 8 : NDFL_PHASE_GROUP >= 4 ? 4 : 2;
    // (one copy of each run group's code, its results selected into place: the loop unrolled made the
    // function 74 KB, more than the instruction cache, with the pass's other code competing)
#pragma unroll 1
    for (uint32_t f = 0; f < 8; f += G) {
        PhOut P[G];
        if (esc4) phase_multi_esc<G>(v, t, ed, nb, s + f, e, esc4, P);
        else phase_multi<G>(v, t, ed, nb, s + f, e, P);  // (past e: empty, ends at s + f)
#pragma unroll
        for (uint32_t h = 0; h < G; h++) {
            const uint32_t g = f + h;
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
                endv[k] = k == g ? P[h].end : endv[k];
                cntv[k] = k == g ? P[h].cnt : cntv[k];
                fbcv[k] = k == g ? P[h].fbc : fbcv[k];
                krv[k] = k == g ? P[h].kr : krv[k];
            }
            const uint32_t fo = (P[h].fb != NOCP && P[h].fb - s < 255u) ? P[h].fb - s : 255u;
            if (g < 4) fbl |= fo << (8 * g); else fbh |= fo << (8 * (g - 4));
        }
    }
#else
    for (uint32_t f = 0; f < 8; f++) {
        uint32_t en, cn, kr, fb, fbc;
        phase_run(v, t, ed, nb, s + f, e, en, cn, kr, fb, fbc);      // (past e: empty, ends at s + f)
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            endv[k] = k == f ? en : endv[k];
            cntv[k] = k == f ? cn : cntv[k];
            fbcv[k] = k == f ? fbc : fbcv[k];
            krv[k] = k == f ? kr : krv[k];
        }
        const uint32_t fo = (fb != NOCP && fb - s < 255u) ? fb - s : 255u;
        if (f < 4) fbl |= fo << (8 * f); else fbh |= fo << (8 * (f - 4));
    }
#endif
    // map of lane j: phase of lane j-1 -> phase of lane j
    uint32_t Q = 0;                             // lane 0: always phase 0
#pragma unroll
    for (uint32_t f = 0; f < 8; f++) {
        const uint32_t x = __shfl_up(endv[f], 1, 64);
        const uint32_t vv = phase_of(x - s, fbl, fbh) & 15u;
        if (lane > 0) Q |= vv << (4 * f);
    }
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t B = __shfl_up(Q, k, 64);
        if (lane >= k) Q = map_compose(Q, B);
    }
    const uint32_t myph = Q & 15u;
    const uint32_t xsel = myph < 8 ? sel8(endv, myph) : NOCP;
    uint32_t x = __shfl_up(xsel, 1, 64);
    if (lane == 0) x = s;
    SegR r;
    r.start = x; r.end = x; r.cnt = 0; r.kind = T_ERR; r.reason = R_INTERNAL;
    bool known = false;
    if (myph < 8) {
        const uint32_t pc = phase_of(x - s, fbl, fbh);
        const uint32_t f = pc & 15u;
        if (f == myph) {
            known = true;
            const uint32_t kr = sel8(krv, f);
            r.end = sel8(endv, f);
            r.cnt = sel8(cntv, f) - ((pc & 16u) ? sel8(fbcv, f) : 0u);
            r.kind = kr >> 5; r.reason = kr & 31u;
        }
    }
    const uint64_t km = __ballot(!known);
    const uint32_t u = km ? (uint32_t)__builtin_ctzll(km) : 64u;
    const uint64_t tm = __ballot(known && r.kind != T_EXIT);
    const uint32_t t0 = tm ? (uint32_t)__builtin_ctzll(tm) : 64u;
    first_term = min(t0, 64u);
    if (u < t0) {
        // in-order decode from lane u on (its predecessor is exact)
        S.exit_[lane] = r.end;
        __syncthreads();
        first_term = 64;
        for (uint32_t j = u; j < 64 && first_term == 64; j++) {
            nfix++;
            if ((uint32_t)lane == j) {
                const uint32_t st = j ? (uint32_t)S.exit_[j - 1] : s;
                uint32_t en, cn, kr, fb, fbc;
                if (esc4) {
                    PhOut P1[1];
                    phase_multi_esc<1>(v, t, ed, nb, st, e, esc4, P1);
                    en = P1[0].end; cn = P1[0].cnt; kr = P1[0].kr;
                } else {
                    phase_run(v, t, ed, nb, st, e, en, cn, kr, fb, fbc);
                }
                r.start = st; r.end = en; r.cnt = cn; r.kind = kr >> 5; r.reason = kr & 31u;
                S.exit_[lane] = en;
                S.kind_[lane] = r.kind;
            }
            __syncthreads();
            if (S.kind_[j] != T_EXIT) first_term = j;
        }
    }
    out.start = g.base + r.start; out.end = g.base + r.end; out.cnt = r.cnt;
    out.kind = r.kind; out.reason = r.reason;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor((unsigned long long)x, o, 64);
    return x;
}
__device__ __forceinline__ uint64_t wave_excl_u64(uint64_t v, int lane) {
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up((unsigned long long)x, o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}

// Is b one of the header candidates (sorted list)?
__device__ __forceinline__ bool is_cand(const uint64_t* cands, uint32_t ncand, uint64_t b, uint32_t* idx = nullptr) {
    uint32_t lo = 0, hi = ncand;
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (cands[mid] < b) lo = mid + 1; else hi = mid; }
    if (idx) *idx = lo;
    return lo < ncand && cands[lo] == b;
}

// Next header candidate strictly after b (sorted list), capped at `limit`.
__device__ __forceinline__ uint64_t next_cand(const uint64_t* cands, uint32_t ncand, uint64_t b, uint64_t limit) {
    uint32_t lo = 0, hi = ncand;
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (cands[mid] <= b) lo = mid + 1; else hi = mid; }
    const uint64_t nx = lo < ncand ? cands[lo] : NONE;
    return min(nx, limit);
}

// Cursor over the sorted candidate list for one chain (wave-uniform): the chain's positions only
// grow, so the next candidate is kept in a register and advanced, instead of a binary search (15
// dependent loads) per round.  at(b) = is_cand (index = first candidate >= b); after(b) = next_cand.
struct CandCur {
    const uint64_t* c;
    uint32_t n, i;
    uint64_t v;
    __device__ __forceinline__ void init(const uint64_t* cands, uint32_t ncand, uint64_t b) {
        c = cands; n = ncand;
        uint32_t lo = 0, hi = n;
        while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (c[mid] < b) lo = mid + 1; else hi = mid; }
        i = lo;
        v = i < n ? c[i] : NONE;
    }
    __device__ __forceinline__ bool at(uint64_t b, uint32_t* idx) {
        while (v < b) { i++; v = i < n ? c[i] : NONE; }
        *idx = i;
        return v == b;
    }
    __device__ __forceinline__ uint64_t after(uint64_t b, uint64_t limit) {
        while (v <= b) { i++; v = i < n ? c[i] : NONE; }
        return min(v, limit);
    }
};

// ---- emit: write pass of one lane ---------------------------------------------------------------
// Literal bytes gather in a 64-bit register and leave as 4-byte stores (unaligned global stores are
// fine on gfx950); before a copy the pending 0..3 bytes go out as one 4-byte store whose spare bytes
// the copy (or, for a deferred copy, the resolve rounds) overwrites -- always the lane's own bytes.
// Copies move 8 or 4 bytes per load/store pair; the last chunk is stored overlapping so that no
// store reaches past the copy's end (the next lane's bytes).
typedef __attribute__((address_space(1))) uint8_t gu8;       // global (not flat) pointers
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

// NDFL_EMIT_NOSTORE (an A/B build, never the product): every output store and copy lands in the
// first 4 KiB of the output, so the emit pass runs its full decode with no write traffic to HBM
#ifdef NDFL_EMIT_NOSTORE
#define NDFL_OA(x) ((x) & 0xFFFull)
#else
#define NDFL_OA(x) (x)
#endif
// NDFL_EMIT_W16: completed literal words are held (up to 3) and leave as one 16-byte store, so a lane
// issues a quarter of the scattered stores (each store instruction of a wave touches 64 lines)
#ifndef NDFL_EMIT_W16
#define NDFL_EMIT_W16 1
#endif
#ifndef NDFL_EMIT_NT
#define NDFL_EMIT_NT 0          // (A/B: non-temporal 16-byte literal stores)
#endif
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4v gu128;
struct Wr {
    uint64_t acc;               // pending literal bytes (low byte first)
    uint32_t an;                // pending byte count (0..3 between tokens)
    uint64_t dst;               // output address of acc's first byte
#if NDFL_EMIT_W16
    uint32_t q0, q1, q2, hn;    // completed words held back (hn of them), at dst - 4 hn
#endif
};
__device__ __forceinline__ void wr_init(Wr& w, uint64_t dst) {
    w.acc = 0; w.an = 0; w.dst = dst;
#if NDFL_EMIT_W16
    w.q0 = 0; w.q1 = 0; w.q2 = 0; w.hn = 0;
#endif
}
// held words out (before a copy or at the end)
__device__ __forceinline__ void wr_drain(Wr& w, gu8* out) {
#if NDFL_EMIT_W16
    if (w.hn) {
        gu8* d = out + NDFL_OA(w.dst - 4 * w.hn);
        if (w.hn >= 2) *(gu64*)d = (uint64_t)w.q0 | ((uint64_t)w.q1 << 32);
        if (w.hn == 1) *(gu32*)d = w.q0;
        if (w.hn == 3) *(gu32*)(d + 8) = w.q2;
        w.hn = 0;
    }
#else
    (void)w; (void)out;
#endif
}
__device__ __forceinline__ void wr_lit(Wr& w, gu8* out, uint32_t val, uint32_t n) {
    w.acc |= (uint64_t)val << (8 * w.an);
    w.an += n;
    if (w.an >= 4) {
        const uint32_t word = (uint32_t)w.acc;
#if NDFL_EMIT_W16
        if (w.hn == 3) {
#if NDFL_EMIT_NT
            __builtin_nontemporal_store(u32x4v{w.q0, w.q1, w.q2, word}, (gu128*)(out + NDFL_OA(w.dst - 12)));
#else
            *(gu128*)(out + NDFL_OA(w.dst - 12)) = u32x4v{w.q0, w.q1, w.q2, word};
#endif
            w.hn = 0;
        } else {
            w.q0 = w.hn == 0 ? word : w.q0;
            w.q1 = w.hn == 1 ? word : w.q1;
            w.q2 = w.hn == 2 ? word : w.q2;
            w.hn++;
        }
#else
        *(gu32*)(out + NDFL_OA(w.dst)) = word;
#endif
        w.acc >>= 32;
        w.an -= 4;
        w.dst += 4;
    }
}
// pending bytes out before a copy at w.dst + w.an (which covers the store's spare bytes)
__device__ __forceinline__ void wr_flush_word(Wr& w, gu8* out) {
    wr_drain(w, out);
    if (w.an) {
        *(gu32*)(out + NDFL_OA(w.dst)) = (uint32_t)w.acc;
        w.dst += w.an;
        w.acc = 0;
        w.an = 0;
    }
}
// pending bytes out exactly (end of the lane's output)
__device__ __forceinline__ void wr_flush_exact(Wr& w, gu8* out) {
    wr_drain(w, out);
    for (uint32_t k = 0; k < w.an; k++) out[NDFL_OA(w.dst + k)] = (uint8_t)(w.acc >> (8 * k));
    w.dst += w.an;
    w.acc = 0;
    w.an = 0;
}
__device__ __forceinline__ uint64_t ld8(const gu8* p) { return *(const gu64*)p; }
__device__ __forceinline__ uint32_t ld4(const gu8* p) { return *(const gu32*)p; }
// out[dst, dst + len) = out[dst - dist, ...), byte-serial semantics; every source byte is final and
// this lane's own (or the window's).  `lastb` is the byte at dst - 1 (known to the lane: a dist-1
// run needs no read back) and is updated to the copy's last byte.
__device__ __forceinline__ void wr_copy(gu8* out, uint64_t dst, uint32_t len, uint32_t dist, uint32_t& lastb) {
    gu8* d = out + NDFL_OA(dst);
    const gu8* sp = out + NDFL_OA(dst - dist);
    if (dist == 1) {
        // a run: 16-byte stores (the last one overlapping back), so the wave's store loop takes
        // at most 17 trips for the longest run instead of 65
        const uint32_t v4 = lastb * 0x01010101u;
#if NDFL_EMIT_W16
        if (len >= 16) {
            const u32x4v x = {v4, v4, v4, v4};
            uint32_t k = 0;
            for (; k + 16 <= len; k += 16) *(gu128*)(d + k) = x;
            if (k < len) *(gu128*)(d + len - 16) = x;
            return;
        }
#endif
        if (len >= 4) {
            uint32_t k = 0;
            for (; k + 4 <= len; k += 4) *(gu32*)(d + k) = v4;
            if (k < len) *(gu32*)(d + len - 4) = v4;
        } else {
            for (uint32_t k = 0; k < len; k++) d[k] = (uint8_t)lastb;
        }
        return;
    }
#if NDFL_EMIT_W16
    if (dist >= 16 && len >= 16) {
        uint32_t k = 0;
        u32x4v x = {0, 0, 0, 0};
        for (; k + 16 <= len; k += 16) { x = *(const gu128*)(sp + k); *(gu128*)(d + k) = x; }
        if (k < len) { x = *(const gu128*)(sp + len - 16); *(gu128*)(d + len - 16) = x; }
        lastb = x.w >> 24;
        return;
    }
#endif
    if (dist >= 8 && len >= 8) {
        uint32_t k = 0;
        uint64_t x = 0;
        for (; k + 8 <= len; k += 8) { x = ld8(sp + k); *(gu64*)(d + k) = x; }
        if (k < len) { x = ld8(sp + len - 8); *(gu64*)(d + len - 8) = x; }
        lastb = (uint32_t)(x >> 56);
        return;
    }
    if (dist >= 4 && len >= 4) {
        uint32_t k = 0, x = 0;
        for (; k + 4 <= len; k += 4) { x = ld4(sp + k); *(gu32*)(d + k) = x; }
        if (k < len) { x = ld4(sp + len - 4); *(gu32*)(d + len - 4) = x; }
        lastb = x >> 24;
        return;
    }
    uint32_t b = lastb;
    for (uint32_t k = 0; k < len; k++) { b = sp[k]; d[k] = (uint8_t)b; }
    lastb = b;
}

}  // namespace wv

// Header records: one lane per header candidate parses it (the count pass's lane-0 parse, which
// leaves 63 lanes idle through a chain of dependent loads, becomes a load of 336 bytes).
extern "C" __global__ void __launch_bounds__(64)
ndfl_inflate_hdr_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* cands, uint32_t ncand,
                        wv::HdrRec* rec, uint32_t* flat_list, uint32_t* nflat, uint32_t* flat_flag) {
    using namespace wv;
    __shared__ __attribute__((aligned(16))) uint32_t lens[64][80];
    __shared__ uint16_t clt[64][128];
    __shared__ uint32_t win[8 * 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x * 64 + lane;
    if (k >= ncand) return;                     // (no barrier below)
    const In in{w, nwords, nbits};
    for (uint32_t q = 0; q < 80; q++) lens[lane][q] = 0;
    const uint64_t p = cands[k];
    Hdr h;
    parse_hdr_core<RdWin>(in, p, (uint8_t*)lens[lane], clt[lane], h, win + lane);
    HdrRec* r = rec + k;
    for (uint32_t q = 0; q < 80; q += 4)
        *(uint4*)&r->lens[q] = make_uint4(lens[lane][q], lens[lane][q + 1], lens[lane][q + 2], lens[lane][q + 3]);
    r->h = h;
    r->at = p;
    // escape-prefix literal code (count_flat_group): no code shorter than 8 bits, every 8-bit code a
    // literal, 256 - 2^k of them (k <= 2) -- the other 2^k prefixes lead to the longer codes
    uint32_t c8 = 0;
    bool bad = false;
    for (uint32_t q = 0; q < 72; q++) {
        const uint32_t v = lens[lane][q];
#pragma unroll
        for (uint32_t b = 0; b < 4; b++) {
            const uint32_t l = (v >> (8 * b)) & 0xFFu;
            c8 += l == 8 ? 1u : 0u;
            bad = bad || (l - 1u < 7u) || (l == 8 && q >= 64);
        }
    }
    const uint32_t esc = 256u - min(c8, 256u);
    const uint32_t kk = esc == 1 ? 1u : esc == 2 ? 2u : esc == 4 ? 3u : 0u;
    r->flat = (flat_list && h.err == 0 && h.btype == 2 && !bad) ? kk : 0u;
    r->pad = 0;
    if (flat_flag) flat_flag[k] = r->flat;
    if (flat_list) {                            // (wave-aggregated append)
        const uint64_t m = __ballot(r->flat != 0);
        uint32_t b = 0;
        if (lane == 0 && m) b = atomicAdd(nflat, (uint32_t)__popcll(m));
        b = __shfl(b, 0, 64);
        if (r->flat) flat_list[b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = k;
    }
}

// Count pass: persistent waves, each claiming candidate chains through `ticket`; the phase-fallback
// arrays live in the wave's own global slot (ph_all[blockIdx.x]); LDS holds the tables and the
// round's staged input.
#ifndef NDFL_COUNT_WPE
#define NDFL_COUNT_WPE 3
#endif
#ifndef NDFL_REC_BATCH
#define NDFL_REC_BATCH 16       // round records claimed per atomic (the pool keeps 65,536 spare)
#endif
#ifndef NDFL_TREC_BATCH
#define NDFL_TREC_BATCH 4       // table records claimed per atomic
#endif
namespace wv {
// ---- escape-prefix literal blocks, one lane per block (round 6) ------------------------------------
// What DEFLATE encoders produce for incompressible data: a literal/length code of 255 literals of 8
// bits (254, 252: 2^k prefixes left) with the few longer codes -- end of block, a rare literal or
// length -- under the remaining all-ones prefix.  In wave form that is the count pass's costliest case:
// the codes never resynchronise from a wrong bit phase, so every round decodes all 8 phases
// (round_decode_phased, ~1.2 ms of wave time per 64 KiB block, a quarter of the pass on the bench
// corpus).  Decoded serially by ONE lane it needs no speculation at all, and "is any of the next 8
// bytes an escape prefix" covers 8 tokens in a few VALU operations.  A wave takes up to 64 such chains
// (a flat group; ndfl_inflate_hdr_kernel lists them), builds each block's tables and table record in
// turn as usual, keeps per lane a 64-entry escape table (the code under the prefix, from the next 6
// bits), and then every lane decodes its own block, writing exactly the round records the wave decode
// would write (the same round geometry; each lane segment from the first token boundary at or past
// its nominal start -- the emit passes check every one) and the chain's result.  Whatever it cannot
// finish this way -- an error, the input's end, a chain that continues past its first block, more
// than NDFL_FLAT_OTHER_MAX tokens that need the full tables -- goes back to the wave decode, from the
// chain's start.
#ifndef NDFL_FLAT_OTHER_MAX
#define NDFL_FLAT_OTHER_MAX 64          // tokens per block decoded through the global table record
#endif
#ifndef NDFL_FLAT_K
#define NDFL_FLAT_K 4                   // steps between the input rings' phase points
#endif
#ifndef NDFL_FLAT_PRIO
#define NDFL_FLAT_PRIO 1                // the group's decode at raised wave priority (s_setprio 3)
#endif
#ifdef NDFL_FLAT_PROF
__device__ unsigned long long g_flat_prof[4];
#endif
constexpr uint32_t FLAT_ESC_WORD = 64;  // escape tables in the stage from this word (the build's scratch below)
static_assert(FLAT_ESC_WORD + 64 * 64 / 4 <= SW * 64, "flat escape tables in the stage");

// escape entry for the stream bits x following a block's all-ones (8 - kk)-bit prefix: code length |
// kind << 4 (kind 0 a literal, 1 end of block), or 0 (a length code, a reserved symbol, a code longer
// than the 6 bits cover: the full tables decide)
__device__ __forceinline__ uint32_t flat_esc_entry(const TabsG& t, uint32_t kk, uint32_t x) {
    const uint32_t pl = 8 - kk;
    const uint32_t w = ((1u << pl) - 1u) | (x << pl);
    uint32_t e = t.lit[w & ((1u << LB) - 1u)];
    uint32_t len, kind;
    if (e >> 31) {                                  // a single literal (no pair: the code has >= 9 bits)
        len = e & 15; kind = 0;
    } else {
        if (!(e & 31)) e = long_lit(e, w, t);
        len = e & 31;
        const uint32_t k = (e >> 9) & 3;
        kind = k == K_LIT ? 0u : k == K_EOB ? 1u : 2u;
    }
    return (kind < 2 && len > pl && len <= pl + 6) ? (len | (kind << 4)) : 0u;
}

// One flat group (flist[0, n), n <= 64).  Returns the number of chains left to the wave decode, listed
// in redo[] (LDS).  All lanes call.
__device__ __forceinline__ uint32_t count_flat_group(const In& in, const uint32_t* flist, uint32_t n,
                                                     const uint64_t* cands, uint32_t ncand, uint64_t limit,
                                                     uint64_t stop_all, ChainRes* res, const SegPool& pool,
                                                     const HdrRec* hrec, Shared& S, uint32_t* stw, int lane,
                                                     uint32_t* redo, uint32_t& tb_next, uint32_t& tb_end,
                                                     uint32_t* whys) {
    lu8* escs = (lu8*)((lu32*)stw + FLAT_ESC_WORD);        // lane j's entries at escs[j * 64]
    // 1. the blocks' tables one after the other; lane k keeps block k's fields
    uint32_t my_c = 0, my_brec = NOREC, my_kk = 0;
    uint64_t my_d0 = 0;
    bool my_ok = false, my_final = false, my_ed = false;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t c = flist[k];
        const HdrRec* hr = hrec + c;
        uint32_t* lw = (uint32_t*)S.lens;
        lw[lane] = hr->lens[lane];
        if (lane < 16) lw[64 + lane] = hr->lens[64 + lane];
        if (lane == 0) hdr_to_shared(hr->h, S);
        const uint32_t kk = hr->flat - 1u;
        __syncthreads();
        bool ed;
        const int te = build_tables(S, lane, ed, stw);
        uint32_t brec = NOREC;
        if (!te) {
            if (c < pool.nslot && pool.nbt) {
                if (tb_next >= tb_end) {
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(pool.bctr, (uint32_t)NDFL_TREC_BATCH);
                    b = __builtin_amdgcn_readfirstlane(b);
                    tb_next = b; tb_end = b + NDFL_TREC_BATCH;
                }
                brec = tb_next++;
                if (brec < pool.nbt) {
                    uint4* dst = (uint4*)(pool.bt + (uint64_t)brec * BT_BYTES);
                    const uint4* src = (const uint4*)&S.t;
                    for (uint32_t q = (uint32_t)lane; q < sizeof(Tabs) / 16; q += 64) dst[q] = src[q];
                    if (lane == 0) {
                        uint64_t* h = (uint64_t*)(pool.bt + (uint64_t)brec * BT_BYTES + sizeof(Tabs));
                        h[0] = cands[c]; h[1] = S.h_d0;
                        uint32_t* h32 = (uint32_t*)(h + 2);
                        h32[0] = S.h_bfinal; h32[1] = S.h_btype; h32[2] = ed ? 1u : 0u;
                        h32[3] = ((1u << (8 - kk)) - 1u) * 0x01010101u;    // (the escape prefix mask)
                    }
                } else {
                    brec = NOREC;
                }
            }
            const TabsG tg{S.t.lit, S.t.dst, S.t.lx, S.t.dx};
            escs[k * 64 + lane] = (uint8_t)flat_esc_entry(tg, kk, (uint32_t)lane);
        }
        if ((uint32_t)lane == k) {
            my_c = c; my_ok = !te; my_d0 = S.h_d0; my_final = S.h_bfinal != 0; my_ed = ed; my_brec = brec; my_kk = kk;
        }
        __syncthreads();                        // (the next block's header and tables overwrite these)
    }
    // 2. the rounds each block needs, claimed for the group at once: a round covers MAX_SPAN bits
    // unless a header candidate ends it first (+1: the last round may end past the next candidate)
    const bool active = (uint32_t)lane < n && my_ok;
    uint32_t ci = my_c;
    uint64_t cv = active ? cands[ci] : NONE;
    auto after = [&](uint64_t b) {
        while (cv <= b) { ci++; cv = ci < ncand ? cands[ci] : NONE; }
        return min(cv, limit);
    };
    uint32_t nr = 0;
    if (active) {
        const uint64_t e0 = after(my_d0);
        nr = (uint32_t)min<uint64_t>((e0 > my_d0 ? (e0 - my_d0 + MAX_SPAN - 1) / MAX_SPAN : 1) + 1, 1024);
    }
    // the next candidates after the first (a false candidate inside the block ends a round early;
    // loaded here, not in the loop)
    uint64_t cv1 = NONE, cv2 = NONE, cv3 = NONE;
    if (active) {
        cv1 = ci + 1 < ncand ? cands[ci + 1] : NONE;
        cv2 = ci + 2 < ncand ? cands[ci + 2] : NONE;
        cv3 = ci + 3 < ncand ? cands[ci + 3] : NONE;
    }
    const uint32_t rpre = (uint32_t)wave_excl_u64(nr, lane), rtot = (uint32_t)wave_sum_u64(nr);
    uint32_t rb = 0;
    if (lane == 0 && rtot) rb = atomicAdd(pool.ctr, rtot);
    rb = __builtin_amdgcn_readfirstlane(rb);
    // 3. every lane decodes its block alone.  A step is a token (up to 8 literals), a segment switch,
    // or a round's start or end.  The input comes through a ring of 24 words per lane in LDS, in the
    // tables' place (three slots of 8 words; word row r of lane j at ring[r * 64 + j]: no bank
    // conflicts), refilled at phase points every FLAT_K steps, all lanes at once: a lane that left its
    // oldest slot writes the next slot's words, loaded into registers at the previous phase point, and
    // loads the slot after.  Those registers are touched at phase points only -- a lane refilling while
    // the others step made the wave wait for the newest load at every step (8 ms per group).
    bool ok = false;
    uint64_t total = 0, endpos = 0;
    uint32_t status = ST_BOUNDARY, next_idx = 0xFFFFFFFFu, why = active ? 4u : 5u;   // (why a chain goes back)
    if (active) {
        const uint32_t pl = 8 - my_kk, M4 = ((1u << pl) - 1u) * 0x01010101u;
        bool recording = my_c < pool.nslot;
        uint32_t rnext = rb + rpre, rlast = rnext + nr;
        uint32_t brec = my_brec, others = 0;
        // positions relative to an origin at a multiple of 8 words before the block's data (u32)
        const uint64_t o64 = (my_d0 >> 8) << 8;
        const uint64_t og4 = o64 >> 7;                  // (its 16-byte group)
        const uint32_t nbo = (uint32_t)min<uint64_t>(in.nbits - min(in.nbits, o64), 0xFFFFFF00ull);
        uint32_t pos = (uint32_t)(my_d0 - o64);
        lu32* ring = (lu32*)&S.t + lane;
        uint32_t fw = (pos >> 5) & ~7u;                 // the ring holds words [fw - 24, fw)
#pragma unroll
        for (uint32_t i = 0; i < 24; i += 4) {
            const u32x4 v = in.ld4(og4 + ((fw + i) >> 2));
            ring[i * 64] = v.x; ring[(i + 1) * 64] = v.y; ring[(i + 2) * 64] = v.z; ring[(i + 3) * 64] = v.w;
        }
        fw += 24;
        uint32_t frow = 0;                              // the ring row of word fw
        u32x4 ra = in.ld4(og4 + (fw >> 2)), rb = in.ld4(og4 + (fw >> 2) + 1);
        // the round [rs, E) in the wave decode's geometry (make_geo, lane_seg); segment j: the tokens
        // starting in [s_j, s_{j+1}) (s_0 = r0, s_64 = re), relative to the round's word-aligned base
        uint32_t base = 0, r0 = 0, re = 0, per = 0, pw = 0, nbr = 0, idx = NOREC, j = 0, p = 0, jst = 0, bytes = 0, sn = 0;
        uint64_t* ps = nullptr;                         // the round record's starts and counts, its meta
        uint32_t* pc = nullptr;
        uint4* mq = nullptr;
        uint32_t* link = pool.head + my_c;              // where the next round record's index goes
        uint32_t st = 0;                                // 0 a round starts at pos, 1 in a round, 2 EOB, 3 back
        // the group is the pass's longest job: it takes the SIMD's issue slots first
        if (NDFL_FLAT_PRIO) __builtin_amdgcn_s_setprio(3);
        // the round's records: segment j ends the block (EOB) or the round (j = 63)
        auto end_round = [&](bool eob) {
            if (ps) {
                const uint64_t ex = o64 + base + p;
                ps[j] = o64 + base + jst;
                pc[j] = bytes;
                for (uint32_t jj = j + 1; jj < 64; jj++) { ps[jj] = ex; pc[jj] = 0; }
                // (the fields as two 16-byte and one 8-byte stores of values at hand: a SegMeta built in
                // registers was partly spilled, and its reload waited for the rings' loads in flight)
                uint32_t kf = eob ? (uint32_t)T_EOB : (uint32_t)T_EXIT;
                asm volatile("" : "+v"(kf));            // (materialised here, not a spilled constant)
                mq[0] = make_uint4(eob ? j : 64u, kf, 0u, NOREC);
                mq[1] = make_uint4((uint32_t)ex, (uint32_t)(ex >> 32), (uint32_t)ex, (uint32_t)(ex >> 32));
                *(uint2*)(mq + 2) = make_uint2(pw, brec);
                *(uint64_t*)((uint2*)(mq + 2) + 1) = o64 + base + r0;
                *link = idx;                            // (the chain's head, then the previous round's next)
                link = (uint32_t*)mq + 3;
                brec = NOREC;                           // (only the block's first round names its tables)
            }
            total += bytes;
            pos = base + p;
        };
        // segment j's record, and the next segment's start
        auto next_seg = [&]() {
            if (ps) { ps[j] = o64 + base + jst; pc[j] = bytes; }
            total += bytes;
            j++; jst = p; bytes = 0;
            sn = j < 63 ? min(r0 + (j + 1) * per, re) : re;
        };
#ifdef NDFL_FLAT_PROF
        unsigned long long fp_ph = 0, fp_t0 = clock64(), fp_n = 0;
#endif
        while (st < 2) {
            {   // phase point
#ifdef NDFL_FLAT_PROF
                const unsigned long long fp_a = clock64();
#endif
                const uint32_t cw = (st == 1 ? base + p : pos) >> 5;
                if (cw + 16 >= fw) {
                    ring[frow * 64] = ra.x; ring[(frow + 1) * 64] = ra.y; ring[(frow + 2) * 64] = ra.z;
                    ring[(frow + 3) * 64] = ra.w; ring[(frow + 4) * 64] = rb.x; ring[(frow + 5) * 64] = rb.y;
                    ring[(frow + 6) * 64] = rb.z; ring[(frow + 7) * 64] = rb.w;
                    fw += 8;
                    frow = frow == 16 ? 0u : frow + 8;
                    ra = in.ld4(og4 + (fw >> 2)); rb = in.ld4(og4 + (fw >> 2) + 1);
                }
#ifdef NDFL_FLAT_PROF
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                fp_ph += clock64() - fp_a;
                fp_n++;
#endif
            }
            for (uint32_t k = 0; k < NDFL_FLAT_K && st < 2; k++) {
                if (st == 0) {
                    const uint64_t rsa = o64 + pos;
                    // (the next candidate was loaded before the loop; a round passing it -- a candidate
                    // inside the block -- goes back to the wave decode: a load here would make every
                    // round start wait for the rings' loads in flight)
                    if (cv <= rsa) { cv = cv1; cv1 = cv2; cv2 = cv3; cv3 = NONE; ci++; }
                    if (cv <= rsa) {                    // (rare: more false candidates in the block)
                        while (cv <= rsa) { ci++; cv = ci < ncand ? cands[ci] : NONE; }
                        cv1 = ci + 1 < ncand ? cands[ci + 1] : NONE;
                        cv2 = ci + 2 < ncand ? cands[ci + 2] : NONE;
                        cv3 = ci + 3 < ncand ? cands[ci + 3] : NONE;
                    }
                    uint64_t E = min(min(cv, limit), rsa + MAX_SPAN);
                    if (E <= rsa) E = rsa + 1;
                    base = pos & ~31u;
                    r0 = pos - base; re = (uint32_t)(E - o64) - base;
                    pw = max((uint32_t)NDFL_PW_MIN, ((re - r0 + 63) / 64 + 31) / 32); per = pw * 32;
                    nbr = nbo - min(nbo, base);
                    idx = NOREC;
                    if (recording) {
                        if (rnext >= rlast) {           // (a header candidate inside the block: more rounds)
                            rnext = atomicAdd(pool.ctr, 8u);
                            rlast = rnext + 8;
                        }
                        if (rnext < pool.nrec) idx = rnext++;
                        else recording = false;
                    }
                    ps = idx != NOREC ? pool.start + (uint64_t)idx * 64 : nullptr;
                    pc = idx != NOREC ? pool.cnt + (uint64_t)idx * 64 : nullptr;
                    mq = idx != NOREC ? (uint4*)(pool.meta + idx) : nullptr;
                    j = 0; p = r0; jst = r0; bytes = 0;
                    sn = min(r0 + per, re);
                    st = 1;                             // (and the round's first step at once)
                }
                if (st != 1) continue;
                // One step, branch-free on its common path (a divergent branch per case made every step
                // pay for the cases of the other 63 lanes): a token (up to 8 literals, or one escape
                // literal) when the lane stands before its segment's end and the ring holds its window,
                // then the segment switch if the lane has reached the end.  End of block, the round's
                // end and the full-table tokens branch.
                const uint32_t ap = base + p, cw = ap >> 5;
                const bool tk_ok = p < sn && cw + 2 < fw;
                uint32_t rr0 = frow + 24 - min(fw - cw, 24u);
                rr0 = rr0 >= 24 ? rr0 - 24 : rr0;
                const uint32_t rr1 = rr0 == 23 ? 0u : rr0 + 1, rr2 = rr1 == 23 ? 0u : rr1 + 1;
                const uint32_t w0 = ring[rr0 * 64], w1 = ring[rr1 * 64], w2 = ring[rr2 * 64];
                const uint32_t sh = ap & 31u;
                const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh), hi = __builtin_amdgcn_alignbit(w2, w1, sh);
                // (the escape entry read at once, whether needed or not: its latency overlaps the scan;
                // the lane index recomputed: a value kept from outside the loop was spilled, and its
                // reload waited for the rings' loads in flight)
                uint32_t ln;
                asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
                const uint32_t ent = escs[ln * 64 + ((lo >> pl) & 63u)], len = ent & 15u;
                const uint32_t q = (sn - min(sn, p) + 7) >> 3, qi = (nbr - min(nbr, p)) >> 3;
                const uint32_t t = tk_ok ? min(min(esc_index(lo, hi, M4), q), qi) : 0u;
                const bool esc = tk_ok && t == 0 && (lo & (M4 & 0xFFu)) == (M4 & 0xFFu) && ent && p + len <= nbr;
                const bool eob = esc && (ent >> 4);
                p += t ? 8 * t : esc ? len : 0u;
                bytes += t ? t : (esc && !eob) ? 1u : 0u;
                bool ended = eob;                       // (the block, a full-table error or the round)
                if (tk_ok && t == 0 && !esc) {
                    // through the block's full tables (global table record)
                    if (my_brec == NOREC || ++others > NDFL_FLAT_OTHER_MAX) {
                        st = 3; why = 2;
                    } else {
                        const uint32_t* tb = (const uint32_t*)(pool.bt + (uint64_t)my_brec * BT_BYTES);
                        const TabsG tg{tb, tb + (1u << LB), tb + offsetof(Tabs, lx) / 4, tb + offsetof(Tabs, dx) / 4};
                        uint32_t pp = 0;
                        Tok tk;
                        tok_e<true>(lo, hi, tg.lit[lo & ((1u << LB) - 1u)], pp, tg, my_ed, sn - p, nbr - min(nbr, p), tk);
                        if (tk.kind == K_LIT || tk.kind == K_LEN) bytes += tk.n;
                        else if (tk.kind == K_EOB) ended = true;
                        else { st = 3; why = 3; }
                        p += pp;
                    }
                    ended = ended || st == 3;
                }
                // the token(s) started before sn: a segment (or the round) ends at the first boundary
                // past it (an empty segment at a round's end switches without a token)
                const bool rend = !ended && p >= sn && j == 63;
                if (ended || rend) {
                    if (st != 3) { end_round(!rend); st = rend ? 0u : 2u; }
                } else {
                    const bool sw = p >= sn;
                    if (sw && ps) { ps[j] = o64 + base + jst; pc[j] = bytes; }
                    total += sw ? bytes : 0u;
                    j += sw ? 1u : 0u;
                    jst = sw ? p : jst;
                    bytes = sw ? 0u : bytes;
                    sn = sw ? (j < 63 ? min(r0 + (j + 1) * per, re) : re) : sn;
                }
            }
        }
        if (NDFL_FLAT_PRIO) __builtin_amdgcn_s_setprio(0);
#ifdef NDFL_FLAT_PROF
        if (lane == 0) {       // (lane 0's view: its loop cycles, of them at phase points, phase points)
            atomicAdd(&g_flat_prof[0], clock64() - fp_t0); atomicAdd(&g_flat_prof[1], fp_ph); atomicAdd(&g_flat_prof[2], fp_n);
        }
#endif
        if (st == 2) {
            // the chain's end: the final block, or a header candidate (or the range end) next
            const uint64_t cur = o64 + pos;
            if (my_final) { status = ST_FINAL; endpos = cur; ok = true; }
            else if (cur >= stop_all) { status = ST_BOUNDARY; endpos = cur; ok = true; }
            else {
                while (cv < cur) { ci++; cv = ci < ncand ? cands[ci] : NONE; }
                next_idx = ci;
                if (cv == cur) { status = ST_BOUNDARY; endpos = cur; ok = true; }
            }
        }
    }
    if (ok) {
        ChainRes o;
        o.end_bit = endpos; o.out_count = total; o.status = status; o.reason = 0; o.next = next_idx; o.pad = 0;
        o.bnd_bit = 0; o.bnd_cnt = 0;
        res[my_c] = o;
    }
    // 4. the rest back to the wave decode
    const bool rd = (uint32_t)lane < n && !ok;
    if (whys && rd) atomicAdd(&whys[why], 1u);
    const uint64_t rm = __ballot(rd);
    if (rd) redo[__popcll(rm & ((1ull << lane) - 1ull))] = my_c;
    __syncthreads();
    return (uint32_t)__popcll(rm);
}
}  // namespace wv

extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NDFL_COUNT_WPE)))
ndfl_inflate_count_wave_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* starts,
                               const uint64_t* stops, uint32_t nchains, const uint64_t* cands, uint32_t ncand,
                               uint64_t limit, ChainRes* res, uint32_t* stats, uint64_t slot_base, SegPool pool,
                               uint32_t* ticket, wv::PhArr* ph_all, const uint32_t* order, uint64_t stop_all,
                               const wv::HdrRec* hrec, const uint32_t* nord, const uint32_t* flist,
                               const uint32_t* nflat) {
    using namespace wv;
    __shared__ __attribute__((aligned(16))) Shared S;
    if (nord) nchains = *nord;                  // (stored-header aliases and flat chains left out of the order)
    __shared__ Stage stg;
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_redo[64];             // a flat group's chains left to the wave decode
    const int lane = threadIdx.x;
    PhArr* ph = ph_all + blockIdx.x;
    const In in{w, nwords, nbits};
    const uint64_t t_begin = stats ? wall_clock64() : 0;
    // round and table records are claimed in batches per wave (one contended atomic per batch
    // instead of one per round; unused slots of a batch stay unused)
    uint32_t rb_next = 0, rb_end = 0, tb_next = 0, tb_end = 0;
    // tickets [0, ngroups) are flat groups of up to 64 chains (count_flat_group), the rest index order[]
    const uint32_t nfl = (nflat && hrec && slot_base == 0) ? *nflat : 0u, ngroups = (nfl + 63) / 64;
    uint32_t nredo = 0;
    for (;;) {
    uint32_t c;
    if (nredo) {
        c = s_redo[--nredo];
    } else {
        __syncthreads();
        if (lane == 0) s_ticket = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t tk = s_ticket;
        if (tk >= ngroups + nchains) break;
        if (tk < ngroups) {
            const uint32_t g0 = tk * 64;
            const uint64_t tf0 = stats ? wall_clock64() : 0;
            nredo = count_flat_group(in, flist + g0, min(64u, nfl - g0), cands, ncand, limit, stop_all, res, pool, hrec,
                                     S, stg.w, lane, s_redo, tb_next, tb_end, stats ? ticket + 10 : nullptr);
            if (stats && lane == 0) {                   // (ticket words 5, 6: chains sent back, group wave time)
                atomicAdd(ticket + 5, nredo);
                atomicAdd((unsigned long long*)(ticket + 6), (unsigned long long)(wall_clock64() - tf0));
            }
            continue;
        }
        c = order[tk - ngroups];
    }
    const uint64_t start = starts[c], stop = stops ? stops[c] : stop_all;
    uint64_t cur = start, total = 0, endpos = start;
    uint32_t status = ST_BOUNDARY, reason = 0, nslow = 0, nfix = 0, nround = 0, next_idx = 0xFFFFFFFFu;
    bool recording = slot_base + c < pool.nslot;
    uint32_t prev_rec = NOREC;
    PhaseClock pcl = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef NDFL_PHASE_CLOCK
    PhaseClock* pc = stats ? &pcl : nullptr;     // costs registers: build with -DNDFL_PHASE_CLOCK to profile
#else
    PhaseClock* pc = nullptr;
#endif
    uint64_t tb = pc ? wall_clock64() : 0;
    const uint64_t t_chain = stats ? wall_clock64() : 0;
    CandCur cc;
    if (slot_base == 0 && c < ncand) {          // the first pass: chain c starts at candidate c (no search)
        cc.c = cands; cc.n = ncand; cc.i = c; cc.v = cands[c];
    } else {
        cc.init(cands, ncand, start);
    }
    uint32_t nblk = 0;
    for (int blk = 0;; blk++) {
        nblk = (uint32_t)blk;
        // a chain ends at the first later block boundary that is itself a header candidate (its own
        // chain links on from there) or at the range end; false candidates are passed over
        if (blk > 0 && (cur >= stop || cc.at(cur, &next_idx))) { status = ST_BOUNDARY; endpos = cur; break; }
        if (hrec && blk == 0 && cc.i < cc.n && cc.v == cur) {
            // the chain starts at a header candidate: its parse is in the header records
            const HdrRec* hr = hrec + cc.i;
            uint32_t* lw = (uint32_t*)S.lens;
            lw[lane] = hr->lens[lane];
            if (lane < 16) lw[64 + lane] = hr->lens[64 + lane];
            if (lane == 0) hdr_to_shared(hr->h, S);
            __syncthreads();
        } else {
            for (uint32_t s = (uint32_t)lane; s < 320; s += 64) S.lens[s] = 0;
            __syncthreads();
            if (lane == 0) parse_hdr(in, cur, S);
            __syncthreads();
        }
        if (S.h_err) { status = ST_ERROR; reason = S.h_err; endpos = S.h_pos; break; }
        const uint64_t d0 = S.h_d0;
        const bool bfinal = S.h_bfinal != 0;
        if (S.h_btype == 0) {
            const uint64_t avail = (nbits - d0) / 8, ln = S.h_len;
            if (avail < ln) { total += avail; status = ST_ERROR; reason = R_UEOS; endpos = d0 + 8 * avail; break; }
            total += ln;
            cur = d0 + 8 * ln;
            if (bfinal) { status = ST_FINAL; endpos = cur; break; }
            continue;
        }
        bool ed;
        if (pc) { const uint64_t x = wall_clock64(); pc->hdr += x - tb; tb = x; }
        const int te = build_tables(S, lane, ed, stg.w);
        if (te) { status = ST_ERROR; reason = (uint32_t)te; endpos = d0; break; }
        // literal/length codes mostly of one length 8 resynchronise rarely: phase-mapped rounds
        bool phased = false;
        uint32_t esc4 = 0;
        {
            uint32_t n8 = 0;
            for (uint32_t q = 0; q < 5; q++) {
                const uint32_t sy = q * 64 + (uint32_t)lane;
                n8 += (uint32_t)__popcll(__ballot(sy < 288 && S.lens[sy] == 8));
            }
            phased = n8 >= 192;
            if (phased && NDFL_PHASE_ESC) esc4 = flat8_mask(S.t, lane);
        }
        // the block's tables and header fields for the emit pass (a table record)
        uint32_t brec = NOREC;
        if (recording && pool.nbt) {
            if (tb_next >= tb_end) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(pool.bctr, (uint32_t)NDFL_TREC_BATCH);
                b = __builtin_amdgcn_readfirstlane(b);
                tb_next = b; tb_end = b + NDFL_TREC_BATCH;
            }
            brec = tb_next++;
            if (brec < pool.nbt) {
                uint4* dst = (uint4*)(pool.bt + (uint64_t)brec * BT_BYTES);
                const uint4* src = (const uint4*)&S.t;
                for (uint32_t q = (uint32_t)lane; q < sizeof(Tabs) / 16; q += 64) dst[q] = src[q];
                if (lane == 0) {
                    uint64_t* h = (uint64_t*)(pool.bt + (uint64_t)brec * BT_BYTES + sizeof(Tabs));
                    h[0] = cur; h[1] = d0;
                    uint32_t* h32 = (uint32_t*)(h + 2);
                    h32[0] = S.h_bfinal; h32[1] = S.h_btype; h32[2] = ed ? 1u : 0u;
                    h32[3] = phased ? (esc4 ? esc4 : 1u) : 0u;      // (emit: 4-literal steps / escape scan)
                }
            } else {
                brec = NOREC;
            }
        }
        if (pc) { const uint64_t x = wall_clock64(); pc->build += x - tb; tb = x; }
        uint64_t rs = d0;
        bool block_done = false, chain_done = false;
        while (!block_done) {
            uint64_t E = min(cc.after(rs, limit), rs + MAX_SPAN);
            if (E <= rs) E = rs + 1;
            Seg r;
            uint32_t ft;
            Geo g;
            if (phased) {
                const uint64_t t0p = pc ? wall_clock64() : 0;
                round_decode_phased(in, S.t, ed, rs, E, S, stg, lane, r, ft, nfix, g, esc4);
                if (pc) pc->phmap += wall_clock64() - t0p;
            } else {
                const uint32_t ns0 = nslow;
                round_decode(in, S.t, ed, rs, E, S, stg, lane, r, ft, nslow, nfix, ph, g, pc);
                if (nslow - ns0 > NDFL_PHASE_SWITCH) phased = true;    // phase-locked code: map the next rounds
            }
            if (pc) tb = wall_clock64();
            if (recording) {
                // record the exact segments of this round (and its geometry) for the emit pass
                const bool live = (uint32_t)lane <= ft;
                uint32_t idx = NOREC;
                if (__all(!live || r.cnt < 0xFFFFFFFFull)) {
                    if (rb_next >= rb_end) {
                        uint32_t b = 0;
                        if (lane == 0) b = atomicAdd(pool.ctr, (uint32_t)NDFL_REC_BATCH);
                        b = __builtin_amdgcn_readfirstlane(b);
                        rb_next = b; rb_end = b + NDFL_REC_BATCH;
                    }
                    idx = rb_next++;
                }
                if (idx < pool.nrec) {
                    pool.start[(uint64_t)idx * 64 + lane] = r.start;
                    pool.cnt[(uint64_t)idx * 64 + lane] = (uint32_t)r.cnt;
                    const int src = ft < 64 ? (int)ft : 63;
                    const uint64_t fe = __shfl((unsigned long long)r.end, src, 64);
                    const uint32_t fk = __shfl(r.kind, src, 64), fr = __shfl(r.reason, src, 64);
                    if (lane == 0) {
                        SegMeta m;
                        m.ft = ft; m.kind_ft = fk; m.reason_ft = fr; m.next = NOREC;
                        m.end_ft = fe; m.exit63 = fe; m.pw = g.pw; m.pad = brec; m.rs = g.base + g.r0;
                        pool.meta[idx] = m;
                        if (prev_rec == NOREC) pool.head[slot_base + c] = idx;
                        else pool.meta[prev_rec].next = idx;
                    }
                    prev_rec = idx;
                    brec = NOREC;               // (only the block's first round names its tables)
                } else {
                    recording = false;          // the emit pass re-derives the remaining rounds
                }
            }
            nround++;
            if (pc) { const uint64_t x = wall_clock64(); pc->rec += x - tb; tb = x; }
            total += wave_sum_u64((uint32_t)lane <= ft ? r.cnt : 0ull);
            if (ft < 64) {
                const uint64_t fe = __shfl((unsigned long long)r.end, (int)ft, 64);
                const uint32_t fk = __shfl(r.kind, (int)ft, 64), fr = __shfl(r.reason, (int)ft, 64);
                block_done = true;
                if (fk == T_ERR) { status = ST_ERROR; reason = fr; endpos = fe; chain_done = true; }
                else {
                    cur = fe;
                    if (bfinal) { status = ST_FINAL; endpos = cur; chain_done = true; }
                }
            } else {
                rs = __shfl((unsigned long long)r.end, 63, 64);
            }
        }
        if (chain_done) break;
    }
    if (lane == 0) {
        ChainRes o;
        o.end_bit = endpos; o.out_count = total; o.status = status; o.reason = reason;
        o.next = next_idx;
        // NDFL_STATS: the chain's wave time (10 us units, 16 bits) and blocks (16 bits)
        o.pad = stats ? (min((uint32_t)((wall_clock64() - t_chain) / 1000), 0xFFFFu) << 16) | min(nblk + 1, 0xFFFFu) : 0u;
        o.bnd_bit = 0; o.bnd_cnt = 0;
        res[c] = o;
        if (stats) {
            atomicAdd(&stats[0], nslow); atomicAdd(&stats[1], nfix); atomicAdd(&stats[2], nround);
            unsigned long long* st64 = (unsigned long long*)(stats + 32);
            atomicAdd(&st64[0], pcl.hdr); atomicAdd(&st64[1], pcl.spec); atomicAdd(&st64[2], pcl.verify);
            atomicAdd(&st64[3], pcl.phases); atomicAdd(&st64[4], pcl.serial); atomicAdd(&st64[5], pcl.rec);
            atomicAdd(&st64[6], pcl.build); atomicAdd(&st64[7], pcl.phmap);
            atomicMax(&st64[12], (unsigned long long)(wall_clock64() - t_chain));
        }
    }
    }
    if (stats && lane == 0) {                   // wave occupancy of the pass: busy sum, first start, last end
        unsigned long long* st64 = (unsigned long long*)(stats + 32);
        const uint64_t t_end = wall_clock64();
        atomicAdd(&st64[8], t_end - t_begin);
        atomicMax(&st64[9], t_end);
        atomicMax(&st64[10], ~t_begin);
        atomicAdd(&st64[11], 1ull);
    }
}

// Emit pass: persistent waves claiming the linked chains through `ticket`.  No lane and no chain
// ever waits on another: a copy whose source lies before the lane's own output (an earlier lane,
// an earlier chain, the window), or covers one of the lane's own deferred bytes, is not executed but
// deferred -- its bytes get a back-reference (ref[i] = distance to a byte holding the same value)
// and a pending bit, and ndfl_inflate_resolve_kernel rounds resolve them afterwards by pointer
// jumping.  So every chain decodes in parallel whatever the LZ77 distances.
#ifndef NDFL_EMIT_WAVES_PER_SIMD
#define NDFL_EMIT_WAVES_PER_SIMD 3
#endif
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NDFL_EMIT_WAVES_PER_SIMD)))
ndfl_inflate_emit_wave_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const EmitChain* chains,
                              uint32_t nlist, uint32_t* ticket, uint8_t* out, ChainRes* res, const uint64_t* cands,
                              uint32_t ncand, uint32_t* ref, uint32_t* pend, SegPool pool, wv::PhArr* ph_all,
                              uint32_t* stats, const uint64_t* info, const uint32_t* eorder,
                              const uint32_t* dnlist) {
    using namespace wv;
    __shared__ __attribute__((aligned(16))) Shared S;
    __shared__ Stage stg;
    __shared__ uint32_t s_ticket;
    const int lane = threadIdx.x;
    gu8* gout = (gu8*)out;
    PhArr* S_ph = ph_all + blockIdx.x;
    const uint64_t t_begin = stats ? wall_clock64() : 0;
    if (info) {                                 // device-side linking: the list length, and nothing
        if (info[LI_FLAGS]) return;             // to emit when the host has to step in (uniform)
        nlist = (uint32_t)info[LI_NCH];
    }
    if (dnlist) {                               // the chains the fast emit pass left (eorder lists them):
        nlist = *dnlist;                        // usually none, and then no wave takes a ticket
        if (nlist == 0) return;
    }
    for (;;) {
    __syncthreads();
    if (lane == 0) s_ticket = atomicAdd(ticket, 1u);
    __syncthreads();
    if (s_ticket >= nlist) break;
    const uint32_t ci = eorder ? eorder[s_ticket] : s_ticket;    // (costliest chains first)
    const In in{w, nwords, nbits};
    const EmitChain ch = chains[ci];
    const uint64_t t_chain = stats ? wall_clock64() : 0;
    uint64_t cur = ch.start_bit, base = ch.out_off;
    uint32_t status = ST_BOUNDARY, reason = 0;
    uint64_t endpos = ch.start_bit;
    uint32_t nslow = 0, nfix = 0;
    uint32_t rec = ch.slot < pool.nslot ? pool.head[ch.slot] : NOREC;
    // the next round's record is loaded one round ahead (its loads overlap this round's decode)
    SegMeta pm = {};
    uint64_t pst = 0;
    uint32_t pcn = 0;
    if (rec != NOREC) { pm = pool.meta[rec]; pst = pool.start[(uint64_t)rec * 64 + lane]; pcn = pool.cnt[(uint64_t)rec * 64 + lane]; }
    uint64_t bnd_bit = cur, bnd_out = base;     // start of the current block (partial-input decodes)
    for (int blk = 0;; blk++) {
        if (blk > 0 && cur == ch.end_bit) { status = ST_BOUNDARY; endpos = cur; break; }
        bnd_bit = cur; bnd_out = base;
        // the count pass's tables of this block, when its first round record names them
        const char* btr = (rec != NOREC && pm.pad < pool.nbt) ? pool.bt + (uint64_t)pm.pad * BT_BYTES : nullptr;
        if (btr && *(const uint64_t*)(btr + sizeof(Tabs)) != cur) btr = nullptr;     // (not this block)
        if (btr) {
            __syncthreads();                    // the previous block's table reads are done
            const uint4* src = (const uint4*)btr;
            uint4* dst = (uint4*)&S.t;
            for (uint32_t q = (uint32_t)lane; q < sizeof(Tabs) / 16; q += 64) dst[q] = src[q];
            if (lane == 0) {
                const uint64_t* h = (const uint64_t*)(btr + sizeof(Tabs));
                const uint32_t* h32 = (const uint32_t*)(h + 2);
                S.h_err = 0; S.h_d0 = h[1]; S.h_bfinal = h32[0]; S.h_btype = h32[1]; S.h_len = h32[2];
            }
            __syncthreads();
        } else {
            for (uint32_t s = (uint32_t)lane; s < 320; s += 64) S.lens[s] = 0;
            __syncthreads();
            if (lane == 0) parse_hdr(in, cur, S);
            __syncthreads();
        }
        if (S.h_err) { status = ST_ERROR; reason = S.h_err; endpos = S.h_pos; break; }
        const uint64_t d0 = S.h_d0;
        const bool bfinal = S.h_bfinal != 0;
        if (S.h_btype == 0) {
            const uint64_t avail = (nbits - d0) / 8, ln = S.h_len;
            const uint64_t take = min(avail, ln);
            const uint64_t ib = d0 >> 3;
            for (uint64_t i = (uint64_t)lane; i < take; i += 64) {
                const uint64_t b = ib + i;
                out[base + i] = (uint8_t)(in.ld(b >> 2) >> (8 * (uint32_t)(b & 3)));
            }
            base += take;
            if (take < ln) { status = ST_ERROR; reason = R_UEOS; endpos = d0 + 8 * avail; break; }
            cur = d0 + 8 * ln;
            if (bfinal) { status = ST_FINAL; endpos = cur; break; }
            continue;
        }
        bool ed;
        if (btr) {
            ed = S.h_len != 0;                  // (the loaded record's empty-distance flag)
        } else {
            const int te = build_tables(S, lane, ed, stg.w);
            if (te) { status = ST_ERROR; reason = (uint32_t)te; endpos = d0; break; }
        }
        uint64_t rs = d0;
        bool block_done = false, chain_done = false;
        while (!block_done) {
            Seg r;
            uint32_t ft;
            Geo g;
            if (rec != NOREC) {
                // exact segments from the count pass, and the round's geometry
                const SegMeta m = pm;
                ft = m.ft;
                r.start = pst;
                r.cnt = pcn;
                rec = m.next;
                if (rec != NOREC) { pm = pool.meta[rec]; pst = pool.start[(uint64_t)rec * 64 + lane]; pcn = pool.cnt[(uint64_t)rec * 64 + lane]; }
                const uint64_t nx = __shfl_down((unsigned long long)r.start, 1, 64);
                r.end = lane < 63 ? nx : m.exit63;
                r.kind = T_EXIT; r.reason = 0;
                if ((uint32_t)lane == ft) { r.end = m.end_ft; r.kind = m.kind_ft; r.reason = m.reason_ft; }
                g = make_geo(in, m.rs, m.rs + 1, m.pw);      // the count pass's staging geometry
                stage_round(in, g, stg, lane);
            } else {
                uint64_t E = min(next_cand(cands, ncand, rs, ch.end_bit), rs + MAX_SPAN);
                if (E <= rs) E = rs + 1;
                round_decode(in, S.t, ed, rs, E, S, stg, lane, r, ft, nslow, nfix, S_ph, g);
            }
            const bool live = (uint32_t)lane <= ft;
            const uint64_t mycnt = live ? r.cnt : 0ull;
            const uint64_t pre = wave_excl_u64(mycnt, lane);
            const uint64_t rsum = wave_sum_u64(mycnt);
            // write pass: every lane runs its segment to the end on its own
            const Lv v = make_lv(stg, g, lane);
            const uint32_t nb = g.nb;
            uint32_t pos = (uint32_t)(r.start - g.base);
            uint32_t end = (uint32_t)(r.end - g.base);
            uint32_t kind = r.kind, rsn = r.reason;
            const uint64_t dst0 = base + pre;
            uint32_t n = 0;                 // bytes produced
            Wr wr;
            wr_init(wr, dst0);
            uint64_t dfr = ~0ull;           // first deferred byte of this lane (absolute)
            uint64_t lastsrc = 0;           // a byte holding the value of the last output byte, when !lsp
            bool lsp = false;               //   (lsp: the byte just before dst0 + n)
            uint32_t lastb = 0;             // the last output byte, when it is final (lastok)
            bool lastok = false;
            bool active = live;
#if NDFL_BITBUF
            Bb bb;
            const uint32_t lim = min(end, nb - min(nb, 48u));
            bool fast = active && pos < lim;           // (pos only grows: once false, it stays false)
            if (fast) bb_init(bb, v, pos);
#endif
            while (active && pos < end) {
                Tok tk;
#if NDFL_BITBUF
                if (fast) {
                    tok_bb<true>(bb, v, S.t, ed, tk, end);
                    pos = bb.pos;
                    fast = pos < lim;
                } else {
                    tok<true>(v, pos, S.t, ed, end, nb, tk);
                }
#else
                if (pos + 48 < end) tok<false>(v, pos, S.t, ed, end, nb, tk);
                else tok<true>(v, pos, S.t, ed, end, nb, tk);
#endif
                if (tk.kind == K_LIT) {
                    wr_lit(wr, gout, tk.val, tk.n);
                    n += tk.n;
                    lsp = true;
                    lastb = tk.val >> (tk.n == 2 ? 8 : 0);
                    lastok = true;
                    continue;
                }
                if (tk.kind != K_LEN) break;            // EOB or error (as verified)
                const uint64_t dst = dst0 + n;
                if ((uint64_t)tk.dist > dst) {
                    kind = T_ERR; rsn = R_COPY_BEFORE; end = pos; break;
                }
                const uint32_t len = tk.n, dist = tk.dist;
                const uint64_t src = dst - dist;
                const uint64_t src_end = src + min(len, dist);          // the copy's bytes before dst
                bool defer = src < dst0;
                if (!defer && src_end > dfr) {
                    // a source at or past our first deferred byte: pending only if its bit is set
                    // (bits of our own range are set by this lane alone, atomically, so an agent-
                    // scope load sees them)
                    for (uint64_t q = src >> 5; q <= (src_end - 1) >> 5 && !defer; q++) {
                        const uint64_t lo = max(src, q << 5), hi = min(src_end, (q + 1) << 5);
                        const uint32_t m = (uint32_t)(((1ull << (hi - lo)) - 1) << (lo & 31));
                        defer = (__hip_atomic_load(&pend[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & m) != 0;
                    }
                }
                wr_flush_word(wr, gout);
                if (!defer && dist == 1 && !lastok) lastb = gout[dst - 1];    // (not one of our bytes yet)
                if (!defer) {
                    wr_copy(gout, dst, len, dist, lastb);           // sources final and our own
                    lastok = true;
                    lsp = true;
                } else {
                    // deferred: back-references (a dist-1 run points at the byte its value comes
                    // from), pending bits; the bytes are written by the resolve rounds
                    const uint64_t anchor = dist == 1 ? (n > 0 ? (lsp ? dst - 1 : lastsrc) : src) : 0;
                    for (uint32_t k = 0; k < len; k++) {
                        const uint64_t back = dst + k - anchor;     // a run > 4 GiB falls back to its previous byte
                        ref[dst + k] = dist == 1 ? (back < (1ull << 32) ? (uint32_t)back : 1u) : dist;
                    }
                    for (uint64_t q = dst >> 5; q <= (dst + len - 1) >> 5; q++) {
                        const uint64_t lo = max(dst, q << 5), hi = min(dst + len, (q + 1) << 5);
                        const uint32_t m = (uint32_t)(((1ull << (hi - lo)) - 1) << (lo & 31));
                        atomicOr(&pend[q], m);
                    }
                    lastsrc = anchor;
                    lsp = dist != 1;
                    dfr = min(dfr, dst);
                    lastok = false;                 // the copy's bytes are pending
                }
                n += len;
                wr.dst = dst0 + n;
            }
            wr_flush_exact(wr, gout);
            // the segment, checked: the write pass lands on the next lane's segment
            // start having produced exactly the bytes the count pass's record (or this round's
            // decode) counts
            if (live && kind != T_ERR && (n != mycnt || pos != end)) { kind = T_ERR; rsn = R_INTERNAL; }
            // the first lane (in stream order) that ended with an error decides
            const uint64_t em = __ballot(live && kind == T_ERR);
            if (em) {
                const int fl = (int)__builtin_ctzll(em);
                status = ST_ERROR;
                reason = __shfl(rsn, fl, 64);
                endpos = g.base + __shfl(end, fl, 64);
                base = __shfl((unsigned long long)(dst0 + n), fl, 64);
                chain_done = true;
                break;
            }
            base += rsum;
            if (ft < 64) {
                block_done = true;
                cur = __shfl((unsigned long long)r.end, (int)ft, 64);
                if (bfinal) { status = ST_FINAL; endpos = cur; chain_done = true; }
            } else {
                rs = __shfl((unsigned long long)r.end, 63, 64);
            }
        }
        if (chain_done) break;
    }
    if (lane == 0) {
        ChainRes o;
        o.end_bit = endpos; o.out_count = base - ch.out_off; o.status = status; o.reason = reason;
        o.next = 0xFFFFFFFFu; o.pad = 0;
        o.bnd_bit = bnd_bit; o.bnd_cnt = bnd_out - ch.out_off;
        res[ci] = o;
        if (stats) atomicMax((unsigned long long*)(stats + 32) + 20, (unsigned long long)(wall_clock64() - t_chain));
    }
    }
    if (stats && lane == 0) {                   // wave occupancy of the pass: busy sum, first start, last end
        unsigned long long* st64 = (unsigned long long*)(stats + 32);
        const uint64_t t_end = wall_clock64();
        atomicAdd(&st64[16], t_end - t_begin);
        atomicMax(&st64[17], t_end);
        atomicMax(&st64[18], ~t_begin);
        atomicAdd(&st64[19], 1ull);
    }
}

// Fast emit pass (the common case): a chain whose every Huffman block has the count pass's table
// record and every round its segment record is replayed from those records alone (no header parse,
// no table build, no round decode), so the kernel holds the registers of the record replay only:
// 128 VGPRs, 11.0 KB of LDS (tables + the staged round), 14 waves per CU where the full emit kernel
// holds 12 (measured: emit 8.81 -> 8.41 ms).  NDFL_EMITF_STAGE=0 reads the input through L1/L2
// instead of the LDS stage (4 waves per SIMD; measured slower, 10.3 ms).  A chain that needs anything else (a block without a table record, a round without a
// segment record, a stored block that is invalid or runs past the input) is listed in `slow` for the
// full kernel, which runs it from its start: the output this kernel wrote for the chain so far is
// rewritten there identically (the same records give the same segments, deferral decisions, bytes,
// back-references and pending bits).
#ifndef NDFL_EMITF_STAGE
#define NDFL_EMITF_STAGE 1
#endif
#ifndef NDFL_EMITF_GX
#define NDFL_EMITF_GX 1         // primary tables in LDS, extension areas read from the table record
#endif
#ifndef NDFL_EMIT_JUMP
#define NDFL_EMIT_JUMP 1        // blocks of mostly 8-bit literal codes: four literals a step where they can
#endif
#ifndef NDFL_EMITF_WAVES_PER_SIMD
#define NDFL_EMITF_WAVES_PER_SIMD 4
#endif
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NDFL_EMITF_WAVES_PER_SIMD)))
ndfl_inflate_emit_fast_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const EmitChain* chains,
                              uint32_t* ticket, uint8_t* out, ChainRes* res, uint32_t* ref, uint32_t* pend,
                              SegPool pool, const uint64_t* info, const uint32_t* eorder, uint32_t* slow,
                              uint32_t* nslow) {
    using namespace wv;
#if NDFL_EMITF_GX
    __shared__ __attribute__((aligned(16))) uint32_t Tp[(1u << LB) + (1u << DB)];     // primary tables
    TabsG T;
    T.lit = Tp;
    T.dst = Tp + (1u << LB);
#else
    __shared__ __attribute__((aligned(16))) Tabs T;
#endif
#if NDFL_EMITF_STAGE
    __shared__ Stage stg;
#endif
    const int lane = threadIdx.x;
    gu8* gout = (gu8*)out;
    if (info[LI_FLAGS]) return;                 // (the host steps in: nothing to emit)
    const uint32_t nlist = (uint32_t)info[LI_NCH];
    const In in{w, nwords, nbits};
    for (;;) {
    uint32_t tk0 = 0;
    if (lane == 0) tk0 = atomicAdd(ticket, 1u);
    const uint32_t t = __builtin_amdgcn_readfirstlane(tk0);
    if (t >= nlist) break;
    const uint32_t ci = eorder[t];              // (costliest chains first)
    const EmitChain ch = chains[ci];
    uint64_t cur = ch.start_bit, base = ch.out_off;
    uint32_t status = ST_BOUNDARY, reason = 0;
    uint64_t endpos = ch.start_bit;
    bool abort = false;
    uint32_t rec = ch.slot < pool.nslot ? pool.head[ch.slot] : NOREC;
    SegMeta pm = {};
    uint64_t pst = 0;
    uint32_t pcn = 0;
    if (rec != NOREC) { pm = pool.meta[rec]; pst = pool.start[(uint64_t)rec * 64 + lane]; pcn = pool.cnt[(uint64_t)rec * 64 + lane]; }
    uint64_t bnd_bit = cur, bnd_out = base;
    for (int blk = 0;; blk++) {
        if (blk > 0 && cur == ch.end_bit) { status = ST_BOUNDARY; endpos = cur; break; }
        bnd_bit = cur; bnd_out = base;
        if (cur + 3 > nbits) { abort = true; break; }
        const uint32_t hb = (uint32_t)(in.win64(cur)) & 7u;
        if ((hb >> 1) == 0) {                   // stored block (D/decomp/Open.java:286-310)
            const uint64_t hp = (cur + 3 + 7) & ~7ull;
            if (hp + 32 > nbits) { abort = true; break; }
            const uint32_t lw = (uint32_t)in.win64(hp);
            if ((lw >> 16) != (~lw & 0xFFFFu)) { abort = true; break; }
            const uint64_t ln = lw & 0xFFFFu, d0 = hp + 32;
            if (d0 + 8 * ln > nbits) { abort = true; break; }
            const uint64_t ib = d0 >> 3;
            for (uint64_t i = (uint64_t)lane; i < ln; i += 64) {
                const uint64_t b = ib + i;
                out[base + i] = (uint8_t)(in.ld(b >> 2) >> (8 * (uint32_t)(b & 3)));
            }
            base += ln;
            cur = d0 + 8 * ln;
            if (hb & 1) { status = ST_FINAL; endpos = cur; break; }
            continue;
        }
        const char* btr = (rec != NOREC && pm.pad < pool.nbt) ? pool.bt + (uint64_t)pm.pad * BT_BYTES : nullptr;
        if (!btr || *(const uint64_t*)(btr + sizeof(Tabs)) != cur) { abort = true; break; }
        __syncthreads();                        // the previous block's table reads are done
        {
            const uint4* src = (const uint4*)btr;
#if NDFL_EMITF_GX
            uint4* dst = (uint4*)Tp;
            for (uint32_t q = (uint32_t)lane; q < sizeof(Tp) / 16; q += 64) dst[q] = src[q];
            T.lx = (const uint32_t*)btr + offsetof(Tabs, lx) / 4;
            T.dx = (const uint32_t*)btr + offsetof(Tabs, dx) / 4;
#else
            uint4* dst = (uint4*)&T;
            for (uint32_t q = (uint32_t)lane; q < sizeof(Tabs) / 16; q += 64) dst[q] = src[q];
#endif
        }
        const uint64_t* h = (const uint64_t*)(btr + sizeof(Tabs));
        const uint32_t* h32 = (const uint32_t*)(h + 2);
        const bool bfinal = h32[0] != 0, ed = h32[2] != 0;
        const bool ph8 = NDFL_EMIT_JUMP && h32[3] != 0;     // mostly 8-bit literal codes
        const uint32_t esc4 = h32[3] > 1 ? h32[3] : 0u;     // escape-prefix literal block (phase_multi_esc)
        __syncthreads();
        bool block_done = false, chain_done = false;
        while (!block_done) {
            if (rec == NOREC) { abort = true; chain_done = true; break; }
            const SegMeta m = pm;
            const uint32_t ft = m.ft;
            const uint64_t rstart = pst;
            const uint32_t rcnt = pcn;
            rec = m.next;
            if (rec != NOREC) { pm = pool.meta[rec]; pst = pool.start[(uint64_t)rec * 64 + lane]; pcn = pool.cnt[(uint64_t)rec * 64 + lane]; }
            const uint64_t nx = __shfl_down((unsigned long long)rstart, 1, 64);
            uint64_t rend = lane < 63 ? nx : m.exit63;
            uint32_t kind = T_EXIT, rsn = 0;
            if ((uint32_t)lane == ft) { rend = m.end_ft; kind = m.kind_ft; rsn = m.reason_ft; }
            const Geo g = make_geo(in, m.rs, m.rs + 1, m.pw);      // the count pass's geometry
            const bool live = (uint32_t)lane <= ft;
            const uint64_t mycnt = live ? rcnt : 0ull;
            const uint64_t pre = wave_excl_u64(mycnt, lane);
            const uint64_t rsum = wave_sum_u64(mycnt);
#if NDFL_EMITF_STAGE
            stage_round(in, g, stg, lane);
            const Lv v = make_lv(stg, g, lane);
#else
            Gv v;
            v.rw = (uint32_t)lane * g.pw;
            v.q = w + (g.base >> 5) + v.rw;
#endif
            const uint32_t nb = g.nb;
            uint32_t pos = (uint32_t)(rstart - g.base);
            uint32_t end = (uint32_t)(rend - g.base);
            const uint64_t dst0 = base + pre;
            uint32_t n = 0;
            Wr wr;
            wr_init(wr, dst0);
            uint64_t dfr = ~0ull, lastsrc = 0;     // (lastsrc when !lsp; lsp: the byte before dst0 + n)
            bool lsp = false;
            uint32_t lastb = 0;
            bool lastok = false;
            Bb bb;
            const uint32_t lim = min(end, nb - min(nb, 48u));
            bool fast = live && pos < lim;
            if (fast) bb_init(bb, v, pos);
            // (two instances of the token loop: blocks of mostly 8-bit literal codes try four literals a
            // step, the others keep the plain loop's code and registers)
            auto token_loop = [&](auto ph) {
                using PH = decltype(ph);
                while (live && pos < end) {
                    Tok tk;
                    if (PH::value && fast && esc4) {
                        // escape-prefix literal block: up to 8 literals, to the first escape byte
                        const uint32_t lo = (uint32_t)bb.buf, hi = (uint32_t)(bb.buf >> 32);
                        const uint32_t t = min(min(esc_index(lo, hi, esc4), bb.nb >> 3), (end - pos + 7) >> 3);
                        if (t) {
                            uint32_t b[8];
#pragma unroll
                            for (uint32_t i = 0; i < 8; i++)
                                b[i] = (T.lit[(i < 4 ? lo >> (8 * i) : hi >> (8 * (i - 4))) & 0xFFu] >> 9) & 0xFFu;
                            const uint32_t v0 = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                            const uint32_t v1 = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
                            const uint32_t n0 = min(t, 4u);
                            wr_lit(wr, gout, n0 == 4 ? v0 : v0 & ((1u << (8 * n0)) - 1u), n0);
                            if (t > 4) wr_lit(wr, gout, t == 8 ? v1 : v1 & ((1u << (8 * (t - 4))) - 1u), t - 4);
                            n += t;
                            lsp = true;
                            lastb = t > 4 ? (v1 >> (8 * (t - 5))) & 0xFFu : (v0 >> (8 * (t - 1))) & 0xFFu;
                            lastok = true;
                            // (a 64-bit shift by 64 is undefined: the hardware shifts by 0)
                            bb.buf = t < 8 ? bb.buf >> (8 * t) : 0ull;
                            bb.nb -= 8 * t;
                            bb.pos += 8 * t;
                            bb_refill(bb, v);
                            pos = bb.pos;
                            fast = pos < lim;
                            continue;
                        }
                    }
                    if (PH::value && fast && !esc4 && bb.nb >= 34 && pos + 24 < end) {
                        // four 8-bit literal codes at once (independent table reads at 0, 8, 16, 24 bits;
                        // the lane's end is a token boundary, so none of the four passes it)
                        const uint32_t lo = (uint32_t)bb.buf, hi = (uint32_t)(bb.buf >> 32);
                        const uint32_t e0 = T.lit[lo & ((1u << LB) - 1u)], e1 = T.lit[(lo >> 8) & ((1u << LB) - 1u)];
                        const uint32_t e2 = T.lit[(lo >> 16) & ((1u << LB) - 1u)];
                        const uint32_t e3 = T.lit[__builtin_amdgcn_alignbit(hi, lo, 24) & ((1u << LB) - 1u)];
                        // a single literal of 8 bits: bit 31, advance 8, first length 8, no pair
                        if (((e0 & 0x800001FFu) == 0x80000088u) && ((e1 & 0x800001FFu) == 0x80000088u) &&
                            ((e2 & 0x800001FFu) == 0x80000088u) && ((e3 & 0x800001FFu) == 0x80000088u)) {
                            const uint32_t b3 = (e3 >> 9) & 0xFFu;
                            wr_lit(wr, gout, ((e0 >> 9) & 0xFFu) | (((e1 >> 9) & 0xFFu) << 8) | (((e2 >> 9) & 0xFFu) << 16) | (b3 << 24), 4);
                            n += 4;
                            lsp = true;
                            lastb = b3;
                            lastok = true;
                            bb_skip(bb, 32);
                            bb_refill(bb, v);
                            pos = bb.pos;
                            fast = pos < lim;
                            continue;
                        }
                    }
                    if (fast) {
                        tok_bb<true>(bb, v, T, ed, tk, end);
                        pos = bb.pos;
                        fast = pos < lim;
                    } else {
                        tok<true>(v, pos, T, ed, end, nb, tk);
                    }
                    if (tk.kind == K_LIT) {
                        wr_lit(wr, gout, tk.val, tk.n);
                        n += tk.n;
                        lsp = true;
                        lastb = tk.val >> (tk.n == 2 ? 8 : 0);
                        lastok = true;
                        continue;
                    }
                    if (tk.kind != K_LEN) break;
                    const uint64_t dst = dst0 + n;
                    if ((uint64_t)tk.dist > dst) { kind = T_ERR; rsn = R_COPY_BEFORE; end = pos; break; }
                    const uint32_t len = tk.n, dist = tk.dist;
                    const uint64_t src = dst - dist;
                    const uint64_t src_end = src + min(len, dist);
                    bool defer = src < dst0;
                    if (!defer && src_end > dfr) {
                        for (uint64_t q = src >> 5; q <= (src_end - 1) >> 5 && !defer; q++) {
                            const uint64_t lo = max(src, q << 5), hi = min(src_end, (q + 1) << 5);
                            const uint32_t mk = (uint32_t)(((1ull << (hi - lo)) - 1) << (lo & 31));
                            defer = (__hip_atomic_load(&pend[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & mk) != 0;
                        }
                    }
                    wr_flush_word(wr, gout);
                    if (!defer && dist == 1 && !lastok) lastb = gout[dst - 1];
                    if (!defer) {
                        wr_copy(gout, dst, len, dist, lastb);
                        lastok = true;
                        lsp = true;
                    } else {
                        const uint64_t anchor = dist == 1 ? (n > 0 ? (lsp ? dst - 1 : lastsrc) : src) : 0;
                        for (uint32_t k = 0; k < len; k++) {
                            const uint64_t back = dst + k - anchor;
                            ref[dst + k] = dist == 1 ? (back < (1ull << 32) ? (uint32_t)back : 1u) : dist;
                        }
                        for (uint64_t q = dst >> 5; q <= (dst + len - 1) >> 5; q++) {
                            const uint64_t lo = max(dst, q << 5), hi = min(dst + len, (q + 1) << 5);
                            const uint32_t mk = (uint32_t)(((1ull << (hi - lo)) - 1) << (lo & 31));
                            atomicOr(&pend[q], mk);
                        }
                        lastsrc = anchor;
                        lsp = dist != 1;
                        dfr = min(dfr, dst);
                        lastok = false;
                    }
                    n += len;
                    wr.dst = dst0 + n;
                }
            };
            if (ph8) token_loop(std::true_type{}); else token_loop(std::false_type{});
            wr_flush_exact(wr, gout);
            // the count pass's record, checked: the lane's replay lands on the next
            // lane's segment start having produced exactly the bytes the record counts
            if (live && kind != T_ERR && (n != rcnt || pos != end)) { kind = T_ERR; rsn = R_INTERNAL; }
            const uint64_t em = __ballot(live && kind == T_ERR);
            if (em) {
                const int fl = (int)__builtin_ctzll(em);
                status = ST_ERROR;
                reason = __shfl(rsn, fl, 64);
                endpos = g.base + __shfl(end, fl, 64);
                base = __shfl((unsigned long long)(dst0 + n), fl, 64);
                chain_done = true;
                break;
            }
            base += rsum;
            if (ft < 64) {
                block_done = true;
                cur = __shfl((unsigned long long)rend, (int)ft, 64);
                if (bfinal) { status = ST_FINAL; endpos = cur; chain_done = true; }
            }
        }
        if (chain_done) break;
    }
    if (lane == 0) {
        if (abort) {
            slow[atomicAdd(nslow, 1u)] = ci;
        } else {
            ChainRes o;
            o.end_bit = endpos; o.out_count = base - ch.out_off; o.status = status; o.reason = reason;
            o.next = 0xFFFFFFFFu; o.pad = 0;
            o.bnd_bit = bnd_bit; o.bnd_cnt = bnd_out - ch.out_off;
            res[ci] = o;
        }
    }
    }
}

// ---- resolve rounds -------------------------------------------------------------------------------
#ifndef NDFL_RESOLVE_HOPS
#define NDFL_RESOLVE_HOPS 4
#endif
// Pending bytes form 32-byte groups (one bitmap word each) listed in `list`.  A wave takes two
// groups, a lane one byte i: with p = i - ref[i], a final p gives out[i] = out[p]; a pending p makes
// i jump (ref[i] += ref[p]), so the remaining distance to a final byte halves each round.  Bits and
// bytes read here were settled by earlier launches; ref[p] may be updated concurrently, but both its
// old and new values point at a byte of the same value.  A lane follows up to NDFL_RESOLVE_HOPS
// pending targets in one launch before it jumps (fewer rounds for deep chains of copies of copies,
// as in LZ77 text).
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_resolve_kernel(const uint32_t* list, const uint32_t* nlist, const uint32_t* pend, uint32_t* ref,
                            uint8_t* out, uint32_t* newbits) {
    const uint32_t n = *nlist;
    const uint32_t b = threadIdx.x & 31;
    for (uint32_t k = (blockIdx.x * 256 + threadIdx.x) >> 5; k < n; k += gridDim.x * 8) {
        const uint64_t wd = list[k];
        const uint32_t bits = pend[wd];
        bool still = false;
        if ((bits >> b) & 1) {
            // follow up to NDFL_RESOLVE_HOPS references in this launch (each keeps the value: every
            // ref, old or new, points at a byte of the same value); a final target copies, else the
            // byte keeps the distance reached
            const uint64_t i = wd * 32 + b;
            uint64_t d = ref[i];
            uint64_t p = i - d;
            bool pending = (pend[p >> 5] >> (p & 31)) & 1;
#pragma unroll 1
            for (int h = 1; h < NDFL_RESOLVE_HOPS && pending; h++) {
                const uint64_t nd = d + ref[p];
                if (nd >= (1ull << 32)) break;                     // (keep d: p still leads to the value)
                d = nd;
                p = i - d;
                pending = (pend[p >> 5] >> (p & 31)) & 1;
            }
            if (pending) {
                const uint64_t nd = d + ref[p];
                ref[i] = (uint32_t)(nd < (1ull << 32) ? nd : d);
                still = true;
            } else {
                out[i] = out[p];
            }
        }
        const uint64_t m = __ballot(still);
        if (b == 0) newbits[k] = (uint32_t)(m >> (threadIdx.x & 32));
    }
}

// Apply a round's bits and compact the list of still-pending groups (grid-stride: the grid is sized
// before the list size is known).
// Block-wide append of the flagged lanes' values to list[*n ...] (one global atomic per block).
__device__ __forceinline__ void block_append(bool flag, uint32_t v, uint32_t* list, uint32_t* n) {
    __shared__ uint32_t wc[4], wbase;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t m = __ballot(flag);
    if (lane == 0) wc[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = wc[0] + wc[1] + wc[2] + wc[3];
        wbase = t ? atomicAdd(n, t) : 0u;
    }
    __syncthreads();
    uint32_t off = wbase;
    for (int k = 0; k < wid; k++) off += wc[k];
    if (flag) list[off + __popcll(m & ((1ull << lane) - 1))] = v;
    __syncthreads();
}

extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_resolve_apply_kernel(const uint32_t* list, const uint32_t* nlist, uint32_t* pend, const uint32_t* newbits,
                                  uint32_t* list_out, uint32_t* nlist_out, uint32_t* nbytes_out) {
    const uint32_t n = *nlist;
    for (uint32_t k0 = blockIdx.x * 256; k0 < n; k0 += gridDim.x * 256) {
        const uint32_t k = k0 + threadIdx.x;
        const bool live = k < n;
        uint32_t nb = 0, wd = 0;
        if (live) { wd = list[k]; nb = newbits[k]; pend[wd] = nb; }
        if (nbytes_out) {
            const uint32_t c = wave_sum((uint32_t)__popc(nb));
            if ((threadIdx.x & 63) == 0 && c) atomicAdd(nbytes_out, c);
        }
        block_append(live && nb != 0, wd, list_out, nlist_out);
    }
}

// Initial list: every non-zero bitmap word in [w0, w1).
extern "C" __global__ void __launch_bounds__(256)
ndfl_inflate_pending_list_kernel(const uint32_t* pend, uint64_t w0, uint64_t w1, uint32_t* list, uint32_t* nlist) {
    // 16 words per thread (four 16-byte loads), one block scan of the non-zero counts, one global
    // atomic per block
    __shared__ uint32_t sh[4], sbase;
    const uint64_t base = w0 + ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    uint32_t v[16];
    if (base + 16 <= w1 && (base & 3) == 0) {
        const u32x4* q = (const u32x4*)(pend + base);
#pragma unroll
        for (int k = 0; k < 4; k++) { const u32x4 x = q[k]; v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w; }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = base + k < w1 ? pend[base + k] : 0u;
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) cnt += v[k] != 0;
    uint32_t tot;
    const uint32_t off = block_excl_scan<uint32_t, 4>(cnt, sh, tot);
    if (threadIdx.x == 0) sbase = tot ? atomicAdd(nlist, tot) : 0u;
    __syncthreads();
    uint32_t o = sbase + off;
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (v[k]) list[o++] = (uint32_t)(base + k);
}
