// lz77_kernels.hip -- MI355X (gfx950) LZ77 encoder for the FULL_* presets and any
// Lz77Huffman(dynamic, minRun, maxRun, minDist, maxDist) (D/comp/Lz77Huffman.java:20-39,62-130).
//
// The reference searches every distance minDist..min(maxDist, index-off) at every parse position
// and keeps the longest run (capped at maxRun and the chunk end), the smallest distance on ties
// (:71-84).  Only candidates whose run reaches minRun (>= 3) can be chosen, and those share the
// 3-byte prefix, so walking every earlier position with the same 3-byte prefix nearest-first and
// keeping strictly longer runs is the same search.  Three launches per batch:
//   1. ndfl_lz_links_kernel   one workgroup per 32 KiB segment: link[q] = distance to the previous
//                             position whose 3-byte prefix hashes like q's (0 if none within
//                             32 KiB); head table in LDS, in-wave duplicates resolved by readlane.
//   2. ndfl_lz_match_kernel   one 1024-thread workgroup per 8 KiB tile: the tile's 32 KiB window
//                             (bytes and links) is staged in LDS and every position's best
//                             (run, distance) is found by walking its chain; written as one u32
//                             per position (run << 16 | distance-1, or the literal byte).
//   3. ndfl_lz_encode_kernel  one 1024-thread workgroup per chunk: the greedy parse (:68-130) is a
//                             walk over the per-position steps (one wave, 64 steps per LDS read,
//                             chased with readlane); then histograms, code construction, token
//                             bits and the look-back/store shared with the RLE encoder.
// D/ = /root/reference/src/io/nayuki/deflate/
#include "ndfl_common.hpp"

namespace {

constexpr int LZ_SEG = 32768;                      // link segment = largest distance
constexpr int LZ_HBITS = 15;                       // hash buckets (head table: 64 KB of u16)
constexpr int LZ_TILE = 8192;                      // match-search positions per workgroup
constexpr int LZ_WIN = 32768;                      // window before the tile
constexpr int LZ_WWORDS = (LZ_WIN + LZ_TILE + 272) / 4;   // window bytes as words (+ lookahead)
constexpr uint32_t LZ_DS = 32768;                  // data start inside the staging buffer

__device__ __forceinline__ uint32_t lz_hash(uint32_t k) { return (k * 2654435761u) >> (32 - LZ_HBITS); }

struct LzArgs {
    const uint8_t* buf;       // staging buffer: [pad | history (H) | data (n)], data at LZ_DS
    uint64_t total;           // LZ_DS + n
    uint64_t vstart;          // LZ_DS - H: first valid history byte
    uint32_t chunk_len;
    uint32_t parent_len;      // history start from the chunk of this length (BinarySplit sub-blocks)
    uint32_t hist_limit;
    uint32_t min_run, max_run, min_dist, max_dist;
    const uint16_t* link;     // link[q - L0]
    uint64_t L0;
    uint64_t p_begin, p_end;  // searched positions (buffer index) of this launch
    uint32_t* match;          // match[q - p_begin]
    unsigned long long* stats;  // optional: [0] searched positions, [1] chain hops, [2] trigram hits, [3] compare words
};

}  // namespace

// ---- 1. hash-chain links ---------------------------------------------------------------------
// Segment s covers positions [L0 + 32K s, +32K) ∩ [.., L1).  The head table is first filled from
// the 32 KiB before the segment (those are the only positions a link can reach), then the
// segment's positions are linked in order, 1024 at a time by one workgroup: every wave finds, for
// its 64 positions, the highest lane below each with the same bucket (all 16 waves at once); then
// the waves take turns on the head table in position order -- a lane with no predecessor in its
// wave reads the head entry, the last lane of each bucket updates it.
extern "C" __global__ void __launch_bounds__(1024)
ndfl_lz_links_kernel(const uint8_t* buf, uint64_t total, uint64_t vstart, uint64_t L0, uint64_t L1, uint16_t* link) {
    __shared__ __attribute__((aligned(16))) uint16_t head[1 << LZ_HBITS];
    __shared__ __attribute__((aligned(16))) uint32_t bb[(1024 + 16) / 4];    // one 1 KiB block + lookahead
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t s0 = L0 + (uint64_t)blockIdx.x * LZ_SEG;
    const uint64_t s1 = min(s0 + LZ_SEG, L1);
    const uint64_t seed0 = max(vstart, s0 >= (uint64_t)LZ_SEG ? s0 - LZ_SEG : 0ull);
    for (int k = tid; k < (1 << LZ_HBITS) / 8; k += 1024) ((u32x4*)head)[k] = u32x4{~0u, ~0u, ~0u, ~0u};
    // bytes are staged 1 KiB at a time, the next block's loads in flight while this one is linked
    // (the staging buffer has 64 zero bytes after `total`)
    auto load16 = [&](uint64_t g) -> u32x4 {
        return g + 16 <= total + 64 ? *(const u32x4*)(buf + g) : u32x4{0u, 0u, 0u, 0u};
    };
    const uint64_t a0 = seed0 & ~15ull;
    u32x4 nx = tid < 65 ? load16(a0 + 16 * (uint64_t)tid) : u32x4{0u, 0u, 0u, 0u};
    for (uint64_t q0 = a0; q0 < s1; q0 += 1024) {
        __syncthreads();
        if (tid < 65) ((u32x4*)bb)[tid] = nx;
        __syncthreads();
        if (q0 + 1024 < s1 && tid < 65) nx = load16(q0 + 1024 + 16 * (uint64_t)tid);
        const uint32_t r = (uint32_t)tid;
        const uint64_t q = q0 + r;
        const bool valid = q >= seed0 && q < s1 && q + 2 < total;
        uint32_t h = 0x10000u + (uint32_t)lane;   // distinct non-bucket for invalid lanes
        if (valid) h = lz_hash(__builtin_amdgcn_alignbyte(bb[(r >> 2) + 1], bb[r >> 2], r & 3) & 0xFFFFFFu);
        int prevLane = -1;
        bool last = true;
#pragma unroll 8
        for (int k = 0; k < 64; k++) {
            const uint32_t hk = __builtin_amdgcn_readlane(h, k);
            const bool eq = hk == h;
            if (eq && k < lane) prevLane = k;
            if (eq && k > lane) last = false;
        }
        const uint32_t off = (uint32_t)(q - seed0);   // < 65536; 0xFFFF is written only by the
        uint32_t d = 0;                               // segment's last position and never read
        if (valid && prevLane >= 0) d = (uint32_t)(lane - prevLane);
        for (int g = 0; g < 16; g++) {
            if (wid == g && valid) {
                if (prevLane < 0) {
                    const uint32_t hv = head[h];
                    if (hv != 0xFFFFu) { d = off - hv; if (d > (uint32_t)LZ_SEG) d = 0; }
                }
                if (last) head[h] = (uint16_t)off;   // one wave: its LDS ops stay in program order
            }
            __syncthreads();
        }
        if (q >= s0 && q < s1) link[q - L0] = (uint16_t)d;
    }
}

// ---- 2. best match at every position ---------------------------------------------------------
namespace {
__device__ __forceinline__ uint32_t lz_word(const uint32_t* w, uint32_t r) {
    return __builtin_amdgcn_alignbyte(w[(r >> 2) + 1], w[r >> 2], r & 3);
}
__device__ __forceinline__ uint32_t lz_byte(const uint32_t* w, uint32_t r) {
    return (w[r >> 2] >> (8 * (r & 3))) & 0xFFu;
}
}  // namespace

extern "C" __global__ void __launch_bounds__(1024)
ndfl_lz_match_kernel(LzArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t wb[LZ_WWORDS + 4];
    __shared__ __attribute__((aligned(16))) uint16_t lk[LZ_WIN + LZ_TILE];
    __shared__ uint32_t s_next;
    const int tid = threadIdx.x;
    if (tid == 0) s_next = 1024;
    const uint64_t p0 = a.p_begin + (uint64_t)blockIdx.x * LZ_TILE;
    const uint64_t p1 = min(p0 + LZ_TILE, a.p_end);
    const int64_t wb0 = (int64_t)p0 - LZ_WIN;         // window base (buffer index); p0 >= LZ_DS
    // stage window bytes [wb0, wb0 + 4*LZ_WWORDS) (zero past the buffer) and links [wb0, p1)
    for (int k = tid; k < LZ_WWORDS + 4; k += 1024) {
        const int64_t g = wb0 + 4 * (int64_t)k;
        uint32_t v = 0;
        if (g >= 0 && g + 4 <= (int64_t)a.total) v = *(const uint32_t*)(a.buf + g);
        else for (int b = 0; b < 4; b++) if (g + b >= 0 && g + b < (int64_t)a.total) v |= (uint32_t)a.buf[g + b] << (8 * b);
        wb[k] = v;
    }
    const int nlk = (int)(p1 - (uint64_t)wb0);
    for (int k = tid; k < nlk; k += 1024) {
        const int64_t g = wb0 + k;
        lk[k] = g >= (int64_t)a.L0 ? a.link[g - (int64_t)a.L0] : (uint16_t)0;
    }
    __syncthreads();
    const uint32_t minRun = a.min_run, maxRun = a.max_run;
    // chunk and parent chunk of the tile's first position (wave-uniform); later positions of the
    // tile step from them with 32-bit divisions (a claim runs beside other lanes' hops, so it must
    // be cheap: no 64-bit division per position)
    const uint64_t cs0 = LZ_DS + ((p0 - LZ_DS) / a.chunk_len) * a.chunk_len;
    const uint64_t pps0 = LZ_DS + ((p0 - LZ_DS) / a.parent_len) * a.parent_len;
    uint32_t st_pos = 0, st_hop = 0, st_hit = 0, st_cmp = 0;
    // Each lane searches positions one hop per iteration and takes the tile's next unclaimed position
    // (LDS counter) as soon as it finishes one: chain lengths vary by orders of magnitude, so static
    // assignment would leave the tile waiting on its unluckiest lanes.  The next link is read
    // together with the candidate.
    uint64_t i = p0 + tid;
    bool have = false;
    uint32_t ri = 0, rlo = 0, rhi = 0, maxlen = 0, wi0 = 0, best = 0, bestd = 0, rj = 0, d = 0, want = 0;
    for (;;) {
        if (!have) {
            while (i < p1) {
                // i - cs0 < LZ_TILE + chunk_len < 2^32
                const uint64_t cs = cs0 + (uint64_t)(((uint32_t)(i - cs0) / a.chunk_len) * a.chunk_len);
                const uint64_t e = min(cs + a.chunk_len, a.total);
                maxlen = (uint32_t)min((uint64_t)maxRun, e - i);
                const uint64_t ps = pps0 + (uint64_t)(((uint32_t)(i - pps0) / a.parent_len) * a.parent_len);
                const uint64_t off = ps - min((uint64_t)a.hist_limit, ps - a.vstart);
                const int64_t lo = max((int64_t)i - (int64_t)a.max_dist, (int64_t)off);
                const int64_t hi = (int64_t)i - (int64_t)a.min_dist;
                ri = (uint32_t)((int64_t)i - wb0);
                if (maxlen >= minRun && hi >= lo) {
                    st_pos++;
                    wi0 = lz_word(wb, ri);
                    rlo = (uint32_t)(lo - wb0);
                    rhi = (uint32_t)(hi - wb0);
                    rj = ri; d = lk[ri];
                    best = 0; bestd = 0; want = 0;
                    have = true;
                    break;
                }
                a.match[i - a.p_begin] = lz_byte(wb, ri);
                i = p0 + atomicAdd(&s_next, 1u);
            }
            if (!have) break;
        }
        // one hop
        bool fin = d == 0 || d > rj - rlo;                      // chain ends, or next candidate below lo
        if (!fin) {
            rj -= d;
            st_hop++;
            d = lk[rj];
            const uint32_t x0 = lz_word(wb, rj) ^ wi0;
            const uint32_t sb = lz_byte(wb, rj + best);
            if (rj <= rhi && (x0 & 0xFFFFFFu) == 0 && (best < 3 || sb == want)) {   // can be longer
                st_hit++;
                uint32_t run;
                if (x0) run = 3;
                else {
                    uint32_t k = 4;
                    for (;;) {
                        if (k >= maxlen) { run = maxlen; break; }
                        const uint32_t y = lz_word(wb, rj + k) ^ lz_word(wb, ri + k);
                        st_cmp++;
                        if (y) { run = k + (__builtin_ctz(y) >> 3); break; }
                        k += 4;
                    }
                }
                run = min(run, maxlen);
                if (run > best) {
                    best = run;
                    bestd = ri - rj;
                    fin = best >= maxlen;
                    if (!fin) want = lz_byte(wb, ri + best);
                }
            }
        }
        if (fin) {
            a.match[i - a.p_begin] = best >= minRun ? (best << 16 | (bestd - 1)) : lz_byte(wb, ri);
            have = false;
            i = p0 + atomicAdd(&s_next, 1u);
        }
    }
    if (a.stats) {
        atomicAdd(&a.stats[0], (unsigned long long)st_pos); atomicAdd(&a.stats[1], (unsigned long long)st_hop);
        atomicAdd(&a.stats[2], (unsigned long long)st_hit); atomicAdd(&a.stats[3], (unsigned long long)st_cmp);
    }
}

// ---- 2'. best match at the positions the greedy parse visits ---------------------------------
// The greedy parse (D/comp/Lz77Huffman.java:68-130) reads the best match only at the positions it
// visits -- about a fifth of the positions on text, and mostly word starts, whose candidate lists are
// short: on the config-3 text the visited positions hold 7 % of the candidates that a search at every
// position walks (tests/lz_parse_stats.c).  So each wave follows the parse through its own 512
// positions of a tile and searches only where the parse lands; a parse started anywhere merges with
// the true one within a few tokens (a literal lands on every position, a match on its end), so
// wave w's path from its segment start is the true path from the first position both visit on.
// After all waves have run, wave w checks the true entry into its segment (wave w-1's exit, in
// order): a position its own path visited means the rest of its path is exact; otherwise it follows
// the true path from the entry until that meets its own (or leaves the segment).  The tile's first
// wave starts LZP_LEAD positions before the tile (unless the tile starts a chunk, where the parse
// starts exactly), so its path has merged with the true one by the tile start -- or, rarely, not: a
// true-path position never searched keeps the sentinel LZP_NONE and the encode kernel searches it
// (lz_match_global).
//
// The search at one position is wave-cooperative: the window's positions are counting-sorted by a
// 13-bit hash of their first three bytes once per tile, and the 64 lanes test the position's whole
// bucket, 64 candidates per step -- a candidate whose run reaches minRun (>= 3) shares the three
// bytes -- keeping the longest run and, among equal runs, the nearest candidate (the reference
// scans distances upwards and keeps strictly longer runs, :71-84).  A long bucket first tests the
// 64 nearest distances: a run reaching the cap there ends the search (nothing farther can win).
namespace {
constexpr int LZP_TILE = 8192;                     // positions written per tile
constexpr int LZP_SEG = 512;                       // positions per wave (16 waves)
constexpr int LZP_LEAD = 256;                      // lead-in of the first wave (tiles inside a chunk)
constexpr int LZP_HBITS = 13;
constexpr int LZP_NPOS = LZP_LEAD + LZ_WIN + LZP_TILE;          // window positions (sorted)
constexpr int LZP_WWORDS = (LZP_NPOS + 272) / 4;                // window bytes as words (+ lookahead)
constexpr uint32_t LZP_NONE = 0xFFFFFFFFu;         // sentinel: position not searched
constexpr int LZP_NEAR = 128;                      // buckets longer than this test the nearest distances first

__device__ __forceinline__ uint32_t lzp_hash(uint32_t k) { return (k * 2654435761u) >> (32 - LZP_HBITS); }

// Wave maximum (all 64 lanes active): rotations within each row of 16 lanes by DPP, then the four
// row maxima through readlane -- a uniform (scalar) result, no LDS crossbar round trips.
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false));   // row_ror:8
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xF, 0xF, false));   // row_ror:4
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x122, 0xF, 0xF, false));   // row_ror:2
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x121, 0xF, 0xF, false));   // row_ror:1
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    return max(max(r0, r1), max(r2, r3));
}

// A wave's current chunk and parent chunk along its path (positions only grow): no division per
// search.  All wave-uniform.
struct LzpBnd {
    uint64_t cs, ps;
    __device__ __forceinline__ void init(const LzArgs& a, uint64_t q) {
        cs = LZ_DS + ((q - LZ_DS) / a.chunk_len) * a.chunk_len;
        ps = LZ_DS + ((q - LZ_DS) / a.parent_len) * a.parent_len;
    }
    __device__ __forceinline__ void advance(const LzArgs& a, uint64_t q) {
        while (q >= cs + a.chunk_len) cs += a.chunk_len;
        while (q >= ps + a.parent_len) ps += a.parent_len;
    }
};

struct LzpS {
    uint32_t wb[LZP_WWORDS + 4];                   // window bytes [wb0, wb0 + 4 * LZP_WWORDS)
    uint16_t sorted[LZP_NPOS];                     // window offsets, grouped by hash bucket
    uint32_t bend[1 << LZP_HBITS];                 // counts -> starts -> bucket ends (after the scatter)
    uint32_t vis[LZP_TILE / 32];                   // positions the waves' paths searched (tile-relative)
    uint32_t xit[16];                              // each wave's exit (tile-relative, may pass the tile)
    uint32_t scan[16];
};

// Wave-cooperative exact search at buffer position q (window-relative rq).  All lanes call with the
// same q; returns the match word (run << 16 | dist - 1, or the literal byte).
__device__ __forceinline__ uint32_t lzp_search(const LzArgs& a, const LzpS& S, int64_t wb0, uint64_t q, LzpBnd& bd,
                                               uint32_t* st) {
    const int lane = threadIdx.x & 63;
    const uint32_t rq = (uint32_t)((int64_t)q - wb0);
    bd.advance(a, q);
    const uint64_t e = min(bd.cs + a.chunk_len, a.total);
    const uint32_t maxlen = (uint32_t)min((uint64_t)a.max_run, e - q);
    const uint64_t off = bd.ps - min((uint64_t)a.hist_limit, bd.ps - a.vstart);
    const int64_t lo = max((int64_t)q - (int64_t)a.max_dist, (int64_t)off);
    const int64_t hi = (int64_t)q - (int64_t)a.min_dist;
    const uint32_t lit = lz_byte(S.wb, rq);
    if (maxlen < a.min_run || hi < lo) return lit;
    const uint32_t wq = lz_word(S.wb, rq);
    const uint32_t rlo = (uint32_t)(lo - wb0), rhi = (uint32_t)(hi - wb0);
    // run of candidate r (window-relative, in [rlo, rhi]) against q, capped at maxlen; 0 when the
    // first three bytes differ
    auto run_of = [&](uint32_t r) -> uint32_t {
        const uint32_t x0 = lz_word(S.wb, r) ^ wq;
        if (x0 & 0xFFFFFFu) return 0u;
        if (x0) return min(3u, maxlen);
        uint32_t k = 4;
        for (;;) {
            if (k >= maxlen) return maxlen;
            const uint32_t y = lz_word(S.wb, r + k) ^ lz_word(S.wb, rq + k);
            if (y) return min(k + (__builtin_ctz(y) >> 3), maxlen);
            k += 4;
        }
    };
    const uint32_t h = lzp_hash(wq & 0xFFFFFFu);
    const uint32_t B0 = h ? S.bend[h - 1] : 0u, B1 = S.bend[h];
    uint32_t best = 0;                                  // run << 16 | r (larger r: nearer)
    if (B1 - B0 > (uint32_t)LZP_NEAR) {
        // the 64 nearest distances: a run reaching the cap among them is the answer
        const uint32_t r = rhi - (uint32_t)lane;
        uint32_t k = 0;
        if ((int64_t)rhi - lane >= (int64_t)rlo) { const uint32_t run = run_of(r); if (run) k = run << 16 | r; }
        k = wave_max_dpp(k);
        if ((k >> 16) >= maxlen) best = k;
        st[1] += 64u;
    }
    if ((best >> 16) < maxlen) {
        for (uint32_t i = B0; i < B1; i += 64) {
            uint32_t k = 0;
            if (i + lane < B1) {
                const uint32_t r = S.sorted[i + lane];
                if (r >= rlo && r <= rhi) { const uint32_t run = run_of(r); if (run) k = run << 16 | r; }
            }
            best = max(best, k);
        }
        best = wave_max_dpp(best);
        st[1] += B1 - B0;
    }
    st[0]++;
    const uint32_t run = best >> 16;
    return run >= a.min_run ? (run << 16 | (rq - (best & 0xFFFFu) - 1)) : lit;
}
}  // namespace

extern "C" __global__ void __launch_bounds__(1024)
ndfl_lz_parse_match_kernel(LzArgs a, uint32_t lead_on) {
    __shared__ __attribute__((aligned(16))) LzpS S;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t p0 = a.p_begin + (uint64_t)blockIdx.x * LZP_TILE;
    const uint64_t p1 = min(p0 + LZP_TILE, a.p_end);
    const uint32_t ntile = (uint32_t)(p1 - p0);
    const int64_t wb0 = (int64_t)p0 - LZP_LEAD - LZ_WIN;
    uint32_t st[2] = {0u, 0u};                         // (NDFL_LZ_STATS: searches, bucket entries scanned)
    const uint64_t tk0 = a.stats ? wall_clock64() : 0;
    // positions never searched read as the sentinel (the searched ones are stored over it below)
    for (uint32_t k = (uint32_t)tid; k < ntile; k += 1024) a.match[p0 + k - a.p_begin] = LZP_NONE;
    for (int k = tid; k < LZP_WWORDS + 4; k += 1024) {
        const int64_t g = wb0 + 4 * (int64_t)k;
        uint32_t v = 0;
        if (g >= 0 && g + 4 <= (int64_t)a.total) v = *(const uint32_t*)(a.buf + g);
        else for (int b = 0; b < 4; b++) if (g + b >= 0 && g + b < (int64_t)a.total) v |= (uint32_t)a.buf[g + b] << (8 * b);
        S.wb[k] = v;
    }
    for (int k = tid; k < (1 << LZP_HBITS); k += 1024) S.bend[k] = 0;
    for (int k = tid; k < LZP_TILE / 32; k += 1024) S.vis[k] = 0;
    __syncthreads();
    // counting sort of the window's positions by hash (candidates: valid bytes, a full trigram)
    const uint32_t nsort = (uint32_t)(p1 - (uint64_t)wb0);
    const int64_t gmin = max((int64_t)a.vstart, wb0);
    for (uint32_t r = (uint32_t)tid; r < nsort; r += 1024) {
        const int64_t g = wb0 + r;
        if (g >= gmin && g + 2 < (int64_t)a.total) atomicAdd(&S.bend[lzp_hash(lz_word(S.wb, r) & 0xFFFFFFu)], 1u);
    }
    __syncthreads();
    {
        constexpr int PER = (1 << LZP_HBITS) / 1024;
        uint32_t v[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) { v[i] = S.bend[tid * PER + i]; sum += v[i]; }
        uint32_t tot;
        uint32_t run = block_excl_scan<uint32_t, 16>(sum, S.scan, tot);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; i++) { S.bend[tid * PER + i] = run; run += v[i]; }
    }
    __syncthreads();
    for (uint32_t r = (uint32_t)tid; r < nsort; r += 1024) {
        const int64_t g = wb0 + r;
        if (g >= gmin && g + 2 < (int64_t)a.total) {
            const uint32_t at = atomicAdd(&S.bend[lzp_hash(lz_word(S.wb, r) & 0xFFFFFFu)], 1u);
            S.sorted[at] = (uint16_t)r;
        }
    }
    __syncthreads();
    const uint64_t tk1 = a.stats ? wall_clock64() : 0;
    // chunk / parent chunk of the tile's lead-in start (positions step from them with 32-bit math)
    const uint64_t q00 = p0 - LZP_LEAD >= a.p_begin ? p0 - LZP_LEAD : p0;
    auto step_of = [&](uint32_t m) -> uint32_t { return (m >> 16) ? (m >> 16) : 1u; };
    // the waves' paths
    const uint64_t s_w = p0 + (uint64_t)w * LZP_SEG;
    const uint64_t e_w = min(s_w + LZP_SEG, p1);
    if (s_w < p1) {
        const bool chunk_start = ((p0 - LZ_DS) % a.chunk_len) == 0;
        uint64_t q = (w == 0 && lead_on && !chunk_start) ? q00 : s_w;
        LzpBnd bd;
        bd.init(a, q);
        while (q < e_w) {
            const uint32_t m = lzp_search(a, S, wb0, q, bd, st);
            if (q >= s_w) {
                const uint32_t t = (uint32_t)(q - p0);
                if (lane == 0) { a.match[q - a.p_begin] = m; atomicOr(&S.vis[t >> 5], 1u << (t & 31)); }
            }
            q += step_of(m);
        }
        if (lane == 0) S.xit[w] = (uint32_t)(q - p0);
    }
    __syncthreads();
    const uint64_t tk2 = a.stats ? wall_clock64() : 0;
    // the true entry of each wave's segment, in order
    const int nw = (int)((ntile + LZP_SEG - 1) / LZP_SEG);
    for (int v = 1; v < nw; v++) {
        if (w == v) {
            const uint32_t ent = S.xit[v - 1];
            const uint32_t sv = (uint32_t)v * LZP_SEG, ev = min(sv + (uint32_t)LZP_SEG, ntile);
            uint32_t x = S.xit[v];
            if (ent >= ev) x = ent;                     // the true path passes over this segment
            else if (!((S.vis[ent >> 5] >> (ent & 31)) & 1u)) {
                uint32_t t = ent;
                LzpBnd bd;
                bd.init(a, p0 + t);
                while (t < ev && !((S.vis[t >> 5] >> (t & 31)) & 1u)) {
                    const uint64_t q = p0 + t;
                    const uint32_t m = lzp_search(a, S, wb0, q, bd, st);
                    if (lane == 0) { a.match[q - a.p_begin] = m; atomicOr(&S.vis[t >> 5], 1u << (t & 31)); }
                    t += step_of(m);
                }
                if (t >= ev) x = t;                     // (else: met its own path, whose exit stands)
            }
            if (lane == 0) S.xit[v] = x;
        }
        __syncthreads();
    }
    if (a.stats && lane == 0) { atomicAdd(&a.stats[0], (unsigned long long)st[0]); atomicAdd(&a.stats[1], (unsigned long long)st[1]); }
    if (a.stats && tid == 0) {                         // tile phase times (wall clock, 100 MHz): stage + sort, paths, entries
        atomicAdd(&a.stats[3], (unsigned long long)(tk1 - tk0)); atomicAdd(&a.stats[4], (unsigned long long)(tk2 - tk1));
        atomicAdd(&a.stats[5], (unsigned long long)(wall_clock64() - tk2)); atomicAdd(&a.stats[6], 1ull);
    }
}

// Exact search at one position from global memory (the encode kernel's rare fallback for a true-path
// position the parse-driven search did not reach): every distance of the window, 64 per step, the
// nearest first; a step whose best run reaches the cap ends the search.  Wave-uniform q.
namespace {
struct LzGlob {
    const uint8_t* buf;
    uint64_t total, vstart;
    uint32_t chunk_len, parent_len, hist_limit, min_run, max_run, min_dist, max_dist;
};
__device__ __noinline__ uint32_t lz_match_global(const LzGlob& g, uint64_t q) {
    const int lane = threadIdx.x & 63;
    const uint64_t cs = LZ_DS + ((q - LZ_DS) / g.chunk_len) * g.chunk_len;
    const uint64_t e = min(cs + g.chunk_len, g.total);
    const uint32_t maxlen = (uint32_t)min((uint64_t)g.max_run, e - q);
    const uint64_t ps = LZ_DS + ((q - LZ_DS) / g.parent_len) * g.parent_len;
    const uint64_t off = ps - min((uint64_t)g.hist_limit, ps - g.vstart);
    const int64_t lo = max((int64_t)q - (int64_t)g.max_dist, (int64_t)off);
    const uint32_t lit = g.buf[q];
    if (maxlen < g.min_run || (int64_t)q - (int64_t)g.min_dist < lo) return lit;
    const uint32_t dmax = (uint32_t)((int64_t)q - lo);
    uint32_t best = 0;                                  // run << 16 | (65535 - dist)
    for (uint32_t d0 = g.min_dist; d0 <= dmax; d0 += 64) {
        const uint32_t d = d0 + (uint32_t)lane;
        uint32_t k = 0;
        if (d <= dmax) {
            const uint8_t* x = g.buf + (q - d);
            const uint8_t* y = g.buf + q;
            uint32_t run = 0;
            while (run < maxlen && x[run] == y[run]) run++;
            if (run) k = run << 16 | (65535u - d);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) k = max(k, (uint32_t)__shfl_xor((int)k, o, 64));
        best = max(best, k);
        if ((best >> 16) >= maxlen) break;
    }
    const uint32_t run = best >> 16;
    return run >= g.min_run ? (run << 16 | ((65535u - (best & 0xFFFFu)) - 1)) : lit;
}
}  // namespace

// ---- 3. parse + block encode ------------------------------------------------------------------
namespace {
struct LzEncArgs {
    const uint32_t* match;    // per data position of this batch: run << 16 | dist-1, or literal
    uint64_t batch_x0;        // data index of match[0]
    uint64_t n;               // data bytes of the call
    uint32_t chunk_len;
    uint32_t chunk_base;      // first chunk of this batch
    uint32_t nchunks_batch;
    uint32_t nchunks;         // chunks of the call
    int32_t final_last;
    int32_t dynamic;
    uint32_t base_bit;
    uint32_t* out;
    uint64_t* status;
    uint32_t* ticket;
    uint64_t* edge_w;
    uint32_t* edge_v;
    uint64_t* chunk_bits;     // optional [nchunks]: block bits
    uint32_t* match_rw;       // = match: positions the parse reaches but the search skipped (LZP_NONE) are
    LzGlob g;                 //   searched here from global memory (lz_match_global) and stored back
    unsigned long long* stats;// optional (NDFL_LZ_STATS): [2] fallback searches
};

// Length symbol / extra of a run (D/comp/Lz77Huffman.java:92-111) and distance symbol / extra of
// d = dist-1 (:112-127).
__device__ __forceinline__ void dist_sym(uint32_t d, uint32_t& sym, uint32_t& ne, uint32_t& ex) {
    if (d < 4) { sym = d; ne = 0; ex = 0; }
    else {
        ne = 30 - __clz(d);
        sym = (ne << 1) + (d >> ne);
        ex = d & ((1u << ne) - 1);
    }
}
}  // namespace

extern "C" __global__ void __launch_bounds__(DT, 1)
ndfl_lz_encode_kernel(LzEncArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t big[32768];   // steps (u16) -> scratch -> bit buffer
    __shared__ uint32_t tokm[2048];                                 // token starts, 1 bit per position
    __shared__ Persist ps;
    __shared__ uint32_t wexit[16];                                  // the parse walk's true exit per wave
    static_assert(OUTW <= 32768, "bit buffer must fit the step array");
    uint32_t* obuf = big;
    char* scr = (char*)big;
    uint16_t* step = (uint16_t*)big;
    uint32_t* hlit = (uint32_t*)(scr + SCR_HLIT);
    uint32_t* hdist = (uint32_t*)(scr + SCR_HDIST);
    uint32_t* misc = (uint32_t*)(scr + SCR_MISC);
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;

    const uint64_t tq0 = a.stats ? wall_clock64() : 0;   // (NDFL_LZ_STATS: phase times of chunk workgroups)
    if (tid == 0) ps.chunk = a.chunk_base + atomicAdd(a.ticket, 1u);
    for (int k = tid; k < 2048; k += DT) tokm[k] = 0;
    __syncthreads();
    const uint32_t c = ps.chunk;
    const uint64_t cs = (uint64_t)c * a.chunk_len;
    const uint32_t len_c = (uint32_t)min((uint64_t)a.chunk_len, a.n - cs);
    const bool is_final = a.final_last && (c + 1 == a.nchunks);
    const uint32_t* mt = a.match + (cs - a.batch_x0);

    // ---- parse: steps in LDS, one wave walks them (D/comp/Lz77Huffman.java:68-130) -----------
    // (1024: a position the match search did not reach).  16-byte loads, four in flight per thread
    auto step_of = [](uint32_t mk) -> uint32_t { const uint32_t m = mk >> 16; return mk == LZP_NONE ? 1024u : m ? m : 1u; };
    if ((((uintptr_t)mt) & 15) == 0) {
        const uint32_t nq = len_c / 4;
#pragma unroll 4
        for (uint32_t k = (uint32_t)tid; k < nq; k += DT) {
            const u32x4 v = *(const u32x4*)(mt + 4 * k);
            *(uint2*)&step[4 * k] = make_uint2(step_of(v.x) | step_of(v.y) << 16, step_of(v.z) | step_of(v.w) << 16);
        }
        for (uint32_t k = 4 * nq + (uint32_t)tid; k < len_c; k += DT) step[k] = (uint16_t)step_of(mt[k]);
    } else {
#pragma unroll 4
        for (uint32_t k = (uint32_t)tid; k < len_c; k += DT) step[k] = (uint16_t)step_of(mt[k]);
    }
    if (tid == 0) ps.P = 0;                                         // (repairs made)
    __syncthreads();
    // The walk is split over the 16 waves: wave w walks its 1/16 of the chunk from the segment start
    // (a multiple of 32 positions, so each wave owns whole words of tokm), as the match kernel's
    // paths do; then, in order, wave w takes the true entry (wave w-1's true exit): its own walk
    // visited it (the common case -- parses merge within a few tokens), or the wave re-walks from it
    // one token at a time until it lands on its own walk.  Token bits its walk set before the entry or
    // between true tokens are cleared.  A step of 1024 marks a position the match search skipped.
    const uint64_t tqa = a.stats ? wall_clock64() : 0;
    const uint32_t lenc = (uint32_t)__builtin_amdgcn_readfirstlane((int)len_c);
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(wid);
    const uint32_t segw = ((lenc + 16 * 32 - 1) / (16 * 32)) * 32;
    const uint32_t sg0 = min(wv * segw, lenc), sg1 = min(sg0 + segw, lenc);
    uint32_t nrep = 0;
    auto fallback = [&](uint32_t q) -> uint32_t {                   // (wave-uniform q) returns the step
        const uint32_t m = lz_match_global(a.g, LZ_DS + cs + q);
        if (lane == 0) a.match_rw[cs + q - a.batch_x0] = m;
        if (lane == 0) step[q] = (uint16_t)((m >> 16) ? (m >> 16) : 1u);
        nrep++;
        return (m >> 16) ? (m >> 16) : 1u;
    };
    auto clear_bits = [&](uint32_t b0, uint32_t b1) {                // tokm bits [b0, b1) (inside this wave's words)
        if (b0 >= b1) return;
        for (uint32_t k = (b0 >> 5) + (uint32_t)lane; k <= ((b1 - 1) >> 5); k += 64) {
            const uint32_t lo = max(b0, k << 5) - (k << 5), hi = min(b1, (k + 1) << 5) - (k << 5);
            const uint32_t m = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
            tokm[k] &= ~m;
        }
    };
    // the walk starts at the segment's first position the match search reached (a wave start of the
    // match kernel for the default 64 KiB chunks), so it follows searched positions
    uint32_t wst = sg1;
    for (uint32_t b = sg0; b < sg1; b += 64) {
        const uint64_t m = __ballot(b + lane < sg1 && step[b + lane] < 1024);
        if (m) { wst = b + (uint32_t)__builtin_ctzll(m); break; }
    }
    wst = (uint32_t)__builtin_amdgcn_readfirstlane((int)wst);
    uint32_t xspec = sg0;                                            // this wave's walk exit
    if (wst < sg1) {
        uint32_t cur = wst;
        while (cur < sg1) {
            const uint32_t s = cur + lane < lenc ? (uint32_t)step[cur + lane] : 64u;
            const uint32_t lim = min(64u, sg1 - cur);
            uint64_t mask = 0;
            uint32_t p = 0;
            do {
                mask |= 1ull << p;
                p += (uint32_t)__builtin_amdgcn_readlane((int)s, (int)p);
            } while (p < lim);
            if (p >= 1024) {
                const uint32_t q = p - 1024;                         // (its token bit is in mask)
                p = q + fallback(cur + q);
            }
            // OR the 64-bit window mask into tokm at bit `cur` (3 words at most)
            const uint32_t sh = cur & 31, w0 = cur >> 5;
            if (lane < 3) {
                const uint32_t piece = lane == 0 ? (uint32_t)(mask << sh)
                                     : lane == 1 ? (uint32_t)(mask >> (32 - sh))
                                     : (sh ? (uint32_t)(mask >> (64 - sh)) : 0u);
                if (piece && w0 + lane < 2048) tokm[w0 + lane] |= piece;
            }
            cur += p;
            cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur);
        }
        xspec = cur;
    }
    __syncthreads();
    const uint64_t tqb = a.stats ? wall_clock64() : 0;
    // true entries, in wave order (wexit[w]: wave w's true exit)
    if (wid == 0 && lane == 0) wexit[0] = xspec;
    __syncthreads();
    for (int v = 1; v < 16; v++) {
        if (wid == v && sg0 < sg1) {
            const uint32_t e = wexit[v - 1];
            uint32_t x = xspec;
            if (e >= sg1) {
                clear_bits(sg0, sg1);                                // the true parse passes over this segment
                x = e;
            } else {
                clear_bits(sg0, e);
                uint32_t t = e;
                for (;;) {
                    if (t >= sg1) { x = t; break; }
                    if ((tokm[t >> 5] >> (t & 31)) & 1u) break;      // on this wave's walk: x = its exit
                    if (lane == 0) tokm[t >> 5] |= 1u << (t & 31);
                    uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)step[t]);
                    if (st >= 1024) st = fallback(t);
                    clear_bits(t + 1, min(t + st, sg1));
                    t += st;
                }
            }
            if (lane == 0) wexit[v] = x;
        } else if (wid == v && lane == 0) {
            wexit[v] = wexit[v - 1];
        }
        __syncthreads();
    }
    if (a.stats && tid == 0) {
        const uint64_t tqc = wall_clock64();
        atomicAdd(&a.stats[14], tqb - tqa); atomicAdd(&a.stats[15], tqc - tqb);
    }
    if (nrep) {
        __threadfence();
        if (lane == 0) atomicAdd((unsigned long long*)&ps.P, (unsigned long long)nrep);
        if (lane == 0 && a.stats) atomicAdd(&a.stats[2], (unsigned long long)nrep);
    }
    __syncthreads();
    if (ps.P) __threadfence();                                      // the stored repairs, seen by every wave

    const uint64_t tq1 = a.stats ? wall_clock64() : 0;
    // ---- histograms --------------------------------------------------------------------------
    if (tid < 288) hlit[tid] = 0;
    if (tid < 32) hdist[tid] = 0;
    __syncthreads();
    const uint32_t t0 = (uint32_t)tid * 64;
    const uint64_t mymask = (uint64_t)tokm[2 * tid] | (uint64_t)tokm[2 * tid + 1] << 32;
#define NDFL_FOR_TOKENS(...)                                                       \
    for (uint64_t mm_ = mymask; mm_; mm_ &= mm_ - 1) {                             \
        const uint32_t pos_ = t0 + (uint32_t)__builtin_ctzll(mm_);                 \
        const uint32_t m = mt[pos_];                                               \
        const uint32_t run = m >> 16;                                              \
        __VA_ARGS__                                                                \
    }
    NDFL_FOR_TOKENS({
        if (!run) { atomicAdd(&hlit[m & 0xFF], 1u); continue; }
        uint32_t sym, ne, ex; run_sym(run, sym, ne, ex);
        atomicAdd(&hlit[sym], 1u);
        dist_sym(m & 0xFFFF, sym, ne, ex);
        atomicAdd(&hdist[sym], 1u);
    })
    if (tid == 0) {
        atomicAdd(&hlit[256], 1u);                              // end of block (:131-132)
        if (a.dynamic && len_c == 0) atomicAdd(&hlit[0], 1u);  // (:146-147)
    }
    __syncthreads();

    const uint64_t tq2 = a.stats ? wall_clock64() : 0;
    // ---- codes ---------------------------------------------------------------------------------
    build_block_codes(a.dynamic != 0, scr, ps);
    const uint32_t packedLo = misc[4], packedHi = misc[5];
    __syncthreads();
    const uint64_t tq3 = a.stats ? wall_clock64() : 0;

    // ---- token bits, block size ------------------------------------------------------------------
    uint32_t mybits = 0;
    NDFL_FOR_TOKENS({
        if (!run) { mybits += ps.litCode[m & 0xFF] >> 16; continue; }
        uint32_t sym, ne, ex; run_sym(run, sym, ne, ex);
        mybits += (ps.litCode[sym] >> 16) + ne;
        dist_sym(m & 0xFFFF, sym, ne, ex);
        mybits += (ps.distCode[sym] >> 16) + ne;
    })
    uint32_t tokTotal;
    const uint32_t myoff = block_excl_scan<uint32_t, NW>(mybits, ps.scan32, tokTotal);
    const uint32_t eobLen = ps.litCode[256] >> 16;
    const uint32_t hdrBits = ps.hdrBits;
    const uint64_t S = (uint64_t)hdrBits + tokTotal + eobLen;
    if (tid == 0) {
        if (c == 0) st_agent(&a.status[0], ST_PRE | (a.base_bit + S));
        else st_agent(&a.status[c], ST_AGG | S);
        if (a.chunk_bits) a.chunk_bits[c] = S;
    }
    const uint32_t nwl = (uint32_t)((S + 31) >> 5) + 1;
    __syncthreads();
    for (uint32_t k = (uint32_t)tid; k < nwl; k += DT) obuf[k] = 0;
    __syncthreads();

    // ---- emit ----------------------------------------------------------------------------------
    emit_block_header(obuf, is_final, a.dynamic != 0, ps, packedLo, packedHi, hdrBits, tokTotal, eobLen);
    {
        BitPut bp; bp.init(obuf, hdrBits + myoff);
        NDFL_FOR_TOKENS({
            if (!run) { const uint32_t lc = ps.litCode[m & 0xFF]; bp.put(lc & 0xFFFF, lc >> 16); continue; }
            uint32_t sym, ne, ex; run_sym(run, sym, ne, ex);
            const uint32_t sc = ps.litCode[sym];
            bp.put(sc & 0xFFFF, sc >> 16);
            bp.put(ex, ne);
            dist_sym(m & 0xFFFF, sym, ne, ex);
            const uint32_t dc = ps.distCode[sym];
            bp.put(dc & 0xFFFF, dc >> 16);
            bp.put(ex, ne);
        })
        bp.flush();
    }
#undef NDFL_FOR_TOKENS
    __syncthreads();
    const uint64_t tq4 = a.stats ? wall_clock64() : 0;
    block_lookback(c, a.base_bit, S, a.status, ps);
    block_store(obuf, ps.P, S, c, a.out, a.edge_w, a.edge_v);
    if (a.stats && tid == 0) {
        const uint64_t tq5 = wall_clock64();
        atomicAdd(&a.stats[8], tq1 - tq0); atomicAdd(&a.stats[9], tq2 - tq1); atomicAdd(&a.stats[10], tq3 - tq2);
        atomicAdd(&a.stats[11], tq4 - tq3); atomicAdd(&a.stats[12], tq5 - tq4); atomicAdd(&a.stats[13], 1ull);
    }
    (void)lane;
}
