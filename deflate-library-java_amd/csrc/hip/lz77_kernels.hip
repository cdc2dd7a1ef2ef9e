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
    static_assert(OUTW <= 32768, "bit buffer must fit the step array");
    uint32_t* obuf = big;
    char* scr = (char*)big;
    uint16_t* step = (uint16_t*)big;
    uint32_t* hlit = (uint32_t*)(scr + SCR_HLIT);
    uint32_t* hdist = (uint32_t*)(scr + SCR_HDIST);
    uint32_t* misc = (uint32_t*)(scr + SCR_MISC);
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;

    if (tid == 0) ps.chunk = a.chunk_base + atomicAdd(a.ticket, 1u);
    for (int k = tid; k < 2048; k += DT) tokm[k] = 0;
    __syncthreads();
    const uint32_t c = ps.chunk;
    const uint64_t cs = (uint64_t)c * a.chunk_len;
    const uint32_t len_c = (uint32_t)min((uint64_t)a.chunk_len, a.n - cs);
    const bool is_final = a.final_last && (c + 1 == a.nchunks);
    const uint32_t* mt = a.match + (cs - a.batch_x0);

    // ---- parse: steps in LDS, one wave walks them (D/comp/Lz77Huffman.java:68-130) -----------
    for (uint32_t k = (uint32_t)tid; k < len_c; k += DT) {
        const uint32_t m = mt[k] >> 16;
        step[k] = (uint16_t)(m ? m : 1u);
    }
    __syncthreads();
    if (wid == 0) {
        uint32_t cur = 0;
        while (cur < len_c) {
            const uint32_t s = cur + lane < len_c ? (uint32_t)step[cur + lane] : 64u;
            uint64_t mask = 0;
            uint32_t p = 0;
            while (p < 64 && cur + p < len_c) {
                mask |= 1ull << p;
                p += (uint32_t)__builtin_amdgcn_readlane((int)s, (int)p);
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
        }
    }
    __syncthreads();

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

    // ---- codes ---------------------------------------------------------------------------------
    build_block_codes(a.dynamic != 0, scr, ps);
    const uint32_t packedLo = misc[4], packedHi = misc[5];
    __syncthreads();

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
    block_lookback(c, a.base_bit, S, a.status, ps);
    block_store(obuf, ps.P, S, c, a.out, a.edge_w, a.edge_v);
    (void)lane;
}
