// deflate_kernels.hip -- MI355X (gfx950) DEFLATE block encoder.
//
// Replaces the per-chunk loop DeflaterOutputStream.writeBuffer -> Lz77Huffman.decide/compressTo
// -> BitOut.writeBits (D/DeflaterOutputStream.java:119-171, D/comp/Lz77Huffman.java:42-286) for
// the RLE_* and LITERAL_* presets.  One 1024-thread workgroup encodes one chunk (<= 64 KiB) in a
// single pass over HBM:
//   1. the chunk is loaded once into registers (64 B per lane, 16-B loads) and CRC-32'd there;
//   2. run pieces are found with a ballot-free bitmask per lane + a block suffix-min;
//   3. the greedy RLE parse is evaluated in closed form per run piece into LDS
//      histograms;
//   4. length-limited package-merge (exact reference tie order: packages before leaves on equal
//      frequency, D/comp/Lz77Huffman.java:319-333) runs as parallel merge-path levels + a prefix
//      backtrack; canonical codes are built from per-length bitmasks;
//   5. each lane's token bits are block-scanned; the chunk's global bit offset comes from a
//      decoupled look-back over per-chunk status words (chunk ids from an atomic ticket, so a
//      workgroup only ever waits on workgroups that already started);
//   6. tokens are packed into a word-aligned LDS bit buffer with LDS atomicOr and streamed out
//      with coalesced stores; the two boundary words of each chunk go to an edge list merged by
//      ndfl_edge_fixup.
// D/ = /root/reference/src/io/nayuki/deflate/
#include "ndfl_common.hpp"

namespace {

constexpr int DT = 1024;                  // threads per workgroup
constexpr int NW = DT / 64;               // waves per workgroup
constexpr int MAX_CHUNK = 65536;
constexpr int OUTW = 18600;               // LDS bit-buffer words (>= 594,362 bits)

constexpr uint64_t ST_AGG = 1ull << 62;
constexpr uint64_t ST_PRE = 2ull << 62;
constexpr uint64_t ST_VAL = (1ull << 62) - 1;

// ---- LDS layout (bytes) -------------------------------------------------------------------
// [0, OUTW*4)          bit buffer; during code construction it is overlaid by scratch below
// then persistent small arrays.
constexpr int SCR_HLIT = 0;                         // u32[288] literal/length histogram
constexpr int SCR_HDIST = SCR_HLIT + 288 * 4;       // u32[32]
constexpr int SCR_LAST = SCR_HDIST + 32 * 4;        // u8[1024] last byte of each lane
constexpr int SCR_KEY = SCR_LAST + 1024;            // u32[288]
constexpr int SCR_LF = SCR_KEY + 288 * 4;           // u32[288] sorted leaf freq
constexpr int SCR_LS = SCR_LF + 288 * 4;            // u32[288] sorted leaf symbol
constexpr int SCR_PFA = SCR_LS + 288 * 4;           // u32[304] packages
constexpr int SCR_PFB = SCR_PFA + 304 * 4;          // u32[304]
constexpr int SCR_MF = SCR_PFB + 304 * 4;           // u32[608] merged list
constexpr int SCR_MPK = SCR_MF + 608 * 4;           // u32[15][20] is-package bits per level
constexpr int SCR_LVL = SCR_MPK + 15 * 20 * 4;      // u32[16] leaves per level
constexpr int SCR_LEN = SCR_LVL + 16 * 4;           // u8[320] code lengths (lit ++ dist)
constexpr int SCR_CLLEN = SCR_LEN + 320;            // u8[32] code-length-code lengths
constexpr int SCR_BLC = SCR_CLLEN + 32;             // u32[16] bl_count
constexpr int SCR_NXC = SCR_BLC + 16 * 4;           // u32[16] next code
constexpr int SCR_MASK = SCR_NXC + 16 * 4;          // u32[16][10] symbols-by-length bitmask
constexpr int SCR_CLH = SCR_MASK + 16 * 10 * 4;     // u32[20] code-length histogram
constexpr int SCR_MISC = SCR_CLH + 20 * 4;          // u32[16]
constexpr int SCR_END = SCR_MISC + 16 * 4;
static_assert(2 * SCR_END <= OUTW * 4, "scratch (two package-merge problems) must fit in the bit buffer");

struct Persist {
    uint32_t litCode[288];    // rev(code) | len << 16
    uint32_t distCode[32];
    uint32_t clCode[20];
    uint8_t clSym[320];
    uint8_t clExtra[320];
    uint16_t clOff[320];      // bit offset of each code-length symbol inside the header body
    uint64_t scan64[NW];
    uint32_t scan32[NW];
    uint32_t chunk;           // ticket
    uint32_t nsym, ncl, hlit, hdist;
    uint32_t hdrBits;         // total header bits (incl. bfinal/btype)
    uint32_t clBodyBits;
    uint64_t P;               // chunk global bit offset
    uint32_t crcAcc[NW];
};

// The split passes (hist, emit) keep no code-construction state: a smaller block of persistent LDS,
// so that two emit workgroups (bit buffer + this) fit a CU.
struct PersistS {
    uint32_t litCode[288];
    uint32_t distCode[32];
    uint64_t scan64[NW];
    uint32_t scan32[NW];
    uint32_t chunk;
    uint32_t hdrBits;
    uint64_t P;
    uint32_t crcAcc[NW];
};

struct Args {
    const uint8_t* in;        // data region of this call (device)
    uint64_t n;
    uint32_t chunk_len;
    uint32_t nchunks;
    int32_t prev_byte;        // byte preceding chunk 0, or -1 if none (no history)
    int32_t hist_enabled;     // historyLookbehindLimit > 0
    int32_t final_last;       // last chunk is bfinal
    int32_t rle;              // 1: RLE preset (dist 1, runs 3..258); 0: LITERAL preset
    int32_t dynamic;
    uint32_t parent_len;      // history start rule: the chunk of this length containing the block
                              // (BinarySplit sub-blocks, D/comp/BinarySplit.java:44-45); = chunk_len otherwise
    uint32_t base_bit;        // bit offset of chunk 0 in `out` (0..7)
    uint32_t* out;            // word-aligned output, words [0, ...)
    uint64_t* status;         // [nchunks], zeroed
    uint32_t* ticket;         // zeroed
    uint64_t* edge_w;         // [2*nchunks]
    uint32_t* edge_v;         // [2*nchunks]
    uint64_t* chunk_bits;     // optional [nchunks]
    uint32_t* crc_raw;        // optional [nchunks]
    const uint32_t* crc_tab;  // slicing-by-4 tables (1024 u32)
    const uint32_t* crc_x;    // x^(8k) k<64 then x^(8*64k) k<1024
    uint64_t* prof;           // optional [nchunks][8] phase timestamps (wall clock)
    // split pipeline (hist -> codes -> offsets -> emit), see ndfl_deflate_codes_kernel
    uint32_t* hist_out;       // [nchunks][HREC] histograms: literal/length [0,288), distance [288,320)
    const uint32_t* codes;    // [nchunks][CREC] code records
    const uint64_t* chunk_off;// [nchunks] global bit offset of each chunk
    uint32_t c0;              // split passes: first chunk of this launch (slab pipeline), grid = chunks
    uint32_t pf_dist;         // split passes: touch chunk c + pf_dist (the next wave of resident
                              // workgroups on this XCD) into L2 while chunk c is processed; 0: off
};

// Split pipeline record layouts.
constexpr int HREC = 320;                 // u32 per chunk histogram record
constexpr int CREC_LIT = 0;               // u32[288] rev(code) | len << 16
constexpr int CREC_DIST = 288;            // u32[32]
constexpr int CREC_HDR = 320;             // u32[HDRW] header bits from local bit 0 (bfinal .. code-length symbols)
constexpr int HDRW = 80;                  // >= 3 + 14 + 57 + 316 * 7 = 2286 bits (every code-length entry costs <= 7 bits)
constexpr int CREC_META = CREC_HDR + HDRW;  // [0] hdrBits
constexpr int CREC = CREC_META + 16;
enum { MODE_FUSED = 0, MODE_HIST = 1, MODE_EMIT = 2 };
// hist pass: HCOPY lane-interleaved histogram copies at a stride of HSTR words (HSTR mod 64 = 20:
// the copies of a symbol fall in different LDS banks)
#ifndef NDFL_HCOPY
#define NDFL_HCOPY 8
#endif
constexpr int HCOPY = NDFL_HCOPY;
constexpr int HSTR = HCOPY > 4 ? 340 : 336;

// Length symbol / extra bits of a run 3..258 (D/comp/Lz77Huffman.java:92-111).
__device__ __forceinline__ void run_sym(uint32_t run, uint32_t& sym, uint32_t& ne, uint32_t& ex) {
    if (run < 11) { sym = run + 254; ne = 0; ex = 0; }
    else if (run == 258) { sym = 285; ne = 0; ex = 0; }
    else {
        uint32_t r = run - 3;
        ne = 29 - __clz(r);
        sym = (ne << 2) + (r >> ne) + 257;
        ex = r & ((1u << ne) - 1);
    }
}

// ---- Package-merge code lengths (D/comp/Lz77Huffman.java:309-335) ---------------------------
// hist: n entries (LDS).  Writes lens[0..n) (LDS, u8).  Every thread of the block must call (the
// barriers are shared); thread `t` of the calling group works on this problem when `active`, so two
// independent problems (literal/length and distance codes) run side by side on disjoint thread
// ranges with their own scratch `s`.
__device__ void pm_lengths(const uint32_t* hist, int n, int L, uint8_t* lens, char* s, int t, bool active) {
    uint32_t* key = (uint32_t*)(s + SCR_KEY);
    uint32_t* lf = (uint32_t*)(s + SCR_LF);
    uint32_t* ls = (uint32_t*)(s + SCR_LS);
    uint32_t* pfA = (uint32_t*)(s + SCR_PFA);
    uint32_t* pfB = (uint32_t*)(s + SCR_PFB);
    uint32_t* mf = (uint32_t*)(s + SCR_MF);
    uint32_t* mpk = (uint32_t*)(s + SCR_MPK);
    uint32_t* lvl = (uint32_t*)(s + SCR_LVL);
    if (active && t < n) {
        uint32_t f = hist[t];
        key[t] = f ? (f << 9 | (uint32_t)t) : 0xFFFFFFFFu;
    }
    if (active && t < 15 * 20) mpk[t] = 0;
    __syncthreads();
    // leaves sorted by (freq, symbol): rank by counting (n <= 288, broadcast LDS reads)
    uint32_t nl = 0;
    if (active) for (int j = 0; j < n; j++) nl += key[j] != 0xFFFFFFFFu;   // uniform per problem
    if (active && t < n) {
        uint32_t k = key[t];
        if (k != 0xFFFFFFFFu) {
            uint32_t r = 0;
            for (int j = 0; j < n; j++) r += key[j] < k;
            lf[r] = k >> 9;
            ls[r] = (uint32_t)t;
        }
        lens[t] = 0;
    }
    __syncthreads();
    const bool work = active && nl >= 2;   // otherwise all zero lengths (callers never need this for litlen/dist)
    uint32_t np = 0;
    uint32_t* pf = pfA;
    uint32_t* pfn = pfB;
    for (int it = 0; it < L; it++) {
        const uint32_t m = np + nl;
        if (work && (uint32_t)t < m) {
            uint32_t f, pos;
            bool isp = (uint32_t)t < np;
            if (isp) {
                f = pf[t];
                // # leaves with freq < f
                uint32_t lo = 0, hi = nl;
                while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (lf[mid] < f) lo = mid + 1; else hi = mid; }
                pos = (uint32_t)t + lo;
            } else {
                uint32_t r = (uint32_t)t - np;
                f = lf[r];
                // # packages with freq <= f
                uint32_t lo = 0, hi = np;
                while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (pf[mid] <= f) lo = mid + 1; else hi = mid; }
                pos = r + lo;
            }
            mf[pos] = f;
            if (isp) atomicOr(&mpk[it * 20 + (pos >> 5)], 1u << (pos & 31));
        }
        __syncthreads();
        const uint32_t np2 = m >> 1;
        if (work && (uint32_t)t < np2) pfn[t] = mf[2 * t] + mf[2 * t + 1];
        __syncthreads();
        np = np2;
        uint32_t* tmp = pf; pf = pfn; pfn = tmp;
    }
    // backtrack: prefix of 2(nl-1) items at the last level; leaves in the prefix of each level.
    if (work && t < 64) {
        uint32_t m = 2 * (nl - 1);
        for (int it = L - 1; it >= 0; it--) {
            uint32_t cnt = 0;
            if (t < 20) {
                uint32_t w = mpk[it * 20 + t];
                uint32_t lo = (uint32_t)t * 32;
                if (lo + 32 <= m) cnt = __popc(w);
                else if (lo < m) cnt = __popc(w & ((1u << (m - lo)) - 1));
            }
            cnt = wave_sum(cnt);
            if (t == 0) lvl[it] = m - cnt;
            m = 2 * cnt;
        }
    }
    __syncthreads();
    if (work && (uint32_t)t < nl) {
        uint32_t c = 0;
        for (int it = 0; it < L; it++) c += (uint32_t)t < lvl[it];
        lens[ls[t]] = (uint8_t)c;
    }
    __syncthreads();
}
__device__ __forceinline__ void pm_lengths(const uint32_t* hist, int n, int L, uint8_t* lens, char* s) {
    pm_lengths(hist, n, L, lens, s, (int)threadIdx.x, true);
}

// Canonical codes (D/comp/Lz77Huffman.java:368-391): rev(code) | len << 16.
__device__ void canon_codes(const uint8_t* lens, int n, uint32_t* codes, char* s) {
    uint32_t* blc = (uint32_t*)(s + SCR_BLC);
    uint32_t* nxc = (uint32_t*)(s + SCR_NXC);
    uint32_t* mask = (uint32_t*)(s + SCR_MASK);
    const int tid = threadIdx.x;
    if (tid < 16) blc[tid] = 0;
    if (tid < 160) mask[tid] = 0;
    __syncthreads();
    if (tid < n) {
        uint32_t l = lens[tid];
        if (l) {
            atomicAdd(&blc[l], 1u);
            atomicOr(&mask[l * 10 + (tid >> 5)], 1u << (tid & 31));
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t code = 0;
        blc[0] = 0;
        for (int b = 1; b < 16; b++) { code = (code + blc[b - 1]) << 1; nxc[b] = code; }
    }
    __syncthreads();
    if (tid < n) {
        uint32_t l = lens[tid];
        uint32_t c = 0;
        if (l) {
            uint32_t rank = 0;
            const int wi = tid >> 5;
            for (int w = 0; w < wi; w++) rank += __popc(mask[l * 10 + w]);
            rank += __popc(mask[l * 10 + wi] & ((1u << (tid & 31)) - 1));
            uint32_t code = nxc[l] + rank;
            c = (__brev(code) >> (32 - l)) | (l << 16);
        }
        codes[tid] = c;
    }
    __syncthreads();
}

// One lane's bits into the LDS bit buffer: a 32-bit accumulator (one shift-or per code); a code that
// crosses the word boundary leaves its top bits as the next word's start (v >> (32 - nb_before),
// 1..30 bits since n <= 30), and the word goes out with one LDS atomicOr.
struct BitPut {
    uint32_t lo;
    uint32_t nb;
    uint32_t wb;         // byte offset of the word being filled
    char* buf;
    __device__ __forceinline__ void init(uint32_t* b, uint32_t bitpos) {
        buf = (char*)b; wb = (bitpos >> 5) * 4; nb = bitpos & 31; lo = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, uint32_t n) {     // v < 2^n, n <= 30
        const uint32_t nb0 = nb;
        lo |= v << nb0;
        nb = nb0 + n;
        if (nb >= 32) {
            atomicOr((uint32_t*)(buf + wb), lo);
            wb += 4;
            nb -= 32;
            lo = v >> (32 - nb0);
        }
    }
    __device__ __forceinline__ void flush() {
        if (nb) atomicOr((uint32_t*)(buf + wb), lo);
    }
};

constexpr uint32_t CL_EXTRA_BITS[3] = {2, 3, 7};

// Code construction for one block, histograms already final (EOB counted).  Dynamic:
// D/comp/Lz77Huffman.java:143-265 (trim, single-distance fix-up, package-merge lengths, canonical
// codes, code-length RLE, code-length code, header sizes); static: the fixed codes of :394-410.
// Leaves the code tables and header layout in `ps` and the reordered 3-bit code-length-code
// lengths packed in misc[4..5] of the scratch.  All threads must call.
__device__ __forceinline__ void build_block_codes(bool dynamic, char* scr, Persist& ps, uint64_t* dbg = nullptr) {
    uint32_t* hlit = (uint32_t*)(scr + SCR_HLIT);
    uint32_t* hdist = (uint32_t*)(scr + SCR_HDIST);
    uint8_t* lens = (uint8_t*)(scr + SCR_LEN);
    uint8_t* clLen = (uint8_t*)(scr + SCR_CLLEN);
    uint32_t* clh = (uint32_t*)(scr + SCR_CLH);
    uint32_t* misc = (uint32_t*)(scr + SCR_MISC);
    const int tid = threadIdx.x;
    if (!dynamic) {
        // fixed codes (D/comp/Lz77Huffman.java:394-410)
        if (tid < 288) {
            uint32_t l = tid < 144 ? 8 : tid < 256 ? 9 : tid < 280 ? 7 : 8;
            uint32_t code = tid < 144 ? 0x30 + tid : tid < 256 ? 0x190 + (tid - 144) : tid < 280 ? (tid - 256) : 0xC0 + (tid - 280);
            ps.litCode[tid] = (__brev(code) >> (32 - l)) | (l << 16);
        }
        if (tid < 32) ps.distCode[tid] = (__brev((uint32_t)tid) >> 27) | (5u << 16);
        if (tid == 0) { ps.hdrBits = 3; ps.nsym = 0; }
        __syncthreads();
    } else {
        // trim litlen histogram, keep >= 257 (:148-151)
        if (tid == 0) {
            int ln = 286;
            while (ln > 257 && hlit[ln - 1] == 0) ln--;
            misc[0] = (uint32_t)ln;
            // single used distance code -> dummy neighbour (:155-171)
            int used = 0, first = -1;
            for (int i = 0; i < 30; i++) if (hdist[i]) { used++; if (first < 0) first = i; }
            if (used == 1) { if (first < 29) hdist[first + 1] = 1; else hdist[first - 1] = 1; }
            int dn = 30;
            while (dn > 1 && hdist[dn - 1] == 0) dn--;
            misc[1] = (uint32_t)dn;
            misc[2] = (dn == 1 && hdist[0] == 0) ? 1u : 0u;   // empty distance code
        }
        __syncthreads();
        if (dbg && tid == 0) dbg[0] = wall_clock64();
        const int ln = (int)misc[0], dn = (int)misc[1];
        const bool emptyDist = misc[2] != 0;
        // literal/length and distance lengths side by side: threads [0, 640) and [640, 1024)
        if (emptyDist && tid == 0) lens[ln] = 0;
        {
            const bool isLit = tid < 640;
            pm_lengths(isLit ? hlit : hdist, isLit ? ln : dn, 15, isLit ? lens : lens + ln,
                       isLit ? scr : scr + SCR_END, isLit ? tid : tid - 640, isLit || !emptyDist);
        }
        if (dbg && tid == 0) dbg[1] = wall_clock64();
        canon_codes(lens, ln, ps.litCode, scr);
        canon_codes(lens + ln, dn, ps.distCode, scr);
        if (dbg && tid == 0) dbg[2] = wall_clock64();
        // code-length sequence RLE (:187-223) as maximal-run decomposition
        const int nc = ln + dn;
        uint32_t rstart = 0xFFFFFFFFu;
        uint32_t v = 0;
        if (tid < nc) {
            v = lens[tid];
            if (tid == 0 || lens[tid - 1] != v) rstart = (uint32_t)tid;
        }
        uint32_t rnext = min(block_excl_suffix_min<NW>(rstart, 0xFFFFFFFFu, ps.scan32), (uint32_t)nc);
        uint32_t cnt = 0, Z = 0;
        if (rstart != 0xFFFFFFFFu) {
            Z = rnext - rstart;
            if (v == 0) {
                uint32_t q = Z / 138, r = Z % 138;
                cnt = q + (r >= 3 ? 1 : r);
            } else {
                uint32_t rest = Z - 1, q = rest / 6, r = rest % 6;
                cnt = 1 + q + (r >= 3 ? 1 : r);
            }
        }
        uint32_t tot;
        uint32_t off = block_excl_scan<uint32_t, NW>(cnt, ps.scan32, tot);
        if (rstart != 0xFFFFFFFFu) {
            uint32_t k = off;
            if (v == 0) {
                uint32_t L = Z;
                while (L > 0) {
                    uint32_t r = min(L, 138u);
                    if (r < 3) { ps.clSym[k] = 0; ps.clExtra[k++] = 0; L -= 1; }
                    else if (r < 11) { ps.clSym[k] = 17; ps.clExtra[k++] = (uint8_t)(r - 3); L -= r; }
                    else { ps.clSym[k] = 18; ps.clExtra[k++] = (uint8_t)(r - 11); L -= r; }
                }
            } else {
                ps.clSym[k] = (uint8_t)v; ps.clExtra[k++] = 0;
                uint32_t L = Z - 1;
                while (L >= 3) { uint32_t r = min(L, 6u); ps.clSym[k] = 16; ps.clExtra[k++] = (uint8_t)(r - 3); L -= r; }
                while (L > 0) { ps.clSym[k] = (uint8_t)v; ps.clExtra[k++] = 0; L--; }
            }
        }
        if (tid < 20) clh[tid] = 0;
        __syncthreads();
        if ((uint32_t)tid < tot) atomicAdd(&clh[ps.clSym[tid]], 1u);
        __syncthreads();
        if (dbg && tid == 0) dbg[3] = wall_clock64();
        pm_lengths(clh, 19, 7, clLen, scr);
        if (dbg && tid == 0) dbg[4] = wall_clock64();
        canon_codes(clLen, 19, ps.clCode, scr);
        if (dbg && tid == 0) dbg[5] = wall_clock64();
        // per-symbol header bit offsets
        uint32_t sb = 0;
        if ((uint32_t)tid < tot) {
            uint32_t sy = ps.clSym[tid];
            sb = (ps.clCode[sy] >> 16) + (sy >= 16 ? CL_EXTRA_BITS[sy - 16] : 0);
        }
        uint32_t body;
        uint32_t so = block_excl_scan<uint32_t, NW>(sb, ps.scan32, body);
        if ((uint32_t)tid < tot) ps.clOff[tid] = (uint16_t)so;
        if (tid == 0) {
            const int order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            int ncl = 19;
            while (ncl > 4 && clLen[order[ncl - 1]] == 0) ncl--;    // (:230-234)
            ps.ncl = (uint32_t)ncl;
            ps.nsym = tot;
            ps.hlit = (uint32_t)(ln - 257);
            ps.hdist = (uint32_t)(dn - 1);
            ps.clBodyBits = body;
            ps.hdrBits = 3 + 14 + 3 * (uint32_t)ncl + body;
            // stash reordered code-length-code lengths in misc[4..] (3 bits each, packed)
            uint64_t packed = 0;
            for (int i = 0; i < ncl; i++) packed |= (uint64_t)clLen[order[i]] << (3 * i);
            misc[4] = (uint32_t)packed; misc[5] = (uint32_t)(packed >> 32);
        }
        __syncthreads();
    }
}

// Block header (bfinal, btype, HLIT/HDIST/HCLEN, code-length-code lengths, code-length symbols:
// D/comp/Lz77Huffman.java:134-135,236-258) and the end-of-block code after `tokTotal` token bits
// (:285), ORed into the LDS bit buffer at local bit 0.  All threads must call (no barrier).
__device__ __forceinline__ void emit_block_header(uint32_t* obuf, bool is_final, bool dynamic, const Persist& ps,
                                                  uint32_t packedLo, uint32_t packedHi, uint32_t hdrBits,
                                                  uint32_t tokTotal, uint32_t eobLen) {
    const int tid = threadIdx.x;
    const uint32_t bit0 = 0;
    if (tid == 0) {
        BitPut bp; bp.init(obuf, bit0);
        bp.put(is_final ? 1u : 0u, 1);
        bp.put(dynamic ? 2u : 1u, 2);
        if (dynamic) {
            bp.put(ps.hlit, 5);
            bp.put(ps.hdist, 5);
            bp.put(ps.ncl - 4, 4);
            uint64_t packed = (uint64_t)packedLo | (uint64_t)packedHi << 32;
            for (uint32_t i = 0; i < ps.ncl; i++) bp.put((uint32_t)(packed >> (3 * i)) & 7u, 3);
        }
        bp.flush();
        // end-of-block symbol
        BitPut be; be.init(obuf, bit0 + hdrBits + tokTotal);
        be.put(ps.litCode[256] & 0xFFFF, eobLen);
        be.flush();
    }
    if (dynamic && (uint32_t)tid < ps.nsym) {
        const uint32_t sy = ps.clSym[tid];
        BitPut bp; bp.init(obuf, bit0 + 17 + 3 * ps.ncl + ps.clOff[tid]);
        bp.put(ps.clCode[sy] & 0xFFFF, ps.clCode[sy] >> 16);
        if (sy >= 16) bp.put(ps.clExtra[tid], CL_EXTRA_BITS[sy - 16]);
        bp.flush();
    }
}

// Decoupled look-back (one wave): the chunk's global bit offset from its predecessors' status words,
// then its inclusive prefix published.  Lane i polls predecessor c-1-i, so 64 predecessors cost one
// round trip; the closest inclusive prefix (PRE) ends the walk, aggregates (AGG) before it are
// summed, and a not-yet-published predecessor closer than it re-polls.  Chunk ids come from a
// ticket, so a workgroup only waits on workgroups that already started.  Result in ps.P.
__device__ __forceinline__ void block_lookback(uint32_t c, uint64_t base_bit, uint64_t S, uint64_t* status, Persist& ps) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    if (wid == 0) {
        // decoupled look-back, one wave: lane i polls predecessor c-1-i, so 64 predecessors cost
        // one round trip; the closest inclusive prefix (PRE) ends the walk, aggregates (AGG)
        // before it are summed, and a not-yet-published predecessor closer than it re-polls.
        uint64_t P = base_bit;
        if (c > 0) {
            uint64_t acc = 0;
            int64_t base = (int64_t)c - 1;
            for (;;) {
                const int64_t j = base - lane;
                const uint64_t st = j >= 0 ? ld_agent(&status[j]) : ST_PRE;
                const uint64_t pre = __ballot((st & ST_PRE) != 0);
                const uint64_t nr = __ballot((st >> 62) == 0);
                const int fp = pre ? (int)__builtin_ctzll(pre) : 64;
                const int fn = nr ? (int)__builtin_ctzll(nr) : 64;
                if (fn < fp) { __builtin_amdgcn_s_sleep(1); continue; }
                acc += wave_sum(lane <= fp ? (st & ST_VAL) : 0ull);
                if (fp < 64) break;
                base -= 64;
            }
            P = acc;
            if (lane == 0) st_agent(&status[c], ST_PRE | (P + S));
        }
        if (lane == 0) ps.P = P;
    }
    __syncthreads();
}

// Store the LDS bit buffer (S bits at local bit 0) at global bit ps.P: interior words with plain
// coalesced stores, the first and last word to the edge list merged by ndfl_edge_fixup_kernel.
__device__ __forceinline__ void block_store(const uint32_t* obuf, uint64_t P, uint64_t S, uint32_t c, uint32_t* out,
                                            uint64_t* edge_w, uint32_t* edge_v) {
    const int tid = threadIdx.x;
    const uint32_t sh = (uint32_t)(P & 31);
    const uint32_t nw = (uint32_t)((sh + S + 31) >> 5);
    const uint64_t W0 = P >> 5;
    auto outw = [&](uint32_t k) -> uint32_t {
        const uint32_t cur = obuf[k];
        const uint32_t prv = k ? obuf[k - 1] : 0u;
        return sh ? (cur << sh) | (prv >> (32 - sh)) : cur;
    };
    for (uint32_t k = (uint32_t)tid + 1; k + 1 < nw; k += DT) out[W0 + k] = outw(k);
    if (tid == 0) {
        edge_w[2 * c] = W0;
        edge_v[2 * c] = outw(0);
        edge_w[2 * c + 1] = W0 + nw - 1;
        edge_v[2 * c + 1] = nw > 1 ? outw(nw - 1) : 0u;
    }
}

}  // namespace

// One chunk, one 1024-thread workgroup.  MODE_FUSED does everything (chunk ids from a ticket,
// look-back for the offset); the split pipeline runs it as MODE_HIST (load, CRC, histograms to
// hist_out) and, after ndfl_deflate_codes_kernel and ndfl_deflate_offsets_kernel, MODE_EMIT (load,
// code tables and header from the record, token bits at the precomputed offset).
template <int MODE, class PS>
__device__ __forceinline__ void deflate_chunk(const Args& a, uint32_t* obuf, PS& ps, uint32_t* hl4 = nullptr,
                                              uint32_t* ctab = nullptr) {
    char* scr = (char*)obuf;
    uint32_t* hlit = (uint32_t*)(scr + SCR_HLIT);
    uint32_t* hdist = (uint32_t*)(scr + SCR_HDIST);
    uint8_t* lastb = (uint8_t*)(scr + SCR_LAST);
    uint32_t* misc = (uint32_t*)(scr + SCR_MISC);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;

    const uint64_t tp0 = wall_clock64();
    if (MODE == MODE_FUSED) {
        if (tid == 0) ps.chunk = atomicAdd(a.ticket, 1u);
    } else {
        if (tid == 0) ps.chunk = a.c0 + blockIdx.x;
    }
    if (MODE == MODE_FUSED) {
        if (tid < 288) hlit[tid] = 0;
        if (tid < 32) hdist[tid] = 0;
    } else if (MODE == MODE_HIST) {
        for (int k = tid; k < HCOPY * HSTR; k += DT) hl4[k] = 0;
        if (a.crc_raw) ctab[tid] = a.crc_tab[tid];          // slicing-by-4 tables to LDS (DT == 1024)
    }
    __syncthreads();
    const uint32_t c = ps.chunk;
    const uint64_t cs = (uint64_t)c * a.chunk_len;
    const uint32_t len_c = (uint32_t)min((uint64_t)a.chunk_len, a.n - cs);
    const bool is_final = a.final_last && (c + 1 == a.nchunks);
    const uint8_t* src = a.in + cs;

    // ---- 1. load 64 bytes per lane into registers --------------------------------------------
    uint32_t w[16];
    const uint32_t t0 = (uint32_t)tid * 64;
    const int vcnt = (int)min(64u, len_c > t0 ? len_c - t0 : 0u);
    if (vcnt == 64 && (((uintptr_t)(src + t0)) & 15) == 0) {
        const u32x4* p = (const u32x4*)(src + t0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            u32x4 v = __builtin_nontemporal_load(p + k);
            w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                int i = 4 * k + b;
                if (i < vcnt) x |= (uint32_t)src[t0 + i] << (8 * b);
            }
            w[k] = x;
        }
    }
    if (vcnt > 0) {
        uint32_t lv = w[15] >> 24;
        if (vcnt < 64) {                    // only the chunk's last lane; static indices keep w[] in registers
#pragma unroll
            for (int i = 0; i < 64; i++) if (i == vcnt - 1) lv = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        }
        lastb[tid] = (uint8_t)lv;
    }

    // ---- CRC-32 (raw, init 0) of this lane's bytes, combined across the chunk ----------------
    if (MODE != MODE_EMIT && a.crc_raw) {
        uint32_t cr = 0;
        const uint32_t* tb = MODE == MODE_HIST ? ctab : a.crc_tab;
        const uint32_t* T0 = tb;
        const uint32_t* T1 = tb + 256;
        const uint32_t* T2 = tb + 512;
        const uint32_t* T3 = tb + 768;
        const int nfull = vcnt >> 2;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (k < nfull) {
                uint32_t x = cr ^ w[k];
                cr = T3[x & 0xFF] ^ T2[(x >> 8) & 0xFF] ^ T1[(x >> 16) & 0xFF] ^ T0[x >> 24];
            }
        }
        if (vcnt & 3) {
#pragma unroll
            for (int i = 0; i < 64; i++)
                if (i >= nfull * 4 && i < vcnt) cr = T0[(cr ^ (w[i >> 2] >> (8 * (i & 3)))) & 0xFF] ^ (cr >> 8);
        }
        uint32_t contrib = 0;
        if (vcnt > 0) {
            // shift by the bytes that follow this lane inside the chunk
            const uint32_t after = len_c - (t0 + (uint32_t)vcnt);
            const uint32_t q = after & 63, k64 = after >> 6;
            uint32_t sh = a.crc_x[64 + k64];
            if (q) sh = crc_multmodp(a.crc_x[q], sh);
            contrib = crc_multmodp(sh, cr);
        }
        contrib = wave_xor(contrib);
        if (lane == 0) ps.crcAcc[wid] = contrib;
    }
    __syncthreads();
    if (MODE != MODE_EMIT && a.crc_raw && tid == 0) {
        uint32_t x = 0;
        for (int k = 0; k < NW; k++) x ^= ps.crcAcc[k];
        a.crc_raw[c] = x;
    }

    const uint64_t tp1 = wall_clock64();
    // The split passes read their chunk once, at the start, and every workgroup of a generation
    // waits on HBM at the same time.  One byte per 128-byte line of the chunk the next generation
    // takes on this XCD (c + pf_dist, dispatch is round-robin over the XCDs) is loaded here, after
    // the pass's last dependent global load, and consumed at the end, so that chunk is in L2 when
    // its workgroup starts.
    uint32_t pfv = 0;
    auto prefetch_next = [&]() {
        const uint64_t cn = (uint64_t)c + a.pf_dist;
        if (a.pf_dist && cn < a.nchunks && tid < 512) {
            const uint64_t off = cn * a.chunk_len + (uint64_t)tid * 128;
            if (off < a.n) pfv = a.in[off];
        }
    };
    // ---- 2. run pieces ------------------------------------------------------------------------
    // a block inside its parent chunk always has the parent's earlier bytes as history
    const bool has_prev0 = (cs % a.parent_len != 0) ? true : (c > 0) ? (a.hist_enabled != 0) : (a.prev_byte >= 0);
    const uint32_t prev0 = (c > 0) ? (uint32_t)src[-1] : (uint32_t)(a.prev_byte & 0xFF);
    uint64_t F = 0;
    if (vcnt > 0) {
        uint32_t prev = tid > 0 ? (uint32_t)lastb[tid - 1] : 0u;
        if (!a.rle) {
            F = vcnt == 64 ? ~0ull : ((1ull << vcnt) - 1);
        } else {
            // four bytes per step: x = word ^ (word shifted by one byte) is nonzero exactly in the
            // bytes that differ from the byte before them; their high bits are gathered into 4 bits
            // by one multiply (bits 0, 8, 16, 24 land on 21..24 with no carries)
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t x = w[k] ^ ((w[k] << 8) | (k ? (w[k - 1] >> 24) : prev));
                const uint32_t hb = ((((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u) >> 7;
                F |= (uint64_t)(((hb * 0x00204081u) >> 21) & 0xFu) << (4 * k);
            }
            if (tid == 0) F |= 1ull;
            if (vcnt < 64) F &= (1ull << vcnt) - 1;
        }
    }
    const uint32_t firstStart = F ? t0 + (uint32_t)__builtin_ctzll(F) : 0xFFFFFFFFu;
    const uint32_t nextStart = min(block_excl_suffix_min<NW>(firstStart, 0xFFFFFFFFu, ps.scan32), len_c);

    // piece visitor: (start_local, length, value, lead)
    auto lead_of = [&](uint32_t gpos, uint32_t v) -> uint32_t {
        if (!a.rle) return 1u;
        if (gpos == 0) return (has_prev0 && prev0 == v) ? 0u : 1u;
        return 1u;
    };
    // Piece classes per lane, over its 64 bytes (F bit i: a piece starts at byte i).  A
    // piece of length plen with lead literal `lead` is R = plen - lead bytes of matches; R < 3 means
    // it is plen literals of one value, whatever its lead (:62-90).  So a start is
    //   mR1: 1 literal (plen 1), mR2: 2 literals (plen 2), mR3: 3 literals (plen 3, lead 1),
    //   mLG: a run with a length token (R >= 3) -- the only class that needs the closed-form parse.
    // plen comes from the next start: the lane's own starts, then nextStart as a marker bit (the
    // chunk end is one).  Only the chunk's first byte can have lead 0 (its value continues the
    // history), where plen 3 is R = 3: a run.
    // The classes of all 64 bytes are formed at once from F and the marker position mp (bit 31 of
    // mpx: the chunk's first piece has lead 0): LM bit i = byte i is a literal of a literal piece (a
    // piece of 2 or 3 equal bytes is that many literals of the same value, so its copies sit on the
    // bytes they cover), LG bit i = a run piece starts at byte i; ce = literal copies past the lane's
    // last byte (the next lane's first bytes, same value).
    uint32_t mpx = 0xFFFFu;
    if (vcnt > 0) {
        mpx = nextStart - t0;
        if (a.rle && tid == 0 && (F & 1) && lead_of(0, w[0] & 0xFFu) == 0) mpx |= 1u << 31;
    }
    uint64_t LM = 0, LG = 0;
    uint32_t ce = 0;
    if (vcnt > 0) {
        const uint32_t mq = mpx & 0xFFFFu;
        const uint64_t wl = F | (mq < 64 ? 1ull << mq : 0ull);
        const uint64_t wh = (mq >= 64 && mq < 67) ? 1ull << (mq - 64) : 0ull;      // bits 64..66
        const uint64_t e1 = (wl >> 1) | (wh << 63), e2 = (wl >> 2) | (wh << 62), e3 = (wl >> 3) | (wh << 61);
        uint64_t r3 = F & ~e1 & ~e2 & e3;
        LG = F & ~(e1 | e2 | e3);
        if ((mpx >> 31) && (r3 & 1ull)) { r3 &= ~1ull; LG |= 1ull; }
        const uint64_t r2 = (F & ~e1 & e2) | r3;
        const uint64_t r1 = (F & e1) | r2;
        LM = r1 | (r2 << 1) | (r3 << 2);
        ce = (uint32_t)(r2 >> 63) + (uint32_t)((r3 >> 62) & 1ull) + (uint32_t)(r3 >> 63);
    }
    // visit this lane's bytes in order, 8 at a time.  Outer loop over 8-byte groups (select tree on
    // the uniform group index: a dynamic register index would put w[] in scratch memory), inner loop
    // unrolled by the caller: byte extraction is a constant shift.  BODY sees the group's bytes
    // (gw0_, gw1_), its literal and run-start bits (lm_, lg_) and whether any lane of the wave starts
    // a run in it (anyL_), so the per-byte work of literal bytes is branch-free.  A macro rather than
    // a lambda: capturing w[] by reference also demotes it to scratch.
#define NDFL_FOR_GROUPS_L(...)                                                                         \
    _Pragma("unroll 1") for (int o_ = 0; o_ < 8; o_++) {                                               \
        const uint32_t lm_ = (uint32_t)(LM >> (8 * o_)) & 0xFFu;                                      \
        const uint32_t lg_ = (uint32_t)(LG >> (8 * o_)) & 0xFFu;                                      \
        if (!__any((lm_ | lg_) != 0)) continue;                                                        \
        const bool o1_ = o_ & 1, o2_ = o_ & 2, o4_ = o_ & 4;                                           \
        const uint32_t a0_ = o1_ ? w[2] : w[0], a1_ = o1_ ? w[6] : w[4];                               \
        const uint32_t a2_ = o1_ ? w[10] : w[8], a3_ = o1_ ? w[14] : w[12];                            \
        const uint32_t b0_ = o1_ ? w[3] : w[1], b1_ = o1_ ? w[7] : w[5];                               \
        const uint32_t b2_ = o1_ ? w[11] : w[9], b3_ = o1_ ? w[15] : w[13];                            \
        const uint32_t gw0_ = o4_ ? (o2_ ? a3_ : a2_) : (o2_ ? a1_ : a0_);                             \
        const uint32_t gw1_ = o4_ ? (o2_ ? b3_ : b2_) : (o2_ ? b1_ : b0_);                             \
        const bool anyL_ = __any(lg_ != 0);                                                            \
        __VA_ARGS__                                                                                    \
    }
#define NDFL_BYTE(j) ((((j) < 4 ? gw0_ : gw1_) >> (8 * ((j) & 3))) & 0xFFu)
// 0 or all ones: byte j of the group is a literal
#define NDFL_LMASK(j) ((uint32_t)((int32_t)(lm_ << (31 - (j))) >> 31))
    // a run starting at group byte j: its value v, start gpos and end pend (next start)
#define NDFL_RUN_L(j, ...)                                                                             \
    if ((lg_ >> (j)) & 1) {                                                                            \
        const int i_ = 8 * o_ + (j);                                                                   \
        const uint32_t v = NDFL_BYTE(j);                                                               \
        const uint32_t gpos = t0 + (uint32_t)i_;                                                       \
        const uint64_t rest_ = i_ < 63 ? (F >> (i_ + 1)) : 0ull;                                       \
        const uint32_t pend = rest_ ? gpos + 1 + (uint32_t)__builtin_ctzll(rest_) : nextStart;         \
        __VA_ARGS__                                                                                    \
    }

    // ---- 3. histograms (closed-form greedy parse per piece, App. A.2) -------------------------
    // MODE_HIST counts into HCOPY lane-interleaved copies (fewer same-address LDS atomics per
    // instruction; see HCOPY / HSTR)
    uint32_t* hl = hlit;
    uint32_t* hd = hdist;
    if (MODE == MODE_HIST) { hl = hl4 + (tid & (HCOPY - 1)) * HSTR; hd = hl + 288; }
    if (MODE == MODE_HIST) {
        asm volatile("" :: "v"(prev0));    // its load is waited for here, not behind the prefetch
        prefetch_next();
    }
    if (MODE != MODE_EMIT) {
    NDFL_FOR_GROUPS_L({
_Pragma("unroll")
        for (int j = 0; j < 8; j++)
            if ((lm_ >> j) & 1) atomicAdd(&hl[NDFL_BYTE(j)], 1u);
        if (!anyL_) continue;                   // (wave-uniform: no run starts in the group)
_Pragma("unroll")
        for (int j = 0; j < 8; j++) {
            NDFL_RUN_L(j, {
                const uint32_t lead = lead_of(gpos, v);
                const uint32_t R = pend - gpos - lead;
                const uint32_t n258 = R / 258, m = R % 258;
                const uint32_t nlit = lead + (m < 3 ? m : 0);
                if (nlit) atomicAdd(&hl[v], nlit);
                if (n258) atomicAdd(&hl[285], n258);
                uint32_t nd = n258;
                if (m >= 3) {
                    uint32_t sym, ne, ex; run_sym(m, sym, ne, ex);
                    atomicAdd(&hl[sym], 1u);
                    nd++;
                }
                if (nd) atomicAdd(&hd[0], nd);
            })
        }
    })
    if (ce) atomicAdd(&hl[w[15] >> 24], ce);
    if (tid == 0) {
        atomicAdd(&hl[256], 1u);                          // end of block (:131-132)
        if (a.dynamic && len_c == 0) atomicAdd(&hl[0], 1u);  // (:146-147)
    }
    __syncthreads();
    }
    if (MODE == MODE_HIST) {
        uint32_t* h = a.hist_out + (uint64_t)c * HREC;
        if (tid < HREC) {
            uint32_t v = 0;
_Pragma("unroll")
            for (int k = 0; k < HCOPY; k++) v += hl4[k * HSTR + tid];
            h[tid] = v;
        }
        asm volatile("" :: "v"(pfv));
        return;
    }

    const uint64_t tp2 = wall_clock64();
    // ---- 4. code construction -------------------------------------------------------------------
    uint32_t packedLo = 0, packedHi = 0;
    if constexpr (MODE == MODE_FUSED) {
        build_block_codes(a.dynamic != 0, scr, ps, a.prof ? a.prof + (uint64_t)c * 16 + 8 : nullptr);
        packedLo = misc[4]; packedHi = misc[5];
    } else {
        const uint32_t* rec = a.codes + (uint64_t)c * CREC;
        if (tid < 288) ps.litCode[tid] = rec[CREC_LIT + tid];
        else if (tid < 320) ps.distCode[tid - 288] = rec[CREC_DIST + tid - 288];
        if (tid == 0) ps.hdrBits = rec[CREC_META];
    }
    __syncthreads();

    const uint64_t tp3 = wall_clock64();
    if (MODE == MODE_EMIT) prefetch_next();
    // ---- 5. token bits per lane, chunk size, decoupled look-back ------------------------------
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(ps.distCode[0]);       // workgroup-uniform: SGPRs
    const uint32_t c285 = __builtin_amdgcn_readfirstlane(ps.litCode[285]);
    uint32_t mybits = 0;
    NDFL_FOR_GROUPS_L({
        uint32_t pf[8];
_Pragma("unroll")
        for (int j = 0; j < 8; j++) pf[j] = ps.litCode[NDFL_BYTE(j)];
        uint32_t gs = 0;                        // (<= 8 x 15: the literal lengths of the group)
_Pragma("unroll")
        for (int j = 0; j < 8; j++) gs += (pf[j] & NDFL_LMASK(j)) >> 16;
        mybits += gs;
        if (anyL_) {                            // (wave-uniform: some lane starts a run in the group)
_Pragma("unroll")
            for (int j = 0; j < 8; j++) {
                NDFL_RUN_L(j, {
                    const uint32_t lv = pf[j] >> 16;
                    const uint32_t lead = lead_of(gpos, v);
                    const uint32_t R = pend - gpos - lead;
                    const uint32_t n258 = R / 258, m = R % 258;
                    mybits += lead * lv + n258 * ((c285 >> 16) + (d0 >> 16));
                    if (m >= 3) {
                        uint32_t sym, ne, ex; run_sym(m, sym, ne, ex);
                        mybits += (ps.litCode[sym] >> 16) + ne + (d0 >> 16);
                    } else {
                        mybits += m * lv;
                    }
                })
            }
        }
    })
    if (ce) mybits += ce * (ps.litCode[w[15] >> 24] >> 16);
    const uint64_t tp3a = wall_clock64();
    uint32_t tokTotal;
    const uint32_t myoff = block_excl_scan<uint32_t, NW>(mybits, ps.scan32, tokTotal);
    const uint64_t tp3b = wall_clock64();
    const uint32_t eobLen = __builtin_amdgcn_readfirstlane(ps.litCode[256] >> 16);
    const uint32_t hdrBits = __builtin_amdgcn_readfirstlane(ps.hdrBits);
    const uint64_t S = (uint64_t)hdrBits + tokTotal + eobLen;
    // publish this chunk's size now; the look-back runs after the chunk is emitted at local bit 0,
    // so predecessors get the emit time to publish theirs
    if (MODE == MODE_FUSED && tid == 0) {
        if (c == 0) st_agent(&a.status[0], ST_PRE | (a.base_bit + S));
        else st_agent(&a.status[c], ST_AGG | S);
        if (a.chunk_bits) a.chunk_bits[c] = S;
    }
    const uint64_t tp4 = wall_clock64();
    // zero the bit buffer (scratch is dead from here on); one spare word for the final shift
    const uint32_t nwl = (uint32_t)((S + 31) >> 5) + 1;
    __syncthreads();
    if (MODE == MODE_FUSED) {
        for (uint32_t k = (uint32_t)tid; k < nwl; k += DT) obuf[k] = 0;
    } else {
        // the record's header words (zero past hdrBits) start the buffer
        const uint32_t* hdr = a.codes + (uint64_t)c * CREC + CREC_HDR;
        const uint32_t hw = (hdrBits + 31) >> 5;
        for (uint32_t k = (uint32_t)tid; k < nwl; k += DT) obuf[k] = k < hw ? hdr[k] : 0u;
    }
    __syncthreads();
    const uint32_t bit0 = 0;

    // ---- 6. emit ------------------------------------------------------------------------------
    if constexpr (MODE == MODE_FUSED) {
        emit_block_header(obuf, is_final, a.dynamic != 0, ps, packedLo, packedHi, hdrBits, tokTotal, eobLen);
    } else if (tid == 0) {
        BitPut be; be.init(obuf, bit0 + hdrBits + tokTotal);
        be.put(ps.litCode[256] & 0xFFFF, eobLen);
        be.flush();
    }
    {
        BitPut bp; bp.init(obuf, bit0 + hdrBits + myoff);
        const uint32_t d0c = d0 & 0xFFFF, d0l = d0 >> 16;
        const uint32_t m258 = (c285 & 0xFFFF) | (d0c << (c285 >> 16));
        const uint32_t m258l = (c285 >> 16) + d0l;
        // one literal code per literal byte (LM), the tokens of a run at its first byte (LG); a group
        // in which no lane of the wave starts a run (wave-uniform) joins two codes per put (<= 30 bits)
        NDFL_FOR_GROUPS_L({
            // codes looked up 4 bytes ahead (8 would spill: the bit buffer state, the chunk's 16
            // words and the lookups share 64 VGPRs)
            uint32_t pf[4];
_Pragma("unroll")
            for (int j = 0; j < 4; j++) pf[j] = ps.litCode[NDFL_BYTE(j)];
            if (!anyL_) {
_Pragma("unroll")
                for (int j = 0; j < 8; j += 2) {
                    const uint32_t e0 = pf[j & 3] & NDFL_LMASK(j);
                    const uint32_t e1 = pf[(j + 1) & 3] & NDFL_LMASK(j + 1);
                    if (j < 4) { pf[j] = ps.litCode[NDFL_BYTE(j + 4)]; pf[j + 1] = ps.litCode[NDFL_BYTE(j + 5)]; }
                    const uint32_t l0 = e0 >> 16;
                    bp.put((e0 & 0xFFFF) | ((e1 & 0xFFFF) << l0), l0 + (e1 >> 16));
                }
                continue;
            }
_Pragma("unroll")
            for (int j = 0; j < 8; j++) {
                const uint32_t lc = pf[j & 3];
                if (j < 4) pf[j] = ps.litCode[NDFL_BYTE(j + 4)];
                const uint32_t e = lc & NDFL_LMASK(j);
                bp.put(e & 0xFFFF, e >> 16);
                NDFL_RUN_L(j, {
                    const uint32_t lead = lead_of(gpos, v);
                    const uint32_t R = pend - gpos - lead;
                    const uint32_t n258 = R / 258, m = R % 258;
                    if (lead) bp.put(lc & 0xFFFF, lc >> 16);
                    for (uint32_t k = 0; k < n258; k++) bp.put(m258, m258l);
                    if (m >= 3) {
                        uint32_t sym, ne, ex; run_sym(m, sym, ne, ex);
                        const uint32_t sc = ps.litCode[sym];
                        bp.put(sc & 0xFFFF, sc >> 16);
                        bp.put(ex, ne);
                        bp.put(d0c, d0l);
                    } else {
                        for (uint32_t k = 0; k < m; k++) bp.put(lc & 0xFFFF, lc >> 16);
                    }
                })
            }
        })
        if (ce) {                               // copies past the lane's last byte (same value)
            const uint32_t lc = ps.litCode[w[15] >> 24];
            bp.put(lc & 0xFFFF, lc >> 16);
            if (ce > 1) bp.put(lc & 0xFFFF, lc >> 16);
        }
        bp.flush();
    }
    __syncthreads();

    const uint64_t tp5e = wall_clock64();
    // ---- 7. look-back, then store shifted to the global bit offset ---------------------------
    if constexpr (MODE == MODE_FUSED) block_lookback(c, a.base_bit, S, a.status, ps);
    const uint64_t tp5 = wall_clock64();
    const uint64_t P = MODE == MODE_FUSED ? ps.P : a.chunk_off[c];
    block_store(obuf, P, S, c, a.out, a.edge_w, a.edge_v);
    if (tid == 0) {
        if (a.prof) {
            uint64_t* q = a.prof + (uint64_t)c * 16;
            q[0] = tp0; q[1] = tp1; q[2] = tp2; q[3] = tp3; q[4] = tp4; q[5] = tp5e; q[6] = tp5;
            q[7] = wall_clock64();
            (void)tp3a; (void)tp3b;
        }
    }
    (void)is_final; (void)packedLo; (void)packedHi;
    asm volatile("" :: "v"(pfv));
}

extern "C" __global__ void __launch_bounds__(DT, 8)
ndfl_deflate_chunks_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t obuf[OUTW];
    __shared__ Persist ps;
    deflate_chunk<MODE_FUSED>(a, obuf, ps);
}

// Split pipeline pass 1: CRC + histograms only (small LDS).
extern "C" __global__ void __launch_bounds__(DT, 8)
ndfl_deflate_hist_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t obuf[(SCR_LAST + 1024) / 4];
    __shared__ __attribute__((aligned(16))) uint32_t hl4[HCOPY * HSTR];
    __shared__ uint32_t ctab[1024];
    __shared__ PersistS ps;
    deflate_chunk<MODE_HIST>(a, obuf, ps, hl4, ctab);
}

// Split pipeline pass 4: token bits at the offset from ndfl_deflate_offsets_kernel.
extern "C" __global__ void __launch_bounds__(DT, 8)
ndfl_deflate_emit_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t obuf[OUTW];
    __shared__ PersistS ps;
    deflate_chunk<MODE_EMIT>(a, obuf, ps);
}

// Merge the boundary words: every word touched by more than one chunk is the OR of all of them.
extern "C" __global__ void ndfl_edge_fixup_kernel(const uint64_t* edge_w, const uint32_t* edge_v, uint32_t n_edges,
                                                  uint32_t* out) {
    uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_edges) return;
    uint64_t wv = edge_w[e];
    if (e > 0 && edge_w[e - 1] == wv) return;
    uint32_t v = 0;
    for (uint32_t k = e; k < n_edges && edge_w[k] == wv; k++) v |= edge_v[k];
    out[wv] = v;
}

// Combine per-chunk raw CRCs into the raw CRC of the call's data: raw = XOR over chunks of
// crc_c * x^(8 * bytes after chunk c).  Grid-stride over chunks, the shift from a table of
// x^(8 * 2^k) (one multiply per set bit), partial XORs folded with one atomicXor per wave into
// *out_raw (zeroed by the caller).
extern "C" __global__ void __launch_bounds__(256)
ndfl_crc_combine_kernel(const uint32_t* crc_raw, uint32_t nchunks, uint32_t chunk_len, uint64_t n,
                        const uint32_t* x8p2, uint32_t* out_raw) {
    uint32_t acc = 0;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += gridDim.x * blockDim.x) {
        const uint64_t end = min((uint64_t)(c + 1) * chunk_len, n);
        uint64_t after = n - end;
        uint32_t p = 1u << 31;                                   // x^0
        for (int k = 0; after; k++, after >>= 1)
            if (after & 1) p = crc_multmodp(x8p2[k], p);
        acc ^= crc_multmodp(p, crc_raw[c]);
    }
    acc = wave_xor(acc);
    if ((threadIdx.x & 63) == 0 && acc) atomicXor(out_raw, acc);
}

// Standalone CRC-32 (raw, init 0) of a device buffer: one 1024-thread workgroup per 64 KiB
// segment, combined by ndfl_crc_combine_kernel.  Used on the decompress side (gunzip trailer).
extern "C" __global__ void __launch_bounds__(1024)
ndfl_crc_segments_kernel(const uint8_t* in, uint64_t n, const uint32_t* crc_tab, const uint32_t* crc_x,
                         uint32_t* seg_raw) {
    __shared__ uint32_t red[16];
    const uint32_t seg = blockIdx.x;
    const uint64_t s0 = (uint64_t)seg * 65536;
    const uint32_t len = (uint32_t)min((uint64_t)65536, n - s0);
    const uint32_t t0 = threadIdx.x * 64;
    const int vcnt = (int)min(64u, len > t0 ? len - t0 : 0u);
    const uint8_t* src = in + s0 + t0;
    uint32_t cr = 0;
    const uint32_t* T0 = crc_tab; const uint32_t* T1 = crc_tab + 256;
    const uint32_t* T2 = crc_tab + 512; const uint32_t* T3 = crc_tab + 768;
    if (vcnt == 64 && (((uintptr_t)src) & 15) == 0) {
        const u32x4* p = (const u32x4*)src;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            u32x4 v = __builtin_nontemporal_load(p + k);
            uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t x = cr ^ ww[j];
                cr = T3[x & 0xFF] ^ T2[(x >> 8) & 0xFF] ^ T1[(x >> 16) & 0xFF] ^ T0[x >> 24];
            }
        }
    } else {
        for (int i = 0; i < vcnt; i++) cr = T0[(cr ^ src[i]) & 0xFF] ^ (cr >> 8);
    }
    uint32_t contrib = 0;
    if (vcnt > 0) {
        const uint32_t after = len - (t0 + (uint32_t)vcnt);
        uint32_t sh = crc_x[64 + (after >> 6)];
        if (after & 63) sh = crc_multmodp(crc_x[after & 63], sh);
        contrib = crc_multmodp(sh, cr);
    }
    contrib = wave_xor(contrib);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = contrib;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = 0;
        for (int k = 0; k < 16; k++) x ^= red[k];
        seg_raw[seg] = x;
    }
}

// Multi-GPU seam step: a shard's bit stream, compressed at bit 0, is moved to bit `shift` (0..7)
// of its first byte, i.e. to its global bit offset mod 8.  One output word per
// thread from input words t-1 and t; bits past `nbits` are cleared.
__device__ __forceinline__ uint32_t seam_word(const uint8_t* in, uint64_t nin, bool aligned, int64_t t) {
    if (t < 0) return 0u;
    const uint64_t b = (uint64_t)t * 4;
    if (aligned && b + 4 <= nin) return *(const uint32_t*)(in + b);
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; k++)
        if (b + k < nin) v |= (uint32_t)in[b + k] << (8 * k);
    return v;
}

extern "C" __global__ void __launch_bounds__(256)
ndfl_bits_shift_kernel(const uint8_t* in, uint64_t nbits, uint32_t shift, uint8_t* out, uint64_t nout) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t b = t * 4;
    if (b >= nout) return;
    const uint64_t nin = (nbits + 7) / 8;
    const bool aligned = (((uintptr_t)in) & 3) == 0;
    uint32_t hi = seam_word(in, nin, aligned, (int64_t)t), lo = seam_word(in, nin, aligned, (int64_t)t - 1);
    // clear bits at or past nbits (in either source word)
    auto keep = [nbits](uint64_t wbit) -> uint32_t {
        return wbit + 32 <= nbits ? 0xFFFFFFFFu : nbits > wbit ? (uint32_t)((1ull << (nbits - wbit)) - 1) : 0u;
    };
    hi &= keep(t * 32);
    if (t > 0) lo &= keep(t * 32 - 32);
    const uint32_t v = shift ? (hi << shift) | (lo >> (32 - shift)) : hi;
    if (b + 4 <= nout && (((uintptr_t)out) & 3) == 0) {
        *(uint32_t*)(out + b) = v;
    } else {
        for (uint32_t k = 0; k < 4; k++)
            if (b + k < nout) out[b + k] = (uint8_t)(v >> (8 * k));
    }
}
