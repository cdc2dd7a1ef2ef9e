// deflate_split.hip -- the split RLE/LITERAL encoder pipeline (gfx950).
//
// The fused ndfl_deflate_chunks_kernel holds a 1024-thread workgroup (and the chunk's bytes in its
// registers) through the whole per-chunk Huffman build, which is a few hundred items of work at a
// time: two chunks per CU spend most of their life in barriers.  The split pipeline gives each
// phase the shape it wants:
//   1. ndfl_deflate_hist_kernel     1024 threads / chunk: load, CRC-32, closed-form RLE parse into
//                                   histograms (hist_out)
//   2. ndfl_deflate_codes_kernel    ONE WAVE / chunk: package-merge code lengths, canonical codes,
//                                   code-length RLE + its code, the header bits, the block size
//                                   (D/comp/Lz77Huffman.java:134-265,309-410) into a code record
//   3. ndfl_deflate_offsets_kernel  exclusive scan of the block sizes -> each chunk's global bit offset
//   4. ndfl_deflate_emit_kernel     1024 threads / chunk: reload, token bits at the known offset
// Every step restates the same reference lines as the fused kernel (deflate_kernels.hip) and yields
// the same bits; the block size is computed from the histograms (every token's code length plus its
// extra bits -- the extra-bit count is a function of the symbol).
// D/ = /root/reference/src/io/nayuki/deflate/

namespace {

// LDS of one code-construction wave (8.8 KB: 18 waves per CU; the round-3 layout's 12.4 KB held
// 13).  Lifetimes share storage: the package-merge input keys live in pf[1] until the leaves are
// ranked (level 0 writes pf[1] only after that), the header bits in pf[0] after the last
// package-merge, the code-length symbols' header offsets in lf after the last package-merge; the
// merged level is never stored (packages are summed as the merge produces them).
struct WScr {
    uint32_t hlit[288];
    uint32_t hdist[32];
    uint32_t hdist0[32];      // distance histogram before the single-code fix-up (token bits)
    union {
        uint32_t lf[288];         // ranked leaf frequencies (package-merge)
        uint16_t clOff[320];      // header bit offset of each code-length symbol (after the last one)
    };
    uint16_t ls[288];
    uint32_t pf[2][304];      // package frequencies of the current / next level
    __device__ __forceinline__ uint32_t* key() { return pf[1]; }     // (292 used: n padded to 4)
    __device__ __forceinline__ uint32_t* hdr() { return pf[0]; }     // (HDRW used)
    uint32_t mpk[15 * 20];
    uint32_t lvl[16];
    uint32_t blc[16], nxc[16], mask[16 * 10];
    uint32_t clh[20];
    uint32_t clCode[20];
    uint32_t misc[8];
    uint8_t clSym[320], clExtra[320];
    uint8_t lens[320];
    uint8_t clLen[32];
};

// Length-limited code lengths by package-merge (D/comp/Lz77Huffman.java:309-335), one wave: the
// same merge-path levels, tie order (packages before leaves on equal frequency) and backtrack as
// pm_lengths, with each lane taking every 64th item.  lens[0..n) receives the lengths.
__device__ void wpm_lengths(const uint32_t* hist, int n, int L, uint8_t* lens, WScr& S) {
    const int lane = threadIdx.x;
    // the used symbols' keys (freq << 9 | symbol) compacted in symbol order, padded to 4 with ~0
    uint32_t nl = 0;
    for (int base = 0; base < n; base += 64) {                // uniform trip count
        const int i = base + lane;
        uint32_t k = 0xFFFFFFFFu;
        if (i < n) { const uint32_t f = hist[i]; if (f) k = f << 9 | (uint32_t)i; lens[i] = 0; }
        const uint64_t m = __ballot(k != 0xFFFFFFFFu);
        if (k != 0xFFFFFFFFu) S.key()[nl + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = k;
        nl += (uint32_t)__popcll(m);
    }
    const uint32_t nlp = (nl + 3) & ~3u;
    if ((uint32_t)lane < nlp - nl) S.key()[nl + lane] = 0xFFFFFFFFu;
    for (int t = lane; t < L * 20; t += 64) S.mpk[t] = 0;
    __syncthreads();
    // leaves sorted by (freq, symbol): rank by counting among the used keys only (a text chunk uses
    // ~100 of the 286 literal/length symbols), up to 5 keys per lane in registers
    {
        const uint32_t nq = (nl + 63) >> 6;                   // uniform: key slots per lane in use
        uint32_t kk[5], r[5];
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t i = (uint32_t)lane + 64u * q;
            kk[q] = i < nl ? S.key()[i] : 0xFFFFFFFFu;
            r[q] = 0;
        }
        for (uint32_t j = 0; j < nlp; j += 4) {
            const uint4 v = *(const uint4*)&S.key()[j];
#pragma unroll
            for (int q = 0; q < 5; q++)
                if ((uint32_t)q < nq)
                    r[q] += (uint32_t)(v.x < kk[q]) + (uint32_t)(v.y < kk[q]) + (uint32_t)(v.z < kk[q]) + (uint32_t)(v.w < kk[q]);
        }
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t i = (uint32_t)lane + 64u * q;
            if (i < nl) { S.lf[r[q]] = kk[q] >> 9; S.ls[r[q]] = (uint16_t)(kk[q] & 511u); }
        }
    }
    __syncthreads();
    if (nl < 2) return;                                       // uniform: all lengths zero
    uint32_t np = 0;
    int cur = 0;
    for (int it = 0; it < L; it++) {
        const uint32_t m = np + nl;
        const uint32_t* pf = S.pf[cur];
        // merged order: package i before leaf j iff pf[i] <= lf[j] (packages first on equal freq).
        // Lane l merges positions [k0, k1): one merge-path search for how many packages precede k0,
        // then a sequential merge (one dependent LDS read per output instead of one binary search
        // per item).  k0 is even, so the lane sums its own pairs into the next level's packages.
        uint32_t* pfn = S.pf[cur ^ 1];
        {
            const uint32_t per = (((m + 63) >> 6) + 1) & ~1u;
            const uint32_t k0 = min(m, (uint32_t)lane * per), k1 = min(m, k0 + per);
            uint32_t lo = k0 > nl ? k0 - nl : 0u, hi = min(k0, np);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (pf[mid] <= S.lf[k0 - mid - 1]) lo = mid + 1; else hi = mid;
            }
            uint32_t i = lo, j = k0 - lo;
            uint32_t pv = i < np ? pf[i] : 0u, lv = j < nl ? S.lf[j] : 0u;
            const uint32_t wb = k0 & ~31u;
            uint64_t bits = 0;
            uint32_t held = 0;
            for (uint32_t pos = k0; pos < k1; pos++) {
                const bool takeP = i < np && (j >= nl || pv <= lv);
                const uint32_t item = takeP ? pv : lv;
                if (pos & 1) pfn[pos >> 1] = held + item;
                held = item;
                if (takeP) {
                    bits |= 1ull << (pos - wb);
                    i++;
                    pv = i < np ? pf[i] : 0u;
                } else {
                    j++;
                    lv = j < nl ? S.lf[j] : 0u;
                }
            }
            if ((uint32_t)bits) atomicOr(&S.mpk[it * 20 + (wb >> 5)], (uint32_t)bits);
            if ((uint32_t)(bits >> 32)) atomicOr(&S.mpk[it * 20 + (wb >> 5) + 1], (uint32_t)(bits >> 32));
        }
        __syncthreads();
        const uint32_t np2 = m >> 1;
        np = np2;
        cur ^= 1;
    }
    // backtrack: prefix of 2(nl-1) items at the last level; leaves in the prefix of each level
    {
        uint32_t m = 2 * (nl - 1);
        for (int it = L - 1; it >= 0; it--) {
            uint32_t cnt = 0;
            if (lane < 20) {
                const uint32_t w = S.mpk[it * 20 + lane];
                const uint32_t lo = (uint32_t)lane * 32;
                if (lo + 32 <= m) cnt = __popc(w);
                else if (lo < m) cnt = __popc(w & ((1u << (m - lo)) - 1));
            }
            cnt = wave_sum(cnt);
            if (lane == 0) S.lvl[it] = m - cnt;
            m = 2 * cnt;
        }
    }
    __syncthreads();
    for (uint32_t t = (uint32_t)lane; t < nl; t += 64) {
        uint32_t cl = 0;
        for (int it = 0; it < L; it++) cl += t < S.lvl[it];
        lens[S.ls[t]] = (uint8_t)cl;
    }
    __syncthreads();
}

// Canonical codes (D/comp/Lz77Huffman.java:368-391), one wave: rev(code) | len << 16 into codes[0..n).
__device__ void wcanon(const uint8_t* lens, int n, uint32_t* codes, WScr& S) {
    const int lane = threadIdx.x;
    if (lane < 16) S.blc[lane] = 0;
    for (int t = lane; t < 160; t += 64) S.mask[t] = 0;
    __syncthreads();
    for (int t = lane; t < n; t += 64) {
        const uint32_t l = lens[t];
        if (l) { atomicAdd(&S.blc[l], 1u); atomicOr(&S.mask[l * 10 + (t >> 5)], 1u << (t & 31)); }
    }
    __syncthreads();
    if (lane == 0) {
        uint32_t code = 0;
        S.blc[0] = 0;
        for (int b = 1; b < 16; b++) { code = (code + S.blc[b - 1]) << 1; S.nxc[b] = code; }
    }
    __syncthreads();
    for (int t = lane; t < n; t += 64) {
        const uint32_t l = lens[t];
        uint32_t cv = 0;
        if (l) {
            uint32_t rank = 0;
            const int wi = t >> 5;
            for (int w = 0; w < wi; w++) rank += __popc(S.mask[l * 10 + w]);
            rank += __popc(S.mask[l * 10 + wi] & ((1u << (t & 31)) - 1));
            cv = (__brev(S.nxc[l] + rank) >> (32 - l)) | (l << 16);
        }
        codes[t] = cv;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t wave_excl_suffix_min(uint32_t v, uint32_t ident) {
    const int lane = threadIdx.x & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_down(x, o, 64);
        if (lane + o < 64) x = min(x, y);
    }
    const uint32_t nxt = __shfl_down(x, 1, 64);
    return lane == 63 ? ident : nxt;
}

// extra bits of literal/length symbol s (257..285) and distance symbol d (:92-127)
__device__ __forceinline__ uint32_t len_extra(uint32_t s) { return (s >= 265 && s < 285) ? (s - 261) >> 2 : 0u; }
__device__ __forceinline__ uint32_t dist_extra(uint32_t d) { return d >= 4 ? (d >> 1) - 1 : 0u; }

}  // namespace

// Pass 2: one wave builds one chunk's codes and header from its histograms (same steps as
// build_block_codes: D/comp/Lz77Huffman.java:143-265 dynamic, :394-410 static).  Writes the code
// record (codes, header bits, hdrBits) and the block size in bits to a.status[c] (+ chunk_bits).
extern "C" __global__ void __launch_bounds__(64)
ndfl_deflate_codes_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) WScr S;
    const uint32_t c = a.c0 + blockIdx.x;
    const int lane = threadIdx.x;
    const uint64_t cs = (uint64_t)c * a.chunk_len;
    const uint32_t len_c = (uint32_t)min((uint64_t)a.chunk_len, a.n - cs);
    const bool is_final = a.final_last && (c + 1 == a.nchunks);
    const uint32_t* h = a.hist_out + (uint64_t)c * HREC;
    uint32_t* rec = (uint32_t*)a.codes + (uint64_t)c * CREC;
    for (int i = lane; i < 288; i += 64) S.hlit[i] = h[i];
    if (lane < 32) { const uint32_t v = h[288 + lane]; S.hdist[lane] = v; S.hdist0[lane] = v; }
    for (int i = lane; i < HDRW; i += 64) S.hdr()[i] = 0;
    __syncthreads();
    uint32_t hdrBits;
    uint64_t tok = 0;                  // token bits incl. the end-of-block code
    if (!a.dynamic) {
        // fixed codes (:394-410)
        for (int t = lane; t < 288; t += 64) {
            const uint32_t l = t < 144 ? 8 : t < 256 ? 9 : t < 280 ? 7 : 8;
            const uint32_t code = t < 144 ? 0x30 + t : t < 256 ? 0x190 + (t - 144) : t < 280 ? (t - 256) : 0xC0 + (t - 280);
            rec[CREC_LIT + t] = (__brev(code) >> (32 - l)) | (l << 16);
            tok += (uint64_t)S.hlit[t] * (l + len_extra((uint32_t)t));
        }
        if (lane < 32) {
            rec[CREC_DIST + lane] = (__brev((uint32_t)lane) >> 27) | (5u << 16);
            if (lane < 30) tok += (uint64_t)S.hdist0[lane] * (5 + dist_extra((uint32_t)lane));
        }
        hdrBits = 3;
        if (lane == 0) S.hdr()[0] = (is_final ? 1u : 0u) | (1u << 1);
        __syncthreads();
    } else {
        // trim litlen histogram, keep >= 257 (:148-151); single used distance code gets a dummy
        // neighbour (:155-171); empty distance code (:172-177)
        {
            const uint64_t lb = __ballot(lane < 29 && S.hlit[257 + lane] != 0);
            uint64_t db = __ballot(lane < 30 && S.hdist[lane] != 0);
            if (__popcll(db) == 1) {
                const int first = (int)__builtin_ctzll(db);
                const int nb = first < 29 ? first + 1 : first - 1;
                if (lane == 0) S.hdist[nb] = 1;
                db |= 1ull << nb;
            }
            if (lane == 0) {
                S.misc[0] = lb ? 258u + (uint32_t)(63 - __builtin_clzll(lb)) : 257u;
                S.misc[1] = db ? 1u + (uint32_t)(63 - __builtin_clzll(db)) : 1u;
                S.misc[2] = db ? 0u : 1u;
            }
        }
        __syncthreads();
        const int ln = (int)S.misc[0], dn = (int)S.misc[1];
        const bool emptyDist = S.misc[2] != 0;
        wpm_lengths(S.hlit, ln, 15, S.lens, S);
        if (emptyDist) { if (lane == 0) S.lens[ln] = 0; __syncthreads(); }
        else wpm_lengths(S.hdist, dn, 15, S.lens + ln, S);
        wcanon(S.lens, ln, rec + CREC_LIT, S);
        wcanon(S.lens + ln, dn, rec + CREC_DIST, S);
        for (int t = ln + lane; t < 288; t += 64) rec[CREC_LIT + t] = 0;
        if (lane >= dn && lane < 32) rec[CREC_DIST + lane] = 0;
        // token bits: code length + extra bits per symbol occurrence; the dummy literal of an empty
        // block (:146-147) is in the histogram but never written
        for (int t = lane; t < ln; t += 64) tok += (uint64_t)S.hlit[t] * (S.lens[t] + len_extra((uint32_t)t));
        if (lane < dn) tok += (uint64_t)S.hdist0[lane] * (S.lens[ln + lane] + dist_extra((uint32_t)lane));
        if (lane == 0 && len_c == 0) tok -= S.lens[0];
        // code-length sequence RLE (:187-223) as maximal-run decomposition; lane owns [5l, 5l+5)
        const int nc = ln + dn;
        uint32_t v[5], rnext[5];
        bool st[5];
        uint32_t firstStart = 0xFFFFFFFFu;
#pragma unroll
        for (int q = 4; q >= 0; q--) {
            const int i = 5 * lane + q;
            v[q] = i < nc ? S.lens[i] : 0u;
            st[q] = i < nc && (i == 0 || S.lens[i - 1] != v[q]);
            if (st[q]) firstStart = (uint32_t)i;
        }
        uint32_t nxt = min(wave_excl_suffix_min(firstStart, 0xFFFFFFFFu), (uint32_t)nc);
        uint32_t cnt[5], mycnt = 0;
#pragma unroll
        for (int q = 4; q >= 0; q--) {
            cnt[q] = 0;
            if (st[q]) {
                const uint32_t Z = nxt - (uint32_t)(5 * lane + q);
                if (v[q] == 0) { const uint32_t qq = Z / 138, r = Z % 138; cnt[q] = qq + (r >= 3 ? 1 : r); }
                else { const uint32_t rest = Z - 1, qq = rest / 6, r = rest % 6; cnt[q] = 1 + qq + (r >= 3 ? 1 : r); }
                rnext[q] = nxt;
                nxt = (uint32_t)(5 * lane + q);
            }
            mycnt += cnt[q];
        }
        const uint32_t incl = wave_incl_scan(mycnt);
        const uint32_t tot = __shfl(incl, 63, 64);
        uint32_t k = incl - mycnt;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            if (!st[q]) continue;
            const uint32_t Z = rnext[q] - (uint32_t)(5 * lane + q);
            if (v[q] == 0) {
                uint32_t Lr = Z;
                while (Lr > 0) {
                    const uint32_t r = min(Lr, 138u);
                    if (r < 3) { S.clSym[k] = 0; S.clExtra[k++] = 0; Lr -= 1; }
                    else if (r < 11) { S.clSym[k] = 17; S.clExtra[k++] = (uint8_t)(r - 3); Lr -= r; }
                    else { S.clSym[k] = 18; S.clExtra[k++] = (uint8_t)(r - 11); Lr -= r; }
                }
            } else {
                S.clSym[k] = (uint8_t)v[q]; S.clExtra[k++] = 0;
                uint32_t Lr = Z - 1;
                while (Lr >= 3) { const uint32_t r = min(Lr, 6u); S.clSym[k] = 16; S.clExtra[k++] = (uint8_t)(r - 3); Lr -= r; }
                while (Lr > 0) { S.clSym[k] = (uint8_t)v[q]; S.clExtra[k++] = 0; Lr--; }
            }
        }
        if (lane < 20) S.clh[lane] = 0;
        __syncthreads();
        for (uint32_t t = (uint32_t)lane; t < tot; t += 64) atomicAdd(&S.clh[S.clSym[t]], 1u);
        __syncthreads();
        wpm_lengths(S.clh, 19, 7, S.clLen, S);
        wcanon(S.clLen, 19, S.clCode, S);
        for (int i = lane; i < HDRW; i += 64) S.hdr()[i] = 0;        // (hdr shares pf[0])
        // per-symbol header bit offsets (exclusive scan, lane owns [5l, 5l+5))
        uint32_t sb[5], lsum = 0;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t i = (uint32_t)(5 * lane + q);
            sb[q] = 0;
            if (i < tot) {
                const uint32_t sy = S.clSym[i];
                sb[q] = (S.clCode[sy] >> 16) + (sy >= 16 ? CL_EXTRA_BITS[sy - 16] : 0);
            }
            lsum += sb[q];
        }
        const uint32_t bincl = wave_incl_scan(lsum);
        const uint32_t body = __shfl(bincl, 63, 64);
        uint32_t so = bincl - lsum;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t i = (uint32_t)(5 * lane + q);
            if (i < tot) S.clOff[i] = (uint16_t)so;
            so += sb[q];
        }
        const int order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        int ncl = 19;
        while (ncl > 4 && S.clLen[order[ncl - 1]] == 0) ncl--;    // (:230-234)
        hdrBits = 3 + 14 + 3 * (uint32_t)ncl + body;
        __syncthreads();
        // header (:134-135,236-258) into the LDS word buffer
        if (lane == 0) {
            BitPut bp; bp.init(S.hdr(), 0);
            bp.put(is_final ? 1u : 0u, 1);
            bp.put(2u, 2);
            bp.put((uint32_t)(ln - 257), 5);
            bp.put((uint32_t)(dn - 1), 5);
            bp.put((uint32_t)ncl - 4, 4);
            for (int i = 0; i < ncl; i++) bp.put(S.clLen[order[i]], 3);
            bp.flush();
        }
        for (uint32_t t = (uint32_t)lane; t < tot; t += 64) {
            const uint32_t sy = S.clSym[t];
            BitPut bp; bp.init(S.hdr(), 17 + 3 * (uint32_t)ncl + S.clOff[t]);
            bp.put(S.clCode[sy] & 0xFFFF, S.clCode[sy] >> 16);
            if (sy >= 16) bp.put(S.clExtra[t], CL_EXTRA_BITS[sy - 16]);
            bp.flush();
        }
        __syncthreads();
    }
    for (int i = lane; i < HDRW; i += 64) rec[CREC_HDR + i] = S.hdr()[i];
    tok = wave_sum(tok);
    if (lane == 0) {
        rec[CREC_META] = hdrBits;
        const uint64_t Sz = (uint64_t)hdrBits + tok;
        a.status[c] = Sz;
        if (a.chunk_bits) a.chunk_bits[c] = Sz;
    }
}

// Pass 3: chunk c's global bit offset = base + sum of the sizes before it; total[0] = end bit.  Two
// launches (ndfl_common.hpp scan_tile_*): the tile sums, then each tile's scan; grid = tiles.
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_deflate_offsets_sum_kernel(const uint64_t* sizes, uint32_t n, uint64_t* part) {
    scan_tile_sum([&](uint32_t i) { return sizes[i]; }, n, part);
}
extern "C" __global__ void __launch_bounds__(SCAN_T)
ndfl_deflate_offsets_kernel(const uint64_t* sizes, uint32_t n, uint64_t base, uint64_t* off, uint64_t* total,
                            const uint64_t* part) {
    scan_tile_apply([&](uint32_t i) { return sizes[i]; }, [&](uint32_t i, uint64_t v) { off[i] = v; }, n, part, base,
                    total);
}
