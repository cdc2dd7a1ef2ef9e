// strategy_kernels.hip -- MI355X (gfx950) block assembly for strategies whose choice depends on
// the output bit position: Uncompressed (D/comp/Uncompressed.java:19-51) and MultiStrategy
// (D/comp/MultiStrategy.java:31-57).
//
// Every Lz77Huffman substrategy encodes all chunks once into its own stream at bit 0 (its block
// bits do not depend on where they land).  The host walks the chunks in order with the output
// position mod 8 -- MultiStrategy.decide keeps, per starting position, the first substrategy with
// the fewest bits, and compressTo picks by BitOutputStream.getBitPosition() -- which fixes each
// chunk's substrategy and global bit offset.  ndfl_assemble_kernel then writes every chunk at its
// offset: a bit-shifted copy of its block from the chosen stream, or stored blocks written in place
// (their padding depends on the position).  Words wholly inside one chunk are plain stores; the
// first/last word of a chunk is shared with its neighbours and merged with atomicOr (the output is
// zeroed first).
// D/ = /root/reference/src/io/nayuki/deflate/
#include "ndfl_common.hpp"

namespace {
constexpr uint32_t ST_MAX_BLOCK = 65535;        // Uncompressed.MAX_BLOCK_LEN (:54)

struct AsmArgs {
    const uint32_t* const* streams;  // per substrategy: its stream (null for Uncompressed)
    const uint8_t* data;             // the call's data (device)
    uint64_t n;
    uint32_t chunk_len;
    uint32_t nchunks;
    int32_t final_last;
    const uint8_t* choice;           // per chunk: substrategy index
    const uint64_t* src_bit;         // per chunk (entry): bit offset of its block in the chosen stream
    const uint64_t* dst_bit;         // per chunk: global output bit offset
    const uint64_t* nbits;           // per chunk: bits
    const uint8_t* setfin;           // optional per entry: set the block's bfinal bit (its first bit)
    int32_t per_entry_stream;        // 1: streams[] has one pointer per entry (choice ignored)
    uint32_t* out;                   // zeroed, word-aligned
};

}  // namespace

extern "C" __global__ void __launch_bounds__(256)
ndfl_assemble_kernel(AsmArgs a) {
    const uint32_t c = blockIdx.x;
    const uint64_t d = a.dst_bit[c], L = a.nbits[c];
    const uint32_t* src = a.per_entry_stream ? a.streams[c] : a.streams[a.choice[c]];
    if (src == nullptr) {
        // stored blocks (D/comp/Uncompressed.java:33-46): bfinal, btype 00, zero pad to a byte,
        // LEN, NLEN, bytes; only the first block can start inside a byte
        const uint64_t cs = (uint64_t)c * a.chunk_len;
        const uint32_t len = (uint32_t)min((uint64_t)a.chunk_len, a.n - cs);
        const bool fin = a.final_last && c + 1 == a.nchunks;
        const uint32_t nblk = max((len + ST_MAX_BLOCK - 1) / ST_MAX_BLOCK, 1u);
        uint8_t* ob = (uint8_t*)a.out;
        uint64_t B = (d + 3 + 7) >> 3;                  // LEN of block 0
        for (uint32_t k = 0; k < nblk; k++) {
            const uint32_t n = min(len - k * ST_MAX_BLOCK, ST_MAX_BLOCK);
            const uint32_t bf = (fin && k + 1 == nblk) ? 1u : 0u;
            if (k == 0) {
                if (threadIdx.x == 0 && bf) atomicOr(&a.out[d >> 5], 1u << (d & 31));
            } else {
                if (threadIdx.x == 0) ob[B] = (uint8_t)bf;
                B += 1;
            }
            if (threadIdx.x == 0) {
                const uint32_t nl = n ^ 0xFFFFu;
                // block 0's LEN may share its word with the previous chunk's last bits only when
                // B-1 holds header bits (a byte store leaves the other bytes alone)
                ob[B] = (uint8_t)n; ob[B + 1] = (uint8_t)(n >> 8);
                ob[B + 2] = (uint8_t)nl; ob[B + 3] = (uint8_t)(nl >> 8);
            }
            const uint8_t* s = a.data + cs + (uint64_t)k * ST_MAX_BLOCK;
            for (uint32_t i = threadIdx.x; i < n; i += 256) ob[B + 4 + i] = s[i];
            B += 4 + n;
        }
        return;
    }
    const uint64_t s = a.src_bit[c];
    const uint64_t w0 = d >> 5, w1 = (d + L - 1) >> 5;
    if (L == 0) return;
    if (a.setfin && a.setfin[c] && threadIdx.x == 0) atomicOr(&a.out[d >> 5], 1u << (d & 31));
    for (uint64_t w = w0 + threadIdx.x; w <= w1; w += 256) {
        // dst bits [32w, 32w+32) <- src bits from q = s + (32w - d)
        const int64_t q = (int64_t)s + (int64_t)(32 * w) - (int64_t)d;
        uint32_t v;
        if (q >= 0) {
            const uint64_t qi = (uint64_t)q >> 5;
            const uint32_t sh = (uint32_t)q & 31;
            const uint32_t lo = src[qi], hi = src[qi + 1];
            v = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
        } else {
            v = src[0] << (uint32_t)(-q);                 // only the first word: bits below d are masked
        }
        const uint64_t b0 = max(d, 32 * w), b1 = min(d + L, 32 * w + 32);
        const uint32_t m = (uint32_t)(((b1 - b0) == 32 ? 0xFFFFFFFFull : ((1ull << (b1 - b0)) - 1)) << (b0 - 32 * w));
        v &= m;
        if (m == 0xFFFFFFFFu && w != w0 && w != w1) a.out[w] = v;
        else atomicOr(&a.out[w], v);
    }
}

// ---- Adler-32 (java.util.zip.Adler32, the zlib container's checksum: D/ZlibOutputStream.java:22,
// D/ZlibInputStream.java:25) -------------------------------------------------------------------
// One 1024-thread workgroup per 64 KiB segment: S = sum of bytes, T = sum of (len - i) * byte_i
// (i from 0), both mod 65521; the host folds the segments in order: b += len*a + T, a += S.
extern "C" __global__ void __launch_bounds__(1024)
ndfl_adler_segments_kernel(const uint8_t* in, uint64_t n, uint32_t* seg_st) {
    __shared__ unsigned long long rs[16], rt[16];
    const uint32_t seg = blockIdx.x;
    const uint64_t s0 = (uint64_t)seg * 65536;
    const uint32_t len = (uint32_t)min((uint64_t)65536, n - s0);
    const uint32_t t0 = threadIdx.x * 64;
    const uint32_t cnt = len > t0 ? min(64u, len - t0) : 0u;
    const uint8_t* p = in + s0 + t0;
    uint32_t ss = 0, tt = 0;                         // sums over this thread's bytes, weights cnt - k
    if (cnt == 64 && (((uintptr_t)p) & 15) == 0) {
        const u32x4* q = (const u32x4*)p;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u32x4 v = __builtin_nontemporal_load(q + k);
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t b = (w4[j >> 2] >> (8 * (j & 3))) & 0xFF;
                ss += b;
                tt += (uint32_t)(64 - (16 * k + j)) * b;
            }
        }
    } else {
        for (uint32_t k = 0; k < cnt; k++) { const uint32_t b = p[k]; ss += b; tt += (cnt - k) * b; }
    }
    // weight of this thread's bytes relative to the segment end: + bytes after them
    const unsigned long long after = (unsigned long long)(len - t0 - cnt);
    unsigned long long S = ss, T = tt + (cnt ? after * ss : 0ull);
    S = wave_sum(S);
    T = wave_sum(T);
    if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = S; rt[threadIdx.x >> 6] = T; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, b = 0;
        for (int k = 0; k < 16; k++) { a += rs[k]; b += rt[k]; }
        seg_st[2 * seg] = (uint32_t)(a % 65521u);
        seg_st[2 * seg + 1] = (uint32_t)(b % 65521u);
    }
}
