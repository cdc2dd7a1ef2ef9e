// ndfl_common.hpp -- shared device helpers for the MI355X (gfx950) DEFLATE kernels.
// Wave64 throughout: every cross-lane idiom below assumes 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

// Switches of a context, read once from the environment when the context is created
// (ndfl_ctx_create).  None is needed in production: they select the decoder's hand-over paths for
// the tests (EMIT_FAST, NO_BT, NO_ALIAS, COUNT_W, FLAT, TEST_SEGFLIP), statistics for profiling (STATS, HOST_TIMES,
// LZ_STATS), and the few A/B alternatives still measured against the defaults.
struct Knobs {
    bool stats = false;          // NDFL_STATS: per-pass counters and phase clocks to stderr
    bool host_times = false;     // NDFL_HOST_TIMES: host-side timestamps of a decode
    bool host_link = false;      // NDFL_HOST_LINK: the host's chain linking instead of the device's
    bool no_hdrrec = false;      // NDFL_NO_HDRREC: chain-first headers parsed by lane 0 (no records)
    bool emit_fast = true;       // NDFL_EMIT_FAST=0: the full emit kernel alone
    bool no_bt = false;          // NDFL_NO_BT: no table records (every Huffman chain handed over)
    bool no_alias = false;       // NDFL_NO_ALIAS: every stored-header alias counted
    uint32_t count_w = 0;        // NDFL_COUNT_W: waves per chain in the count pass (0: automatic)
    bool deflate_pf = true;      // NDFL_DEFLATE_PF=0: no L2 touch of the next chunk in the encoder
    bool deflate_profile = false;  // NDFL_DEFLATE_PROFILE: per-phase encoder clocks (one-kernel encoder)
    bool deflate_fused = false;  // NDFL_DEFLATE_FUSED: the one-kernel encoder instead of the split passes
    bool lz_stats = false;       // NDFL_LZ_STATS
    bool lz_chain = false;       // NDFL_LZ_SEARCH=chain: the round-3 hash-chain LZ77 search
    int lz_lead = -1;            // NDFL_LZ_LEAD: parse-driven search lead-in (-1: default)
    bool flat = true;            // NDFL_FLAT=0: escape-prefix literal blocks counted in wave form too
    uint32_t flat_min = 49152;   // NDFL_FLAT_MIN: chains to count at least for flat groups (their latency)
    bool test_segflip = false;   // NDFL_TEST_SEGFLIP: one count-pass record's byte count perturbed
                                 //   before the emit pass (the emit-side check must fail the decode)
    void read() {
        auto on = [](const char* n) { const char* e = getenv(n); return e && strcmp(e, "0") != 0; };
        auto num = [](const char* n, int dflt) { const char* e = getenv(n); return e ? atoi(e) : dflt; };
        stats = on("NDFL_STATS"); host_times = on("NDFL_HOST_TIMES"); host_link = on("NDFL_HOST_LINK");
        no_hdrrec = on("NDFL_NO_HDRREC");
        emit_fast = num("NDFL_EMIT_FAST", 1) != 0;
        no_bt = on("NDFL_NO_BT"); no_alias = on("NDFL_NO_ALIAS");
        count_w = (uint32_t)num("NDFL_COUNT_W", 0);
        deflate_pf = num("NDFL_DEFLATE_PF", 1) != 0; deflate_profile = on("NDFL_DEFLATE_PROFILE");
        deflate_fused = on("NDFL_DEFLATE_FUSED");
        lz_stats = on("NDFL_LZ_STATS");
        const char* se = getenv("NDFL_LZ_SEARCH");
        lz_chain = se && !strcmp(se, "chain");
        lz_lead = num("NDFL_LZ_LEAD", -1);
        test_segflip = on("NDFL_TEST_SEGFLIP");
        flat = num("NDFL_FLAT", 1) != 0;
        flat_min = (uint32_t)num("NDFL_FLAT_MIN", 49152);
    }
    // the effective switches, one line (printed by ndfl_ctx_create when stats are on)
    void print(FILE* f) const {
        fprintf(f, "[ndfl] context knobs: stats=%d host_times=%d host_link=%d no_hdrrec=%d emit_fast=%d no_bt=%d "
                   "no_alias=%d count_w=%u deflate_pf=%d deflate_profile=%d deflate_fused=%d lz_stats=%d "
                   "lz_search=%s lz_lead=%d test_segflip=%d flat=%d flat_min=%u\n",
                (int)stats, (int)host_times, (int)host_link, (int)no_hdrrec, (int)emit_fast, (int)no_bt,
                (int)no_alias, count_w, (int)deflate_pf, (int)deflate_profile, (int)deflate_fused, (int)lz_stats,
                lz_chain ? "chain" : "parse", lz_lead, (int)test_segflip, (int)flat, flat_min);
    }
};

#define NDFL_WAVE 64

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// CRC-32/ISO-HDLC (java.util.zip.CRC32) in the reflected domain.
#define NDFL_CRC_POLY 0xEDB88320u

// a*b mod P for reflected 32-bit polynomials (x^0 is the MSB).
__host__ __device__ inline uint32_t crc_multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ NDFL_CRC_POLY : b >> 1;
    }
    return p;
}

// x^(8*n) mod P.
__host__ __device__ inline uint32_t crc_x8n(uint64_t n) {
    uint32_t p = 1u << 31;          // x^0
    uint32_t sq = 1u << 23;         // x^8
    while (n) {
        if (n & 1) p = crc_multmodp(sq, p);
        sq = crc_multmodp(sq, sq);
        n >>= 1;
    }
    return p;
}

// Wave-level inclusive scan (sum) over 64 lanes.
template <typename T>
__device__ inline T wave_incl_scan(T x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

template <typename T>
__device__ inline T wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

template <typename T>
__device__ inline T wave_xor(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    return x;
}

// Block-wide exclusive scan.  `sh` needs NWAVES entries.  All threads must call.
template <typename T, int NWAVES>
__device__ inline T block_excl_scan(T v, T* sh, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = wave_incl_scan(v);
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        T w = lane < NWAVES ? sh[lane] : T(0);
        w = wave_incl_scan(w);
        if (lane < NWAVES) sh[lane] = w;
    }
    __syncthreads();
    T pre = (wid > 0 ? sh[wid - 1] : T(0)) + x - v;
    total = sh[NWAVES - 1];
    __syncthreads();
    return pre;
}

// Device-wide exclusive scan in two launches over tiles of SCAN_TILE items (SCAN_T threads x
// SCAN_PER items, loads in flight together): scan_tile_sum writes each tile's sum, scan_tile_apply
// scans a tile from the sum of the tiles before it (each block adds those partials up itself: no
// third launch, no block waits on another).  One workgroup over the whole list ran at the bandwidth
// one CU draws from data other XCDs wrote (~0.1 ms for 65,536 items).  n >= 1.
constexpr uint32_t SCAN_T = 256, SCAN_PER = 8, SCAN_TILE = SCAN_T * SCAN_PER;
template <class Ld>
__device__ __forceinline__ void scan_tile_sum(Ld ld, uint32_t n, uint64_t* part) {
    __shared__ uint64_t sh[SCAN_T / 64];
    const uint32_t i0 = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
    uint64_t x[SCAN_PER], v = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) x[k] = ld(min(i0 + k, n - 1));
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) v += i0 + k < n ? x[k] : 0ull;
    uint64_t tot;
    block_excl_scan<uint64_t, SCAN_T / 64>(v, sh, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
// st(i, exclusive prefix of item i + init); *grand (if set) = init + the sum of all n items
template <class Ld, class St>
__device__ __forceinline__ void scan_tile_apply(Ld ld, St st, uint32_t n, const uint64_t* part, uint64_t init,
                                                uint64_t* grand) {
    __shared__ uint64_t sh[SCAN_T / 64], sp[SCAN_T / 64];
    uint64_t p = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += SCAN_T) p += part[t];
    uint64_t before;
    block_excl_scan<uint64_t, SCAN_T / 64>(p, sp, before);
    const uint32_t i0 = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
    uint64_t x[SCAN_PER], v = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) x[k] = ld(min(i0 + k, n - 1));
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) { if (i0 + k >= n) x[k] = 0; v += x[k]; }
    uint64_t tot;
    uint64_t run = init + before + block_excl_scan<uint64_t, SCAN_T / 64>(v, sh, tot);
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++)
        if (i0 + k < n) { st(i0 + k, run); run += x[k]; }
    if (grand && blockIdx.x + 1 == gridDim.x && threadIdx.x == 0) *grand = init + before + tot;
}

// Block-wide exclusive suffix minimum: min over threads t' > t of v[t'] (or `ident`).
template <int NWAVES>
__device__ inline uint32_t block_excl_suffix_min(uint32_t v, uint32_t ident, uint32_t* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // inclusive suffix min within the wave
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_down(x, o, 64);
        if (lane + o < 64) x = min(x, y);
    }
    if (lane == 0) sh[wid] = x;       // wave's min
    __syncthreads();
    uint32_t after = ident;           // min over later waves
    for (int w = wid + 1; w < NWAVES; w++) after = min(after, sh[w]);
    uint32_t nxt = __shfl_down(x, 1, 64);
    uint32_t r = (lane == 63) ? after : min(nxt, after);
    __syncthreads();
    return r;
}

// Agent-scope relaxed atomics on 64-bit status words (decoupled look-back).
__device__ inline uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
