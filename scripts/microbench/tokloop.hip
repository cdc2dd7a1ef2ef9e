// tokloop.hip -- microbenchmark of the decoder's Huffman token loop on one MI355X (not part of the
// library).  A synthetic literal/length/distance stream (text-like literal code, all codes <= 10 bits
// so every token resolves in the primary table, literal pairs as in wv::group_lits) is decoded in
// rounds staged into LDS exactly like wv::stage_round (word i of lane j at w[i * 64 + j], 14-word
// lane segments), one wave per workgroup, LDS padded so that occupancy matches the count pass
// (NDFL_MB_LDS bytes per wave).  Variants of the per-lane loop:
//   0  window: every token re-reads its 64-bit window from LDS (ds_read2st64 + ds_read, alignbit),
//      then the table -- two dependent LDS round trips per token (the library's tok<false>)
//   1  bit buffer: a 64-bit register buffer refilled one word at a time from a word loaded ahead,
//      so the table read is the only LDS round trip on the token's dependency chain
//   2  window, two half-segments per lane decoded in lockstep (two independent chains)
//   3  bit buffer, two half-segments per lane in lockstep
// Every variant must report the same byte count.  Build: hipcc -O3 --offload-arch=gfx950 -o tokloop tokloop.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <queue>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t LB = 10, DB = 8;
constexpr uint32_t LPW = 14, SW = LPW + 4;
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3 };

#ifndef NDFL_MB_LDS
#define NDFL_MB_LDS 13000
#endif
constexpr uint32_t TAB_BYTES = ((1u << LB) + (1u << DB)) * 4;
constexpr uint32_t STG_BYTES = SW * 64 * 4;
constexpr uint32_t PAD_BYTES = NDFL_MB_LDS > TAB_BYTES + STG_BYTES ? NDFL_MB_LDS - TAB_BYTES - STG_BYTES : 4;

struct Sh {
    uint32_t lit[1u << LB];
    uint32_t dst[1u << DB];
    uint32_t w[SW * 64];
    uint32_t pad[PAD_BYTES / 4];
};

__device__ __forceinline__ void stage(const uint32_t* in, uint64_t nwords, uint64_t w0base, Sh& S, int lane) {
    const uint64_t w0 = w0base + (uint64_t)lane * LPW;
    __syncthreads();
#pragma unroll 4
    for (uint32_t i = 0; i < SW; i++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(in + min(w0 + i, nwords - 1)),
                                         (__attribute__((address_space(3))) void*)&S.w[i * 64], 4, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// ---- variant 0/2: window re-read per token ----------------------------------------------------
struct Win {
    const uint32_t* p;
    __device__ __forceinline__ void win(uint32_t pos, uint32_t& lo, uint32_t& hi) const {
        const uint32_t* q = p + (pos >> 5) * 64;
        const uint32_t a = q[0], b = q[64], c = q[128];
        lo = __builtin_amdgcn_alignbit(b, a, pos & 31);
        hi = __builtin_amdgcn_alignbit(c, b, pos & 31);
    }
};
// one token at pos (no end checks: caller keeps pos + 48 < stop); returns bytes
__device__ __forceinline__ uint32_t tok_win(const Win& v, uint32_t& pos, const Sh& S) {
    uint32_t lo, hi;
    v.win(pos, lo, hi);
    const uint32_t e = S.lit[lo & ((1u << LB) - 1u)];
    if (e >> 31) { pos += e & 15; return 1u + ((e >> 8) & 1u); }
    const uint32_t cl = e & 31, xb = (e >> 5) & 15;
    const uint32_t run = (e >> 16) + ((lo >> cl) & ((1u << xb) - 1u));
    const uint32_t sh = cl + xb;
    const uint32_t dw = __builtin_amdgcn_alignbit(hi, lo, sh);
    const uint32_t d = S.dst[dw & ((1u << DB) - 1u)];
    const uint32_t dl = d & 31, dxb = (d >> 5) & 15;
    pos += sh + dl + dxb;
    return run;
}

// ---- variant 1/3: bit buffer ---------------------------------------------------------------------
struct BB {
    uint64_t buf;      // bits from pos on
    uint32_t nb;       // valid bits in buf (32..64 at a token start)
    uint32_t wi;       // index of the next word to append (relative to the lane region)
    uint32_t nxt;      // that word, loaded ahead
    uint32_t pos;
};
__device__ __forceinline__ void bb_init(BB& b, const uint32_t* p, uint32_t pos) {
    const uint32_t i = pos >> 5, s = pos & 31;
    b.buf = ((uint64_t)p[i * 64] | ((uint64_t)p[(i + 1) * 64] << 32)) >> s;
    b.nb = 64 - s;
    b.wi = i + 2;
    b.nxt = p[b.wi * 64];
    b.pos = pos;
}
__device__ __forceinline__ void bb_refill(BB& b, const uint32_t* p) {
    if (b.nb < 32) {
        b.buf |= (uint64_t)b.nxt << b.nb;
        b.nb += 32;
        b.wi++;
        b.nxt = p[b.wi * 64];
    }
}
__device__ __forceinline__ uint32_t tok_bb(BB& b, const uint32_t* p, const Sh& S) {
    const uint32_t e = S.lit[(uint32_t)b.buf & ((1u << LB) - 1u)];
    uint32_t n;
    if (e >> 31) {
        const uint32_t adv = e & 15;
        b.buf >>= adv; b.nb -= adv; b.pos += adv;
        n = 1u + ((e >> 8) & 1u);
    } else {
        const uint32_t cl = e & 31, xb = (e >> 5) & 15;
        const uint32_t lo = (uint32_t)b.buf;
        n = (e >> 16) + ((lo >> cl) & ((1u << xb) - 1u));
        const uint32_t sh = cl + xb;
        b.buf >>= sh; b.nb -= sh; b.pos += sh;
        bb_refill(b, p);
        const uint32_t d = S.dst[(uint32_t)b.buf & ((1u << DB) - 1u)];
        const uint32_t dl = d & 31, dxb = (d >> 5) & 15;
        b.buf >>= dl + dxb; b.nb -= dl + dxb; b.pos += dl + dxb;
    }
    bb_refill(b, p);
    return n;
}

template <int V>
__global__ void __launch_bounds__(64) tok_kernel(const uint32_t* in, uint64_t nwords, uint32_t nrounds,
                                                 const uint32_t* lit, const uint32_t* dst, unsigned long long* out) {
    __shared__ Sh S;
    const int lane = threadIdx.x;
    for (uint32_t k = lane; k < (1u << LB); k += 64) S.lit[k] = lit[k];
    for (uint32_t k = lane; k < (1u << DB); k += 64) S.dst[k] = dst[k];
    if (lane == 0) S.pad[0] = 0;
    uint64_t total = 0;
    const uint32_t seg = LPW * 32;
    for (uint32_t r = blockIdx.x; r < nrounds; r += gridDim.x) {
        stage(in, nwords, (uint64_t)r * 64 * LPW, S, lane);
        const uint32_t* p = S.w + lane;
        uint32_t cnt = 0;
        if (V == 0) {
            Win v{p};
            uint32_t pos = 0;
            while (pos + 48 < seg) cnt += tok_win(v, pos, S);
        } else if (V == 1) {
            BB b;
            bb_init(b, p, 0);
            while (b.pos + 48 < seg) cnt += tok_bb(b, p, S);
        } else if (V == 2) {
            Win v{p};
            uint32_t pa = 0, pb = seg / 2;
            const uint32_t ea = seg / 2, eb = seg;
            for (;;) {
                const bool fa = pa + 48 < ea, fb = pb + 48 < eb;
                if (!fa && !fb) break;
                if (fa) cnt += tok_win(v, pa, S);
                if (fb) cnt += tok_win(v, pb, S);
            }
        } else {
            BB a, b;
            bb_init(a, p, 0);
            bb_init(b, p, seg / 2);
            const uint32_t ea = seg / 2, eb = seg;
            for (;;) {
                const bool fa = a.pos + 48 < ea, fb = b.pos + 48 < eb;
                if (!fa && !fb) break;
                if (fa) cnt += tok_bb(a, p, S);
                if (fb) cnt += tok_bb(b, p, S);
            }
        }
        total += cnt;
    }
    atomicAdd(out, (unsigned long long)total);
}

// ---- host: a text-like code and stream ----------------------------------------------------------
static void huff_lengths(const std::vector<double>& f, std::vector<int>& len) {
    const int n = (int)f.size();
    std::vector<int> parent(2 * n, -1);
    typedef std::pair<double, int> P;
    std::priority_queue<P, std::vector<P>, std::greater<P>> q;
    for (int i = 0; i < n; i++) q.push({f[i], i});
    int nx = n;
    while (q.size() > 1) {
        P a = q.top(); q.pop();
        P b = q.top(); q.pop();
        parent[a.second] = nx; parent[b.second] = nx;
        q.push({a.first + b.first, nx++});
    }
    len.assign(n, 0);
    for (int i = 0; i < n; i++) { int d = 0, x = i; while (parent[x] >= 0) { x = parent[x]; d++; } len[i] = d; }
}

int main(int argc, char** argv) {
    const uint64_t nbits_target = (argc > 1 ? strtoull(argv[1], 0, 10) : 2048ull) << 20;   // Mbit
    const int reps = 5;
    // symbols: 256 literals (Zipf-like) + length symbols 257..264 (runs 3..10); distance: 2 codes
    std::vector<double> f(265, 0.0);
    for (int i = 0; i < 256; i++) f[i] = 1.0 / (1.0 + (i * 37 % 256));
    double lsum = 0; for (int i = 0; i < 256; i++) lsum += f[i];
    for (int i = 257; i < 265; i++) f[i] = lsum * 0.06 / 8;
    f[256] = 1e-9;                       // EOB: present, never emitted
    std::vector<int> len;
    for (int it = 0; it < 40; it++) {
        huff_lengths(f, len);
        int mx = *std::max_element(len.begin(), len.end());
        if (mx <= 10) break;
        for (auto& x : f) x = x + lsum * 0.002;      // flatten until every code fits the primary
    }
    // canonical codes
    int blc[16] = {0}, nxc[16];
    for (int l : len) if (l) blc[l]++;
    int code = 0; blc[0] = 0;
    for (int b = 1; b < 16; b++) { code = (code + blc[b - 1]) << 1; nxc[b] = code; }
    std::vector<uint32_t> cw(265);
    auto rev = [](uint32_t v, int l) { uint32_t r = 0; for (int i = 0; i < l; i++) r |= ((v >> i) & 1) << (l - 1 - i); return r; };
    for (int s = 0; s < 265; s++) if (len[s]) cw[s] = rev(nxc[len[s]]++, len[s]);
    // primary table with literal pairs (wv::lit_entry + group_lits)
    std::vector<uint32_t> lit(1u << LB, 0), dst(1u << DB, 0);
    for (int s = 0; s < 265; s++) {
        if (!len[s]) continue;
        uint32_t e;
        if (s < 256) e = (uint32_t)len[s] | (K_LIT << 9) | ((uint32_t)s << 16);
        else if (s == 256) e = (uint32_t)len[s] | (K_EOB << 9);
        else e = (uint32_t)len[s] | (K_LEN << 9) | ((uint32_t)(s - 257 + 3) << 16);
        for (uint32_t k = cw[s]; k < (1u << LB); k += 1u << len[s]) lit[k] = e;
    }
    std::vector<uint32_t> nv(1u << LB);
    for (uint32_t k = 0; k < (1u << LB); k++) {
        const uint32_t e1 = lit[k], l1 = e1 & 31;
        uint32_t v = e1;
        if (l1 && ((e1 >> 9) & 3) == K_LIT) {
            const uint32_t b1 = (e1 >> 16) & 0xFF;
            v = (1u << 31) | l1 | (l1 << 4) | (b1 << 9);
            const uint32_t e2 = lit[k >> l1], l2 = e2 & 31;
            if (l1 < LB && l2 && l1 + l2 <= LB && ((e2 >> 9) & 3) == K_LIT)
                v = (1u << 31) | (l1 + l2) | (l1 << 4) | (1u << 8) | (b1 << 9) | (((e2 >> 16) & 0xFF) << 17);
        }
        nv[k] = v;
    }
    lit = nv;
    for (uint32_t k = 0; k < (1u << DB); k++) dst[k] = 1u | ((1u + (k & 1)) << 16);     // 2 codes of length 1
    // stream
    std::vector<uint32_t> words((nbits_target >> 5) + 64, 0);
    uint64_t bp = 0;
    double ftot = 0; for (int s = 0; s < 265; s++) if (s != 256) ftot += f[s];
    std::vector<double> cdf; std::vector<int> sym;
    double acc = 0; for (int s = 0; s < 265; s++) if (s != 256) { acc += f[s] / ftot; cdf.push_back(acc); sym.push_back(s); }
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    auto put = [&](uint32_t v, int n) { for (int i = 0; i < n; i++, bp++) if ((v >> i) & 1) words[bp >> 5] |= 1u << (bp & 31); };
    uint64_t nsyms = 0, nbytes = 0;
    while (bp + 64 < nbits_target) {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        const double u = (rng >> 11) * (1.0 / 9007199254740992.0);
        const int s = sym[std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin() < (long)sym.size() ? std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin() : sym.size() - 1];
        put(cw[s], len[s]);
        if (s > 256) { put(rng & 1, 1); nbytes += s - 257 + 3; } else nbytes++;
        nsyms++;
    }
    printf("code: max len %d, %.2f bits/symbol, stream %llu Mbit, %.2f bytes/symbol\n",
           *std::max_element(len.begin(), len.end()), (double)bp / nsyms, (unsigned long long)(bp >> 20), (double)nbytes / nsyms);
    const uint64_t nwords = words.size();
    const uint32_t nrounds = (uint32_t)((bp >> 5) / (64 * LPW)) - 1;
    uint32_t *d_in, *d_lit, *d_dst;
    unsigned long long* d_out;
    CHECK(hipMalloc(&d_in, nwords * 4));
    CHECK(hipMalloc(&d_lit, lit.size() * 4));
    CHECK(hipMalloc(&d_dst, dst.size() * 4));
    CHECK(hipMalloc(&d_out, 8));
    CHECK(hipMemcpy(d_in, words.data(), nwords * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_lit, lit.data(), lit.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_dst, dst.data(), dst.size() * 4, hipMemcpyHostToDevice));
    hipDeviceProp_t pr;
    CHECK(hipGetDeviceProperties(&pr, 0));
    const int grid = pr.multiProcessorCount * 32;      // every wave slot the LDS / VGPR budget allows
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    printf("LDS/wave %u B (%u waves/CU by LDS), grid %d, rounds %u\n", (unsigned)sizeof(Sh),
           (unsigned)(163840 / sizeof(Sh)), grid, nrounds);
    auto run = [&](int v) {
        unsigned long long res = 0;
        float best = 1e30f;
        for (int r = 0; r < reps; r++) {
            CHECK(hipMemset(d_out, 0, 8));
            CHECK(hipEventRecord(e0));
            if (v == 0) tok_kernel<0><<<grid, 64>>>(d_in, nwords, nrounds, d_lit, d_dst, d_out);
            if (v == 1) tok_kernel<1><<<grid, 64>>>(d_in, nwords, nrounds, d_lit, d_dst, d_out);
            if (v == 2) tok_kernel<2><<<grid, 64>>>(d_in, nwords, nrounds, d_lit, d_dst, d_out);
            if (v == 3) tok_kernel<3><<<grid, 64>>>(d_in, nwords, nrounds, d_lit, d_dst, d_out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            CHECK(hipMemcpy(&res, d_out, 8, hipMemcpyDeviceToHost));
        }
        const double bits = (double)nrounds * 64 * LPW * 32;
        printf("variant %d: %.3f ms, %.1f GB/s of stream, %.1f GB/s of output, bytes %llu\n", v, best,
               bits / 8 / best / 1e6, (double)res / best / 1e6, res);
    };
    for (int v = 0; v < 4; v++) run(v);
    return 0;
}
