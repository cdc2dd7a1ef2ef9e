// build_bench.hip -- the decoder's per-block table build (wv::build_tables, inflate_wave.hpp) in
// isolation (measurement tooling, not product code): every wave builds the tables of real block
// headers (scripts/r06/make_hdr_set.py: the dynamic headers of the oracle's RLE_DYNAMIC encoding of
// the config-4 corpus) over and over, at the count pass's occupancy (3 waves per SIMD) and alone
// (1 wave per SIMD), and reports cycles per build; every record's tables are also written out once
// and compared with the build compiled as the reference (-DREF_BUILD=1 in a second binary, or the
// same binary: the dump file of one run is the reference of the next).
// Build: hipcc -O3 --offload-arch=gfx950 -w -I. -o build_bench build_bench.hip [-DNDFL_...]
// Run:   ./build_bench hdrs.bin [dump_out.bin] [ref_dump.bin]
#include "../../deflate-library-java_amd/csrc/hip/inflate_kernels.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

struct HRec {
    uint32_t btype, numlit, numdist, pad;
    uint8_t lens[320];
};

__device__ __forceinline__ void load_rec(const HRec& r, wv::Shared& S, int lane) {
    for (uint32_t s = (uint32_t)lane; s < 320; s += 64) S.lens[s] = r.lens[s];
    if (lane == 0) {
        S.h_btype = r.btype; S.h_numlit = r.numlit; S.h_numdist = r.numdist; S.h_err = 0; S.h_bfinal = 0;
    }
    __syncthreads();
}

// MODE 0: build_tables; 1: the literal/length build_code alone; 2: + group_lits; 3: the distance build_code
template <int MODE>
__device__ __forceinline__ int build_part(wv::Shared& S, int lane, bool& ed, uint32_t* scr) {
    using namespace wv;
    ed = false;
    if (MODE == 0) return build_tables(S, lane, ed, scr);
#if NDFL_BUILD_V2
    LShared* L = (LShared*)&S;
    if (MODE == 3) return build_code_l<false, DB>(L, 288, 32, L->t.dst, L->t.dx, DX, false, lane, (lu32*)scr);
    const int e = MODE == 2 ? build_code_l<false, LB, true>(L, 0, 288, L->t.lit, L->t.lx, LX, true, lane, (lu32*)scr)
                            : build_code_l<false, LB>(L, 0, 288, L->t.lit, L->t.lx, LX, true, lane, (lu32*)scr);
#else
    if (MODE == 3) return build_code(S, 288, 32, S.t.dst, DB, S.t.dx, DX, false, lane);
    const int e = build_code(S, 0, 288, S.t.lit, LB, S.t.lx, LX, true, lane);
    if (MODE == 2 && !e) group_lits(S.t, lane);
#endif
    return e;
}

template <int WPE, int MODE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
bench_kernel(const HRec* recs, uint32_t nrec, uint32_t iters, unsigned long long* cyc, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) wv::Shared S;
    __shared__ wv::Stage stg;
    const int lane = threadIdx.x;
    unsigned long long tot = 0;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; it++) {
        const HRec& r = recs[(blockIdx.x * 7u + it) % nrec];
        load_rec(r, S, lane);
        const unsigned long long t0 = clock64();
        bool ed;
        const int e = build_part<MODE>(S, lane, ed, stg.w);
        __syncthreads();
        tot += clock64() - t0;
        acc += S.t.lit[lane * 16 + (it & 15)] ^ S.t.dst[lane * 4] ^ (uint32_t)e ^ (ed ? 7u : 0u);
    }
    if (lane == 0) atomicAdd(cyc, tot);
    if (acc == 0x9E3779B9u) sink[lane] = acc;
}

__global__ void __launch_bounds__(64) dump_kernel(const HRec* recs, uint32_t nrec, wv::Tabs* out, int* err) {
    __shared__ __attribute__((aligned(16))) wv::Shared S;
    __shared__ wv::Stage stg;
    const int lane = threadIdx.x;
    for (uint32_t k = blockIdx.x; k < nrec; k += gridDim.x) {
        for (uint32_t q = (uint32_t)lane; q < sizeof(wv::Tabs) / 4; q += 64) ((uint32_t*)&S.t)[q] = 0;
        load_rec(recs[k], S, lane);
        bool ed;
        const int e = wv::build_tables(S, lane, ed, stg.w);
        __syncthreads();
        const uint32_t* src = (const uint32_t*)&S.t;
        uint32_t* dst = (uint32_t*)(out + k);
        for (uint32_t q = (uint32_t)lane; q < sizeof(wv::Tabs) / 4; q += 64) dst[q] = src[q];
        if (lane == 0) err[k] = e | (ed ? 0x100 : 0);
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: build_bench hdrs.bin [dump_out] [ref_dump]\n"); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    std::vector<HRec> h;
    HRec r;
    while (fread(&r, sizeof r, 1, f) == 1) h.push_back(r);
    fclose(f);
    const uint32_t n = (uint32_t)h.size();
    HRec* d_recs;
    wv::Tabs* d_tabs;
    int* d_err;
    unsigned long long* d_cyc;
    uint32_t* d_sink;
    if (hipMalloc(&d_recs, n * sizeof(HRec)) || hipMalloc(&d_tabs, n * sizeof(wv::Tabs)) || hipMalloc(&d_err, n * 4) ||
        hipMalloc(&d_cyc, 8) || hipMalloc(&d_sink, 256)) return 1;
    (void)hipMemcpy(d_recs, h.data(), n * sizeof(HRec), hipMemcpyHostToDevice);
    // correctness: every record's tables, optionally against a reference dump
    hipLaunchKernelGGL(dump_kernel, dim3(256), dim3(64), 0, 0, d_recs, n, d_tabs, d_err);
    std::vector<wv::Tabs> t(n);
    std::vector<int> e(n);
    (void)hipMemcpy(t.data(), d_tabs, n * sizeof(wv::Tabs), hipMemcpyDeviceToHost);
    (void)hipMemcpy(e.data(), d_err, n * 4, hipMemcpyDeviceToHost);
    if (argc > 2) {
        FILE* o = fopen(argv[2], "wb");
        fwrite(t.data(), sizeof(wv::Tabs), n, o);
        fwrite(e.data(), 4, n, o);
        fclose(o);
    }
    int bad = -1;
    if (argc > 3) {
        FILE* rf = fopen(argv[3], "rb");
        std::vector<wv::Tabs> rt(n);
        std::vector<int> re(n);
        if (!rf || fread(rt.data(), sizeof(wv::Tabs), n, rf) != n || fread(re.data(), 4, n, rf) != n) { fprintf(stderr, "ref\n"); return 1; }
        fclose(rf);
        // the words a decoder reads: both primary tables, and of each extension area its used part
        // -- the second-level tables (up to the last one a primary entry points at), or the slow
        // path's arrays (n entries + 16 limits + 16 u16 first codes + 16 u16 offsets)
        auto used = [](const uint32_t* prim, uint32_t np, uint32_t n) {
            uint32_t u = 0;
            bool any_long = false, any_two = false;
            for (uint32_t k = 0; k < np; k++) {
                const uint32_t e = prim[k];
                if ((e >> 31) || (e & 31)) continue;
                any_long = true;
                const uint32_t sd = (e >> 5) & 15;
                if (sd) { any_two = true; u = std::max(u, (e >> 16) + (1u << sd)); }
            }
            return !any_long ? 0u : any_two ? u : n + 32;
        };
        bad = 0;
        for (uint32_t k = 0; k < n; k++) {
            const wv::Tabs& A = rt[k];
            const wv::Tabs& B = t[k];
            const uint32_t ul = used(A.lit, 1024, 288), ud = used(A.dst, 256, 32);
            const bool same = !memcmp(A.lit, B.lit, sizeof A.lit) && !memcmp(A.dst, B.dst, sizeof A.dst) &&
                              !memcmp(A.lx, B.lx, ul * 4) && !memcmp(A.dx, B.dx, ud * 4) && re[k] == e[k];
            if (!same) {
                if (bad < 5) fprintf(stderr, "record %u differs (lx used %u, dx used %u, err %x / %x)\n", k, ul, ud, re[k], e[k]);
                bad++;
            }
        }
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t iters = 64;
    typedef void (*KF)(const HRec*, uint32_t, uint32_t, unsigned long long*, uint32_t*);
    const KF kf[2][4] = {{bench_kernel<1, 0>, bench_kernel<1, 1>, bench_kernel<1, 2>, bench_kernel<1, 3>},
                         {bench_kernel<3, 0>, bench_kernel<3, 1>, bench_kernel<3, 2>, bench_kernel<3, 3>}};
    const char* mname[4] = {"build_tables", "lit build_code", "lit + group_lits", "dist build_code"};
    for (int mode = 0; mode < 4; mode++)
    for (int wpe : {1, 3}) {
        const uint32_t grid = (uint32_t)ncu * 4 * wpe;
        for (int rep = 0; rep < 2; rep++) {
            (void)hipMemset(d_cyc, 0, 8);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(kf[wpe == 3][mode], dim3(grid), dim3(64), 0, 0, d_recs, n, iters, d_cyc, d_sink);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
        }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        unsigned long long cyc = 0;
        (void)hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
        const double builds = (double)grid * iters;
        printf("%-18s waves/SIMD %d: %u waves x %u builds: %.3f ms, %.1f ns per build (chip), %.0f cycles per build (wave)\n",
               mname[mode], wpe, grid, iters, ms, ms * 1e6 / builds, (double)cyc / builds);
    }
#ifdef NDFL_BUILD_PROF
    {
        std::vector<unsigned long long> all(8192 * 8);
        (void)hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(wv::g_bprof), all.size() * 8);
        unsigned long long pr[8] = {};
        for (size_t i = 0; i < all.size(); i++) pr[i % 8] += all[i];
        unsigned long long tot = 0;
        for (int i = 0; i < 6; i++) tot += pr[i];
        printf("build_code_v2 sections (share of cycles, all runs): ranks %.3f d %.3f scatter %.3f long %.3f pull %.3f sub %.3f\n",
               pr[0] / (double)tot, pr[1] / (double)tot, pr[2] / (double)tot, pr[3] / (double)tot, pr[4] / (double)tot,
               pr[5] / (double)tot);
    }
#endif
    printf("records %u, compared %s\n", n, bad < 0 ? "no reference" : bad == 0 ? "all equal" : "DIFFER");
    return bad > 0 ? 1 : 0;
}
