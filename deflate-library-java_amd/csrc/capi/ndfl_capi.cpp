// ndfl_capi.cpp -- host side of the C ABI declared in include/ndfl.h.
// Compiled as HIP for gfx950 together with the kernels (single translation unit).
#include "../../../include/ndfl.h"
#include "../hip/deflate_kernels.hip"
#include "../hip/deflate_split.hip"
#include "../hip/lz77_kernels.hip"
#include "../hip/strategy_kernels.hip"
#include "../hip/inflate_kernels.hip"

#include <hip/hip_runtime.h>
#include <string.h>
#include <stdio.h>
#include <algorithm>
#include <stdlib.h>
#include <vector>
#include <functional>
#include <map>

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) { hipFree(p); p = nullptr; cap = 0; }
        size_t want = n < 4096 ? 4096 : n;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() { if (p) hipFree(p); p = nullptr; cap = 0; }
    template <class T> T* as() const { return (T*)p; }
};

uint32_t host_crc_tab[1024];
uint32_t host_crc_x[64 + 1024];
uint32_t host_crc_p2[64];          // x^(8 * 2^k)
bool host_tabs_ready = false;

void init_host_tables() {
    if (host_tabs_ready) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ NDFL_CRC_POLY : c >> 1;
        host_crc_tab[i] = c;
    }
    for (int t = 1; t < 4; t++)
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = host_crc_tab[(t - 1) * 256 + i];
            host_crc_tab[t * 256 + i] = (c >> 8) ^ host_crc_tab[c & 0xFF];
        }
    for (uint32_t k = 0; k < 64; k++) host_crc_x[k] = crc_x8n(k);
    for (uint32_t k = 0; k < 1024; k++) host_crc_x[64 + k] = crc_x8n((uint64_t)k * 64);
    host_crc_p2[0] = 1u << 23;
    for (int k = 1; k < 64; k++) host_crc_p2[k] = crc_multmodp(host_crc_p2[k - 1], host_crc_p2[k - 1]);
    host_tabs_ready = true;
}

}  // namespace

struct ndfl_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    bool user_stream = false;       // ndfl_ctx_set_stream named the caller's stream
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_order = nullptr;
    double last_ms = 0;
    double deflate_ms = 0;
    DevBuf d_in, d_out, d_status, d_ticket, d_edge_w, d_edge_v, d_crc, d_crc1, d_tabs, d_hostio;
    DevBuf d_hist, d_codes, d_off;  // split RLE/LITERAL pipeline: histograms, code records, offsets
    DevBuf d_lz, d_link, d_match;   // LZ77 path: staging [pad|hist|data], hash links, per-position matches
    DevBuf d_mdata, d_mstreams[16], d_mbits[16], d_masm;   // strategy composition
    uint64_t* cb_out = nullptr;     // internal: when set, encoders also write per-chunk block bits here
    uint32_t parent_len = 0;        // internal: history rule of BinarySplit sub-blocks (0: chunk_len)
    InflateScratch inf;
    uint32_t* h_pinned = nullptr;   // small pinned area for results
    Knobs knobs;                    // switches read once at ndfl_ctx_create (ndfl_common.hpp)
    int err_sym = -1;               // the last decode's reserved symbol (ndfl_ctx_error_symbol), or -1
};

#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return NDFL_E_DEVICE; } while (0)

// The ordering contract of include/ndfl.h: unless the caller named its stream (ndfl_ctx_set_stream),
// a call's device work starts only after everything queued before the call on the device's default
// stream -- e.g. the torch kernel that produced an NDFL_IN_DEVICE buffer, or the torch kernel still
// using a block the caching allocator has just handed out again as an NDFL_OUT_DEVICE buffer.  (The
// context's own stream is also a blocking stream, which the null stream orders implicitly; the
// event makes the wait explicit.)  Every call synchronizes its stream before returning, so results
// are complete when the call returns.
static hipStream_t ordered_stream(ndfl_ctx* c) {
    if (!c->user_stream) {
        hipEventRecord(c->ev_order, nullptr);
        hipStreamWaitEvent(c->stream, c->ev_order, 0);
    }
    return c->stream;
}

// Raw CRC of `len` bytes from the raw CRCs of its consecutive parts of `part_len` bytes into *out.
static hipError_t launch_crc_combine(ndfl_ctx* c, hipStream_t s, const uint32_t* parts, uint32_t nparts,
                                     uint32_t part_len, uint64_t len, uint32_t* out) {
    hipError_t e = hipMemsetAsync(out, 0, 4, s);
    if (e != hipSuccess) return e;
    const uint32_t* p2 = c->d_tabs.as<uint32_t>() + 1024 + 64 + 1024;
    const uint32_t grid = std::max(1u, std::min(1024u, (nparts + 255) / 256));
    hipLaunchKernelGGL(ndfl_crc_combine_kernel, dim3(grid), dim3(256), 0, s, parts, nparts, part_len, len, p2, out);
    return hipGetLastError();
}

extern "C" {

uint32_t ndfl_abi_version(void) { return NDFL_ABI_VERSION; }

const char* ndfl_error_string(int code) {
    static const char* reasons[] = {
        "Unexpected end of stream", "Reserved block type", "len/nlen mismatch in uncompressed block",
        "This canonical code produces an under-full Huffman code tree",
        "This canonical code produces an over-full Huffman code tree", "No code length value to copy",
        "Run exceeds number of codes", "End-of-block symbol has zero code length", "Reserved run length symbol",
        "Reserved distance symbol", "Length symbol encountered with empty distance code",
        "Attempting to copy from before start of dictionary", "Header checksum mismatch",
        "Unsupported compression method", "Decompression checksum mismatch", "Decompressed size mismatch",
        "Invalid GZIP magic number", "Reserved flags are set", "Unsupported operating system value"};
    if (code == 0) return "ok";
    if (code >= 1 && code <= 19) return reasons[code - 1];
    switch (code) {
        case NDFL_E_ARG: return "invalid argument";
        case NDFL_E_UNSUPPORTED: return "configuration not supported on the GPU path";
        case NDFL_E_CAPACITY: return "output buffer too small";
        case NDFL_E_DEVICE: return "HIP device error";
        case NDFL_E_STATE: return "invalid state";
        default: return "internal error";
    }
}

int ndfl_ctx_create(ndfl_ctx** out, int device, uint32_t flags) {
    (void)flags;
    if (!out) return NDFL_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return NDFL_E_DEVICE;
    HIPCHK(hipSetDevice(device));
    init_host_tables();
    ndfl_ctx* c = new ndfl_ctx();
    c->device = device;
    c->knobs.read();
    c->inf.knobs = c->knobs;
    if (c->knobs.stats) c->knobs.print(stderr);
    if (hipStreamCreateWithFlags(&c->own, hipStreamDefault) != hipSuccess) { delete c; return NDFL_E_DEVICE; }
    c->stream = c->own;
    hipEventCreate(&c->ev0);
    hipEventCreate(&c->ev1);
    if (hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming) != hipSuccess) { delete c; return NDFL_E_DEVICE; }
    if (c->d_tabs.ensure(sizeof(host_crc_tab) + sizeof(host_crc_x) + sizeof(host_crc_p2)) != hipSuccess) { delete c; return NDFL_E_DEVICE; }
    hipMemcpy(c->d_tabs.p, host_crc_tab, sizeof(host_crc_tab), hipMemcpyHostToDevice);
    hipMemcpy((char*)c->d_tabs.p + sizeof(host_crc_tab), host_crc_x, sizeof(host_crc_x), hipMemcpyHostToDevice);
    hipMemcpy((char*)c->d_tabs.p + sizeof(host_crc_tab) + sizeof(host_crc_x), host_crc_p2, sizeof(host_crc_p2),
              hipMemcpyHostToDevice);
    if (hipHostMalloc((void**)&c->h_pinned, 4096, 0) != hipSuccess) { delete c; return NDFL_E_DEVICE; }
    *out = c;
    return NDFL_OK;
}

int ndfl_ctx_destroy(ndfl_ctx* c) {
    if (!c) return NDFL_OK;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->d_in, &c->d_out, &c->d_status, &c->d_ticket, &c->d_edge_w, &c->d_edge_v,
                      &c->d_crc, &c->d_crc1, &c->d_tabs, &c->d_hostio, &c->d_lz, &c->d_link, &c->d_match,
                      &c->d_mdata, &c->d_masm, &c->d_hist, &c->d_codes, &c->d_off};
    for (DevBuf* b : bufs) b->release();
    for (int k = 0; k < 16; k++) { c->d_mstreams[k].release(); c->d_mbits[k].release(); }
    c->inf.release();
    if (c->h_pinned) hipHostFree(c->h_pinned);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->ev_order) hipEventDestroy(c->ev_order);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
    return NDFL_OK;
}

int ndfl_ctx_set_stream(ndfl_ctx* c, void* s) {
    if (!c) return NDFL_E_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    c->user_stream = s != nullptr;
    return NDFL_OK;
}

double ndfl_ctx_last_kernel_ms(ndfl_ctx* c) { return c ? c->last_ms : 0.0; }

int ndfl_ctx_timings(ndfl_ctx* c, double* ms, int n) {
    if (!c || !ms) return NDFL_E_ARG;
    double v[9] = {c->deflate_ms, c->inf.last_ms_find, c->inf.last_ms_count, c->inf.last_ms_emit,
                   c->inf.last_ms_wall, (double)c->inf.chains, (double)c->inf.repairs, (double)c->inf.candidates,
                   (double)c->inf.flat_chains};
    for (int i = 0; i < n && i < 9; i++) ms[i] = v[i];
    return n < 9 ? n : 9;
}

uint64_t ndfl_deflate_bound(uint64_t len, uint32_t chunk_len) {
    if (chunk_len == 0) return 0;
    uint64_t nch = len / chunk_len + 1;
    // per chunk: <= 9 bits per byte (+ EOB) + header (<= 4,500 bits) + word alignment slack
    return (9 * len + nch * 4640) / 8 + 64;
}

uint32_t ndfl_crc32_combine(uint32_t a, uint32_t b, uint64_t len_b) {
    return crc_multmodp(crc_x8n(len_b), a) ^ b;
}

int ndfl_deflate_chunks(ndfl_ctx* c, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                        const uint8_t* data, uint64_t len, uint32_t chunk_len, int strategy,
                        int final_flag, uint32_t start_bitpos, uint8_t* out, uint64_t out_cap,
                        uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags) {
    if (!c || !out_end_bits || (!data && len) || (!hist && hist_len) || !out) return NDFL_E_ARG;
    if (start_bitpos > 7 || hist_limit > 32768 || hist_len > hist_limit || chunk_len == 0) return NDFL_E_ARG;
    if (!final_flag && (len == 0 || len % chunk_len != 0)) return NDFL_E_ARG;
    int rle, dyn;
    switch (strategy) {
        case NDFL_LITERAL_STATIC: rle = 0; dyn = 0; break;
        case NDFL_LITERAL_DYNAMIC: rle = 0; dyn = 1; break;
        case NDFL_RLE_STATIC: rle = 1; dyn = 0; break;
        case NDFL_RLE_DYNAMIC: rle = 1; dyn = 1; break;
        case NDFL_FULL_STATIC: case NDFL_FULL_DYNAMIC:
            return ndfl_deflate_chunks_lz77(c, hist, hist_len, hist_limit, data, len, chunk_len,
                                            strategy == NDFL_FULL_DYNAMIC, 3, 258, 1, 32768, final_flag,
                                            start_bitpos, out, out_cap, out_end_bits, crc_inout, flags);
        case NDFL_UNCOMPRESSED: {
            ndfl_strategy_desc u = {NDFL_KIND_UNCOMPRESSED, 0, 0, 0, 0, 0};
            return ndfl_deflate_chunks_multi(c, hist, hist_len, hist_limit, data, len, chunk_len, &u, 1, final_flag,
                                             start_bitpos, out, out_cap, out_end_bits, crc_inout, flags);
        }
        default: return NDFL_E_ARG;
    }
    if (chunk_len > (uint32_t)MAX_CHUNK) return NDFL_E_UNSUPPORTED;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t nch64 = final_flag ? (len == 0 ? 1 : (len + chunk_len - 1) / chunk_len) : len / chunk_len;
    if (nch64 > 0xFFFFFFFFull) return NDFL_E_UNSUPPORTED;
    const uint32_t nch = (uint32_t)nch64;
    hipStream_t s = ordered_stream(c);

    // input
    const uint8_t* d_data = data;
    int prev_byte = -1;
    if (hist_len > 0) {
        if (flags & NDFL_IN_DEVICE) {
            uint8_t pb = 0;
            HIPCHK(hipMemcpyAsync(&pb, hist + hist_len - 1, 1, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            prev_byte = pb;
        } else {
            prev_byte = hist[hist_len - 1];
        }
    }
    if (!(flags & NDFL_IN_DEVICE) && len) {
        HIPCHK(c->d_in.ensure(len));
        HIPCHK(hipMemcpyAsync(c->d_in.p, data, len, hipMemcpyHostToDevice, s));
        d_data = c->d_in.as<uint8_t>();
    }
    // output
    const uint64_t bound = ndfl_deflate_bound(len, chunk_len);
    const uint64_t bound_words = (bound + 3) / 4 + 2;
    uint32_t* d_out;
    bool direct = (flags & NDFL_OUT_DEVICE) && (((uintptr_t)out & 3) == 0) && out_cap >= bound_words * 4;
    if (direct) d_out = (uint32_t*)out;
    else { HIPCHK(c->d_out.ensure(bound_words * 4)); d_out = c->d_out.as<uint32_t>(); }
    HIPCHK(c->d_status.ensure(nch * sizeof(uint64_t)));
    HIPCHK(c->d_ticket.ensure(64));
    HIPCHK(c->d_edge_w.ensure(2ull * nch * sizeof(uint64_t)));
    HIPCHK(c->d_edge_v.ensure(2ull * nch * sizeof(uint32_t)));
    if (crc_inout) { HIPCHK(c->d_crc.ensure(nch * sizeof(uint32_t))); HIPCHK(c->d_crc1.ensure(64)); }
    HIPCHK(hipMemsetAsync(c->d_status.p, 0, nch * sizeof(uint64_t), s));
    HIPCHK(hipMemsetAsync(c->d_ticket.p, 0, 64, s));

    Args a;
    a.in = d_data; a.n = len; a.chunk_len = chunk_len; a.nchunks = nch;
    a.prev_byte = prev_byte; a.hist_enabled = hist_limit > 0; a.final_last = final_flag ? 1 : 0;
    a.rle = rle; a.dynamic = dyn; a.base_bit = start_bitpos;
    a.parent_len = c->parent_len ? c->parent_len : chunk_len;
    a.out = d_out; a.status = c->d_status.as<uint64_t>(); a.ticket = c->d_ticket.as<uint32_t>();
    a.edge_w = c->d_edge_w.as<uint64_t>(); a.edge_v = c->d_edge_v.as<uint32_t>();
    a.chunk_bits = c->cb_out;
    a.crc_raw = crc_inout ? c->d_crc.as<uint32_t>() : nullptr;
    a.crc_tab = c->d_tabs.as<uint32_t>();
    a.crc_x = c->d_tabs.as<uint32_t>() + 1024;
    a.prof = nullptr;
    const bool prof = c->knobs.deflate_profile;
    if (prof) { HIPCHK(hipMalloc(&a.prof, (size_t)nch * 128)); HIPCHK(hipMemsetAsync(a.prof, 0, (size_t)nch * 128, s)); }
    a.hist_out = nullptr; a.codes = nullptr; a.chunk_off = nullptr;
    {
        // next generation of resident split-pass workgroups: 2 per CU (1024 threads, <= 75 KB LDS)
        static int ncu = 0;
        if (!ncu && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) ncu = 0;
        a.pf_dist = c->knobs.deflate_pf ? 2u * (uint32_t)ncu : 0u;     // (NDFL_DEFLATE_PF=0: no L2 touch)
    }
    // split pipeline by default (deflate_split.hip); NDFL_DEFLATE_FUSED=1 (or the per-phase profile)
    // selects the one-kernel encoder
    const bool split = !c->knobs.deflate_fused && !prof;
    uint64_t* d_total = nullptr;
    if (split) {
        HIPCHK(c->d_hist.ensure((size_t)nch * HREC * 4));
        HIPCHK(c->d_codes.ensure((size_t)nch * CREC * 4));
        HIPCHK(c->d_off.ensure((size_t)nch * 8 + 64 + (size_t)((nch + SCAN_TILE - 1) / SCAN_TILE) * 8));
        a.hist_out = c->d_hist.as<uint32_t>();
        a.codes = c->d_codes.as<uint32_t>();
        a.chunk_off = c->d_off.as<uint64_t>();
        d_total = c->d_off.as<uint64_t>() + nch;
    }
    a.c0 = 0;
    HIPCHK(hipEventRecord(c->ev0, s));
    if (split) {
        hipLaunchKernelGGL(ndfl_deflate_hist_kernel, dim3(nch), dim3(1024), 0, s, a);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_deflate_codes_kernel, dim3(nch), dim3(64), 0, s, a);
        HIPCHK(hipGetLastError());
        const uint32_t ntile = (nch + SCAN_TILE - 1) / SCAN_TILE;
        uint64_t* d_part = c->d_off.as<uint64_t>() + nch + 8;
        hipLaunchKernelGGL(ndfl_deflate_offsets_sum_kernel, dim3(ntile), dim3(SCAN_T), 0, s, (const uint64_t*)a.status,
                           nch, d_part);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_deflate_offsets_kernel, dim3(ntile), dim3(SCAN_T), 0, s, (const uint64_t*)a.status, nch,
                           (uint64_t)start_bitpos, c->d_off.as<uint64_t>(), d_total, (const uint64_t*)d_part);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(ndfl_deflate_emit_kernel, dim3(nch), dim3(1024), 0, s, a);
    } else {
        hipLaunchKernelGGL(ndfl_deflate_chunks_kernel, dim3(nch), dim3(1024), 0, s, a);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev1, s));
    const uint32_t ne = 2 * nch;
    hipLaunchKernelGGL(ndfl_edge_fixup_kernel, dim3((ne + 255) / 256), dim3(256), 0, s,
                       (const uint64_t*)a.edge_w, (const uint32_t*)a.edge_v, ne, d_out);
    HIPCHK(hipGetLastError());
    if (crc_inout) {
        HIPCHK(launch_crc_combine(c, s, (const uint32_t*)a.crc_raw, nch, chunk_len, len, c->d_crc1.as<uint32_t>()));
        HIPCHK(hipMemcpyAsync(c->h_pinned + 4, c->d_crc1.p, 4, hipMemcpyDeviceToHost, s));
    }
    if (split) HIPCHK(hipMemcpyAsync(c->h_pinned, d_total, 8, hipMemcpyDeviceToHost, s));
    else HIPCHK(hipMemcpyAsync(c->h_pinned, a.status + (nch - 1), 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->last_ms = ms;
    c->deflate_ms = ms;
    if (prof) {
        std::vector<uint64_t> h((size_t)nch * 16);
        HIPCHK(hipMemcpy(h.data(), a.prof, (size_t)nch * 128, hipMemcpyDeviceToHost));
        hipFree(a.prof);
        double sum[7] = {0}, tmin = 1e300, tmax = 0, sub[6] = {0};
        uint64_t nsub = 0;
        for (uint32_t k = 0; k < nch; k++) {
            const uint64_t* q = &h[k * 16];
            for (int p = 0; p < 7; p++) sum[p] += (double)(q[p + 1] - q[p]);
            tmin = std::min(tmin, (double)q[0]); tmax = std::max(tmax, (double)q[7]);
            if (q[8]) {   // codes sub-phases: trim, package-merge pair, canonical, cl RLE, cl PM, cl canon/header
                const uint64_t t[7] = {q[2], q[8], q[9], q[10], q[11], q[12], q[13]};
                for (int p = 0; p < 6; p++) sub[p] += (double)(t[p + 1] - t[p]);
                nsub++;
            }
        }
        if (nsub)
            fprintf(stderr, "[ndfl] deflate codes sub-phases (us/chunk): trim %.2f pm(lit,dist) %.2f canon %.2f cl-rle %.2f "
                    "pm(cl) %.2f canon(cl) %.2f\n", sub[0] / nsub / 100, sub[1] / nsub / 100, sub[2] / nsub / 100,
                    sub[3] / nsub / 100, sub[4] / nsub / 100, sub[5] / nsub / 100);
        // wall_clock64 runs at 100 MHz
        fprintf(stderr, "[ndfl] deflate phases (us/chunk): load+crc %.2f hist %.2f codes %.2f bits+scan %.2f emit %.2f "
                "lookback %.2f store %.2f; span %.2f ms\n", sum[0] / nch / 100, sum[1] / nch / 100, sum[2] / nch / 100,
                sum[3] / nch / 100, sum[4] / nch / 100, sum[5] / nch / 100, sum[6] / nch / 100, (tmax - tmin) / 1e5);
    }
    uint64_t st;
    memcpy(&st, c->h_pinned, 8);
    const uint64_t end_bits = st & ST_VAL;
    *out_end_bits = end_bits;
    const uint64_t nbytes = (end_bits + 7) / 8;
    if (crc_inout) {
        uint32_t raw = c->h_pinned[4];
        uint32_t dc = ~(crc_multmodp(crc_x8n(len), 0xFFFFFFFFu) ^ raw);
        *crc_inout = ndfl_crc32_combine(*crc_inout, dc, len);
    }
    if (!direct) {
        if (nbytes > out_cap) return NDFL_E_CAPACITY;
        HIPCHK(hipMemcpyAsync(out, d_out, nbytes,
                              (flags & NDFL_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return NDFL_OK;
}

// Lz77Huffman(dynamic, minRun, maxRun, minDist, maxDist) over K chunks (D/comp/Lz77Huffman.java:20-130):
// staging copy, then per batch of chunks links -> matches -> parse/encode; edges and CRC at the end.
int ndfl_deflate_chunks_lz77(ndfl_ctx* c, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                             const uint8_t* data, uint64_t len, uint32_t chunk_len, int dynamic, int min_run,
                             int max_run, int min_dist, int max_dist, int final_flag, uint32_t start_bitpos,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_end_bits, uint32_t* crc_inout,
                             uint32_t flags) {
    if (!c || !out_end_bits || (!data && len) || (!hist && hist_len) || !out) return NDFL_E_ARG;
    if (start_bitpos > 7 || hist_limit > 32768 || hist_len > hist_limit || chunk_len == 0) return NDFL_E_ARG;
    if (!final_flag && (len == 0 || len % chunk_len != 0)) return NDFL_E_ARG;
    const bool literal_only = min_run == 0 && max_run == 0 && min_dist == 0 && max_dist == 0;   // (:29-31)
    if (!literal_only && !(3 <= min_run && min_run <= max_run && max_run <= 258 && 1 <= min_dist &&
                           min_dist <= max_dist && max_dist <= 32768))
        return NDFL_E_ARG;                                                                     // (:32-38)
    if (literal_only || (min_run == 3 && max_run == 258 && min_dist == 1 && max_dist == 1))
        return ndfl_deflate_chunks(c, hist, hist_len, hist_limit, data, len, chunk_len,
                                   literal_only ? (dynamic ? NDFL_LITERAL_DYNAMIC : NDFL_LITERAL_STATIC)
                                                : (dynamic ? NDFL_RLE_DYNAMIC : NDFL_RLE_STATIC),
                                   final_flag, start_bitpos, out, out_cap, out_end_bits, crc_inout, flags);
    if (chunk_len > (uint32_t)MAX_CHUNK) return NDFL_E_UNSUPPORTED;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t nch64 = final_flag ? (len == 0 ? 1 : (len + chunk_len - 1) / chunk_len) : len / chunk_len;
    if (nch64 > 0xFFFFFFFFull) return NDFL_E_UNSUPPORTED;
    const uint32_t nch = (uint32_t)nch64;
    hipStream_t s = ordered_stream(c);

    // staging buffer: data at LZ_DS, the history right before it
    const uint64_t total = LZ_DS + len;
    HIPCHK(c->d_lz.ensure(total + 64));
    uint8_t* buf = c->d_lz.as<uint8_t>();
    const hipMemcpyKind kin = (flags & NDFL_IN_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (hist_len) HIPCHK(hipMemcpyAsync(buf + LZ_DS - hist_len, hist, hist_len, kin, s));
    if (len) HIPCHK(hipMemcpyAsync(buf + LZ_DS, data, len, kin, s));
    HIPCHK(hipMemsetAsync(buf + total, 0, 64, s));

    const uint64_t bound = ndfl_deflate_bound(len, chunk_len);
    const uint64_t bound_words = (bound + 3) / 4 + 2;
    uint32_t* d_out;
    bool direct = (flags & NDFL_OUT_DEVICE) && (((uintptr_t)out & 3) == 0) && out_cap >= bound_words * 4;
    if (direct) d_out = (uint32_t*)out;
    else { HIPCHK(c->d_out.ensure(bound_words * 4)); d_out = c->d_out.as<uint32_t>(); }
    HIPCHK(c->d_status.ensure(nch * sizeof(uint64_t)));
    HIPCHK(c->d_ticket.ensure(64));
    HIPCHK(c->d_edge_w.ensure(2ull * nch * sizeof(uint64_t)));
    HIPCHK(c->d_edge_v.ensure(2ull * nch * sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(c->d_status.p, 0, nch * sizeof(uint64_t), s));

    // batches of whole chunks, <= 256 MiB of data each (matches: 4 B per byte, links: 2 B)
    const uint32_t batch_ch = std::max<uint32_t>(1, (uint32_t)((256ull << 20) / chunk_len));
    const uint64_t batch_bytes = std::min<uint64_t>((uint64_t)batch_ch * chunk_len, std::max<uint64_t>(len, 1));
    HIPCHK(c->d_match.ensure(batch_bytes * 4));
    HIPCHK(c->d_link.ensure((batch_bytes + LZ_SEG) * 2));

    LzArgs la;
    la.buf = buf; la.total = total; la.vstart = LZ_DS - hist_len; la.chunk_len = chunk_len;
    la.parent_len = c->parent_len ? c->parent_len : chunk_len;
    la.hist_limit = hist_limit; la.min_run = (uint32_t)min_run; la.max_run = (uint32_t)max_run;
    la.min_dist = (uint32_t)min_dist; la.max_dist = (uint32_t)max_dist;
    la.link = c->d_link.as<uint16_t>(); la.match = c->d_match.as<uint32_t>();
    const bool lz_stats = c->knobs.lz_stats;
    la.stats = nullptr;
    if (lz_stats) {
        HIPCHK(hipMalloc(&la.stats, 128));
        HIPCHK(hipMemsetAsync(la.stats, 0, 128, s));
    }
    LzEncArgs ea;
    ea.match = c->d_match.as<uint32_t>(); ea.n = len; ea.chunk_len = chunk_len; ea.nchunks = nch;
    ea.final_last = final_flag ? 1 : 0; ea.dynamic = dynamic ? 1 : 0; ea.base_bit = start_bitpos;
    ea.out = d_out; ea.status = c->d_status.as<uint64_t>(); ea.ticket = c->d_ticket.as<uint32_t>();
    ea.edge_w = c->d_edge_w.as<uint64_t>(); ea.edge_v = c->d_edge_v.as<uint32_t>();
    ea.chunk_bits = c->cb_out;
    ea.match_rw = c->d_match.as<uint32_t>();
    ea.g.buf = buf; ea.g.total = total; ea.g.vstart = la.vstart; ea.g.chunk_len = chunk_len;
    ea.g.parent_len = la.parent_len; ea.g.hist_limit = hist_limit; ea.g.min_run = la.min_run;
    ea.g.max_run = la.max_run; ea.g.min_dist = la.min_dist; ea.g.max_dist = la.max_dist;
    ea.stats = la.stats;
    // match search: at the positions the greedy parse visits (default), or at every position by hash
    // chains (NDFL_LZ_SEARCH=chain, the round-3 search); NDFL_LZ_LEAD=0 drops the tiles' lead-in (so
    // the encode kernel's fallback search runs at most tile starts: a test of that path)
    const bool chain_search = c->knobs.lz_chain;
    const uint32_t lead_on = c->knobs.lz_lead == 0 ? 0u : 1u;

    HIPCHK(hipEventRecord(c->ev0, s));
    for (uint32_t cb = 0; cb < nch; cb += batch_ch) {
        const uint32_t ce = std::min(nch, cb + batch_ch);
        const uint64_t x0 = (uint64_t)cb * chunk_len, x1 = std::min<uint64_t>((uint64_t)ce * chunk_len, len);
        const uint64_t P0 = LZ_DS + x0, P1 = LZ_DS + x1;
        if (P1 > P0 && !chain_search) {
            la.L0 = P0; la.p_begin = P0; la.p_end = P1;
            hipLaunchKernelGGL(ndfl_lz_parse_match_kernel, dim3((uint32_t)((P1 - P0 + LZP_TILE - 1) / LZP_TILE)), dim3(1024),
                               0, s, la, lead_on);
            HIPCHK(hipGetLastError());
        } else if (P1 > P0) {
            const uint64_t L0 = std::max<uint64_t>(la.vstart, P0 - LZ_SEG);
            hipLaunchKernelGGL(ndfl_lz_links_kernel, dim3((uint32_t)((P1 - L0 + LZ_SEG - 1) / LZ_SEG)), dim3(1024), 0, s,
                               (const uint8_t*)buf, total, la.vstart, L0, P1, c->d_link.as<uint16_t>());
            HIPCHK(hipGetLastError());
            la.L0 = L0; la.p_begin = P0; la.p_end = P1;
            hipLaunchKernelGGL(ndfl_lz_match_kernel, dim3((uint32_t)((P1 - P0 + LZ_TILE - 1) / LZ_TILE)), dim3(1024), 0, s, la);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemsetAsync(c->d_ticket.p, 0, 64, s));
        ea.batch_x0 = x0; ea.chunk_base = cb; ea.nchunks_batch = ce - cb;
        hipLaunchKernelGGL(ndfl_lz_encode_kernel, dim3(ce - cb), dim3(1024), 0, s, ea);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(c->ev1, s));
    if (la.stats) {
        unsigned long long st[16];
        HIPCHK(hipMemcpyAsync(st, la.stats, 128, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        hipFree(la.stats);
        if (chain_search)
            fprintf(stderr, "[ndfl] lz match: %llu searched positions, %.2f hops/pos, %.2f trigram hits/pos, %.2f compare words/pos\n",
                    st[0], (double)st[1] / std::max(1ull, st[0]), (double)st[2] / std::max(1ull, st[0]),
                    (double)st[3] / std::max(1ull, st[0]));
        else
            fprintf(stderr, "[ndfl] lz parse-driven match: %llu searches for %llu positions (%.2f %%), %.2f bucket entries per search, "
                    "%llu fallback searches in the encode kernel\n",
                    st[0], (unsigned long long)len, 100.0 * (double)st[0] / std::max<double>(1.0, (double)len),
                    (double)st[1] / std::max(1ull, st[0]), st[2]);
        if (!chain_search)
            fprintf(stderr, "[ndfl] lz parse-driven tiles %llu: stage+sort %.1f us, paths %.1f us, entries %.1f us per tile\n",
                    st[6], st[3] / 100.0 / std::max(1ull, st[6]), st[4] / 100.0 / std::max(1ull, st[6]),
                    st[5] / 100.0 / std::max(1ull, st[6]));
        {
            const double k = 100.0 * (double)std::max(1ull, st[13]);
            fprintf(stderr, "[ndfl] lz encode chunks %llu: fill+parse %.1f us (walks %.1f, true entries %.1f), histograms %.1f us, "
                    "codes %.1f us, token bits %.1f us, look-back+store %.1f us per chunk\n", st[13], st[8] / k, st[14] / k,
                    st[15] / k, st[9] / k, st[10] / k, st[11] / k, st[12] / k);
        }
    }
    const uint32_t ne = 2 * nch;
    hipLaunchKernelGGL(ndfl_edge_fixup_kernel, dim3((ne + 255) / 256), dim3(256), 0, s,
                       (const uint64_t*)ea.edge_w, (const uint32_t*)ea.edge_v, ne, d_out);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->h_pinned, ea.status + (nch - 1), 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->last_ms = ms;
    c->deflate_ms = ms;
    uint64_t st;
    memcpy(&st, c->h_pinned, 8);
    const uint64_t end_bits = st & ST_VAL;
    *out_end_bits = end_bits;
    const uint64_t nbytes = (end_bits + 7) / 8;
    if (crc_inout && len) {
        uint32_t cr = *crc_inout;
        int rc = ndfl_crc32(c, &cr, buf + LZ_DS, len, NDFL_IN_DEVICE);
        if (rc) return rc;
        *crc_inout = cr;
        c->last_ms = ms;
    }
    if (!direct) {
        if (nbytes > out_cap) return NDFL_E_CAPACITY;
        HIPCHK(hipMemcpyAsync(out, d_out, nbytes,
                              (flags & NDFL_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return NDFL_OK;
}

// MultiStrategy over Lz77Huffman / Uncompressed substrategies (D/comp/MultiStrategy.java:31-57,
// D/comp/Uncompressed.java:19-51): every Lz77Huffman substrategy encodes all chunks into its own
// stream; the host walks the chunks with the bit position mod 8 and keeps, per chunk, the first
// substrategy with the fewest bits at that position; ndfl_assemble_kernel writes the result.
int ndfl_deflate_chunks_multi(ndfl_ctx* c, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                              const uint8_t* data, uint64_t len, uint32_t chunk_len, const ndfl_strategy_desc* strats,
                              uint32_t n_strats, int final_flag, uint32_t start_bitpos, uint8_t* out, uint64_t out_cap,
                              uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags) {
    if (!c || !out_end_bits || (!data && len) || (!hist && hist_len) || !out || !strats) return NDFL_E_ARG;
    if (n_strats == 0 || n_strats > 8) return n_strats == 0 ? NDFL_E_ARG : NDFL_E_UNSUPPORTED;
    if (start_bitpos > 7 || hist_limit > 32768 || hist_len > hist_limit || chunk_len == 0) return NDFL_E_ARG;
    if (!final_flag && (len == 0 || len % chunk_len != 0)) return NDFL_E_ARG;
    if (chunk_len > (uint32_t)MAX_CHUNK) return NDFL_E_UNSUPPORTED;
    for (uint32_t k = 0; k < n_strats; k++) {
        const ndfl_strategy_desc& d = strats[k];
        if (d.kind == NDFL_KIND_UNCOMPRESSED) continue;
        if (d.kind != NDFL_KIND_LZ77) return NDFL_E_ARG;
        const bool lit = d.min_run == 0 && d.max_run == 0 && d.min_dist == 0 && d.max_dist == 0;
        if (!lit && !(3 <= d.min_run && d.min_run <= d.max_run && d.max_run <= 258 && 1 <= d.min_dist &&
                      d.min_dist <= d.max_dist && d.max_dist <= 32768))
            return NDFL_E_ARG;
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = ordered_stream(c);
    const uint64_t nch64 = final_flag ? (len == 0 ? 1 : (len + chunk_len - 1) / chunk_len) : len / chunk_len;
    if (nch64 > 0xFFFFFFFFull) return NDFL_E_UNSUPPORTED;
    const uint32_t nch = (uint32_t)nch64;
    // device copies of the inputs (the substrategy calls below take device pointers)
    const uint8_t* d_data = data;
    const uint8_t* d_hist = hist;
    if (!(flags & NDFL_IN_DEVICE)) {
        HIPCHK(c->d_mdata.ensure(len + hist_len + 16));
        if (hist_len) HIPCHK(hipMemcpyAsync(c->d_mdata.p, hist, hist_len, hipMemcpyHostToDevice, s));
        if (len) HIPCHK(hipMemcpyAsync(c->d_mdata.as<uint8_t>() + hist_len, data, len, hipMemcpyHostToDevice, s));
        d_hist = c->d_mdata.as<uint8_t>();
        d_data = d_hist + hist_len;
    }
    const uint64_t bound = ndfl_deflate_bound(len, chunk_len);
    const uint64_t bound_words = (bound + 3) / 4 + 2;
    std::vector<std::vector<uint64_t>> bits(n_strats);
    std::vector<const uint32_t*> streams(n_strats, nullptr);
    for (uint32_t k = 0; k < n_strats; k++) {
        const ndfl_strategy_desc& d = strats[k];
        if (d.kind == NDFL_KIND_UNCOMPRESSED) continue;
        HIPCHK(c->d_mstreams[k].ensure(bound_words * 4 + 64));
        HIPCHK(c->d_mbits[k].ensure(nch * 8ull));
        c->cb_out = c->d_mbits[k].as<uint64_t>();
        uint64_t eb = 0;
        const int rc = ndfl_deflate_chunks_lz77(c, d_hist, hist_len, hist_limit, d_data, len, chunk_len, d.dynamic,
                                                d.min_run, d.max_run, d.min_dist, d.max_dist, final_flag, 0,
                                                c->d_mstreams[k].as<uint8_t>(), bound_words * 4 + 64, &eb, nullptr,
                                                NDFL_IN_DEVICE | NDFL_OUT_DEVICE);
        c->cb_out = nullptr;
        if (rc) return rc;
        bits[k].resize(nch);
        HIPCHK(hipMemcpyAsync(bits[k].data(), c->d_mbits[k].p, nch * 8ull, hipMemcpyDeviceToHost, s));
        streams[k] = c->d_mstreams[k].as<uint32_t>();
    }
    HIPCHK(hipStreamSynchronize(s));
    // choose (D/comp/MultiStrategy.java:35-44: strictly fewer bits wins, so ties keep the earlier one)
    std::vector<uint8_t> choice(nch);
    std::vector<uint64_t> src_bit(nch), dst_bit(nch), nb(nch), soff(n_strats, 0);
    uint64_t pos = start_bitpos;
    for (uint32_t ci = 0; ci < nch; ci++) {
        const uint64_t cl = std::min<uint64_t>(chunk_len, len - (uint64_t)ci * chunk_len);
        const uint32_t p8 = (uint32_t)(pos & 7);
        uint64_t best = UINT64_MAX;
        uint32_t bk = 0;
        for (uint32_t k = 0; k < n_strats; k++) {
            uint64_t b;
            if (strats[k].kind == NDFL_KIND_UNCOMPRESSED) {
                const uint64_t nblk = std::max<uint64_t>((cl + 65534) / 65535, 1);   // (:23-25)
                b = cl * 8 + nblk * 40 + (uint64_t)((int)((13 - p8) % 8) - 5);
            } else {
                b = bits[k][ci];
            }
            if (b < best) { best = b; bk = k; }
        }
        choice[ci] = (uint8_t)bk;
        dst_bit[ci] = pos;
        nb[ci] = best;
        for (uint32_t k = 0; k < n_strats; k++)
            if (strats[k].kind != NDFL_KIND_UNCOMPRESSED) {
                if (k == bk) src_bit[ci] = soff[k];
                soff[k] += bits[k][ci];
            }
        pos += best;
    }
    const uint64_t end_bits = pos;
    const uint64_t need_words = (end_bits + 31) / 32 + 2;
    uint32_t* d_out;
    const bool direct = (flags & NDFL_OUT_DEVICE) && (((uintptr_t)out & 3) == 0) && out_cap >= need_words * 4;
    if (direct) d_out = (uint32_t*)out;
    else { HIPCHK(c->d_out.ensure(need_words * 4)); d_out = c->d_out.as<uint32_t>(); }
    HIPCHK(hipMemsetAsync(d_out, 0, need_words * 4, s));
    // per-chunk tables + stream pointers in one device block
    const size_t tb = nch * (3 * 8ull) + nch + 8 * n_strats + 64;
    HIPCHK(c->d_masm.ensure(tb));
    char* base = (char*)c->d_masm.p;
    uint64_t* d_src = (uint64_t*)base;
    uint64_t* d_dst = d_src + nch;
    uint64_t* d_nb = d_dst + nch;
    const uint32_t** d_streams = (const uint32_t**)(d_nb + nch);
    uint8_t* d_choice = (uint8_t*)(d_streams + n_strats);
    std::vector<char> host(tb);
    memcpy(host.data(), src_bit.data(), nch * 8ull);
    memcpy(host.data() + nch * 8ull, dst_bit.data(), nch * 8ull);
    memcpy(host.data() + nch * 16ull, nb.data(), nch * 8ull);
    memcpy(host.data() + nch * 24ull, streams.data(), 8ull * n_strats);
    memcpy(host.data() + nch * 24ull + 8ull * n_strats, choice.data(), nch);
    HIPCHK(hipMemcpyAsync(base, host.data(), tb, hipMemcpyHostToDevice, s));
    AsmArgs aa;
    aa.streams = d_streams; aa.data = d_data; aa.n = len; aa.chunk_len = chunk_len; aa.nchunks = nch;
    aa.final_last = final_flag ? 1 : 0; aa.choice = d_choice; aa.src_bit = d_src; aa.dst_bit = d_dst; aa.nbits = d_nb;
    aa.setfin = nullptr; aa.per_entry_stream = 0; aa.out = d_out;
    HIPCHK(hipEventRecord(c->ev0, s));
    hipLaunchKernelGGL(ndfl_assemble_kernel, dim3(nch), dim3(256), 0, s, aa);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev1, s));
    HIPCHK(hipStreamSynchronize(s));
    *out_end_bits = end_bits;
    if (crc_inout && len) {
        uint32_t cr = *crc_inout;
        const int rc = ndfl_crc32(c, &cr, d_data, len, NDFL_IN_DEVICE);
        if (rc) return rc;
        *crc_inout = cr;
    }
    const uint64_t nbytes = (end_bits + 7) / 8;
    if (!direct) {
        if (nbytes > out_cap) return NDFL_E_CAPACITY;
        HIPCHK(hipMemcpyAsync(out, d_out, nbytes,
                              (flags & NDFL_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return NDFL_OK;
}

// BinarySplit(sub, minBlockLen) over an Lz77Huffman substrategy (D/comp/BinarySplit.java:21-82):
// each chunk is halved recursively while both halves are longer than minBlockLen, and a split is
// kept when the halves' decisions take fewer bits.  Every halving level of the full chunks is
// encoded by one call (block length L/2^k, history from the parent chunk -- the sub-decide keeps
// `off`, :44-45), a partial final chunk node by node; the host runs the reference's recursion on
// the bit counts and ndfl_assemble_kernel copies the chosen blocks (bfinal set on the last one).
int ndfl_deflate_chunks_binsplit(ndfl_ctx* c, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                                 const uint8_t* data, uint64_t len, uint32_t chunk_len, const ndfl_strategy_desc* sub,
                                 int32_t min_block_len, int final_flag, uint32_t start_bitpos, uint8_t* out,
                                 uint64_t out_cap, uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags) {
    if (!c || !out_end_bits || (!data && len) || (!hist && hist_len) || !out || !sub) return NDFL_E_ARG;
    if (min_block_len < 1) return NDFL_E_ARG;                                      // (:23-24)
    if (start_bitpos > 7 || hist_limit > 32768 || hist_len > hist_limit || chunk_len == 0) return NDFL_E_ARG;
    if (!final_flag && (len == 0 || len % chunk_len != 0)) return NDFL_E_ARG;
    if (chunk_len > (uint32_t)MAX_CHUNK) return NDFL_E_UNSUPPORTED;
    if (sub->kind != NDFL_KIND_LZ77) return NDFL_E_UNSUPPORTED;     // position-independent substrategies only
    {
        const ndfl_strategy_desc& d = *sub;
        const bool lit = d.min_run == 0 && d.max_run == 0 && d.min_dist == 0 && d.max_dist == 0;
        if (!lit && !(3 <= d.min_run && d.min_run <= d.max_run && d.max_run <= 258 && 1 <= d.min_dist &&
                      d.min_dist <= d.max_dist && d.max_dist <= 32768))
            return NDFL_E_ARG;
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = ordered_stream(c);
    const uint32_t M = (uint32_t)min_block_len;
    // device copy [hist | data]
    HIPCHK(c->d_mdata.ensure(len + hist_len + 16));
    const hipMemcpyKind kin = (flags & NDFL_IN_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (hist_len) HIPCHK(hipMemcpyAsync(c->d_mdata.p, hist, hist_len, kin, s));
    if (len) HIPCHK(hipMemcpyAsync(c->d_mdata.as<uint8_t>() + hist_len, data, len, kin, s));
    const uint8_t* base = c->d_mdata.as<uint8_t>();            // base[hist_len + x] = data[x]
    // uniform halving levels of a full chunk
    std::vector<uint32_t> lv{chunk_len};
    while (true) {
        const uint32_t sz = lv.back();
        if (!(sz / 2 > M)) break;                               // min((n+1)/2, n/2) > minBlockLen (:41-42)
        if (sz & 1) return NDFL_E_UNSUPPORTED;                  // uneven halves: not on the GPU path
        lv.push_back(sz / 2);
    }
    const uint32_t nlev = (uint32_t)lv.size();
    if (nlev > 16) return NDFL_E_UNSUPPORTED;
    const bool partial = final_flag && (len == 0 || len % chunk_len != 0);
    const uint64_t nfull = len / chunk_len;
    const uint64_t bound = ndfl_deflate_bound(len, chunk_len) + 64;
    const uint64_t need_words = (bound + 3) / 4 + 4;
    uint32_t* d_out;
    const bool direct = (flags & NDFL_OUT_DEVICE) && (((uintptr_t)out & 3) == 0) && out_cap >= need_words * 4;
    if (direct) d_out = (uint32_t*)out;
    else { HIPCHK(c->d_out.ensure(need_words * 4)); d_out = c->d_out.as<uint32_t>(); }
    HIPCHK(hipMemsetAsync(d_out, 0, need_words * 4, s));

    // encode data [a, a + n) as blocks of `blk` into dst (device), block bits to `bits`.  `level`:
    // a is a chunk boundary and the blocks' history starts at their chunk's (parent_len = chunk_len);
    // otherwise one block whose history is that of the partial chunk starting at `pstart`
    auto encode = [&](uint64_t a, uint64_t n, uint32_t blk, bool level, uint64_t pstart, bool fin, uint8_t* dst,
                      uint64_t cap, uint64_t* d_bits, std::vector<uint64_t>& bits) -> int {
        uint64_t hl, hlim;
        if (level) {
            hl = std::min<uint64_t>(hist_limit, hist_len + a);
            hlim = hist_limit;
            c->parent_len = chunk_len;
        } else {
            const uint64_t off = hist_len + pstart - std::min<uint64_t>(hist_limit, hist_len + pstart);   // in base
            hl = std::min<uint64_t>(32768, hist_len + a - off);
            hlim = hl;
            c->parent_len = 0;
        }
        c->cb_out = d_bits;
        uint64_t eb = 0;
        const int rc = ndfl_deflate_chunks_lz77(c, base + hist_len + a - hl, (uint32_t)hl, (uint32_t)hlim,
                                                base + hist_len + a, n, blk, sub->dynamic, sub->min_run,
                                                sub->max_run, sub->min_dist, sub->max_dist, fin ? 1 : 0, 0, dst, cap,
                                                &eb, nullptr, NDFL_IN_DEVICE | NDFL_OUT_DEVICE);
        c->cb_out = nullptr;
        c->parent_len = 0;
        if (rc) return rc;
        const uint64_t nb = n ? n / blk : 1;
        bits.resize(nb);
        HIPCHK(hipMemcpyAsync(bits.data(), d_bits, nb * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return 0;
    };
    struct Ent { const uint32_t* st; uint64_t src, nb; uint8_t fin; };
    uint64_t pos = start_bitpos;
    // write a group of entries at pos (one assemble launch)
    auto assemble = [&](std::vector<Ent>& ents) -> int {
        const uint32_t ne = (uint32_t)ents.size();
        if (ne == 0) return 0;
        std::vector<uint64_t> src(ne), dst(ne), nb(ne);
        std::vector<const uint32_t*> st(ne);
        std::vector<uint8_t> fin(ne), ch(ne);
        for (uint32_t k = 0; k < ne; k++) {
            src[k] = ents[k].src; dst[k] = pos; nb[k] = ents[k].nb; st[k] = ents[k].st; fin[k] = ents[k].fin;
            ch[k] = 0;
            pos += ents[k].nb;
        }
        // per-entry stream pointers: one "substrategy" per entry (choice = 0 and streams + k)
        const size_t tb = ne * 32ull + 2 * ne + 64;
        HIPCHK(c->d_masm.ensure(tb));
        char* bp = (char*)c->d_masm.p;
        std::vector<char> host(tb);
        memcpy(host.data(), src.data(), ne * 8ull);
        memcpy(host.data() + ne * 8ull, dst.data(), ne * 8ull);
        memcpy(host.data() + ne * 16ull, nb.data(), ne * 8ull);
        memcpy(host.data() + ne * 24ull, st.data(), ne * 8ull);
        memcpy(host.data() + ne * 32ull, fin.data(), ne);
        memcpy(host.data() + ne * 32ull + ne, ch.data(), ne);
        HIPCHK(hipMemcpyAsync(bp, host.data(), tb, hipMemcpyHostToDevice, s));
        AsmArgs aa;
        aa.data = nullptr; aa.n = 0; aa.chunk_len = 1; aa.nchunks = ne; aa.final_last = 0;
        aa.src_bit = (const uint64_t*)bp; aa.dst_bit = (const uint64_t*)(bp + ne * 8ull);
        aa.nbits = (const uint64_t*)(bp + ne * 16ull); aa.streams = (const uint32_t* const*)(bp + ne * 24ull);
        aa.setfin = (const uint8_t*)(bp + ne * 32ull); aa.choice = (const uint8_t*)(bp + ne * 32ull + ne);
        aa.per_entry_stream = 1;
        aa.out = d_out;
        hipLaunchKernelGGL(ndfl_assemble_kernel, dim3(ne), dim3(256), 0, s, aa);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(s));
        return 0;
    };
    // recursion of BinarySplit.decide (:33-66) on bit counts (position-independent substrategy)
    std::vector<std::vector<uint64_t>> lb(nlev);
    std::function<uint64_t(uint32_t, uint64_t, std::vector<std::pair<uint32_t, uint64_t>>&)> decide_lv =
        [&](uint32_t k, uint64_t idx, std::vector<std::pair<uint32_t, uint64_t>>& leaves) -> uint64_t {
            const uint64_t cur = lb[k][idx];
            if (k + 1 < nlev) {
                const uint64_t d0 = lb[k + 1][2 * idx], d1 = lb[k + 1][2 * idx + 1];
                if (d0 + d1 < cur) {                            // improved: recurse into both halves
                    std::vector<std::pair<uint32_t, uint64_t>> l2;
                    const uint64_t t = decide_lv(k + 1, 2 * idx, l2) + decide_lv(k + 1, 2 * idx + 1, l2);
                    if (t < cur) { leaves.insert(leaves.end(), l2.begin(), l2.end()); return t; }
                }
            }
            leaves.push_back({k, idx});
            return cur;
        };
    const uint32_t BCH = std::max<uint32_t>(1, (uint32_t)((64ull << 20) / chunk_len));
    const bool last_is_full = !partial;
    for (uint64_t cb = 0; cb < nfull; cb += BCH) {
        const uint64_t ce = std::min<uint64_t>(nfull, cb + BCH);
        const uint64_t a = cb * chunk_len, n = (ce - cb) * chunk_len;
        std::vector<uint64_t> soff[16];
        for (uint32_t k = 0; k < nlev; k++) {
            const uint64_t capk = (ndfl_deflate_bound(n, lv[k]) + 3) / 4 * 4 + 64;
            HIPCHK(c->d_mstreams[k].ensure(capk));
            HIPCHK(c->d_mbits[k].ensure((n / lv[k]) * 8 + 64));
            const int rc = encode(a, n, lv[k], true, 0, false, c->d_mstreams[k].as<uint8_t>(), capk,
                                  c->d_mbits[k].as<uint64_t>(), lb[k]);
            if (rc) return rc;
            soff[k].resize(lb[k].size() + 1);
            soff[k][0] = 0;
            for (size_t q = 0; q < lb[k].size(); q++) soff[k][q + 1] = soff[k][q] + lb[k][q];
        }
        std::vector<Ent> ents;
        for (uint64_t j = 0; j < ce - cb; j++) {
            std::vector<std::pair<uint32_t, uint64_t>> leaves;
            decide_lv(0, j, leaves);
            for (auto& lf : leaves)
                ents.push_back({c->d_mstreams[lf.first].as<uint32_t>(), soff[lf.first][lf.second], lb[lf.first][lf.second], 0});
        }
        if (ce == nfull && last_is_full && final_flag && !ents.empty()) ents.back().fin = 1;
        const int rc = assemble(ents);
        if (rc) return rc;
    }
    if (partial) {
        const uint64_t P = nfull * chunk_len, lp = len - P;
        std::vector<DevBuf> bufs;
        int nenc = 0, err = 0;
        std::vector<uint64_t> tmpbits;
        HIPCHK(c->d_mbits[0].ensure(64));
        // node [a, a+n): bits and the buffer holding its block (encoded once, kept for assembly)
        std::map<std::pair<uint64_t, uint64_t>, std::pair<size_t, uint64_t>> memo;
        auto node = [&](uint64_t a2, uint64_t n2) -> std::pair<size_t, uint64_t> {
            auto it = memo.find({a2, n2});
            if (it != memo.end()) return it->second;
            if (++nenc > 8192) { err = NDFL_E_UNSUPPORTED; return {0, 0}; }
            bufs.emplace_back();
            const uint64_t capn = (ndfl_deflate_bound(n2, (uint32_t)std::max<uint64_t>(n2, 1)) + 3) / 4 * 4 + 64;
            if (bufs.back().ensure(capn) != hipSuccess) { err = NDFL_E_DEVICE; return {0, 0}; }
            const int rc = encode(P + (a2 - P), n2, (uint32_t)std::max<uint64_t>(n2, 1), false, P, n2 == 0,
                                  bufs.back().as<uint8_t>(), capn, c->d_mbits[0].as<uint64_t>(), tmpbits);
            if (rc) { err = rc; return {0, 0}; }
            auto r = std::make_pair(bufs.size() - 1, tmpbits[0]);
            memo[{a2, n2}] = r;
            return r;
        };
        std::vector<std::pair<uint64_t, uint64_t>> leaves;     // (a, n)
        std::function<uint64_t(uint64_t, uint64_t, std::vector<std::pair<uint64_t, uint64_t>>&)> decide_node =
            [&](uint64_t a2, uint64_t n2, std::vector<std::pair<uint64_t, uint64_t>>& out_l) -> uint64_t {
                const uint64_t cur = node(a2, n2).second;
                const uint64_t h1 = (n2 + 1) / 2, h2 = n2 - h1;
                if (!err && std::min(h1, h2) > M) {
                    const uint64_t d0 = node(a2, h1).second, d1 = node(a2 + h1, h2).second;
                    if (!err && d0 + d1 < cur) {
                        std::vector<std::pair<uint64_t, uint64_t>> l2;
                        const uint64_t t = decide_node(a2, h1, l2) + decide_node(a2 + h1, h2, l2);
                        if (t < cur) { out_l.insert(out_l.end(), l2.begin(), l2.end()); return t; }
                    }
                }
                out_l.push_back({a2, n2});
                return cur;
            };
        decide_node(P, lp, leaves);
        if (err) return err;
        std::vector<Ent> ents;
        for (auto& lf : leaves) {
            auto nd = memo[lf];
            ents.push_back({bufs[nd.first].as<uint32_t>(), 0, nd.second, 0});
        }
        if (!ents.empty() && lp > 0) ents.back().fin = 1;     // (an empty final block was encoded final)
        const int rc = assemble(ents);
        if (rc) return rc;
    }
    const uint64_t end_bits = pos;
    *out_end_bits = end_bits;
    if (crc_inout && len) {
        uint32_t cr = *crc_inout;
        const int rc = ndfl_crc32(c, &cr, base + hist_len, len, NDFL_IN_DEVICE);
        if (rc) return rc;
        *crc_inout = cr;
    }
    const uint64_t nbytes = (end_bits + 7) / 8;
    if (!direct) {
        if (nbytes > out_cap) return NDFL_E_CAPACITY;
        HIPCHK(hipMemcpyAsync(out, d_out, nbytes,
                              (flags & NDFL_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return NDFL_OK;
}

int ndfl_crc32(ndfl_ctx* c, uint32_t* crc_inout, const uint8_t* data, uint64_t len, uint32_t flags) {
    if (!c || !crc_inout || (!data && len)) return NDFL_E_ARG;
    if (len == 0) return NDFL_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = ordered_stream(c);
    const uint8_t* d = data;
    if (!(flags & NDFL_IN_DEVICE)) {
        HIPCHK(c->d_in.ensure(len));
        HIPCHK(hipMemcpyAsync(c->d_in.p, data, len, hipMemcpyHostToDevice, s));
        d = c->d_in.as<uint8_t>();
    }
    const uint64_t nseg = (len + 65535) / 65536;
    HIPCHK(c->d_crc.ensure(nseg * 4));
    HIPCHK(c->d_crc1.ensure(64));
    HIPCHK(hipEventRecord(c->ev0, s));
    hipLaunchKernelGGL(ndfl_crc_segments_kernel, dim3((uint32_t)nseg), dim3(1024), 0, s, d, len,
                       (const uint32_t*)c->d_tabs.as<uint32_t>(), (const uint32_t*)(c->d_tabs.as<uint32_t>() + 1024),
                       c->d_crc.as<uint32_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev1, s));
    HIPCHK(launch_crc_combine(c, s, (const uint32_t*)c->d_crc.as<uint32_t>(), (uint32_t)nseg, 65536u, len,
                              c->d_crc1.as<uint32_t>()));
    HIPCHK(hipMemcpyAsync(c->h_pinned, c->d_crc1.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->last_ms = ms;
    uint32_t raw = c->h_pinned[0];
    uint32_t dc = ~(crc_multmodp(crc_x8n(len), 0xFFFFFFFFu) ^ raw);
    *crc_inout = ndfl_crc32_combine(*crc_inout, dc, len);
    return NDFL_OK;
}

int ndfl_adler32(ndfl_ctx* c, uint32_t* adler_inout, const uint8_t* data, uint64_t len, uint32_t flags) {
    if (!c || !adler_inout || (!data && len)) return NDFL_E_ARG;
    if (len == 0) return NDFL_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = ordered_stream(c);
    const uint8_t* d = data;
    if (!(flags & NDFL_IN_DEVICE)) {
        HIPCHK(c->d_in.ensure(len));
        HIPCHK(hipMemcpyAsync(c->d_in.p, data, len, hipMemcpyHostToDevice, s));
        d = c->d_in.as<uint8_t>();
    }
    const uint64_t nseg = (len + 65535) / 65536;
    HIPCHK(c->d_crc.ensure(nseg * 8));
    HIPCHK(hipEventRecord(c->ev0, s));
    hipLaunchKernelGGL(ndfl_adler_segments_kernel, dim3((uint32_t)nseg), dim3(1024), 0, s, d, len, c->d_crc.as<uint32_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev1, s));
    std::vector<uint32_t> st(nseg * 2);
    HIPCHK(hipMemcpyAsync(st.data(), c->d_crc.p, nseg * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->last_ms = ms;
    uint64_t a = *adler_inout & 0xFFFF, b = *adler_inout >> 16;
    for (uint64_t k = 0; k < nseg; k++) {
        const uint64_t sl = std::min<uint64_t>(65536, len - k * 65536);
        b = (b + sl % 65521 * a + st[2 * k + 1]) % 65521;
        a = (a + st[2 * k]) % 65521;
    }
    *adler_inout = (uint32_t)(b << 16 | a);
    return NDFL_OK;
}

// A decode's Reason as it leaves the library: the decoder reports the second reserved symbol of each
// alphabet (length 287, distance 31) with an internal code; both become the reference's Reason, and
// the symbol -- which the reference puts in its message, "Reserved run length symbol: " + sym
// (D/decomp/Open.java:516, 659) and "Reserved distance symbol: " + sym (:550, 674) -- is kept for
// ndfl_ctx_error_symbol.
static int public_reason(ndfl_ctx* c, int r) {
    c->err_sym = -1;
    switch (r) {
        case inf::R_RESERVED_LEN: c->err_sym = 286; break;
        case inf::R_RESERVED_LEN_HI: c->err_sym = 287; r = inf::R_RESERVED_LEN; break;
        case inf::R_RESERVED_DIST: c->err_sym = 30; break;
        case inf::R_RESERVED_DIST_HI: c->err_sym = 31; r = inf::R_RESERVED_DIST; break;
        case inf::R_INTERNAL: r = NDFL_E_INTERNAL; break;   // (a failed consistency check, not the data)
        default: break;
    }
    return r;
}

int ndfl_ctx_error_symbol(ndfl_ctx* c) { return c ? c->err_sym : -1; }

int ndfl_inflate(ndfl_ctx* c, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
                 uint64_t* out_len, uint64_t* consumed_bits, uint32_t flags) {
    if (!c || !out_len || !consumed_bits || (!in && in_len)) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    return public_reason(c, inflate_run(c->inf, ordered_stream(c), in, in_len, 0, inf::NONE, out, 0, out_cap, out_len,
                                        consumed_bits, flags, false, &c->last_ms));
}

int ndfl_inflate_range(ndfl_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t start_bit, uint64_t end_bit,
                       uint8_t* out, uint64_t dict_len, uint64_t out_cap, uint64_t* out_len, uint64_t* consumed_bits,
                       uint32_t flags) {
    if (!c || !out_len || !consumed_bits || (!in && in_len) || (!out && (dict_len || out_cap))) return NDFL_E_ARG;
    if (dict_len > 32768 || start_bit > in_len * 8 || end_bit <= start_bit) return NDFL_E_ARG;
    const bool deferred = (flags & NDFL_DICT_DEFERRED) != 0;
    const bool partial = (flags & NDFL_IN_PARTIAL) != 0;
    if (deferred && !(flags & NDFL_OUT_DEVICE)) return NDFL_E_ARG;
    if (partial && (deferred || end_bit != UINT64_MAX)) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    return public_reason(c, inflate_run(c->inf, ordered_stream(c), in, in_len, start_bit, end_bit, out, dict_len,
                                        out_cap, out_len, consumed_bits, flags, deferred, &c->last_ms, partial));
}

int ndfl_inflate_sync(ndfl_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t from_bit, uint64_t window_bits,
                      uint64_t* sync_bit, uint32_t flags) {
    if (!c || !sync_bit || (!in && in_len) || from_bit > in_len * 8) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    return inflate_sync(c->inf, ordered_stream(c), in, in_len, from_bit, window_bits, flags, sync_bit, &c->last_ms);
}

int ndfl_inflate_headers(ndfl_ctx* c, const uint8_t* in, uint64_t in_len, uint32_t flags, uint64_t* headers,
                         uint64_t cap, uint64_t* n_headers, uint64_t* survivors, uint64_t surv_cap, uint64_t* stats) {
    if (!c || !n_headers || (!in && in_len) || (!headers && cap) || (!survivors && surv_cap)) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    const int r = inflate_headers(c->inf, ordered_stream(c), in, in_len, flags, headers, cap, n_headers, survivors,
                                  surv_cap, stats);
    return r == -4 ? NDFL_E_DEVICE : r < 0 ? NDFL_E_INTERNAL : r;
}

int ndfl_inflate_resolve(ndfl_ctx* c, uint64_t* n_reemitted) {
    if (!c || !n_reemitted) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    return inflate_resolve(c->inf, ordered_stream(c), n_reemitted);
}

int ndfl_inflate_tail(ndfl_ctx* c, uint64_t tail_len, uint8_t* dst) {
    if (!c || (!dst && tail_len)) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    const int r = inflate_tail(c->inf, ordered_stream(c), tail_len, dst);
    return r == -5 ? NDFL_E_STATE : r == -6 ? NDFL_E_UNSUPPORTED : r == -1 ? NDFL_E_ARG : r;
}

int ndfl_inflate_tail_map(ndfl_ctx* c, uint64_t tail_len, uint32_t* dst) {
    if (!c || (!dst && tail_len)) return NDFL_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    const int r = inflate_tail_map(c->inf, ordered_stream(c), tail_len, dst);
    return r == -5 ? NDFL_E_STATE : r == -6 ? NDFL_E_UNSUPPORTED : r == -1 ? NDFL_E_ARG : r;
}

int ndfl_bits_shift(ndfl_ctx* c, const uint8_t* in, uint64_t nbits, uint32_t shift, uint8_t* out, uint64_t out_cap,
                    uint32_t flags) {
    if (!c || (!in && nbits) || !out || shift > 7) return NDFL_E_ARG;
    if ((flags & (NDFL_IN_DEVICE | NDFL_OUT_DEVICE)) != (NDFL_IN_DEVICE | NDFL_OUT_DEVICE)) return NDFL_E_ARG;
    const uint64_t nout = (nbits + shift + 7) / 8;
    if (nout > out_cap) return NDFL_E_CAPACITY;
    const uint64_t nin = (nbits + 7) / 8;
    if (nout && in < out + nout && out < in + nin) return NDFL_E_ARG;     // no in-place shifting
    if (nout == 0) return NDFL_OK;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t nthr = (nout + 3) / 4;
    hipLaunchKernelGGL(ndfl_bits_shift_kernel, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, ordered_stream(c), in,
                       nbits, shift, out, nout);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return NDFL_OK;
}

}  // extern "C"

#include "ndfl_plugin.cpp"
