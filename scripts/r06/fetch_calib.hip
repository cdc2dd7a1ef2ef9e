// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the load and
// store shapes the ndfl kernels use (measurement tooling, not product code).  Each kernel moves a
// KNOWN byte count of a 2 GiB buffer (far past the 256 MiB Infinity Cache, so every byte comes from
// HBM) with one access shape; FETCH_SIZE (or WRITE_SIZE) per dispatch / that count is the correction
// a kernel of that shape needs (MI355X_MICROARCH.md, HBM: "calibrate on a known byte count in your
// own access pattern").
//   rd_dword      4 B per lane, a wave reads one 256-B row      (the strict stage's and links' reads)
//   rd_dwordx4    16 B per lane, 1 KiB per wave instruction      (finder ld4, encoder hist/emit chunks)
//   rd_lds_dword  LDS-DMA, 4 B per lane, one 256-B row per instr (count / emit round staging)
//   rd_byte_line  one byte per 128-B line                         (the encoder's L2 touch)
//   wr_dword      4 B per lane coalesced stores                   (encoder interior words)
//   wr_dwordx4    16 B per lane coalesced stores
//   wr_scatter16  16-B stores, the 64 lanes of a wave at 64 cursors 4 KiB apart, each cursor walking
//                 its own 4 KiB run (the emit pass's literal stores)
// Build: hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib   (and again with WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t NB = 2ull << 30;

__global__ void __launch_bounds__(256) rd_dword(const uint32_t* __restrict__ p, uint64_t n, uint32_t* sink) {
    uint32_t x = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 4; i += (uint64_t)gridDim.x * 256) x ^= p[i];
    if (x == 0x12345678u) sink[threadIdx.x] = x;
}
__global__ void __launch_bounds__(256) rd_dwordx4(const u32x4* __restrict__ p, uint64_t n, uint32_t* sink) {
    uint32_t x = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = p[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[threadIdx.x] = x;
}
__global__ void __launch_bounds__(256) rd_lds_dword(const uint32_t* __restrict__ p, uint64_t n, uint32_t* sink) {
    __shared__ uint32_t st[16 * 256];
    const uint32_t w = threadIdx.x >> 6;
    uint32_t x = 0;
    // each wave: 16 rows of 256 B per batch, one LDS-DMA dword per lane per row
    for (uint64_t r0 = ((uint64_t)blockIdx.x * 4 + w) * 16; r0 * 256 < n; r0 += (uint64_t)gridDim.x * 4 * 16) {
        for (uint32_t i = 0; i < 16; i++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + (r0 + i) * 64 + (threadIdx.x & 63)),
                                             (__attribute__((address_space(3))) void*)&st[w * 1024 + (i & 3) * 256], 4, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        x ^= st[w * 1024 + (threadIdx.x & 63)];
    }
    if (x == 0x12345678u) sink[threadIdx.x] = x;
}
__global__ void __launch_bounds__(256) rd_byte_line(const uint8_t* __restrict__ p, uint64_t n, uint32_t* sink) {
    uint32_t x = 0;       // (a sum: a byte xor could never equal the sentinel, and the loads were folded away)
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 128; i += (uint64_t)gridDim.x * 256) x += p[i * 128];
    if (x == 0x12345678u) sink[threadIdx.x] = x;
}
__global__ void __launch_bounds__(256) wr_dword(uint32_t* __restrict__ p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 4; i += (uint64_t)gridDim.x * 256) p[i] = (uint32_t)i;
}
__global__ void __launch_bounds__(256) wr_dwordx4(u32x4* __restrict__ p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * 256)
        p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}
__global__ void __launch_bounds__(256) wr_scatter16(u32x4* __restrict__ p, uint64_t n) {
    // wave-run of 64 x 4 KiB: lane j writes its own 4 KiB run 16 B at a time
    const uint64_t lane = threadIdx.x & 63;
    for (uint64_t base = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * 4096; base < n;
         base += (uint64_t)gridDim.x * 4 * 64 * 4096) {
        u32x4* q = p + (base + lane * 4096) / 16;
        for (uint32_t k = 0; k < 4096 / 16; k++) q[k] = u32x4{k, 1u, 2u, 3u};
    }
}

int main() {
    void* buf = nullptr;
    uint32_t* sink = nullptr;
    if (hipMalloc(&buf, NB) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) { fprintf(stderr, "alloc\n"); return 1; }
    hipMemset(buf, 1, NB);
    hipDeviceSynchronize();
    const uint32_t grid = 256 * 8;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timed = [&](const char* name, auto launch) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("%-14s %8.3f ms  %7.1f GB/s (of %llu B)\n", name, ms, NB / (ms * 1e6), (unsigned long long)NB);
    };
    for (int rep = 0; rep < 2; rep++) {
        timed("rd_dword", [&] { hipLaunchKernelGGL(rd_dword, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, NB, sink); });
        timed("rd_dwordx4", [&] { hipLaunchKernelGGL(rd_dwordx4, dim3(grid), dim3(256), 0, 0, (const u32x4*)buf, NB, sink); });
        timed("rd_lds_dword", [&] { hipLaunchKernelGGL(rd_lds_dword, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, NB, sink); });
        timed("rd_byte_line", [&] { hipLaunchKernelGGL(rd_byte_line, dim3(grid), dim3(256), 0, 0, (const uint8_t*)buf, NB, sink); });
        timed("wr_dword", [&] { hipLaunchKernelGGL(wr_dword, dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, NB); });
        timed("wr_dwordx4", [&] { hipLaunchKernelGGL(wr_dwordx4, dim3(grid), dim3(256), 0, 0, (u32x4*)buf, NB); });
        timed("wr_scatter16", [&] { hipLaunchKernelGGL(wr_scatter16, dim3(grid), dim3(256), 0, 0, (u32x4*)buf, NB); });
    }
    printf("bytes per kernel: %llu (rd_byte_line touches every 128-B line once)\n", (unsigned long long)NB);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
