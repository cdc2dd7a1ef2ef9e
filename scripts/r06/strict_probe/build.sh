#!/bin/bash
# Round 6: rebuild the round-4 strict stage's lossy builds with a per-survivor verdict
# probe (scripts/r06/strict_probe.patch on the sources of commit a5b0dbe~1, the last round-4 tree) --
#   sw3     3 waves/SIMD, strict_stored a non-inlined call (lost 2-4 % of the headers, round 5)
#   sw3inl  3 waves/SIMD, strict_stored inlined, no scratch (lost none)
#   sw5inl  5 waves/SIMD, inlined, 95 spilled VGPRs (lost ~4 %)
# into scripts/r06/strict_probe/r4/ (git-ignored; it travels to the GPU box with the tree).  CPU side.
set -e
cd "$(dirname "$0")"
rm -rf r4 && mkdir r4
git -C ../../.. archive a5b0dbe~1 deflate-library-java_amd/csrc deflate-library-java_amd/python include | tar x -C r4
(cd r4 && patch -p0 -s < ../strict_probe.patch)
# NDFL_STRICT_GRID: the strict kernel's grid (workgroups of 256), to run it at a chosen concurrency
sed -i 's/static const uint32_t strict_grid = \[\] {/static const uint32_t strict_grid = [] { if (const char* g = getenv("NDFL_STRICT_GRID")) return (uint32_t)atoi(g);/' \
    r4/deflate-library-java_amd/csrc/hip/inflate_kernels.hip
cd r4/deflate-library-java_amd && mkdir -p lib
SRC=csrc/capi/ndfl_capi.cpp
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -w -x hip -shared"
$H -DNDFL_STRICT_WPE=3 -o lib/libndfl_sw3.so $SRC &
sed 's/__device__ __noinline__ bool strict_stored/__device__ __forceinline__ bool strict_stored/' csrc/hip/inflate_kernels.hip > csrc/hip/inflate_kernels_inl.hip
sed 's/inflate_kernels.hip/inflate_kernels_inl.hip/' $SRC > csrc/capi/ndfl_capi_inl.cpp
$H -DNDFL_STRICT_WPE=3 -o lib/libndfl_sw3inl.so csrc/capi/ndfl_capi_inl.cpp &
$H -DNDFL_STRICT_WPE=5 -o lib/libndfl_sw5inl.so csrc/capi/ndfl_capi_inl.cpp &
wait
ls -la lib
