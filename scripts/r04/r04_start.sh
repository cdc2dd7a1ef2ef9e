#!/bin/bash
# Round-4 start: the GPU parity suite, the default bench line, then an A/B of count-pass widths
# (NDFL_COUNT_W) with the dense and the partitioned header finder.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SKIP_BENCH=${SKIP_BENCH:-} bash scripts/gpu_tests.sh || exit 1
bash scripts/ab_env.sh "NDFL_DEFLATE_SLAB=0" "NDFL_DEFLATE_SLAB=1024" "NDFL_DEFLATE_SLAB=4096" "NDFL_COUNT_W=1" "NDFL_COUNT_W=2" "NDFL_COUNT_W=4" "NDFL_COUNT_W=8" \
  "NDFL_COUNT_W=4 NDFL_FIND_PART_BITS=4194304" "NDFL_COUNT_W=8 NDFL_FIND_PART_BITS=4194304" \
  "NDFL_COUNT_W=8 NDFL_FIND_PART_BITS=16777216" "NDFL_COUNT_W=8 NDFL_FIND_PART_BITS=auto"
