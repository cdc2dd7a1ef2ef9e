#!/bin/bash
# LZ77 (FULL_* presets) on one MI355X: the GPU LZ77 tests, then config 3 with match statistics,
# two-level chains (default) and trigram chains only (NDFL_LZ_L4=0).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ablz
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz77.py tests/test_gpu_strategies.py tests/test_gpu_plugin.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 1 0; do
  NDFL_LZ_STATS=1 NDFL_LZ_L4=$v timeout -k 10 300 python -u scripts/bench_configs.py c3 > $OUT/c3_l4_$v.log 2>&1 || { tail -20 $OUT/c3_l4_$v.log; exit 1; }
  echo "L4=$v"; grep -h '^\[ndfl\] lz\|^{' $OUT/c3_l4_$v.log | tail -2
done
