#!/bin/bash
# Round 4: record-replay fast emit kernel -- decoder parity tests, the slow-list count, then A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py tests/test_gpu_lz77.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/fast_stats.log 2>&1 || { tail -20 gpurun_out/fast_stats.log; exit 1; }
grep -E "fast emit|emit waves" gpurun_out/fast_stats.log | tail -4
bash scripts/ab_env.sh "NDFL_EMIT_FAST=0" "NDFL_EMIT_FAST=1" "NDFL_EMIT_FAST=0" "NDFL_EMIT_FAST=1" && \
bash scripts/ab_libs.sh libndfl_f4.so libndfl_f5.so libndfl_f4.so libndfl_f5.so
