#!/bin/bash
# Round 4: bit buffer up to the stop (run_to / emit) + 16-byte run stores -- decoder parity tests on
# the current build, then A/B of the builds with the full emit kernel only (f4: before; bs: bit
# buffer; r16: + run stores; x64/x96: r16's parent bs with XCP1 64/96), and the LDS-staged fast
# emit variant (fs4)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NDFL_EMIT_FAST=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bs.log 2>&1 || { tail -40 gpurun_out/pytest_bs.log; exit 1; }
tail -2 gpurun_out/pytest_bs.log
bash scripts/ab_libs.sh libndfl_f4.so libndfl_bs.so libndfl_r16.so libndfl_n32.so libndfl_tc.so libndfl_x64.so libndfl_x96.so libndfl_f4.so libndfl_bs.so libndfl_r16.so libndfl_n32.so libndfl_tc.so libndfl_x64.so libndfl_x96.so && \
NDFL_EMIT_FAST=1 bash scripts/ab_libs.sh libndfl_fs4.so libndfl_fs4.so
NDFL_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_stats.log 2>&1 || { tail -20 gpurun_out/c2_stats.log; exit 1; }
grep -E "^\[ndfl\]" gpurun_out/c2_stats.log | sort | uniq -c | sort -rn | head -30
