#!/bin/bash
# Round 4: decoder tests after the phase-trigger change, config 3 (parse-driven search, timed and with
# statistics), then the sparse-finder window A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_parse.log 2>&1 || { tail -20 gpurun_out/c3_parse.log; exit 1; }
tail -1 gpurun_out/c3_parse.log
NDFL_LZ_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_parse_stats.log 2>&1 || { tail -20 gpurun_out/c3_parse_stats.log; exit 1; }
head -1 gpurun_out/c3_parse_stats.log
bash scripts/r04/r04_win.sh
