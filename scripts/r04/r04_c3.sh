#!/bin/bash
# Config 3 timed, then with LZ statistics (searches, bucket entries, fallback searches)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_parse.log 2>&1 || { tail -20 gpurun_out/c3_parse.log; exit 1; }
tail -1 gpurun_out/c3_parse.log | cut -c1-200
NDFL_LZ_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_parse_stats.log 2>&1 || { tail -20 gpurun_out/c3_parse_stats.log; exit 1; }
grep "lz parse" gpurun_out/c3_parse_stats.log | head -4
bash scripts/r04/r04_c3prof.sh
