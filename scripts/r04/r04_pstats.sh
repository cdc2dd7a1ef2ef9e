#!/bin/bash
# Round 4: count-pass statistics (rounds, fix-ups, chain outcomes) on the bench and on config 5
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > gpurun_out/ps_bench.log 2>&1 || { tail -20 gpurun_out/ps_bench.log; exit 1; }
grep -E "^\[ndfl\] (count|device link)" gpurun_out/ps_bench.log | tail -6
NDFL_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c5 > gpurun_out/ps_c5.log 2>&1 || { tail -20 gpurun_out/ps_c5.log; exit 1; }
grep -E "^\[ndfl\] (count|device link)" gpurun_out/ps_c5.log | tail -6
