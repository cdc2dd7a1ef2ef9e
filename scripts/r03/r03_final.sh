#!/bin/bash
# Round-3 final evidence on one MI355X: the GPU parity suite, the profile of the default bench
# (kernel stats, FETCH/WRITE, SQ passes), the default bench line, configurations 1/2/3/5.
cd "$GRAFT_REPO_ROOT"
SKIP_BENCH=1 bash scripts/gpu_tests.sh || exit 1
bash scripts/profile_bench.sh || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
bash scripts/r03/r03_configs_final.sh
