#!/bin/bash
# Round 4: config 2 kernel trace (where the decode's 9.4 ms go)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 scripts/bench_configs.py c2 > gpurun_out/c2prof.log 2>&1 || { tail -20 gpurun_out/c2prof.log; exit 1; }
f=$(find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -1); head -30 "$f" | cut -d, -f1-4
