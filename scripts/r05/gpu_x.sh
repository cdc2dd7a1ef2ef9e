#!/bin/bash
# Round 5: pending (deferred) output groups on the bench stream (NDFL_STATS).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify > gpurun_out/bx_stats.log 2>&1 || { tail -20 gpurun_out/bx_stats.log; exit 1; }
grep -h "emit:\|fast emit\|device link" gpurun_out/bx_stats.log | tail -4
