#!/bin/bash
# Round 6: flat-group statistics at 1 GiB (chains sent back, group wave time).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06k
mkdir -p $O
NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/stats.log 2>&1 || { tail -30 $O/stats.log; exit 1; }
grep "flat=\|flat groups\|count waves\|count chains\|longest" $O/stats.log
