#!/bin/bash
# Round 6: why flat-group chains go back to the wave decode (1 GiB, stats).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06t
mkdir -p $O
NDFL_FLAT_MIN=0 NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/why.log 2>&1 || { tail -30 $O/why.log; exit 1; }
grep "flat=\|flat groups" $O/why.log
