#!/bin/bash
# Round 6: flat groups alone (random data only: no other count work on the chip) -- intrinsic step cost.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06o
mkdir -p $O
NDFL_COUNT_W=1 PROBE_DATA=random NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_fprof.so NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 256 1 0 > $O/fprof_rand.log 2>&1 || { tail -30 $O/fprof_rand.log; exit 1; }
grep "flat=\|flat groups\|flat decode\|count waves" $O/fprof_rand.log
