#!/bin/bash
# Round 6: where the flat groups' time goes (clock64 around the input rings' phase points).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06m
mkdir -p $O
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_fprof.so NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/fprof.log 2>&1 || { tail -30 $O/fprof.log; exit 1; }
grep "flat=\|flat groups\|flat decode" $O/fprof.log
