#!/bin/bash
# Round 6: flat groups at raised wave priority vs not (lib/libndfl_noprio.so), group wave time at 1 GiB,
# then the 4 GiB decode with flat groups on and off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06l
mkdir -p $O
NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/prio.log 2>&1 || { tail -30 $O/prio.log; exit 1; }
grep "flat=\|flat groups" $O/prio.log
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_noprio.so NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/noprio.log 2>&1 || { tail -30 $O/noprio.log; exit 1; }
grep "flat=\|flat groups" $O/noprio.log
timeout -k 10 300 python -u scripts/r06/flat_probe.py 4096 1 0 > $O/probe4g.log 2>&1 || { tail -30 $O/probe4g.log; exit 1; }
grep flat= $O/probe4g.log
