#!/bin/bash
# Round 6: where the count pass's time goes at one rank's 512 MiB share and at the full 4 GiB
# (NDFL_STATS chain table + phase clocks of a -DNDFL_PHASE_CLOCK build), and the byte-line FETCH
# calibration.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06b
mkdir -p $O
for sz in 536870912 4294967296; do
  NDFL_STATS=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_pc.so timeout -k 10 300 python -u bench.py --size $sz --steps 1 --warmup 1 --no-cpu --no-verify > $O/stats_$sz.log 2>&1 || { tail -30 $O/stats_$sz.log; exit 1; }
  grep -E "count chain|count waves|count bits|wave-time|ms_per_step" $O/stats_$sz.log | tail -40
done
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/scripts/r06/fetch_calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/cf -o run --output-format csv -- $B > $GRAFT_REPO_ROOT/$O/calib_fetch.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/calib_fetch.log; exit 1; }
echo ok
