#!/bin/bash
# Round-3 configuration runs on one MI355X (scripts/bench_configs.py): configs 1, 2, 3 and 5, then
# config 3 again with the LZ77 match statistics, with and without the 6-byte-prefix chains
# (NDFL_LZ_L6=0: trigram chains only).  Each step has its own time limit; the first failure ends it.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03cfg
mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  grep -h '^\[ndfl\] lz\|^{' $OUT/$name.log | tail -3; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $OUT/$name.log; exit 1; }; }
step c123 600 python -u scripts/bench_configs.py c1 c2 c3
step c3_l6_stats 300 env NDFL_LZ_STATS=1 python -u scripts/bench_configs.py c3
step c3_l3_stats 300 env NDFL_LZ_STATS=1 NDFL_LZ_L6=0 python -u scripts/bench_configs.py c3
[ -n "$SKIP_C5" ] || step c5 600 python -u scripts/bench_configs.py c5
echo all-ok
