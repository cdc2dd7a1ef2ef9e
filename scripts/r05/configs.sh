#!/bin/bash
# Configurations 1, 2, 3 and 5 of BASELINE.json on one MI355X with the round-5 library
# (scripts/bench_configs.py); each step has its own time limit, the first failure ends it.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05cfg
mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  grep -h '^{' $OUT/$name.log | tail -3; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $OUT/$name.log; exit 1; }; }
step c123 600 python -u scripts/bench_configs.py c1 c2 c3
[ -n "$SKIP_C5" ] || step c5 600 python -u scripts/bench_configs.py c5
echo all-ok
