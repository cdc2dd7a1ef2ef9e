#!/bin/bash
# Round 6: configurations 1, 2, 3 and 5 (scripts/bench_configs.py) and the per-data-type decode
# profile (1 GiB of each config-4 component alone).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06cfg
mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  grep -h '^{' $OUT/$name.log | tail -3; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $OUT/$name.log; exit 1; }; }
step c123 600 python -u scripts/bench_configs.py c1 c2 c3
step c5 600 python -u scripts/bench_configs.py c5
timeout -k 10 300 python -u scripts/prof_types.py 1073741824 > $OUT/types.log 2>&1 || { tail -20 $OUT/types.log; exit 1; }
cat $OUT/types.log
echo all-ok
