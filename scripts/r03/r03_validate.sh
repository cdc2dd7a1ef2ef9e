#!/bin/bash
# Round-3 validation on one MI355X: the default bench line (full-stream bit_exact), the 2-rank
# strong-scaling rehearsal as the driver would launch it (bench.py spawns the ranks), config 5 at
# 16 GiB, and the config-3 profile.  Each GPU step has its own time limit; the first failure ends it.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03
mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  tail -2 $OUT/$name.log; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $OUT/$name.log; exit 1; }; }
[ -n "$SKIP_N1" ] || step bench_n1 400 python -u bench.py
[ -n "$SKIP_N2" ] || step bench_n2_gloo_strong 600 python -u bench.py --gpus 2 --backend gloo --scaling strong --steps 3 --warmup 1
[ -n "$SKIP_C5" ] || step c5 600 python -u scripts/bench_configs.py c5
[ -n "$SKIP_C3" ] || step c3prof 900 bash scripts/c3_profile.sh
echo all-ok
