#!/bin/bash
# A/B of the header finder's scan pattern (NDFL_FIND_WIN / NDFL_FIND_PERIOD, 32-bit words): how the
# count / emit passes behave with fewer, longer chains.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abfind
mkdir -p $OUT
for cfg in "0 0" "4096 16384" "2048 16384" "4096 32768" "8192 32768"; do
  set -- $cfg
  if [ "$1" = 0 ]; then unset NDFL_FIND_WIN NDFL_FIND_PERIOD; else export NDFL_FIND_WIN=$1 NDFL_FIND_PERIOD=$2; fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $OUT/w$1_p$2.log 2>&1 || { tail -20 $OUT/w$1_p$2.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/w$1_p$2.log') if l.startswith('{')][-1])
print('win=$1 per=$2', d['ms_per_step'], json.dumps(d['phases_ms']))"
done
