#!/bin/bash
# Round-3 A/B on the default bench: finder slices (NDFL_FIND_SLICES), and the emit pass without
# HBM output traffic (libndfl_nostore.so, an A/B build: output garbage, so --no-verify).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab3
mkdir -p $OUT
run() { local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 $EXTRA > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1])
print('$name', d['ms_per_step'], json.dumps(d['phases_ms']))"; }
run slices1 NDFL_FIND_SLICES=1
run slices16 NDFL_FIND_SLICES=16
run slices48 NDFL_FIND_SLICES=48
EXTRA=--no-verify run nostore NDFL_LIB_PATH=$GRAFT_REPO_ROOT/deflate-library-java_amd/lib/libndfl_nostore.so
