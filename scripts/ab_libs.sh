#!/bin/bash
# A/B of library builds on the default bench (NDFL_LIB_PATH selects the build): bash scripts/ab_libs.sh a.so b.so ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_$lib.log 2>&1 || { tail -20 gpurun_out/ab_$lib.log; exit 1; }
  echo "$lib $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$lib.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phases_ms'])")"
done
