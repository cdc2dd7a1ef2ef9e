#!/bin/bash
# Round 4: strict stage at 3 waves/SIMD with and without a wait on LDS after each table build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in sw3 sw3l sw3 sw3l; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_$lib.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > gpurun_out/cdl_$lib.log 2>&1 || { tail -20 gpurun_out/cdl_$lib.log; exit 1; }
  echo "$lib $(python -c "import json; d=json.loads(open('gpurun_out/cdl_$lib.log').read().strip().splitlines()[-1]); print(d['phases_ms']['inflate_candidates'])")"
done
