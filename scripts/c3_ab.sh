#!/bin/bash
# Config 3 A/B of library builds (NDFL_LIB_PATH): bash scripts/c3_ab.sh a.so b.so ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$lib timeout -k 10 300 python3 scripts/bench_configs.py c3 > gpurun_out/c3_$lib.log 2>&1 || { tail -20 gpurun_out/c3_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/c3_$lib.log)"
done
