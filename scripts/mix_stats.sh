#!/bin/bash
# NDFL_STATS / phase-clock counters of the host-linked decode of the config-4 mix, per build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SZ=${SZ:-4294967296}
for L in "$@"; do
  NDFL_HOST_LINK=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$L NDFL_STATS=1 timeout -k 10 300 python -u scripts/prof_inflate.py $SZ 2 > gpurun_out/mix_$L.log 2>&1 || { tail -20 gpurun_out/mix_$L.log; exit 1; }
  echo "== $L"; grep -v "count chain\|resolve round\|amdgpu.ids" gpurun_out/mix_$L.log | tail -7
done
