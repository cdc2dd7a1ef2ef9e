#!/bin/bash
# NDFL_STATS counters of the default decode and a sparse-window decode (config-4 mix, 1 GiB)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for envs in "NDFL_COUNT_W=1" "NDFL_FIND_WIN=8192 NDFL_FIND_PERIOD=16384"; do
  i=$((i+1))
  env $envs NDFL_HOST_LINK=1 NDFL_STATS=1 timeout -k 10 300 python -u scripts/prof_inflate.py 1073741824 1 > gpurun_out/winstats_$i.log 2>&1 || { tail -20 gpurun_out/winstats_$i.log; exit 1; }
  echo "== $envs"; grep -v "count chain\|resolve round\|amdgpu.ids" gpurun_out/winstats_$i.log | tail -9
done
