#!/bin/bash
# Per-data-type decode profile (scripts/prof_types.py): the NDFL_STATS / phase-clock counters of the
# host-linked path for each build given (lib/ names, built with -DNDFL_PHASE_CLOCK).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SZ=${SZ:-1073741824}
for L in "$@"; do
  NDFL_HOST_LINK=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$L NDFL_STATS=1 timeout -k 10 300 python -u scripts/prof_types.py $SZ > gpurun_out/types_$L.log 2>&1 || { tail -20 gpurun_out/types_$L.log; exit 1; }
  echo "== $L"; grep -v "count chain\|resolve round" gpurun_out/types_$L.log | awk 'NR%2==1 || /ratio/'
done
