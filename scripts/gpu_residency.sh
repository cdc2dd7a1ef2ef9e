#!/bin/bash
# Count-pass residency check (wave occupancy under NDFL_STATS) and bench A/B of LDS-footprint builds
cd "$GRAFT_REPO_ROOT"
for L in l14pc s16pc; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_$L.so NDFL_STATS=1 timeout -k 10 200 python -u scripts/prof_inflate.py 4294967296 1 > gpurun_out/res_$L.log 2>&1 || exit 1
  echo "$L: $(grep 'occupancy' gpurun_out/res_$L.log | tr '\n' ' ')"
done
bash scripts/ab_libs.sh libndfl_l16.so libndfl_s16.so libndfl_l14.so libndfl_s14.so libndfl_s16.so libndfl_l16.so
