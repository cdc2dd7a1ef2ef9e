#!/bin/bash
# Round 6: count-pass phase clocks per data type (256 MiB of each c4 component alone, -DNDFL_PHASE_CLOCK build)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06c
mkdir -p $O
NDFL_COUNT_W=1 NDFL_STATS=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_pc.so timeout -k 10 300 python -u scripts/prof_types.py 268435456 > $O/types.log 2>&1 || { tail -30 $O/types.log; exit 1; }
grep -E "^(text|binary|random|runs)|wave-time|count waves|slow-verify" $O/types.log
