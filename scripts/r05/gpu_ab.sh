#!/bin/bash
# Round 5: per-data-type count-pass profile with the final round-5 code (phase clocks, -DNDFL_PHASE_CLOCK
# build libndfl_pc.so; 256 MiB of each c4 component alone).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_COUNT_W=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_pc.so NDFL_STATS=1 timeout -k 10 300 python -u scripts/prof_types.py 268435456 runs,binary,text > gpurun_out/types_r05.log 2>&1 || { tail -20 gpurun_out/types_r05.log; exit 1; }
grep -h "wave-time\|count waves\|count bits\|ratio" gpurun_out/types_r05.log
echo done
