#!/bin/bash
# Round 5: count-pass phase clocks (NDFL_STATS with a -DNDFL_PHASE_CLOCK build) on the bench stream.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
NDFL_STATS=1 NDFL_LIB_PATH=$L/libndfl_pc.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify > gpurun_out/bs_pc.log 2>&1 || { tail -20 gpurun_out/bs_pc.log; exit 1; }
grep -h "wave-time\|count waves\|count chains\|strict stage\|count pass" gpurun_out/bs_pc.log | tail -12
