#!/bin/bash
# Round 5: the scratch-free strict stage -- accepted sets on the bench stream for the default build
# (5 waves/SIMD) and 3/4-wave builds of the same code, each 3 runs; then the finder-phase time of
# each build in the bench (no CPU leg, no verify).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u scripts/r05/headers_ab.py $L/libndfl.so $L/libndfl_n3.so $L/libndfl_n4.so > gpurun_out/hab3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/hab3.log; [ $rc -eq 0 ] || exit $rc
for lib in libndfl.so libndfl_n3.so libndfl_n4.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-verify > gpurun_out/b_$lib.log 2>&1 || { tail -20 gpurun_out/b_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/b_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done
