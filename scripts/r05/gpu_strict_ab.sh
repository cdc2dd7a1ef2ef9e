#!/bin/bash
# Round 5: strict-stage variants on the bench stream (scripts/r05/headers_ab.py), then the
# multi-rank GPU protocol tests (window maps).  Stops at a timeout / crash.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u scripts/r05/headers_ab.py $L/libndfl.so ${VARIANTS:-$L/libndfl_sw3.so} > gpurun_out/hab2.log 2>&1
rc=$?; cat gpurun_out/hab2.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_headers.py -x -v --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; tail -25 gpurun_out/par.log; exit $rc
