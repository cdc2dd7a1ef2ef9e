#!/bin/bash
# Round 5: the header-set parity test on the default build and the 3/5-wave strict builds, then the
# bench-stream A/B of the accepted sets (scripts/r05/headers_ab.py).  Stops at a timeout / crash.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {   # name, then the command; pytest rc 1 (failed asserts) goes on, anything else stops
  local name=$1; shift
  timeout -k 10 600 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -15 gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
T="python -u -m pytest tests/test_gpu_headers.py -v --timeout 300 --timeout-method thread"
run hdr_default $T
run hdr_sw3 env NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_sw3.so $T
run hdr_sw5 env NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_sw5.so $T
L=$PWD/deflate-library-java_amd/lib
run hdr_ab python -u scripts/r05/headers_ab.py $L/libndfl.so $L/libndfl_sw3.so $L/libndfl_sw5.so
