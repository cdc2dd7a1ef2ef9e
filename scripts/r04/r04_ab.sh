#!/bin/bash
# Round-4 A/B: the GPU parity suite on the default build, then the default bench per library build
# (LIBS, in lib/), then the token-loop microbenchmark.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
bash scripts/ab_libs.sh $LIBS || exit 1
if [ -n "$MICRO" ]; then
  cd scripts/microbench && for L in $MICRO; do echo "== LDS $L"; timeout -k 5 60 ./tokloop_$L 2048 || exit 1; done
fi
