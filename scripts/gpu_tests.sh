#!/bin/bash
# GPU parity suite (one process, per-test timeout), then the default bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python -u bench.py > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
fi
