#!/bin/bash
# Round-end style GPU pass: GPU parity tests, then the default bench line (with the CPU leg).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
