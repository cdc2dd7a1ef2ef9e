#!/bin/bash
# Round 4: the whole GPU test suite on the current build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
