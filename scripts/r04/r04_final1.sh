#!/bin/bash
# Round 4: decoder parity tests and the bench on the current build
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_configs.py tests/test_gpu_parallel.py tests/test_gpu_gzip.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_f1.log 2>&1 || { tail -40 gpurun_out/pytest_f1.log; exit 1; }
tail -1 gpurun_out/pytest_f1.log
bash scripts/ab_env.sh "NDFL_X=1" "NDFL_X=2"
