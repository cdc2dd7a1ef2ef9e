#!/bin/bash
# Round 4: fast emit pass with only the primary tables in LDS (9.5 KB: 16 waves per CU) -- emit
# parity tests, then A/B against the 11.0 KB layout (gx0)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_long_codes.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gx.log 2>&1 || { tail -40 gpurun_out/pytest_gx.log; exit 1; }
tail -2 gpurun_out/pytest_gx.log
bash scripts/ab_libs.sh libndfl_gx0.so libndfl_gx.so libndfl_gx0.so libndfl_gx.so libndfl_gx0.so libndfl_gx.so
