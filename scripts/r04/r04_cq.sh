#!/bin/bash
# Round 4: copies gathered across lanes before the emit copy path runs (NDFL_EMIT_CQ) -- emit parity
# tests on the default (16), then A/B of 0 (every iteration) / 8 / 16 / 32 / 64
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_long_codes.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cq.log 2>&1 || { tail -40 gpurun_out/pytest_cq.log; exit 1; }
tail -2 gpurun_out/pytest_cq.log
bash scripts/ab_libs.sh libndfl_cq0.so libndfl_cq8.so libndfl_cq16.so libndfl_cq32.so libndfl_cq64.so libndfl_cq0.so libndfl_cq8.so libndfl_cq16.so libndfl_cq32.so libndfl_cq64.so
