#!/bin/bash
# Round 4: LDS-staged record-replay fast emit kernel -- inflate parity tests on that build, then A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_fs4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fs4.log 2>&1 || { tail -40 gpurun_out/pytest_fs4.log; exit 1; }
tail -2 gpurun_out/pytest_fs4.log
NDFL_EMIT_FAST=0 bash scripts/ab_libs.sh libndfl_fs4.so && bash scripts/ab_libs.sh libndfl_fs4.so && NDFL_EMIT_FAST=0 bash scripts/ab_libs.sh libndfl_fs4.so && bash scripts/ab_libs.sh libndfl_fs4.so
