#!/bin/bash
# Decoder fix-up A/B: decoder parity tests on the first build, then the default bench per build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
first=$1
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$first timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_long_codes.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_fix_tests.log 2>&1 || { tail -30 gpurun_out/ab_fix_tests.log; exit 1; }
tail -2 gpurun_out/ab_fix_tests.log
bash scripts/ab_libs.sh "$@"
