#!/bin/bash
# Encoder A/B: encoder parity tests on the first build, then the default bench per build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_strategies.py tests/test_gpu_configs.py tests/test_gpu_gzip.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_enc_tests.log 2>&1 || { tail -30 gpurun_out/ab_enc_tests.log; exit 1; }
tail -2 gpurun_out/ab_enc_tests.log
bash scripts/ab_libs.sh "$@"
