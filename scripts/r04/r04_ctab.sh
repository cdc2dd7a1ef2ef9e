#!/bin/bash
# Round 4: candidate tables built before the count pass -- decoder parity tests, then the bench A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
bash scripts/ab_env.sh "NDFL_NO_CTAB=1" "NDFL_COUNT_W=1" "NDFL_NO_CTAB=1" "NDFL_COUNT_W=1"
