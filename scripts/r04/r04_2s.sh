#!/bin/bash
# Round 4: two decode streams per lane in the emit pass -- decoder parity tests, then the bench A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py tests/test_gpu_lz77.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
bash scripts/ab_libs.sh ${LIBS:-libndfl_base.so libndfl_2s.so libndfl_base.so libndfl_2s.so}
