#!/bin/bash
# Round 4: parse-driven LZ77 search -- LZ77 parity tests, config 3 with statistics for both searches,
# then the sparse-finder window A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz77.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lz.log 2>&1 || { tail -40 gpurun_out/pytest_lz.log; exit 1; }
tail -2 gpurun_out/pytest_lz.log
NDFL_LZ_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_parse.log 2>&1 || { tail -20 gpurun_out/c3_parse.log; exit 1; }
tail -3 gpurun_out/c3_parse.log
NDFL_LZ_SEARCH=chain timeout -k 10 300 python -u scripts/bench_configs.py c3 > gpurun_out/c3_chain.log 2>&1 || { tail -20 gpurun_out/c3_chain.log; exit 1; }
tail -1 gpurun_out/c3_chain.log
bash scripts/r04/r04_win.sh
