#!/bin/bash
# Decoder stats on 1 GiB, inflate GPU tests, N=1 bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_STATS=1 timeout -k 10 200 python scripts/prof_inflate.py 1073741824 1 > gpurun_out/stats.log 2>&1 || { tail -20 gpurun_out/stats.log; exit 1; }
tail -2 gpurun_out/stats.log
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
