#!/bin/bash
# GPU parity tests, a short bench, and a kernel-trace profile of the bench (split encoder check).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_split.log 2>&1 || { tail -30 gpurun_out/bench_split.log; exit 1; }
tail -1 gpurun_out/bench_split.log
NDFL_DEFLATE_FUSED=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_fused.log 2>&1 || { tail -30 gpurun_out/bench_fused.log; exit 1; }
tail -1 gpurun_out/bench_fused.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_split -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_split.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_split.log; exit 1; }
echo prof done
