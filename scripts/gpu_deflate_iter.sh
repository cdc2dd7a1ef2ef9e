#!/bin/bash
# Encoder iteration: GPU parity tests (unless SKIP_TESTS), encoder timings on the 4 GiB c4 corpus,
# per-kernel stats under rocprofv3.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 200 python -u scripts/perf_deflate.py c4:4096 > gpurun_out/perf_deflate.log 2>&1 || { tail -30 gpurun_out/perf_deflate.log; exit 1; }
grep -v amdgpu.ids gpurun_out/perf_deflate.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_def -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/perf_deflate.py c4:4096 > $GRAFT_REPO_ROOT/gpurun_out/prof_def.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_def.log; exit 1; }
grep -E "ndfl_" $GRAFT_REPO_ROOT/gpurun_out/prof_def/run_kernel_stats.csv | cut -d, -f1-8
