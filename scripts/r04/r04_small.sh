#!/bin/bash
# Round 4: register sort in the candidate compaction, wave-aggregated bucket counters in the order
# kernels -- decoder parity tests, a bench pair, and the kernel stats of a short bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_count_wg.py tests/test_gpu_parallel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_small.log 2>&1 || { tail -40 gpurun_out/pytest_small.log; exit 1; }
tail -1 gpurun_out/pytest_small.log
bash scripts/ab_env.sh "NDFL_X=1" "NDFL_X=2" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_small.log 2>&1 || { tail -20 gpurun_out/prof_small.log; exit 1; }
grep -E "compact_kernel|order_kernel|segscan|alias" gpurun_out/prof_small/run_kernel_stats.csv | cut -d, -f1-4
