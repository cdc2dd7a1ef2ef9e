#!/bin/bash
# Round 5: header-record kernel reads each header through a lane-private LDS window (one load wait per
# 256 bits): decoder tests, bench, kernel stats.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_headers.py tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py tests/test_gpu_long_codes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bq_$k.log 2>&1 || { tail -20 gpurun_out/bq_$k.log; exit 1; }
  echo "libndfl.so $(grep -h '^{' gpurun_out/bq_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_q -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_q.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_q.log; exit 1; }
grep -h '"ndfl_' $GRAFT_REPO_ROOT/gpurun_out/prof_q/run_kernel_stats.csv | cut -d, -f1-4 | head -12
