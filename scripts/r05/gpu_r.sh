#!/bin/bash
# Round 5: strict stage claims its survivor slices one ahead (list entries loaded into registers
# while the current slice is checked; 64 per slice) + header kernel rows padded against bank
# conflicts: header-set parity and determinism, decoder tests, bench, kernel stats.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_headers.py tests/test_gpu_inflate.py tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r.log 2>&1 || { tail -30 gpurun_out/pytest_r.log; exit 1; }
tail -2 gpurun_out/pytest_r.log
timeout -k 10 600 python -u scripts/r05/headers_ab.py $L/libndfl.so > gpurun_out/hab_r.log 2>&1 || { tail -20 gpurun_out/hab_r.log; exit 1; }
grep -h '^{' gpurun_out/hab_r.log | cut -c1-200
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/br_$k.log 2>&1 || { tail -20 gpurun_out/br_$k.log; exit 1; }
  echo "libndfl.so $(grep -h '^{' gpurun_out/br_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_r.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_r.log; exit 1; }
grep -h '"ndfl_' $GRAFT_REPO_ROOT/gpurun_out/prof_r/run_kernel_stats.csv | cut -d, -f1-4 | head -12
