#!/bin/bash
# Round 4: fast emit pass (LDS-staged record replay) + XCP1 64 as defaults -- decoder parity tests
# (incl. the fast/full/hand-over modes), then the bench twice and its kernel stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py tests/test_gpu_count_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ef.log 2>&1 || { tail -40 gpurun_out/pytest_ef.log; exit 1; }
tail -2 gpurun_out/pytest_ef.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ef_bench_$i.log 2>&1 || { tail -20 gpurun_out/ef_bench_$i.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ef_bench_$i.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phases_ms'])"
done
bash scripts/ab_libs.sh libndfl_x32.so libndfl_x48.so libndfl_x64.so libndfl_x32.so libndfl_x48.so libndfl_x64.so
