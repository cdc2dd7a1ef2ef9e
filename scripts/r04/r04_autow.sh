#!/bin/bash
# Round 4: automatic count width (4 waves per chain when the counted chains are fewer than the
# count waves) -- decoder parity tests, config 2, then the bench twice
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py tests/test_gpu_count_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_autow.log 2>&1 || { tail -40 gpurun_out/pytest_autow.log; exit 1; }
tail -2 gpurun_out/pytest_autow.log
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_auto$i.log 2>&1 || { tail -20 gpurun_out/c2_auto$i.log; exit 1; }
  echo "c2 $(grep -h '^{' gpurun_out/c2_auto$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])")"
done
bash scripts/ab_env.sh "NDFL_X=1" "NDFL_X=2"
