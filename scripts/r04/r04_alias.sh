#!/bin/bash
# Round 4: stored-header aliases counted once -- decoder parity tests, config 2 with and without
# (NDFL_NO_ALIAS) and count stats, then the bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_inflate.py tests/test_gpu_finder_partitions.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py tests/test_gpu_parallel.py tests/test_gpu_count_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_alias.log 2>&1 || { tail -40 gpurun_out/pytest_alias.log; exit 1; }
tail -2 gpurun_out/pytest_alias.log
for mode in alias noalias alias noalias; do
  if [ $mode = noalias ]; then export NDFL_NO_ALIAS=1; else unset NDFL_NO_ALIAS; fi
  NDFL_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_$mode.log 2>&1 || { tail -20 gpurun_out/c2_$mode.log; exit 1; }
  echo "$mode"; grep -E "^\[ndfl\] (count waves|device link|count chains)" gpurun_out/c2_$mode.log | tail -5
  grep -h '^{' gpurun_out/c2_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])"
done
unset NDFL_NO_ALIAS
bash scripts/ab_env.sh "NDFL_NO_ALIAS=1" "NDFL_X=1" "NDFL_NO_ALIAS=1" "NDFL_X=1"
