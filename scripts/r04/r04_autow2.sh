#!/bin/bash
# Round 4: automatic count width, threshold 4 chains per count wave -- config 2 with stats, c3, bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_autow2.log 2>&1 || { tail -40 gpurun_out/pytest_autow2.log; exit 1; }
tail -1 gpurun_out/pytest_autow2.log
NDFL_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_autos.log 2>&1 || { tail -20 gpurun_out/c2_autos.log; exit 1; }
grep -E "^\[ndfl\] count pass:" gpurun_out/c2_autos.log | head -2
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_auto$i.log 2>&1 || { tail -20 gpurun_out/c2_auto$i.log; exit 1; }
  echo "c2 $(grep -h '^{' gpurun_out/c2_auto$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])")"
done
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/bench_autos.log 2>&1 || { tail -20 gpurun_out/bench_autos.log; exit 1; }
grep -E "^\[ndfl\] count pass:" gpurun_out/bench_autos.log | head -1
for lib in h1 h4 h1 h4; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_$lib.so timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_$lib.log 2>&1 || { tail -20 gpurun_out/c2_$lib.log; exit 1; }
  echo "c2 $lib $(grep -h '^{' gpurun_out/c2_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])")"
done
bash scripts/ab_libs.sh libndfl_h1.so libndfl_h4.so libndfl_h1.so libndfl_h4.so
