#!/bin/bash
# Round 5: codes pass ranks only the used symbols, trims by ballots: encoder
# parity tests, then bench A/B against libndfl_emit2.so (the previous commit).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_strategies.py tests/test_gpu_plugin.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1 || { tail -30 gpurun_out/pytest_j.log; exit 1; }
tail -2 gpurun_out/pytest_j.log
for k in 1 2; do for lib in libndfl.so libndfl_emit2.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bj_$lib$k.log 2>&1 || { tail -20 gpurun_out/bj_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bj_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms']['deflate_kernel'])")"
done; done
cd /tmp && export TMPDIR=/tmp
for lib in libndfl.so libndfl_emit2.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_l_$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_l_$lib.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_l_$lib.log; exit 1; }
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_l_$lib -name '*kernel_stats.csv' | head -1)
  echo "$lib"; grep -h '"ndfl_' $f | cut -d, -f1-4
done
