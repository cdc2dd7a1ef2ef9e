#!/bin/bash
# Round 5: encoder hist, token-bit and emit passes on precomputed 64-bit piece-class masks: encoder
# parity tests, then bench A/B against libndfl_emit1.so (the previous commit).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_strategies.py tests/test_gpu_plugin.py tests/test_gpu_gzip.py tests/test_gpu_zlib.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1 || { tail -30 gpurun_out/pytest_j.log; exit 1; }
tail -2 gpurun_out/pytest_j.log
for k in 1 2; do for lib in libndfl.so libndfl_emit1.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bj_$lib$k.log 2>&1 || { tail -20 gpurun_out/bj_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bj_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms']['deflate_kernel'])")"
done; done
