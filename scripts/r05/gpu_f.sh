#!/bin/bash
# Round 5: encoder emit pass with one literal code per byte of literal pieces, two codes per put:
# encoder parity tests, then bench A/B against the previous emit (libndfl_emit0.so).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_strategies.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 || { tail -30 gpurun_out/pytest_f.log; exit 1; }
tail -2 gpurun_out/pytest_f.log
for k in 1 2; do for lib in libndfl.so libndfl_emit0.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bf_$lib$k.log 2>&1 || { tail -20 gpurun_out/bf_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bf_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms']['deflate_kernel'])")"
done; done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bf_verify.log 2>&1 || { tail -20 gpurun_out/bf_verify.log; exit 1; }
grep -h '^{' gpurun_out/bf_verify.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('verify', d['ms_per_step'], d['bit_exact'])"
