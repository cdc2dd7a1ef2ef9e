#!/bin/bash
# Round 5: decode tables -- codes shorter than the primary bits - 4 filled by all lanes one symbol at
# a time: decoder tests, bench A/B against libndfl_head.so (the previous commit), phase clocks.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py tests/test_gpu_long_codes.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1 || { tail -30 gpurun_out/pytest_t.log; exit 1; }
tail -2 gpurun_out/pytest_t.log
for k in 1 2; do for lib in libndfl.so libndfl_head.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bt_$lib$k.log 2>&1 || { tail -20 gpurun_out/bt_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bt_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
NDFL_STATS=1 NDFL_LIB_PATH=$L/libndfl_pc.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify > gpurun_out/bt_pc.log 2>&1 || { tail -20 gpurun_out/bt_pc.log; exit 1; }
grep -h "wave-time\|count waves" gpurun_out/bt_pc.log | tail -2
