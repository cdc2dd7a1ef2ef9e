#!/bin/bash
# Round 5: count claim order by a cost key from the header records (fixed NDFL_ORDER_FIX_KBIT per chain,
# twice the bits of mostly-8-bit-code blocks; libndfl.so = 96, _of32, _of192) against bits alone (_oc0).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_count_wg.py tests/test_gpu_emit_fast.py tests/test_gpu_configs.py tests/test_gpu_headers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_al.log 2>&1 || { tail -30 gpurun_out/pytest_al.log; exit 1; }
tail -1 gpurun_out/pytest_al.log
for k in 1 2; do for lib in libndfl.so libndfl_oc0.so libndfl_of32.so libndfl_of192.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bl_$lib$k.log 2>&1 || { tail -20 gpurun_out/bl_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bl_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
for lib in libndfl.so libndfl_oc0.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --size 536870912 --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bls_$lib.log 2>&1 || { tail -20 gpurun_out/bls_$lib.log; exit 1; }
  echo "512M $lib $(grep -h '^{' gpurun_out/bls_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done
echo done
