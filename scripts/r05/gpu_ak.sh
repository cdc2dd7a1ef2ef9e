#!/bin/bash
# Round 5: fast emit pass with two token-loop instances (four-literal steps only in blocks of mostly
# 8-bit codes; libndfl.so) against no four-literal step (libndfl_ej0.so).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_emit_fast.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ak.log 2>&1 || { tail -30 gpurun_out/pytest_ak.log; exit 1; }
tail -1 gpurun_out/pytest_ak.log
for k in 1 2; do for lib in libndfl.so libndfl_ej0.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bk_$lib$k.log 2>&1 || { tail -20 gpurun_out/bk_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bk_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
for lib in libndfl.so libndfl_ej0.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u scripts/prof_types.py 1073741824 random,text > gpurun_out/bkt_$lib.log 2>&1 || { tail -20 gpurun_out/bkt_$lib.log; exit 1; }
  echo "== $lib"; grep ratio gpurun_out/bkt_$lib.log | cut -c1-120
done
echo done
