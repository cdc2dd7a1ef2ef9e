#!/bin/bash
# Round 5: the next round's input touched into L2 after each round's staging (LDS-DMA into a scratch
# row) vs -DNDFL_STAGE_TOUCH=0: decoder tests, bench A/B, kernel stats.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py tests/test_gpu_parallel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1 || { tail -30 gpurun_out/pytest_u.log; exit 1; }
tail -2 gpurun_out/pytest_u.log
for k in 1 2 3; do for lib in libndfl.so libndfl_notouch.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bu_$lib$k.log 2>&1 || { tail -20 gpurun_out/bu_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bu_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
