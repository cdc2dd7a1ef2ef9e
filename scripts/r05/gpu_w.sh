#!/bin/bash
# Round 5: finder words of the next word step loaded while the current one is scanned (unconditional,
# clamped into the padding): header-set parity and determinism, decoder tests, bench A/B
# against libndfl_head.so (the previous commit).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_headers.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1 || { tail -30 gpurun_out/pytest_w.log; exit 1; }
tail -2 gpurun_out/pytest_w.log
timeout -k 10 600 python -u scripts/r05/headers_ab.py $L/libndfl.so $L/libndfl_head.so > gpurun_out/hab_w.log 2>&1 || { tail -20 gpurun_out/hab_w.log; exit 1; }
grep -h '^{' gpurun_out/hab_w.log | cut -c1-200
for k in 1 2 3; do for lib in libndfl.so libndfl_head.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bw_$lib$k.log 2>&1 || { tail -20 gpurun_out/bw_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bw_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms']['inflate_find'])")"
done; done
