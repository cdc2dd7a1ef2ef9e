#!/bin/bash
# Round 5: strict stage with the wave-wide window reader + encoder emit (two codes per put):
# header-set parity, decode/encode GPU tests, the bench stream's accepted set (3 runs), then the
# finder-phase and encoder A/B against libndfl_emit0.so (round-5 code before both changes).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_headers.py tests/test_gpu_inflate.py tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 || { tail -30 gpurun_out/pytest_g.log; exit 1; }
tail -2 gpurun_out/pytest_g.log
timeout -k 10 600 python -u scripts/r05/headers_ab.py $L/libndfl.so > gpurun_out/hab_g.log 2>&1 || { tail -20 gpurun_out/hab_g.log; exit 1; }
grep -h '^{' gpurun_out/hab_g.log | cut -c1-300
for k in 1 2; do for lib in libndfl.so libndfl_emit0.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bg_$lib$k.log 2>&1 || { tail -20 gpurun_out/bg_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bg_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > gpurun_out/bg_stats.log 2>&1 || { tail -20 gpurun_out/bg_stats.log; exit 1; }
grep -h "strict stage" gpurun_out/bg_stats.log | head -3
