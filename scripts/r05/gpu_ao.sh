#!/bin/bash
# Round 5: fixed-Huffman tables in the stepped literal form (four-literal phase steps reach
# configuration 2's phase-locked fixed-Huffman text): decoder tests, config 2 and the bench against
# the build before (libndfl_base.so).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_count_wg.py tests/test_gpu_emit_fast.py tests/test_gpu_configs.py tests/test_gpu_gzip.py tests/test_gpu_long_codes.py tests/test_gpu_zlib.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ao.log 2>&1 || { tail -30 gpurun_out/pytest_ao.log; exit 1; }
tail -1 gpurun_out/pytest_ao.log
for k in 1 2; do for lib in libndfl.so libndfl_base.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/bo_$lib$k.log 2>&1 || { tail -20 gpurun_out/bo_$lib$k.log; exit 1; }
  echo "c2 $lib $(grep -h '^{' gpurun_out/bo_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])")"
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bob_$lib$k.log 2>&1 || { tail -20 gpurun_out/bob_$lib$k.log; exit 1; }
  echo "bench $lib $(grep -h '^{' gpurun_out/bob_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
echo done
