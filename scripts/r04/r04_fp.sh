#!/bin/bash
# Round 4: fixed-Huffman blocks in phase-mapped rounds from their first round -- decoder tests with
# fixed blocks, then config 2 A/B (fp0: switch only after a failing round) with count stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py tests/test_gpu_configs.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fp.log 2>&1 || { tail -40 gpurun_out/pytest_fp.log; exit 1; }
tail -2 gpurun_out/pytest_fp.log
for lib in fp0 fp1 fp0 fp1; do
  NDFL_STATS=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_$lib.so timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_$lib.log 2>&1 || { tail -20 gpurun_out/c2_$lib.log; exit 1; }
  echo "$lib"; grep -E "^\[ndfl\] (count waves|device link)" gpurun_out/c2_$lib.log | tail -2
  grep -h '^{' gpurun_out/c2_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])"
done
