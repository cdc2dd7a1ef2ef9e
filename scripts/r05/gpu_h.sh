#!/bin/bash
# Round 5: fast emit pass with the extension areas (codes longer than the primary tables) in LDS
# (-DNDFL_EMITF_GX=0; 4 and 3 waves/SIMD) vs the default (extension areas read from the table
# record in global memory): emit parity for the variant, then bench A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
NDFL_LIB_PATH=$L/libndfl_gx0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_long_codes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1 || { tail -30 gpurun_out/pytest_h.log; exit 1; }
tail -2 gpurun_out/pytest_h.log
for k in 1 2; do for lib in libndfl.so libndfl_gx0.so libndfl_gx0w3.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bh_$lib$k.log 2>&1 || { tail -20 gpurun_out/bh_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bh_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
