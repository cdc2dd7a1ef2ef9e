#!/bin/bash
# Round 5: finder Kraft test by ten lookups of a 64-entry two-length table (one entry per LDS bank,
# no conflicts) vs five lookups of the 4,096-entry four-length table (libndfl_kr4.so): header-set
# parity, the bench stream's accepted set, bench A/B (+ libndfl_base.so: the previous commit).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_headers.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 || { tail -30 gpurun_out/pytest_n.log; exit 1; }
tail -2 gpurun_out/pytest_n.log
timeout -k 10 600 python -u scripts/r05/headers_ab.py $L/libndfl.so > gpurun_out/hab_n.log 2>&1 || { tail -20 gpurun_out/hab_n.log; exit 1; }
grep -h '^{' gpurun_out/hab_n.log | cut -c1-200
for k in 1 2; do for lib in libndfl.so libndfl_kr4.so libndfl_base.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bn_$lib$k.log 2>&1 || { tail -20 gpurun_out/bn_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bn_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
