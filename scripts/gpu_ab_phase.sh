#!/bin/bash
# A/B of decoder builds on the default bench and on config 2 (phase-locked fixed-Huffman text)
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_configs.py tests/test_gpu_long_codes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_inf.log 2>&1 && tail -2 gpurun_out/t_inf.log || { tail -30 gpurun_out/t_inf.log; exit 1; }
bash scripts/ab_libs.sh "$@" || exit 1
for l in "$@"; do
  NDFL_LIB_PATH=$GRAFT_REPO_ROOT/deflate-library-java_amd/lib/$l timeout -k 10 200 python -u scripts/bench_configs.py c2 > gpurun_out/c2_$l.log 2>&1 || exit 1
  echo "c2 $l $(python -c "import json; d=json.loads(open('gpurun_out/c2_$l.log').read().strip().splitlines()[-1]); print(d['ms'], round(d['timings']['inflate_count'],3))")"
done
