#!/bin/bash
# Config 2 (stored + fixed-Huffman .gz decode) across library builds (lib/ names in LIBS)
cd "$GRAFT_REPO_ROOT"
for L in ${LIBS:-libndfl_cur.so libndfl_ad.so libndfl_f2.so libndfl_s2.so libndfl_f4.so libndfl_p1.so libndfl_base.so}; do
  NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/$L timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_$L.log 2>&1 || { tail -5 gpurun_out/c2_$L.log; exit 1; }
  echo "$L $(grep '^{' gpurun_out/c2_$L.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms"], d["timings"]["inflate_count"], d["timings"]["inflate_emit"], d["timings"]["inflate_find"])')"
done
