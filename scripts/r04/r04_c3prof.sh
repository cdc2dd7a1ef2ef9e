#!/bin/bash
# Config 3 kernel stats, parse-driven search (default) and the round-3 chain search
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_c3
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/parse -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/parse.log 2>&1 || { tail -20 $OUT/parse.log; exit 1; }
NDFL_LZ_SEARCH=chain timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/chain -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/chain.log 2>&1 || { tail -20 $OUT/chain.log; exit 1; }
for m in parse chain; do echo "== $m"; grep ndfl_lz $OUT/$m/run_kernel_stats.csv | cut -d, -f1-4; done
