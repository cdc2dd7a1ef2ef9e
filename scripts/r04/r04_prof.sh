#!/bin/bash
# Round-4 profile: kernel trace + stats of the default bench and of config 3.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_r04
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
tail -1 $OUT/c3.log
find $OUT -name "*kernel_stats.csv" | head
