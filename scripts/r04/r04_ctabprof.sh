#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_ctab
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/on -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $OUT/on.log 2>&1 || { tail -5 $OUT/on.log; exit 1; }
NDFL_NO_CTAB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/off -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $OUT/off.log 2>&1 || { tail -5 $OUT/off.log; exit 1; }
for m in on off; do echo "== $m"; grep ndfl_ $OUT/$m/run_kernel_stats.csv | cut -d, -f1-4; done
