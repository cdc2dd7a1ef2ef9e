#!/bin/bash
# Round profile: kernel trace + stats of the bench command, then HBM traffic counters in separate
# --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_bench
mkdir -p $OUT
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $CMD > $OUT/write.log 2>&1
echo done
