#!/bin/bash
# Round profile: kernel trace + stats of the bench command, then HBM traffic counters in separate
# --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_bench
mkdir -p $OUT
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ARGS > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ARGS > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
echo done
