#!/bin/bash
# Round profile of the default bench: kernel trace + stats, then HBM traffic (FETCH_SIZE, WRITE_SIZE)
# and SQ issue/wait counters, each in its own --pmc pass (FETCH_SIZE and WRITE_SIZE do not fit one
# TCC pass on gfx950; no trace domain is mixed with --pmc).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_bench
mkdir -p $OUT
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ARGS > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ARGS > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/sq1 -o run --output-format csv -- python3 $ARGS > $OUT/sq1.log 2>&1 || { tail -20 $OUT/sq1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 $ARGS > $OUT/sq2.log 2>&1 || { tail -20 $OUT/sq2.log; exit 1; }
echo done
