#!/bin/bash
# Config 3 (FULL_DYNAMIC LZ77, 1 GiB text): LZ match statistics, kernel trace + stats, and one SQ
# counter pass (LDS issue / bank conflicts / waits) -- each rocprofv3 pass its own run.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c3prof
mkdir -p $OUT
cd $R
NDFL_LZ_STATS=1 timeout -k 10 300 python3 scripts/bench_configs.py c3 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
tail -3 $OUT/stats.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -5
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/sq1 -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/sq1.log 2>&1 || { tail -20 $OUT/sq1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $OUT/sq2.log 2>&1 || { tail -20 $OUT/sq2.log; exit 1; }
echo done
