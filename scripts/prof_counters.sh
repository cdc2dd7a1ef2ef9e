#!/bin/bash
# Counter passes (separate --pmc runs; no trace domains mixed in), then a kernel-trace --stats run.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof
mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/prof_inflate.py 1073741824 2 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc1 -o run --output-format csv -- python3 $R/scripts/prof_inflate.py 1073741824 1 > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- python3 $R/scripts/prof_inflate.py 1073741824 1 > $OUT/pmc2.log 2>&1
echo done
