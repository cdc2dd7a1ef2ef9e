#!/bin/bash
# Counter passes of the decoder (1 GiB config-4 corpus): separate --pmc runs, no trace domains mixed in.
# SQ_* cycle counters count quad-cycles; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_ctr
mkdir -p $OUT
P="python3 $R/scripts/prof_inflate.py 1073741824 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc1 -o run --output-format csv -- $P > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- $P > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; }
echo counters done
