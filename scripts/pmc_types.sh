#!/bin/bash
# SQ counter passes over the per-type decode driver (one counter group per run, no trace domains).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmct
mkdir -p $OUT
T=${1:-text}
i=0
for grp in "SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
           "SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/scripts/prof_types.py 268435456 $T > $OUT/p$i.log 2>&1 || exit 1
done
echo done
