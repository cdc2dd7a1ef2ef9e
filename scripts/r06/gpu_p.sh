#!/bin/bash
# Round 6: the counters this gfx950 exposes (instruction cache and wait counters for the count pass).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -20 $O/counters.txt; exit 1; }
grep -i "icache\|SQ_WAIT\|SQ_INST_CYCLES\|IFETCH\|SQ_BUSY\|SQC_" $O/counters.txt | head -60
