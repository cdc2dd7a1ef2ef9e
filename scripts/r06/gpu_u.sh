#!/bin/bash
# Round 6: SQ counters of the count pass when it is nearly all flat groups (256 MiB of random bytes,
# one wave per chain, flat groups at any size).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/scripts/r06/flat_probe.py
export NDFL_COUNT_W=1 NDFL_FLAT_MIN=0 PROBE_DATA=random
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $O/a -o run --output-format csv -- python3 -u $P 256 1 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d $O/b -o run --output-format csv -- python3 -u $P 256 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/summarize_sq.py $O/a/run_counter_collection.csv $O/b/run_counter_collection.csv | grep -A20 count_wave
cd $GRAFT_REPO_ROOT
unset NDFL_COUNT_W NDFL_FLAT_MIN PROBE_DATA
NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 4096 1 > $O/stats4g.log 2>&1 || { tail -20 $O/stats4g.log; exit 1; }
grep "flat=\|flat groups\|count waves" $O/stats4g.log
