#!/bin/bash
# Timing experiments: encoder kernels under NDFL_DBG variants (outputs are not valid for dbg != 0).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for d in ${DBGS:-0 1 2 16 4 8}; do
  NDFL_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dbg_$d -o run --output-format csv -- python3 $R/scripts/perf_deflate.py c4:4096 > $R/gpurun_out/dbg_$d.log 2>&1 || { tail -20 $R/gpurun_out/dbg_$d.log; exit 1; }
  echo "dbg=$d"; grep -E "ndfl_" $R/gpurun_out/dbg_$d/run_kernel_stats.csv | cut -d, -f1,4
done
