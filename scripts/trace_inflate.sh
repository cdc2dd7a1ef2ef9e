#!/bin/bash
# Kernel trace + stats of the 1 GiB decode driver.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace -o run --output-format csv -- python3 $R/scripts/prof_inflate.py ${1:-1073741824} 2 > $R/gpurun_out/prof/trace.log 2>&1
