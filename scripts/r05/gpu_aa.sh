#!/bin/bash
# Round 5: count-pass wave time against chain bits (NDFL_STATS) at a 512 MiB share and the full 4 GiB bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for size in 536870912 4294967296; do
NDFL_STATS=1 timeout -k 10 300 python -u bench.py --size $size --steps 1 --warmup 1 --no-cpu --no-verify > gpurun_out/baa_$size.log 2>&1 || { tail -20 gpurun_out/baa_$size.log; exit 1; }
echo "== size $size"; grep -h "count bits\|count longest\|count waves" gpurun_out/baa_$size.log | tail -40
done
echo done
