#!/bin/bash
# Round 5: the count pass's tail at one rank's 8-GPU share (512 MiB): chain wave times (NDFL_STATS),
# widths 1 and 4.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in 1 4; do
NDFL_COUNT_W=$w NDFL_STATS=1 timeout -k 10 300 python -u bench.py --size 536870912 --steps 2 --warmup 1 --no-cpu --no-verify > gpurun_out/by_w$w.log 2>&1 || { tail -20 gpurun_out/by_w$w.log; exit 1; }
echo "== W=$w"; grep -h "count chains\|count waves\|count pass:" gpurun_out/by_w$w.log | tail -5
grep -h '^{' gpurun_out/by_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
done
