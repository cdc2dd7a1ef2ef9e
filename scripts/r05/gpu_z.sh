#!/bin/bash
# Round 5: split count pass (long chains by four waves first, then the rest by one wave) against
# the one-wave pass, at one rank's 8-GPU (512 MiB) and 4-GPU (1 GiB) shares; NDFL_COUNT_SPLIT = the
# long-chain threshold in 32 Kibit (0: off).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for size in 536870912 1073741824; do
for t in 0 12 0 8 16 12; do
NDFL_COUNT_SPLIT=$t timeout -k 10 300 python -u bench.py --size $size --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bz_${size}_$t.log 2>&1 || { tail -20 gpurun_out/bz_${size}_$t.log; exit 1; }
echo -n "size $size split $t: "
grep -h '^{' gpurun_out/bz_${size}_$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
done
done
NDFL_COUNT_SPLIT=12 NDFL_STATS=1 timeout -k 10 300 python -u bench.py --size 536870912 --steps 2 --warmup 1 --no-cpu > gpurun_out/bz_stats.log 2>&1 || { tail -20 gpurun_out/bz_stats.log; exit 1; }
grep -h "count chains\|count waves\|count pass:" gpurun_out/bz_stats.log | tail -5
grep -h '^{' gpurun_out/bz_stats.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['phases_ms'])"
echo done
