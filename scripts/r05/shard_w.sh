#!/bin/bash
# Round 5: the count pass's width on one rank's share at 8 GPUs (512 MiB of config 4: ~8 K single-
# block chains, fewer than 4 per count wave, so the automatic rule picks 4 waves per chain):
# automatic vs NDFL_COUNT_W=1 vs 4, and the same at 1 GiB (4 GPUs) and 2 GiB (2 GPUs).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for sz in 536870912 1073741824 2147483648; do
  for w in auto 1 4; do
    if [ $w = auto ]; then E=""; else E="NDFL_COUNT_W=$w"; fi
    env $E timeout -k 10 300 python -u bench.py --size $sz --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/sw_${sz}_$w.log 2>&1 || { tail -20 gpurun_out/sw_${sz}_$w.log; exit 1; }
    echo "size $sz W=$w $(grep -h '^{' gpurun_out/sw_${sz}_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print(d['ms_per_step'], 'count', p['inflate_count'], 'emit', p['inflate_emit'], 'span', p['inflate_device_span'], 'chains', p['inflate_chains'])")"
  done
done
