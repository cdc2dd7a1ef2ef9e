#!/bin/bash
# Partitioned finder A/B: partition length (NDFL_FIND_PART_BITS; 0 = every position) vs the count /
# emit passes, with the decoder's NDFL_STATS lines (wave occupancy, chains, rounds).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abparts
mkdir -p $OUT
for pb in ${PARTS:-0 default 524288 1048576 2097152}; do
  if [ "$pb" = default ]; then unset NDFL_FIND_PART_BITS; else export NDFL_FIND_PART_BITS=$pb; fi
  NDFL_STATS=${STATS:-1} timeout -k 10 300 python -u bench.py --no-cpu --steps ${STEPS:-1} --warmup 1 > $OUT/p$pb.log 2>&1 || { tail -20 $OUT/p$pb.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/p$pb.log') if l.startswith('{')][-1])
print('part=$pb', d['ms_per_step'], json.dumps(d['phases_ms']))"
  grep "\[ndfl\]" $OUT/p$pb.log | tail -6
done
