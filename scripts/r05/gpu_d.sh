#!/bin/bash
# Round 5: the emit pass without its output stores (-DNDFL_EMIT_NOSTORE: the decode part), the count
# pass's width on one rank's share at 2/4/8 GPUs, then the 8-rank one-GPU rehearsal.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
for k in 1 2; do for lib in libndfl.so libndfl_nostore.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-verify > gpurun_out/bd_$lib$k.log 2>&1 || { tail -20 gpurun_out/bd_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bd_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
bash scripts/r05/shard_w.sh || exit 1
bash scripts/r05/rehearse8.sh || exit 1
