#!/bin/bash
# A/B of runtime knobs on the default bench: bash scripts/ab_env.sh "VAR=1 VAR2=2" "VAR=3" ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/abenv_$i.log 2>&1 || { tail -20 gpurun_out/abenv_$i.log; exit 1; }
  echo "[$envs] $(python -c "import json; d=json.loads(open('gpurun_out/abenv_$i.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phases_ms'])")"
done
