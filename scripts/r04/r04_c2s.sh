#!/bin/bash
# Round 4: config 2 count-pass statistics (device-linked path): chains by outcome and wave time
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NDFL_STATS=1 timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2s.log 2>&1 || { tail -20 gpurun_out/c2s.log; exit 1; }
grep -E "^\[ndfl\]" gpurun_out/c2s.log | tail -8
grep -h '^{' gpurun_out/c2s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])"
