#!/bin/bash
# Round 5 closing check: smoke() and the default bench line on the committed build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_am.log 2>&1 || { tail -20 gpurun_out/smoke_am.log; exit 1; }
tail -2 gpurun_out/smoke_am.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_am.log 2>&1 || { tail -20 gpurun_out/bench_am.log; exit 1; }
grep -h '^{' gpurun_out/bench_am.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['bit_exact'], d['roofline']['frac'], d['phases_ms'])"
echo done
