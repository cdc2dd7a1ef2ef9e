#!/bin/bash
# Round 6: flat groups with the LDS input ring -- parity tests, then the 1 GiB probe (stats, flat on/off).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_emit_fast.py -x -q --timeout 120 --timeout-method thread > $O/pytest_flat.log 2>&1 || { tail -40 $O/pytest_flat.log; exit 1; }
tail -1 $O/pytest_flat.log
NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 0 > $O/stats.log 2>&1 || { tail -30 $O/stats.log; exit 1; }
grep "flat=\|fast emit\|count waves" $O/stats.log
timeout -k 10 300 python -u scripts/r06/flat_probe.py 4096 1 0 > $O/probe4g.log 2>&1 || { tail -30 $O/probe4g.log; exit 1; }
cat $O/probe4g.log | grep flat=
