#!/bin/bash
# Round 6: flat groups (count_flat_group) -- their parity tests first, then the whole GPU suite, and
# the bench with the flat groups on and off (NDFL_FLAT=0), twice each, alternating.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -v --timeout 120 --timeout-method thread > $O/pytest_flat.log 2>&1 || { tail -40 $O/pytest_flat.log; exit 1; }
tail -2 $O/pytest_flat.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_on_$i.log 2>&1 || { tail -30 $O/bench_on_$i.log; exit 1; }
  NDFL_FLAT=0 timeout -k 10 400 python -u bench.py > $O/bench_off_$i.log 2>&1 || { tail -30 $O/bench_off_$i.log; exit 1; }
done
for f in $O/bench_*.log; do echo "$(basename $f): $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], p["inflate_find"], p["inflate_count"], p["inflate_emit"], p["inflate_device_span"], d["bit_exact"])')"; done
