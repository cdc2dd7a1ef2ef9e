#!/bin/bash
# Round 6: the phased round with one copy of its run-group code (74 -> 28 KB): parity + 4 GiB on/off;
# and the counter list (instruction cache counters).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_emit_fast.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/r06/flat_probe.py 4096 1 0 > $O/probe4g.log 2>&1 || { tail -30 $O/probe4g.log; exit 1; }
grep flat= $O/probe4g.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -20 $O/counters.txt; exit 1; }
grep -i "icache\|SQ_WAIT_INST\|IFETCH\|SQ_INSTS_VALU\b\|SQC_" $O/counters.txt | head -40
