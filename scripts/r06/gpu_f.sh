#!/bin/bash
# Round 6: the strict-probe co-residency sweep, the whole GPU parity suite (with the emit-side
# segment check), one bench line, and the FETCH_SIZE calibration of the corrected byte-line kernel.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06f
mkdir -p $O
bash scripts/r06/strict_probe/gpu_probe3.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/scripts/r06/fetch_calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cf -o run --output-format csv -- $B > $O/calib_fetch.log 2>&1 || { tail $O/calib_fetch.log; exit 1; }
echo calib-ok
