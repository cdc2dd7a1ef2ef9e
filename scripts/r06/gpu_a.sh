#!/bin/bash
# Round 6, first GPU call: the parity suite on the new tests (reserved symbols, tail maps, small
# shards), the default bench line, and the FETCH_SIZE / WRITE_SIZE calibration on known byte counts.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "reserved_symbol_in_the_message or tail_map_composes or small_shards_one_gpu or known_answer" \
  > gpurun_out/r06a/pytest_new.log 2>&1 || { tail -40 gpurun_out/r06a/pytest_new.log; exit 1; }
tail -3 gpurun_out/r06a/pytest_new.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06a/bench.log 2>&1 || { tail -30 gpurun_out/r06a/bench.log; exit 1; }
tail -1 gpurun_out/r06a/bench.log
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/scripts/r06/fetch_calib
O=$GRAFT_REPO_ROOT/gpurun_out/r06a
timeout -k 10 120 $B > $O/calib_plain.log 2>&1 || { cat $O/calib_plain.log; exit 1; }
cat $O/calib_plain.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cf -o run --output-format csv -- $B > $O/calib_fetch.log 2>&1 || { tail $O/calib_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cw -o run --output-format csv -- $B > $O/calib_write.log 2>&1 || { tail $O/calib_write.log; exit 1; }
echo calib-ok
