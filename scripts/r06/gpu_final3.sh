#!/bin/bash
# Round 6 evidence (final pass): the whole GPU parity suite, the default bench line, then the bench
# under rocprofv3 -- kernel trace + stats, FETCH_SIZE, WRITE_SIZE and two SQ counter passes, each its
# own run (scripts/profile_bench.sh) -- into gpurun_out/r06_final3.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06_final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 1000 bash scripts/profile_bench.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
cp -r gpurun_out/prof_bench $O/ && echo profiled
