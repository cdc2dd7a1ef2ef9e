#!/bin/bash
# Round 6: flat groups without cursor loads in the loop, escape entry read early: parity, group time,
# 4 GiB on/off, and a 512 MiB share (one rank at 8 GPUs: flat groups gated off by NDFL_FLAT_MIN).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_emit_fast.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
NDFL_FLAT_MIN=0 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_fprof.so NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 > $O/fprof.log 2>&1 || { tail -30 $O/fprof.log; exit 1; }
grep "flat=\|flat groups\|flat decode" $O/fprof.log
timeout -k 10 300 python -u scripts/r06/flat_probe.py 4096 1 0 > $O/probe4g.log 2>&1 || { tail -30 $O/probe4g.log; exit 1; }
grep flat= $O/probe4g.log
timeout -k 10 300 python -u scripts/r06/flat_probe.py 512 1 > $O/probe512.log 2>&1 || { tail -30 $O/probe512.log; exit 1; }
grep flat= $O/probe512.log
