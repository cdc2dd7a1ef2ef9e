#!/bin/bash
# Round 6: the new table build in the library -- GPU parity suite, A/B against the old build, count
# phase clocks.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -40 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
bash scripts/r06/ab.sh r06e head b0 || exit 1
NDFL_STATS=1 NDFL_LIB_PATH=$PWD/deflate-library-java_amd/lib/libndfl_pc.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify > gpurun_out/r06e/pc.log 2>&1 || { tail -20 gpurun_out/r06e/pc.log; exit 1; }
grep -E "wave-time|count waves" gpurun_out/r06e/pc.log | tail -2
