#!/bin/bash
# Round 5: single-workgroup kernels made multi-workgroup (two-launch tile scans for the encoder offsets
# and the segment counts, two-launch bucket orders, first-error search over tiles): the whole GPU
# suite, then bench A/B against libndfl_base.so (the round-5 code before the small-kernel work)
# and a kernel-stats profile.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { tail -30 gpurun_out/pytest_p.log; exit 1; }
tail -2 gpurun_out/pytest_p.log
for k in 1 2; do for lib in libndfl.so libndfl_base.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bp_$lib$k.log 2>&1 || { tail -20 gpurun_out/bp_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bp_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_p.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_p.log; exit 1; }
grep -h '"ndfl_' $GRAFT_REPO_ROOT/gpurun_out/prof_p/run_kernel_stats.csv | cut -d, -f1-4
