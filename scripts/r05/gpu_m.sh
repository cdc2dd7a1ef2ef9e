#!/bin/bash
# Round 5: small decoder/encoder kernels without serial load waits (candidate compaction as a
# wave-per-segment rank sort; 8 loads in flight in the offsets / segscan / order / emit-order /
# summary kernels): the whole GPU suite, then bench A/B against libndfl_base.so (the previous
# commit) and a kernel-stats profile.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1 || { tail -30 gpurun_out/pytest_m.log; exit 1; }
tail -2 gpurun_out/pytest_m.log
for k in 1 2; do for lib in libndfl.so libndfl_base.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bm_$lib$k.log 2>&1 || { tail -20 gpurun_out/bm_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bm_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_m.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_m.log; exit 1; }
grep -h '"ndfl_' $GRAFT_REPO_ROOT/gpurun_out/prof_m/run_kernel_stats.csv | cut -d, -f1-4
