#!/bin/bash
# Round 5: small single-workgroup kernels with their loads in flight together (clamped indices):
# decoder tests, bench A/B against libndfl_base.so, kernel stats of both.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_headers.py tests/test_gpu_emit_fast.py tests/test_gpu_parallel.py tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 || { tail -30 gpurun_out/pytest_o.log; exit 1; }
tail -2 gpurun_out/pytest_o.log
for k in 1 2; do for lib in libndfl.so libndfl_base.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bo_$lib$k.log 2>&1 || { tail -20 gpurun_out/bo_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bo_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
cd /tmp && export TMPDIR=/tmp
for lib in libndfl.so libndfl_base.so; do
NDFL_LIB_PATH=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_o_$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/prof_o_$lib.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_o_$lib.log; exit 1; }
echo "## $lib"; grep -h '"ndfl_' $GRAFT_REPO_ROOT/gpurun_out/prof_o_$lib/run_kernel_stats.csv | cut -d, -f1-4 | grep "order\|summary\|offsets\|segscan\|compact\|hdr_kernel"
done
