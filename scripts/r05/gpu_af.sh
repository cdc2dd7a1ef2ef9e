#!/bin/bash
# Round 5: decoder GPU tests after the count-pass synchronisation changes, then the bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_emit_fast.py tests/test_gpu_count_wg.py tests/test_gpu_long_codes.py tests/test_gpu_configs.py tests/test_gpu_headers.py tests/test_gpu_parallel.py tests/test_gpu_zlib.py tests/test_gpu_gzip.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_af.log 2>&1 || { tail -30 gpurun_out/pytest_af.log; exit 1; }
tail -2 gpurun_out/pytest_af.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_af.log 2>&1 || { tail -20 gpurun_out/bench_af.log; exit 1; }
grep -h '^{' gpurun_out/bench_af.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('bit_exact'), d['phases_ms'])"
echo done
