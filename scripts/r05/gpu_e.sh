#!/bin/bash
# Round 5: the count-width rule at one rank's 8-GPU share (auto must now equal W=1), the workgroup
# count tests, then configurations 1, 2, 3 and 5.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --size 536870912 --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/se_auto.log 2>&1 || { tail -20 gpurun_out/se_auto.log; exit 1; }
echo "size 536870912 W=auto(r5) $(grep -h '^{' gpurun_out/se_auto.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print(d['ms_per_step'], 'count', p['inflate_count'], 'emit', p['inflate_emit'], 'span', p['inflate_device_span'], 'chains', p['inflate_chains'])")"
timeout -k 10 600 python -u -m pytest tests/test_gpu_count_wg.py tests/test_gpu_headers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { tail -30 gpurun_out/pytest_e.log; exit 1; }
tail -2 gpurun_out/pytest_e.log
bash scripts/r05/configs.sh
