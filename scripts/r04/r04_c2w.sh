#!/bin/bash
# Config 2 (stored + fixed-Huffman: long chains, the finder sees no fixed headers) by count-pass width
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_emit_fast.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2w.log 2>&1 || { tail -30 gpurun_out/pytest_c2w.log; exit 1; }
tail -1 gpurun_out/pytest_c2w.log
for W in 1 2 4 8; do
  NDFL_COUNT_W=$W timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/c2_w$W.log 2>&1 || { tail -20 gpurun_out/c2_w$W.log; exit 1; }
  echo "W=$W $(grep -h '^{' gpurun_out/c2_w$W.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['bit_exact'], d['timings'])")"
done
