#!/bin/bash
# GPU tests + 2-rank rehearsal of the sharded bench on one GPU (gloo) + N=1 bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --size 1073741824 --backend gloo --no-cpu \
    > gpurun_out/bench2.log 2>&1 || { tail -30 gpurun_out/bench2.log; exit 1; }
tail -2 gpurun_out/bench2.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -2 gpurun_out/bench1.log
