#!/bin/bash
# One-GPU rehearsal of the driver's 8-GPU command: bench.py --gpus 8 starts 8 ranks itself
# (torch.distributed.run), here over gloo on one card (host-staged exchanges, ranks time-sharing
# cuda:0): strong scaling, the whole 4 GiB config-4 corpus, the global stream gathered onto rank 0,
# every shard and the gathered stream compared with the oracle.  A plumbing check, not a scaling
# number (the RCCL run on an 8-GPU node is the driver's).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 20 1000 python -u bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --cpu-sample 268435456 --verify-threads 2 \
  > gpurun_out/rehearse8.log 2>&1 || { tail -40 gpurun_out/rehearse8.log; exit 1; }
tail -1 gpurun_out/rehearse8.log
