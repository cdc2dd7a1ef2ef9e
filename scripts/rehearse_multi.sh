#!/bin/bash
# One-GPU rehearsal of the multi-GPU bench: 2 ranks time-share cuda:0 over gloo (host-staged
# exchanges), strong scaling (config 4 split over the ranks, gathered onto rank 0).  Not a scaling
# measurement -- the driver runs the RCCL one on an 8-GPU node.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SIZE=${SIZE:-1073741824}
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --scaling strong --size $SIZE --steps 2 --warmup 1 --cpu-sample 268435456 > gpurun_out/rehearse_strong.log 2>&1 || { tail -30 gpurun_out/rehearse_strong.log; exit 1; }
tail -1 gpurun_out/rehearse_strong.log
