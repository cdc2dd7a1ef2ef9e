#!/bin/bash
# Round 4: sparse finder windows (NDFL_FIND_WIN of every NDFL_FIND_PERIOD input words scanned; chains
# then decode on through the blocks that start outside the windows) against the dense scan.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/ab_env.sh "NDFL_COUNT_W=1" "NDFL_FIND_WIN=8192 NDFL_FIND_PERIOD=16384" "NDFL_FIND_WIN=4096 NDFL_FIND_PERIOD=8192" \
  "NDFL_FIND_WIN=2048 NDFL_FIND_PERIOD=4096" "NDFL_FIND_WIN=16384 NDFL_FIND_PERIOD=32768" "NDFL_FIND_WIN=4096 NDFL_FIND_PERIOD=16384" \
  "NDFL_FIND_WIN=8192 NDFL_FIND_PERIOD=12288"
