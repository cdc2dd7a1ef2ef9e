#!/bin/bash
# Round-4 evidence run: the whole GPU parity suite, the default bench line, configurations 1/2/3/5.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit 1
bash scripts/r04/r04_configs.sh || exit 1
