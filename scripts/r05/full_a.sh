#!/bin/bash
# Round 5: GPU parity suite + default bench line, the round profile (kernel trace + PMC passes),
# then the 8-rank one-GPU rehearsal of the driver's command.
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh || exit 1
bash scripts/profile_bench.sh || exit 1
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/rehearse8.sh || exit 1
