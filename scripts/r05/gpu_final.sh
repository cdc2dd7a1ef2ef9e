#!/bin/bash
# Round 5 evidence run with the final code: GPU parity suite + default bench line, the round profile
# (kernel trace + FETCH/WRITE/SQ passes), configurations 1/2/3/5, the 8-rank one-GPU rehearsal.
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh || exit 1
bash scripts/profile_bench.sh || exit 1
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/configs.sh || exit 1
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/rehearse8.sh || exit 1
echo final-ok
