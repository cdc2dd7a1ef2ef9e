#!/bin/bash
# Round 5 evidence (second pass, after the count-pass synchronisation changes), part 1: GPU parity
# suite + default bench line, then the round profile (kernel trace + FETCH/WRITE/SQ passes).
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh || exit 1
bash scripts/profile_bench.sh || exit 1
echo final-a-ok
