#!/bin/bash
# Round 5 evidence (second pass), part 2: configurations 1/2/3/5 and the 8-rank one-GPU rehearsal.
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/configs.sh || exit 1
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/rehearse8.sh || exit 1
echo final-b-ok
