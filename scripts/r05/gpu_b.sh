#!/bin/bash
# Round 5: count-pass phase clocks and strict-stage counters on the config-4 mix (NDFL_STATS, a
# -DNDFL_PHASE_CLOCK build), then the 8-rank one-GPU rehearsal of the driver's command.
cd "$GRAFT_REPO_ROOT"
bash scripts/mix_stats.sh libndfl_pc.so || exit 1
bash scripts/r05/rehearse8.sh || exit 1
