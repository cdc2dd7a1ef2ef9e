#!/bin/bash
# Full GPU parity suite on the default build, then an A/B of builds on the default bench.
cd "$GRAFT_REPO_ROOT"
SKIP_BENCH=1 bash scripts/gpu_tests.sh || exit 1
bash scripts/ab_libs.sh "$@"
