#!/bin/bash
# GPU call (round 6, second probe): is the scratch builds' header loss a matter of concurrency?
# sw5inl (spilling) at the full grid twice, then with the strict kernel limited to 1 and 4
# workgroups (NDFL_STRICT_GRID); sw3 (non-inlined call) at the full grid twice; each compared with
# the no-scratch build (sw3inl).
cd "$GRAFT_REPO_ROOT/scripts/r06/strict_probe"
O=$GRAFT_REPO_ROOT/gpurun_out/r06_strict2
mkdir -p $O
run() {  # name lib grid
  NDFL_LIB_PATH=$PWD/r4/deflate-library-java_amd/lib/libndfl_$2.so NDFL_STRICT_PROBE=/tmp/probe_$1.bin env ${3:+NDFL_STRICT_GRID=$3} \
    timeout -k 10 300 python -u probe.py > $O/probe_$1.log 2>&1 || { cat $O/probe_$1.log; exit 1; }
  echo "$1 (grid ${3:-full}): $(tail -1 $O/probe_$1.log)"
}
run good sw3inl "" && run sw5_a sw5inl "" && run sw5_b sw5inl "" && run sw5_g1 sw5inl 1 && run sw5_g4 sw5inl 4 && \
run sw5_g64 sw5inl 64 && run sw3_a sw3 "" && run sw3_b sw3 "" && \
timeout -k 10 300 python -u analyze.py /tmp/probe_good.bin /tmp/probe_sw5_a.bin /tmp/probe_sw5_b.bin /tmp/probe_sw5_g1.bin \
  /tmp/probe_sw5_g4.bin /tmp/probe_sw5_g64.bin /tmp/probe_sw3_a.bin /tmp/probe_sw3_b.bin > $O/analysis.txt && \
grep "==\|accepted\|lost " $O/analysis.txt
