#!/bin/bash
# GPU call (round 6, third probe): the spilling build (sw5inl) with the strict kernel at 1, 2, 3 and
# 4 workgroups of 256 per CU (256 CUs): at which co-residency does the loss begin?
cd "$GRAFT_REPO_ROOT/scripts/r06/strict_probe"
O=$GRAFT_REPO_ROOT/gpurun_out/r06_strict3
mkdir -p $O
run() {  # name lib grid
  NDFL_LIB_PATH=$PWD/r4/deflate-library-java_amd/lib/libndfl_$2.so NDFL_STRICT_PROBE=/tmp/probe_$1.bin env ${3:+NDFL_STRICT_GRID=$3} \
    timeout -k 10 300 python -u probe.py > $O/probe_$1.log 2>&1 || { cat $O/probe_$1.log; exit 1; }
  echo "$1 (grid ${3:-full}): $(tail -1 $O/probe_$1.log)"
}
run good sw3inl "" && run sw5_g256 sw5inl 256 && run sw5_g512 sw5inl 512 && run sw5_g768 sw5inl 768 && \
run sw5_g1024 sw5inl 1024 && run sw5_g128 sw5inl 128 && \
timeout -k 10 300 python -u analyze.py /tmp/probe_good.bin /tmp/probe_sw5_g128.bin /tmp/probe_sw5_g256.bin \
  /tmp/probe_sw5_g512.bin /tmp/probe_sw5_g768.bin /tmp/probe_sw5_g1024.bin > $O/analysis.txt && \
grep "==\|accepted\|lost " $O/analysis.txt
