#!/bin/bash
# GPU call: the three probe builds on the 4 GiB bench stream, each in its own process, then the
# comparison with the no-scratch build (sw3inl).
cd "$GRAFT_REPO_ROOT/scripts/r06/strict_probe"
O=$GRAFT_REPO_ROOT/gpurun_out/r06_strict
mkdir -p $O
for v in sw3inl sw3 sw5inl; do
  NDFL_LIB_PATH=$PWD/r4/deflate-library-java_amd/lib/libndfl_$v.so NDFL_STRICT_PROBE=/tmp/probe_$v.bin \
    timeout -k 10 300 python -u probe.py > $O/probe_$v.log 2>&1 || { cat $O/probe_$v.log; exit 1; }
  cat $O/probe_$v.log
done
timeout -k 10 300 python -u analyze.py /tmp/probe_sw3inl.bin /tmp/probe_sw3.bin /tmp/probe_sw5inl.bin | tee $O/analysis.txt
