#!/bin/bash
# Round 6: the table build in isolation (scripts/r06/build_bench.hip) -- reference build, and any
# variant binaries present (build_bench_<name>), each checked against the reference's tables.
cd "$GRAFT_REPO_ROOT/scripts/r06"
O=$GRAFT_REPO_ROOT/gpurun_out/r06d
mkdir -p $O
timeout -k 10 120 ./build_bench_ref hdrs.bin $O/ref_dump.bin > $O/ref.log 2>&1 || { cat $O/ref.log; exit 1; }
cat $O/ref.log
for b in build_bench_v*; do
  [ -x "$b" ] || continue
  echo "== $b"
  timeout -k 10 120 ./$b hdrs.bin $O/${b}_dump.bin $O/ref_dump.bin > $O/$b.log 2>&1; rc=$?
  cat $O/$b.log
  [ $rc -le 1 ] || exit 1
done
echo ok
