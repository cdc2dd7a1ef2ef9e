#!/bin/bash
# Round 5: phase runs stepping four 8-bit literals at once (libndfl.so) vs one (libndfl_nj.so), G=4 (libndfl_g4.so) plus
# NDFL_PH_FALLBACK lanes failed to synchronise or after NDFL_PH_FRONTIER frontier misses; variants
# (lib/libndfl_<v>.so) against the default: 4 GiB bench, binary-only count pass, configuration 2.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/deflate-library-java_amd/lib
for k in 1 2; do for lib in libndfl.so libndfl_g1.so; do
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/bc_$lib$k.log 2>&1 || { tail -20 gpurun_out/bc_$lib$k.log; exit 1; }
  echo "$lib $(grep -h '^{' gpurun_out/bc_$lib$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])")"
done; done
for lib in libndfl.so libndfl_g1.so; do
  echo "== $lib types"
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u scripts/prof_types.py 1073741824 random,binary,text > gpurun_out/bct_$lib.log 2>&1 || { tail -20 gpurun_out/bct_$lib.log; exit 1; }
  cut -c1-200 gpurun_out/bct_$lib.log
  echo "== $lib c2"
  NDFL_LIB_PATH=$L/$lib timeout -k 10 300 python -u scripts/bench_configs.py c2 > gpurun_out/bcc_$lib.log 2>&1 || { tail -20 gpurun_out/bcc_$lib.log; exit 1; }
  grep -h '^{' gpurun_out/bcc_$lib.log | cut -c1-300
done
echo done
