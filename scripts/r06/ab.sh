#!/bin/bash
# A/B of library variants on the default bench (4 GiB), alternating: scripts/r06/ab.sh OUT name1 name2 ...
# (name "head" = lib/libndfl.so, others lib/libndfl_<name>.so), 2 alternations, 5 steps each.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = head ]; then L=$PWD/deflate-library-java_amd/lib/libndfl.so; else L=$PWD/deflate-library-java_amd/lib/libndfl_$v.so; fi
    NDFL_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-verify > $O/b_${v}_$rep.log 2>&1 || { tail -20 $O/b_${v}_$rep.log; exit 1; }
    echo "$v $(grep -h '^{' $O/b_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print(d['ms_per_step'], {k: p[k] for k in ('deflate_kernel','inflate_find','inflate_count','inflate_emit','inflate_device_span')})")"
  done
done
