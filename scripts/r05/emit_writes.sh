#!/bin/bash
# Round 5: does the emit pass's WRITE_SIZE (3.6 x its output bytes) come from partly written lines
# leaving L2?  WRITE_SIZE of the fast emit kernel at 4 / 8 / 16 waves per CU (NDFL_EMITF_WPC: the
# persistent grid's size): fewer resident waves keep fewer lines open at once.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/emitw
mkdir -p $OUT
for wpc in 4 8 16; do
  NDFL_EMITF_WPC=$wpc timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/w$wpc -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/w$wpc.log 2>&1 || { tail -20 $OUT/w$wpc.log; exit 1; }
  python3 - $OUT/w$wpc/run_counter_collection.csv $wpc <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); d = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("ndfl_inflate_emit_fast"):
        tot[k] += float(r["Counter_Value"]); d[k].add(r["Dispatch_Id"])
for k, v in tot.items():
    print(f"waves/CU {sys.argv[2]}: {k} WRITE_SIZE per launch {v * 1024 / max(1, len(d[k])) / 1e9:.2f} GB ({len(d[k])} launches)")
PY
  tail -1 $OUT/w$wpc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  emit ms', d['phases_ms']['inflate_emit'])"
done
