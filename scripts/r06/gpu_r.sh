#!/bin/bash
# Round 6: instruction-cache and wait counters of the count pass (1 GiB decode, flat groups on), one
# pass per counter group.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/scripts/r06/flat_probe.py
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $O/ic -o run --output-format csv -- python3 -u $P 1024 1 > $O/ic.log 2>&1 || { tail -20 $O/ic.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/wt -o run --output-format csv -- python3 -u $P 1024 1 > $O/wt.log 2>&1 || { tail -20 $O/wt.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r06r"
for d in ("ic", "wt"):
    f = glob.glob(f"{O}/{d}/**/run_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "ndfl_inflate_count" in k or "emit_fast" in k or "find_compact" in k:
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(d, k, {c: f"{x:.3g}" for c, x in v.items()})
PY
