#!/bin/bash
# Round 5: does the count pass's WRITE_SIZE come from register spills?  WRITE_SIZE of
# the default build (3 waves/SIMD: 240 B/lane of spills) vs a 2-waves/SIMD build (256 VGPRs, no
# VGPR spill), one --pmc pass each over bench.py --steps 2 --warmup 1.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/deflate-library-java_amd/lib
OUT=$R/gpurun_out/count_writes
mkdir -p $OUT
ARGS="$R/bench.py --steps 2 --warmup 1 --no-cpu --no-verify"
for lib in libndfl.so libndfl_cw2.so; do
  NDFL_LIB_PATH=$L/$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$lib -o run --output-format csv -- python3 $ARGS > $OUT/w_$lib.log 2>&1 || { tail -20 $OUT/w_$lib.log; exit 1; }
  grep -h '^{' $OUT/w_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], d['phases_ms']['inflate_count'])"
done
python3 - <<'PY'
import csv, glob, os
R = os.environ["GRAFT_REPO_ROOT"]
for lib in ("libndfl.so", "libndfl_cw2.so"):
    fs = glob.glob(f"{R}/gpurun_out/count_writes/w_{lib}/**/*counter_collection*.csv", recursive=True)
    tot = {}; n = {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
            if "count_wave" not in k and "emit_fast" not in k: continue
            v = float(r.get("Counter_Value", r.get("Counter-Value", 0)))
            key = (k.split("(")[0], r.get("Dispatch_Id", r.get("Dispatch-Id")))
            tot[key] = tot.get(key, 0) + v
    per = {}
    for (k, d), v in tot.items(): per.setdefault(k, []).append(v)
    for k, vs in per.items(): print(lib, k, "launches", len(vs), "WRITE_SIZE per launch (raw counter)", sum(vs) / len(vs))
PY
