#!/bin/bash
# A/B of library builds on the default bench, each with a WRITE_SIZE pass (count / emit write bytes):
#   bash scripts/ab_w16.sh base.so phreg.so w16.so ...   (files under deflate-library-java_amd/lib)
# The bench runs verify the whole stream (bit_exact), so a build that decodes wrong fails here.
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/abw
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for lib in "$@"; do
  L=$R/deflate-library-java_amd/lib/$lib
  NDFL_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > $OUT/$lib.log 2>&1 || { tail -20 $OUT/$lib.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/$lib.log') if l.startswith('{')][-1])
print('$lib', d['ms_per_step'], d['cpu_baseline'].get('bit_exact') if d.get('cpu_baseline') else d.get('bit_exact'), json.dumps(d['phases_ms']))"
  (cd /tmp && export TMPDIR=/tmp && NDFL_LIB_PATH=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$lib -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-verify > $OUT/w_$lib.log 2>&1) || { tail -20 $OUT/w_$lib.log; exit 1; }
  python3 - <<EOF
import csv, collections, glob
f = glob.glob("$OUT/w_$lib/**/run_counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("ndfl_inflate_count") or k.startswith("ndfl_inflate_emit"):
        tot[k] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k in sorted(tot):
    print("   $lib", k, "write GB/launch %.3f" % (tot[k] * 1024 / len(n[k]) / 1e9))
EOF
done
