#!/bin/bash
# Round 6: why the emit pass slows with the flat groups: stats and kernel trace, flat on and off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06i
mkdir -p $O
NDFL_STATS=1 timeout -k 10 300 python -u scripts/r06/flat_probe.py 1024 1 0 > $O/stats.log 2>&1 || { tail -30 $O/stats.log; exit 1; }
grep "flat=\|fast emit\|count chains\|count waves\|emit:" $O/stats.log
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  NDFL_FLAT=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$f -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/scripts/r06/flat_probe.py 1024 $f > $O/prof_$f.log 2>&1 || { tail -20 $O/prof_$f.log; exit 1; }
done
for f in 1 0; do echo "== flat $f"; find $O/prof_$f -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv,sys
rows=list(csv.DictReader(open('{}')))
for r in rows[:12]: print(r['Name'][:48].ljust(48), r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"; done
