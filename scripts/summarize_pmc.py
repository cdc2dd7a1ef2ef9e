"""Summarize rocprofv3 counter_collection CSVs per kernel (sums over dispatches)."""
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:44]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
for k, v in agg.items():
    if 'ndfl' not in k:
        continue
    print(k, 'dispatches', len(disp[k]))
    for a, b in sorted(v.items()):
        print('   %-22s %16.0f' % (a, b))
