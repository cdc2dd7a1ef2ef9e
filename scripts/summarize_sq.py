"""Per-kernel SQ counter summary from rocprofv3 --pmc CSVs (sums over dispatches and XCDs).
Cycle counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*, SQ_BUSY_CYCLES) count quad-cycles.
Usage: python scripts/summarize_sq.py run_counter_collection.csv [more.csv ...]"""
import collections
import csv
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("ndfl"):
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, c in sorted(tot.items()):
    n = max(1, len(disp[k]) // max(1, len(sys.argv) - 1))
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k}  (dispatches/pass {n})")
    for name in sorted(c):
        v = c[name] / n
        extra = f"  ({100 * c[name] / wc:5.1f}% of wave cycles)" if name.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"   {name:24s} {v:16.4g}{extra}")
    w = c.get("SQ_WAVES", 0)
    if w and c.get("SQ_INSTS_VALU"):
        print(f"   VALU insts per wave {c['SQ_INSTS_VALU'] / w:.4g}, LDS {c.get('SQ_INSTS_LDS', 0) / w:.4g}, SALU {c.get('SQ_INSTS_SALU', 0) / w:.4g}")
