"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: python tools/pmc_summary_k.py CSV [substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    name = r.get("Kernel_Name", "")
    if sub not in name:
        continue
    key = name[:90]
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
for k, v in acc.items():
    n = len(disp[k])
    print(f"{k} ({n} dispatches)")
    for c, x in sorted(v.items()):
        print(f"  {c:32s} {x / n:16.0f} per dispatch")
