"""Sum rocprofv3 --pmc counter_collection.csv values per (kernel, counter) for kernels matching a
substring; prints per-dispatch means."""
import csv
import sys
from collections import defaultdict

path, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
acc = defaultdict(float)
disp = defaultdict(set)
for r in csv.DictReader(open(path)):
    name = r.get("Kernel_Name", "")
    if pat not in name:
        continue
    key = (name[:60], r["Counter_Name"])
    acc[key] += float(r["Counter_Value"])
    disp[key].add(r.get("Dispatch_Id", ""))
for (k, c), v in sorted(acc.items()):
    n = max(1, len(disp[(k, c)]))
    print(f"{k:60s} {c:28s} per-dispatch {v / n:16.0f}  dispatches {n}")
