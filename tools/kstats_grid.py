"""Per (kernel, grid size) launch statistics of a rocprofv3 kernel_trace.csv (the stats file merges launches of
one kernel at different grids, e.g. search_res_kernel for config 2 (256 roots) and config 1 (8 roots)).

    python tools/kstats_grid.py TRACE_CSV [substring ...] > kernel_stats_by_grid.csv
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
subs = sys.argv[2:]
acc = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if subs and not any(s in name for s in subs):
        continue
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    acc[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
w = csv.writer(sys.stdout)
w.writerow(["Name", "Grid_Size_X", "Calls", "AverageNs", "MinNs", "MaxNs"])
for (name, grid), d in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, grid, len(d), round(sum(d) / len(d), 1), min(d), max(d)])
