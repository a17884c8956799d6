"""Summarise a rocprofv3 kernel_stats.csv: total ms, then the top kernels (ms, calls, avg us, name)."""
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{f}: total {tot / 1e6:.2f} ms")
    for r in rows[:int(18)]:
        print(f'{float(r["TotalDurationNs"]) / 1e6:8.2f}ms {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:8.1f}us  '
              f'{r["Name"][:100]}')
