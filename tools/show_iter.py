"""Summary of a gpu_res_iter.sh output directory: test tail, bench values, SQ LDS counters."""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
try:
    print(open(os.path.join(d, "tests.log")).read().strip().splitlines()[-1])
except OSError as e:
    print(e)
for f in ("bench", "bench_zero_heads", "bench_philox"):
    try:
        x = json.loads(open(os.path.join(d, f + ".json")).read().strip().splitlines()[-1])
        print(f"{f:18s} {x['value'] / 1e6:7.3f} M sims/s  {x['ms_per_step']:.4f} ms  kernel {x['roofline']['launch_us']} us")
    except Exception as e:  # noqa: BLE001
        print(f, e)
p = os.path.join(d, "pmc", "pmc_counter_collection.csv")
if os.path.exists(p):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(p)):
        if "search_res_kernel" in r["Kernel_Name"]:
            disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(disp)
    for k in sorted({k for v in disp.values() for k in v}):
        print(f"  {k:24s} {sum(v[k] for v in disp.values()) / n:14.0f}")
