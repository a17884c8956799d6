"""Build profiles/pmc_latest.json from a profile_round.sh output directory: per-dispatch means of
FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum / TCC_MISS_sum for each named kernel (the bench's dominant
kernels: search_res_kernel for config 2, search_conv_kernel for config 5), with the gfx950 FETCH_SIZE
correction of MI355X_MICROARCH.md (x2: 128-B streaming reads tallied at 64 B).

    python tools/pmc_latest.py gpurun_out/<dir> search_res_kernel search_conv_kernel search_conv_ez_kernel \
        az_search_fused_kernel > profiles/pmc_latest.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root, pat):
    acc, disp, kname = defaultdict(float), defaultdict(set), ""
    paths = sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True))
    # the bench line's own launch of the kernel: the largest grid (config 1 also runs search_res_kernel, on 8 roots)
    grid = max((int(r.get("Grid_Size") or 0) for path in paths for r in csv.DictReader(open(path))
                if pat in r.get("Kernel_Name", "")), default=0)
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", "")
            if pat not in name or int(r.get("Grid_Size") or 0) != grid:
                continue
            kname = name
            c = r["Counter_Name"]
            acc[c] += float(r["Counter_Value"])
            disp[c].add((path, r.get("Dispatch_Id", "")))
    per = {c: round(v / max(1, len(disp[c])), 1) for c, v in acc.items()}
    fetch = 2 * per.get("FETCH_SIZE", 0.0) * 1024
    write = per.get("WRITE_SIZE", 0.0) * 1024
    req = (per.get("TCC_HIT_sum", 0.0) + per.get("TCC_MISS_sum", 0.0))
    return {
        "kernel": kname,
        "command": "python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline (one rocprofv3 --kernel-trace --pmc pass per group)",
        "per_dispatch": per,
        "fetch_bytes_corrected": int(fetch),
        "write_bytes": int(write),
        "traffic_bytes": int(fetch + write),
        "l2_hit_rate": round(per.get("TCC_HIT_sum", 0.0) / req, 5) if req else None,
        "l2_request_bytes": int(req * 128),
        "notes": "FETCH_SIZE/WRITE_SIZE are KB; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B "
                 "streaming-read requests at 64 B) - an upper bound here, the kernel's HBM reads mix 16-B and 4-B "
                 "lanes. TCC_HIT+MISS x 128 B = bytes requested from L2.",
    }


def main():
    import datetime
    import subprocess
    root = sys.argv[1]
    try:
        head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    except OSError:
        head = None
    # where the numbers come from: bench.py copies this into roofline.traffic_source, so the field cannot be
    # read as measured in the run that prints it
    source = {"pmc_dir": os.path.normpath(root), "built": datetime.datetime.utcnow().strftime("%Y-%m-%d %H:%M UTC"),
              "head": head, "passes": "one rocprofv3 --kernel-trace --pmc run per counter group (tools/profile_round.sh)"}
    print(json.dumps({"source": source, "kernels": {pat: summarise(root, pat) for pat in sys.argv[2:]}}, indent=1))


if __name__ == "__main__":
    main()
