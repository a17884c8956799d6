"""The kernels of one timed step from a rocprofv3 kernel_trace.csv: the launches between two consecutive
launches of the step's dominant kernel (the median such window of the run), in order, with their durations and
the gaps between them — what one step of the bench runs, without the setup and check kernels around the timed
region that the run's kernel_stats.csv also counts.

    python tools/step_kernels.py TRACE_CSV DOMINANT_SUBSTRING > step_sequence.txt
"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
wins = [(idx[j], idx[j + 1]) for j in range(len(idx) - 1)]
spans = [int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) for a, b in wins]
med = statistics.median(spans)
a, b = min(wins, key=lambda w: abs(int(rows[w[1]]["Start_Timestamp"]) - int(rows[w[0]]["Start_Timestamp"]) - med))
print(f"one step: {len(idx)} launches of '{key}'; median window {med / 1e3:.1f} us (start to start)")
prev = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(e - s) / 1e3:10.2f} us  gap {gap:6.2f}  {r['Kernel_Name'][:100]}")
    prev = e
