"""Summarise a rocprofv3 csv trace directory: per-kernel stats and the
timeline of the last few engine steps (start offsets and durations in us)."""
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append(("K", r["Kernel_Name"][:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append(("M", r.get("Direction", "copy")[:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    print(open(f).read())
rows.sort(key=lambda x: x[2])
# last 3 steps: find the last three k_count launches
idx = [i for i, r in enumerate(rows) if "k_count" in r[1]]
if idx:
    start = idx[-3] - 8 if len(idx) >= 3 else 0
    t0 = rows[max(start, 0)][2]
    prev_end = None
    for kind, name, s, e in rows[max(start, 0):]:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print(f"{kind} {(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {name}")
        prev_end = e
