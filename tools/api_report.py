"""Merge a rocprofv3 HIP API trace with the kernel trace: the last engine step
as one timeline (host API calls and kernels, start offsets and durations)."""
import csv
import glob
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append(("API", r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append(("GPU", r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
ev.sort(key=lambda x: x[2])
ks = [i for i, e in enumerate(ev) if e[0] == "GPU" and "k_count" in e[1]]
if len(ks) >= 2:
    a, b = ks[-2], ks[-1]
    t0 = ev[a][2]
    for kind, name, s, e in ev[a:b + 1]:
        print(f"{kind} {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  {name}")
