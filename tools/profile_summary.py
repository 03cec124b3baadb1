"""Turn one scripts/gpu_profile.sh run (gpurun_out/prof) into the committed
profile artefacts under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_summary.json       per-kernel average durations, the PMC
                                    HBM bytes of k_count per launch
  profiles/traffic_k<K>_L<L>.json   what bench.py reports as roofline.traffic

HBM bytes per k_count launch follow MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KiB) is doubled on gfx950 for 16-B-per-lane streaming reads,
WRITE_SIZE (KiB) is taken as is; each comes from its own --pmc pass.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tag = sys.argv[2] if len(sys.argv) > 2 else "r01_k6_L0"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 6
L = int(sys.argv[4]) if len(sys.argv) > 4 else 0
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(repo, "profiles")
os.makedirs(out, exist_ok=True)


# the dominant kernel: k_count (k <= 7 or >= 13), k_part (8 <= k <= 12)
main = "k_part" if 8 <= k <= 12 else "k_count"


def counter(pass_dir, name, kernel=None):
    kernel = kernel or main
    vals = []
    for f in glob.glob(os.path.join(src, pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
summary = {"tag": tag, "k": k, "fasta_line": L, "kernels": {}}
if stats:
    shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats.csv"))
    for r in csv.DictReader(open(stats[0])):
        name = r["Name"].split("(")[0].replace("void ", "")
        summary["kernels"][name] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                    "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
fetch = counter("pmc1", "FETCH_SIZE")
write = counter("pmc2", "WRITE_SIZE")
if fetch and write:
    f_kib = statistics.mean(fetch)
    w_kib = statistics.mean(write)
    hbm = f_kib * 1024 * 2 + w_kib * 1024
    summary[main + "_pmc"] = {"launches": len(fetch), "fetch_size_kib": f_kib, "write_size_kib": w_kib,
                              "hbm_bytes_per_launch": hbm}
    input_bytes = int(sys.argv[5]) if len(sys.argv) > 5 else None
    json.dump({"kernel": main, "k": k, "fasta_line": L, "input_bytes": input_bytes,
               "hbm_bytes_per_launch": hbm,
               "fetch_size_kib": f_kib, "write_size_kib": w_kib,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                         f"`bench.py --k {k} --fasta-line {L}`; bytes = 2*FETCH_SIZE*1024 (gfx950 "
                         "streaming-read correction, MI355X_MICROARCH.md) + WRITE_SIZE*1024, mean per launch",
               "source": tag},
              open(os.path.join(out, f"traffic_k{k}_L{L}.json"), "w"), indent=1)
for p in ("pmc3", "pmc4"):
    for f in glob.glob(os.path.join(src, p, "**", "*counter_collection.csv"), recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if main in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        summary.setdefault(main + "_sq", {}).update({n: statistics.mean(v) for n, v in agg.items()})
json.dump(summary, open(os.path.join(out, f"{tag}_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1)[:3000])
