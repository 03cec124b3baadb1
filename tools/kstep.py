"""Print a profile directory's step time, top kernels and HBM bytes per step
(the profiles/<tag>_summary.json profile_summary.py wrote)."""
import json, sys
tag = sys.argv[1]
d = json.load(open(f"profiles/{tag}_summary.json"))
for n, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"])[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    print("  %-60s %4d calls avg %9.1f us" % (n[:60], v["calls"], v["avg_us"]))
sp = d.get("step_pmc", {})
print("  HBM per step %.2f GB" % (sp.get("hbm_bytes_per_step", 0) / 1e9))
for n, v in sp.get("per_kernel_bytes_per_step", {}).items():
    if v > 1e8:
        print("    %-58s %.2f GB" % (n[:58], v / 1e9))
