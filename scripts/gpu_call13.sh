# SQ counters of the sparse k = 20 step (k_kp_sort, k_repart<u32>, k_sp_wpart)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sq20 K=20 L=80 BASES=10000000000 STEPS=2 SQ=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ("pmc1", "pmc2", "pmc3", "pmc4"):
    f = glob.glob(f"gpurun_out/sq20/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no csv", d); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0][-28:]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[name].add(r["Dispatch_Id"])
    for name, cs in agg.items():
        if any(x in name for x in ("k_kp_sort", "k_repart", "k_sp_wpart")):
            print(d, name, len(n[name]), {k: "%.3g" % (v / len(n[name])) for k, v in sorted(cs.items())})
PY
