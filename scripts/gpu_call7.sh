# SQ counters of the sparse k = 17 step (one pass per counter group)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sq17 K=17 L=80 BASES=10000000000 STEPS=2 SQ=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ("pmc3", "pmc4"):
    f = glob.glob(f"gpurun_out/sq17/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no csv", d); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0][-40:]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    for name, cs in agg.items():
        if any(x in name for x in ("k_kp_count", "k_repart", "k_kpart", "k_sp_emit")):
            print(d, name, {k: "%.3g" % v for k, v in sorted(cs.items())})
PY
