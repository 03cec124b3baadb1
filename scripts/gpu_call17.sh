# kernel traces of k = 16 (1 G bases) and k = 17 (10 G) after the one-pass k_repart
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/seg_k16 K=16 BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
OUT=gpurun_out/seg_k15 K=15 BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
OUT=gpurun_out/seg_k17 K=17 STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
python3 - <<'PY'
import csv, glob
for k in (15, 16, 17):
    f = glob.glob(f"gpurun_out/seg_k{k}/trace/**/run_kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    print(k, [(r["Name"][:28], round(float(r["AverageNs"]) / 1e6, 3)) for r in rows[:5]])
PY
