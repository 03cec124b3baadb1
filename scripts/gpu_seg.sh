# Per-kernel time per step (rocprofv3 kernel trace) of the k=11 10 G-base
# bench with the feed cut into segments of SEGS KiB (FINDKMER_TUNE seg_kb):
# how much of k_part + k_bucket_count the Infinity Cache saves when a
# segment's codes stay on die.  BARGS adds bench options (e.g. --k 14 --bases 1e9).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ST=${STEPS:-3}
for s in ${SEGS:-0 262144 131072 65536}; do
  FINDKMER_TUNE=seg_kb=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/seg_$s -o run -- python3 bench.py --steps $ST --warmup 1 --north-star-bases 0 --no-cpu-baseline ${BARGS:-} > gpurun_out/seg_$s.log 2>&1 || { tail -20 gpurun_out/seg_$s.log; exit 1; }
  echo "== seg_kb=$s: $(tail -1 gpurun_out/seg_$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step %.3f ms" % d["ms_per_step"])')"
  python3 - gpurun_out/seg_$s $((ST + 1)) <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2])
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print("  %-50s %7s calls  %8.3f ms/step  avg %9.1f us" % (r["Name"][:50], r["Calls"], float(r["TotalDurationNs"]) / 1e6 / n, float(r["AverageNs"]) / 1e3))
PY
done
