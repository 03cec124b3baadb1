# kernel trace (rocprofv3 --kernel-trace --stats) of a short bench run, per
# library (LIBS="product build/exp/libfk_x.so ..."): average kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps ${STEPS:-5} --warmup 2 --north-star-bases 0 --no-cpu-baseline ${BARGS:-}"
for lib in ${LIBS:-product}; do
  tag=$(basename $lib .so)
  if [ $lib = product ]; then L=""; else L=$lib; fi
  FINDKMER_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$tag -o run -- python3 $B > gpurun_out/tr_$tag.log 2>&1 || { tail -20 gpurun_out/tr_$tag.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/tr_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step %.3f ms" % d["ms_per_step"])')"
  python3 - "gpurun_out/tr_$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print("  %-60s %6s calls  avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
