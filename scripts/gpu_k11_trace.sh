# kernel breakdown of the k=11 bench step (L=80 and L=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in 80 0; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k11tr_$L -o run -- python3 bench.py --no-cpu-baseline --k 11 --fasta-line $L --steps 10 --warmup 3 > gpurun_out/k11tr_$L.log 2>&1 || { tail -5 gpurun_out/k11tr_$L.log; exit 1; }
python3 - $L <<'PY'
import csv,sys
L=sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/k11tr_{L}/run_kernel_stats.csv")):
    print(L, r['Name'][:28].ljust(30), r['Calls'].rjust(4), ('%.1f' % (float(r['AverageNs'])/1000)).rjust(9), 'us')
PY
done
