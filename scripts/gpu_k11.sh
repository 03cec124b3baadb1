# full GPU suite, k=11 benches (FASTA and pure), k=6 bench, k=11 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_all.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
for L in 80 0; do
  timeout -k 10 200 python bench.py --k 11 --fasta-line $L --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b11_$L.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/b11_$L.log').read().strip().splitlines()[-1]); print('k11 L=$L', round(d['roofline']['kernel_ms']*1000,1), 'us k_count', round(d['ms_per_step']*1000,1), 'us/step', '%.3g' % d['value'])"
done
VARIANTS=prod bash scripts/exp_run.sh || exit 1
K=11 L=80 STEPS=5 bash scripts/gpu_trace.sh > /dev/null || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/trace/run_kernel_stats.csv')): print(r['Name'][:28], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')"
