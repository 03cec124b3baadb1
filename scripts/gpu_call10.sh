# fused walks for every sparse k: the sparse parity tests, then the 10 G-base
# steps at k = 20 (fused, and sp_walk=0) and k = 17, 18
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "sparse" \
  > gpurun_out/c10_tests.log 2>&1 || { tail -40 gpurun_out/c10_tests.log; exit 1; }
tail -3 gpurun_out/c10_tests.log
for kt in "17:" "20:"; do
  IFS=: read k tune <<< "$kt"
  FINDKMER_TUNE=$tune timeout -k 10 240 python bench.py --k $k --fasta-line 80 --bases 10000000000 --steps 4 --warmup 2 \
    --north-star-bases 0 --no-cpu-baseline > gpurun_out/c10_b.json 2> gpurun_out/c10_b.err || { tail -20 gpurun_out/c10_b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c10_b.json').read().strip().splitlines()[-1]); print('k=$k tune=$tune', round(d['ms_per_step'],2), 'ms')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c10_prof -o run -- python3 bench.py --k 20 --fasta-line 80 --bases 10000000000 --steps 2 --warmup 1 --north-star-bases 0 --no-cpu-baseline > gpurun_out/c10_prof.log 2>&1 || { tail -20 gpurun_out/c10_prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c10_prof/**/run_kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls avg {float(r["AverageNs"])/1e6:8.3f}  {r["Name"][:90]}')
PY
