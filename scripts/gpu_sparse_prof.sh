# 17 <= k <= 20: kernel trace of the key-range passes (bench k, 1 G bases)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${K:-17}
N=${N:-1000000000}
for i in 1 2; do timeout -k 10 180 python3 bench.py --k $K --bases $N --fasta-line 80 --north-star-bases 0 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/sp_plain.log 2>&1 || { tail -20 gpurun_out/sp_plain.log; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/sp_plain.log').read().strip().splitlines()[-1]); print('plain', round(d['ms_per_step'],3))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof -o run -- python3 bench.py --k $K --bases $N --fasta-line 80 --north-star-bases 0 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/sp_prof.log 2>&1 || { tail -20 gpurun_out/sp_prof.log; exit 1; }
tail -1 gpurun_out/sp_prof.log | cut -c1-300
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/sp_prof/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
