# k = 13..16 (dense table, global atomics): bench lines + a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 13 14 16; do
  timeout -k 10 180 python3 bench.py --k $k --bases 1000000000 --fasta-line 80 --north-star-bases 0 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bk.log 2>&1 || { tail -20 gpurun_out/bk.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bk.log').read().strip().splitlines()[-1]); print('k=$k', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'ms k_count', round(d['roofline']['frac'],4))"
done
OUT=gpurun_out/prof_k16 K=16 L=80 BASES=1000000000 STEPS=5 bash scripts/gpu_profile.sh
for k in 17 20; do
  for n in 100000000 1000000000; do
    timeout -k 10 180 python3 bench.py --k $k --bases $n --fasta-line 80 --north-star-bases 0 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bk.log 2>&1 || { tail -20 gpurun_out/bk.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bk.log').read().strip().splitlines()[-1]); print('k=$k n=$n', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'ms main')"
  done
done
