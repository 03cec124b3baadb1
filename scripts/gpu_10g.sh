# 10 GB single-run k=6 step: one-pass (falls back at the int32 zone) vs multi-launch, with a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
FK_NO_ONEPASS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --bases 10000000000 --steps 6 --warmup 2 > gpurun_out/b10_$v.log 2>&1 || { tail -5 gpurun_out/b10_$v.log; exit 1; }
tail -1 gpurun_out/b10_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('noonepass=$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p10 -o run -- python3 bench.py --no-cpu-baseline --bases 10000000000 --steps 3 --warmup 1 > gpurun_out/p10.log 2>&1 || { tail -5 gpurun_out/p10.log; exit 1; }
f=$(find gpurun_out/p10 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
