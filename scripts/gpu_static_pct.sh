# k=6 1 GB: static share of the ranges (FK_STATIC_PCT; 100 = no dynamic ranges), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for p in 100 95 90 80; do
FK_STATIC_PCT=$p timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/sp_$p.log 2>&1 || { tail -20 gpurun_out/sp_$p.log; exit 1; }
echo "pct=$p $(grep '^{' gpurun_out/sp_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['kernel_ms']*1000,1))")"
done; done
