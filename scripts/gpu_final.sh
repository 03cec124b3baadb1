# round-end measurements: the default bench line, the k=11 10 G-base trace +
# PMC profile, and the world-1 RCCL exchange times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json | cut -c1-400
OUT=gpurun_out/prof bash scripts/gpu_profile.sh || exit 1
bash scripts/gpu_rccl1.sh
