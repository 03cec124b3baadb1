# round-4 headline: default bench line, then kernel trace + PMC passes of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json
OUT=gpurun_out/prof bash scripts/gpu_profile.sh
