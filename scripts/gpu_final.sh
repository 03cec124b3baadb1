# round-end measurements: the default bench line, the k=11 10 G-base trace +
# PMC profile (the headline), the k=6 north-star profile, 1 G-base traces of
# k = 12..16 and 10 G-base traces of the sparse k = 17, 20; then
#   python3 tools/profile_summary.py gpurun_out/<dir> <tag> ... per workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json | cut -c1-300
OUT=gpurun_out/prof_k11 bash scripts/gpu_profile.sh || exit 1
OUT=gpurun_out/prof_k6 K=6 L=0 SEED=1 bash scripts/gpu_profile.sh || exit 1
for k in 12 13 14 15 16; do
  OUT=gpurun_out/prof_k$k K=$k BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
done
for k in 17 20; do
  OUT=gpurun_out/prof_k$k K=$k STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
done
echo final-done
