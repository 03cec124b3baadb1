# round-6 end (r06b): the default bench line, and traces of what changed since
# r06 -- k = 15, 16 (1 G bases), sparse k = 17, 18, 20 (10 G bases); then
#   python3 tools/profile_summary.py gpurun_out/r06b_k<K> r06b_... per workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err || { tail -20 gpurun_out/r06b_bench.err; exit 1; }
tail -1 gpurun_out/r06b_bench.json | cut -c1-200
OUT=gpurun_out/r06b_k15 K=15 BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
OUT=gpurun_out/r06b_k16 K=16 BASES=1000000000 bash scripts/gpu_profile.sh || exit 1
for k in 17 18 20; do
  OUT=gpurun_out/r06b_k$k K=$k STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
done
echo final-done
