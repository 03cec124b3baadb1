# round-6 end (r06e): traces of k = 15, 16 (1 G bases) and k = 17 (10 G)
# after the segment gather's prefetch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 15 16; do
  OUT=gpurun_out/r06e_k$k K=$k BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
done
OUT=gpurun_out/r06e_k17 K=17 STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
echo final-done
