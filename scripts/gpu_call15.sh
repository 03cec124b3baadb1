# round-6 end (r06c): traces of the sparse k = 17, 20 steps after the walk's
# window extraction and k_kp_sort's run detection changed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 17 20; do
  OUT=gpurun_out/r06c_k$k K=$k STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
done
echo final-done
