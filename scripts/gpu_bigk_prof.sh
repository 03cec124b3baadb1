# trace + FETCH/WRITE passes of k = 14, 15, 16 over 1 G bases of FASTA
set -o pipefail
cd $GRAFT_REPO_ROOT
for k in ${KS:-14 15 16}; do
  K=$k BASES=1000000000 STEPS=${STEPS:-5} TLIM=200 OUT=gpurun_out/prof_k$k bash scripts/gpu_profile.sh || exit 1
done
