# k = 20 sparse over 10 G bases, and k = 12, 13 trace + PMC at 1 G bases
set -o pipefail
cd $GRAFT_REPO_ROOT
K=20 N=10000000000 bash scripts/gpu_sparse_prof.sh || exit 1
KS="12 13" bash scripts/gpu_bigk_prof.sh
