# sparse (17 <= k <= 20) parity, then the k=17 and k=20 10 G-base profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH=0 FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py" SEL="sparse or large_k or sweep_matches_separate or cli_matches_reference" TLIM=900 bash scripts/gpu_quick.sh || exit 1
K=20 N=10000000000 bash scripts/gpu_sparse_prof.sh
