# k >= 14 parity (incl. sparse) then big-k and sparse profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH=0 FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" SEL="k15_and_k16 or k16_dense or table_range or k14 or sparse or large_k" TLIM=900 bash scripts/gpu_quick.sh || exit 1
KS="14 15 16" bash scripts/gpu_bigk_prof.sh || exit 1
K=17 N=10000000000 bash scripts/gpu_sparse_prof.sh
