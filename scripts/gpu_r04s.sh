# sparse (17 <= k <= 20) and k = 14..16 parity, then the k=17 10 G-base
# and k = 15, 16 profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH=0 FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py" SEL="sparse or large_k or k15_and_k16 or k16_dense or table_range or int32_zone_partitioned" TLIM=900 bash scripts/gpu_quick.sh || exit 1
K=${K:-17} N=10000000000 bash scripts/gpu_sparse_prof.sh || exit 1
KS="15 16" bash scripts/gpu_bigk_prof.sh
