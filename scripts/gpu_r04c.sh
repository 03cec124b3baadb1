# k = 14..16 parity, then their profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH=0 FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py" SEL="k15_and_k16 or k16_dense or table_range or k14 or int32_zone_partitioned or (sharded_table and 16)" TLIM=900 bash scripts/gpu_quick.sh || exit 1
KS="${KS:-15 16}" bash scripts/gpu_bigk_prof.sh
