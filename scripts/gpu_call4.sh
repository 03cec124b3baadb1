# k_repart round-6 check: its parity tests, then traces of k = 16, 15 (1 G bases) and the k = 17 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "${SEL:-k16 or k15 or partition_k15 or fresh_table or sparse or routed or sharded_table or low_complexity or table_range}" \
  > gpurun_out/call4.log 2>&1 || { tail -40 gpurun_out/call4.log; exit 1; }
tail -2 gpurun_out/call4.log
KS="16 15" LIBS="product build/exp/libfk_old.so" bash scripts/gpu_call3.sh || exit 1
VARIANTS="old" ROUNDS=1 STEPS=5 WORK="17:80:10000000000 20:80:10000000000" bash scripts/gpu_ab.sh
