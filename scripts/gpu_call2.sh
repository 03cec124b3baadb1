# targeted parity for the span-streamed k_repart (k = 15, 16 dense, sparse k >= 17, the
# routed gloo tables, the skewed 2 G-base stream), then an A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py -m gpu -x -v \
  --timeout 300 --timeout-method thread --durations=15 -k "${SEL:-k16 or k15 or partition_k15 or fresh_table or sparse or routed or sharded_table or low_complexity or table_range}" \
  > gpurun_out/call2.log 2>&1 || { tail -40 gpurun_out/call2.log; exit 1; }
tail -22 gpurun_out/call2.log
VARIANTS="old" ROUNDS=2 STEPS=5 WORK="16:80:1000000000 15:80:1000000000 17:80:10000000000" bash scripts/gpu_ab.sh
