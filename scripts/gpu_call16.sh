# k_repart in one pass (SEG: segment table, consumers gather): k = 15..17
# parity tests, then A/B against the source before it (exp_variant base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py -m gpu -x -v --timeout 150 --timeout-method thread -k "sparse or 15 or 16 or partition" \
  > gpurun_out/c16_tests.log 2>&1 || { tail -40 gpurun_out/c16_tests.log; exit 1; }
tail -2 gpurun_out/c16_tests.log
VARIANTS="base" WORK="16:80:1000000000 15:80:1000000000 17:80:10000000000" STEPS=6 ROUNDS=1 bash scripts/gpu_ab.sh
