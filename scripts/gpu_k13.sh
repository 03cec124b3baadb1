# k = 13 through the partition: parity tests, then the big-k bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "13 or partition or int32_zone or sparse" > gpurun_out/k13_tests.log 2>&1 || { tail -40 gpurun_out/k13_tests.log; exit 1; }
tail -2 gpurun_out/k13_tests.log
bash scripts/gpu_bigk.sh
