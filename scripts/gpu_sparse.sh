# 17 <= k <= 20: sparse parity tests, then the kernel trace of a 1 G-base bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "sparse" > gpurun_out/sparse_tests.log 2>&1 || { tail -40 gpurun_out/sparse_tests.log; exit 1; }
tail -2 gpurun_out/sparse_tests.log
bash scripts/gpu_sparse_prof.sh
