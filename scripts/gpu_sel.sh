# the GPU tests matching SEL (pytest -k), then optional extra command EXTRA
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-900} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "$SEL" > gpurun_out/sel_tests.log 2>&1 || { tail -60 gpurun_out/sel_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/sel_tests.log | tail -3
