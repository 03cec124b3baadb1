# the whole -m gpu suite (as the driver runs it) plus smoke(), logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=40 ${SEL:-} \
  > gpurun_out/suite.log 2>&1 || { tail -60 gpurun_out/suite.log; exit 1; }
tail -30 gpurun_out/suite.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
