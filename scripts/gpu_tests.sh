set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests/ -q -m gpu -x ${PYTEST_ARGS} > gpurun_out/tests.log 2>&1; rc=$?
tail -40 gpurun_out/tests.log
exit $rc
