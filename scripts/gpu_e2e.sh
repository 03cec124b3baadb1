# new CLI tests (ingest, sweep) + golden CLI, then end-to-end CLI timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "cli" > gpurun_out/cli_tests.log 2>&1 || { tail -30 gpurun_out/cli_tests.log; exit 1; }
tail -2 gpurun_out/cli_tests.log
timeout -k 10 600 python -u tools/e2e_cli.py ${E2E_BYTES:-2e9} gpurun_out/e2e.json > gpurun_out/e2e.log 2>&1 || { tail -20 gpurun_out/e2e.log; exit 1; }
tail -1 gpurun_out/e2e.log
