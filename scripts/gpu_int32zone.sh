# the partitioned path's recount in the int32 seqSize zone: tests, then the one-run timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "int32" > gpurun_out/int32.log 2>&1 || { tail -40 gpurun_out/int32.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/int32.log | tail -8
bash scripts/gpu_onerun.sh
