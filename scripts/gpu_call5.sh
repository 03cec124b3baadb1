# the sparse tests and the k = 17 / 20 A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "${SEL:-sparse or low_complexity}" > gpurun_out/call5.log 2>&1 || { tail -40 gpurun_out/call5.log; exit 1; }
tail -2 gpurun_out/call5.log
VARIANTS="${VARIANTS:-old}" ROUNDS=${ROUNDS:-1} STEPS=5 WORK="${WORK:-20:80:10000000000 17:80:10000000000}" bash scripts/gpu_ab.sh
