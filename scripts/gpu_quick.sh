# targeted GPU parity (SEL = pytest -k expression, FILES = test files) then
# the headline bench line; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-600} python -u -m pytest ${FILES:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread -k "${SEL:-partition}" \
  > gpurun_out/quick.log 2>&1 || { tail -40 gpurun_out/quick.log; exit 1; }
tail -2 gpurun_out/quick.log
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --north-star-bases 0 --no-cpu-baseline ${BARGS:-} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_q.json')); r=d['roofline']
print('step %.3f ms  %s %.3f ms  frac %.3f' % (d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac']))"
fi
