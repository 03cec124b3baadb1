# k_tail with deferred stores: timeline probe, bench, one-pass parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/tailprof.py 6 > gpurun_out/tailprof.log 2>&1 || { tail -20 gpurun_out/tailprof.log; exit 1; }
grep step gpurun_out/tailprof.log
timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/t2.log 2>&1 || { tail -20 gpurun_out/t2.log; exit 1; }
grep '^{' gpurun_out/t2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
