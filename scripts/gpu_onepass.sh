# one-pass k_count check: GPU parity, then bench with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_op.log 2>&1 || { tail -20 gpurun_out/bench_op.log; exit 1; }
tail -1 gpurun_out/bench_op.log | cut -c1-400
FK_NO_ONEPASS=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_noop.log 2>&1 || { tail -20 gpurun_out/bench_noop.log; exit 1; }
tail -1 gpurun_out/bench_noop.log | cut -c1-400
timeout -k 10 200 python bench.py --no-cpu-baseline --k 7 > gpurun_out/bench_k7.log 2>&1 || { tail -20 gpurun_out/bench_k7.log; exit 1; }
tail -1 gpurun_out/bench_k7.log | cut -c1-400
timeout -k 10 200 python bench.py --no-cpu-baseline --fasta-line 80 > gpurun_out/bench_fa.log 2>&1 || { tail -20 gpurun_out/bench_fa.log; exit 1; }
tail -1 gpurun_out/bench_fa.log | cut -c1-400
