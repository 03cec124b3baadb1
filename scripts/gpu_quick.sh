# quick loop: smoke, a parity subset, bench (k=6 and k=11)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q ${PYTEST_ARGS:--k "golden_inputs or mixed_random or edge_sizes or streaming or shards"} > gpurun_out/tq.log 2>&1; rc=$?
tail -15 gpurun_out/tq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_k6.log 2>&1 || { tail -20 gpurun_out/bench_k6.log; exit 1; }
tail -1 gpurun_out/bench_k6.log
timeout -k 10 300 python bench.py --k 11 --fasta-line 80 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_k11.log 2>&1 || { tail -20 gpurun_out/bench_k11.log; exit 1; }
tail -1 gpurun_out/bench_k11.log
