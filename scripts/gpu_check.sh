set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke" 
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke-failed; cat gpurun_out/smoke.log | tail -30; exit 1; }
tail -3 gpurun_out/smoke.log
echo "== golden gpu tests"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "golden_inputs or edge_sizes" > gpurun_out/t1.log 2>&1; rc=$?; tail -30 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.log 2>&1; rc=$?; tail -5 gpurun_out/bench1.log; exit $rc
