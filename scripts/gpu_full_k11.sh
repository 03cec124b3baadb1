# full GPU suite, then the k=11 FASTA step (k_part path) and plain k=6
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for L in 80 0; do
timeout -k 10 120 python bench.py --no-cpu-baseline --k 11 --fasta-line $L --steps 10 --warmup 3 > gpurun_out/bench_k11_$L.log 2>&1 || { tail -20 gpurun_out/bench_k11_$L.log; exit 1; }
tail -1 gpurun_out/bench_k11_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k11 L$L step_ms', d['ms_per_step'], 'main_kernel_ms', d['roofline']['kernel_ms'])"
done
