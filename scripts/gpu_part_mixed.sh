# k_part mixed path: partition/mixed tests, k=11 plain bench, header-dense engine times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${PYK:-mixed_tiles or part_resume or partition_skewed or golden_inputs or mixed_random or shards}" > gpurun_out/pm_tests.log 2>&1 || { tail -40 gpurun_out/pm_tests.log; exit 1; }
tail -2 gpurun_out/pm_tests.log
for L in 80 0; do
timeout -k 10 120 python bench.py --no-cpu-baseline --k 11 --fasta-line $L --steps 10 --warmup 3 > gpurun_out/bench_k11_$L.log 2>&1 || { tail -20 gpurun_out/bench_k11_$L.log; exit 1; }
tail -1 gpurun_out/bench_k11_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k11 L$L step_ms', d['ms_per_step'], 'main_kernel_ms', d['roofline']['kernel_ms'])"
done
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
echo "mixed   $(timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 8 11 12 2>/dev/null | tail -1)"
