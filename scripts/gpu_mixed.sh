# mixed tiles: new parity tests, full GPU suite, plain bench (no regression),
# header-dense engine time with and without mixed tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mixed_tiles or part_resume or partition_skewed or golden_inputs" > gpurun_out/mixed_tests.log 2>&1 || { tail -40 gpurun_out/mixed_tests.log; exit 1; }
tail -2 gpurun_out/mixed_tests.log
if [ "${FULL:-1}" = 1 ]; then
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
fi
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_plain.log 2>&1 || { tail -20 gpurun_out/bench_plain.log; exit 1; }
tail -1 gpurun_out/bench_plain.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain k6 step_ms', d['ms_per_step'], 'k_count_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --fasta-line 80 > gpurun_out/bench_fa80.log 2>&1 || { tail -20 gpurun_out/bench_fa80.log; exit 1; }
tail -1 gpurun_out/bench_fa80.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fasta80 k6 step_ms', d['ms_per_step'], 'k_count_ms', d['roofline']['kernel_ms'])"
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
echo "mixed   $(timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 8 11 12 13 2>/dev/null | tail -1)"
echo "nomixed $(FK_NO_MIXED=1 timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 8 11 12 13 2>/dev/null | tail -1)"
