# k=11: parity subset, then kernel times for k_table_stats grid sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "11 or 12 or 9" > gpurun_out/k11_tests.log 2>&1 || { tail -30 gpurun_out/k11_tests.log; exit 1; }
tail -2 gpurun_out/k11_tests.log
for tb in 0 256 64; do
FK_TS_BLOCKS=$tb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k11tb$tb -o run -- python3 bench.py --k 11 --fasta-line 80 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/k11tb$tb.log 2>&1 || { tail -5 gpurun_out/k11tb$tb.log; exit 1; }
echo "tb=$tb"; tail -1 gpurun_out/k11tb$tb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
f=$(find gpurun_out/k11tb$tb -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-60,120-200
done
