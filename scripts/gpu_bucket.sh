# k_bucket_count batching: parity for 8 <= k <= 12, bench, profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "8 or 9 or 10 or 11 or 12" > gpurun_out/bucket_tests.log 2>&1 || { tail -40 gpurun_out/bucket_tests.log; exit 1; }
tail -1 gpurun_out/bucket_tests.log
for K in 11 12 9; do
for L in 80 0; do
timeout -k 10 300 python bench.py --k $K --fasta-line $L --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "k=$K L=$L $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k11b -o run -- python3 bench.py --k 11 --fasta-line 80 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/k11b.log 2>&1 || { tail -5 gpurun_out/k11b.log; exit 1; }
