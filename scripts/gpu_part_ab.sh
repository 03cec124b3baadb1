# k_part block-size A/B: parity (8 <= k <= 12) with the product build, then bench both
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "8 or 9 or 11 or 12" > gpurun_out/part_tests.log 2>&1 || { tail -30 gpurun_out/part_tests.log; exit 1; }
tail -1 gpurun_out/part_tests.log
for K in 11 8 12; do
for lib in "" build/exp/libfk_pw8.so; do
FINDKMER_LIB=$lib timeout -k 10 300 python bench.py --k $K --fasta-line 80 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "k=$K lib=${lib:-product} $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
done
