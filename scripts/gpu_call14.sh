# k_repart's run words as 16-B loads, k_kp_sort's run detection from registers:
# k = 15..20 parity tests, then the steps of k = 16 (1 G bases), 17 and 20 (10 G)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "sparse or 15 or 16" \
  > gpurun_out/c14_tests.log 2>&1 || { tail -40 gpurun_out/c14_tests.log; exit 1; }
tail -2 gpurun_out/c14_tests.log
for kb in "16:1000000000" "17:10000000000" "20:10000000000"; do
  IFS=: read k n <<< "$kb"
  timeout -k 10 240 python bench.py --k $k --fasta-line 80 --bases $n --steps 6 --warmup 2 \
    --north-star-bases 0 --no-cpu-baseline > gpurun_out/c14_b.json 2> gpurun_out/c14_b.err || { tail -20 gpurun_out/c14_b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c14_b.json').read().strip().splitlines()[-1]); print('k=$k', round(d['ms_per_step'],2), 'ms')"
done
