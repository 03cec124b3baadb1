# k = 15, 16: parity tests, then the 1 G-base step with k_count_parts2
# (default) against k_count_parts (cp2=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "15 or 16 or wrap or poly or zone" \
  > gpurun_out/c9_tests.log 2>&1 || { tail -40 gpurun_out/c9_tests.log; exit 1; }
tail -3 gpurun_out/c9_tests.log
for k in 15 16; do
for tune in "" "cp2=0" "" "cp2=0"; do
  FINDKMER_TUNE=$tune timeout -k 10 240 python bench.py --k $k --fasta-line 80 --bases 1000000000 --steps 10 --warmup 3 \
    --north-star-bases 0 --no-cpu-baseline > gpurun_out/c9_b.json 2> gpurun_out/c9_b.err || { tail -20 gpurun_out/c9_b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c9_b.json').read().strip().splitlines()[-1]); print('k=$k tune=$tune', round(d['ms_per_step'],3), 'ms')"
done
done
