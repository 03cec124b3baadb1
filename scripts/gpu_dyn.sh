# dynamic k_count ranges: full GPU suite, then bench with 1 (static) vs 4 ranges per wave, wave times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "${PYTEST_K:-gpu}" > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for rpw in 4 1 2 8; do
FK_RANGES_PER_WAVE=$rpw timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "rpw=$rpw $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])")"
done
FINDKMER_LIB=build/exp/libfk_wt.so timeout -k 10 300 python tools/wave_times.py > gpurun_out/wt.log 2>&1; grep waves gpurun_out/wt.log
