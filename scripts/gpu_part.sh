# k_part changes: the partition parity tests, then the k = 8..12 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${SEL:-partition or golden_inputs or mixed_random or int32_zone or full_size or 10g or mixed_tiles or part_resume or streaming or shards or device_feed}" \
  > gpurun_out/part_tests.log 2>&1 || { tail -40 gpurun_out/part_tests.log; exit 1; }
tail -2 gpurun_out/part_tests.log
for a in "--k 11 --bases 10000000000" "--k 11 --bases 1000000000" "--k 12 --bases 1000000000" "--k 8 --bases 1000000000" "--k 10 --bases 1000000000"; do
  timeout -k 10 120 python3 bench.py $a --fasta-line 80 --north-star-bases 0 --no-cpu-baseline --steps 10 > gpurun_out/bp.log 2>&1 || { tail -20 gpurun_out/bp.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bp.log').read().strip().splitlines()[-1]); print('$a', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'ms k_part', round(d['roofline']['frac'],3))"
done
if [ -f build/exp/libfk_probe.so ]; then
  timeout -k 10 200 python3 tools/part_probe_run.py 11 10e9 80 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/probe.log
fi
