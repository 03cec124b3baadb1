# one-off measurements: tools/chunk_probe (code layouts), the RCCL bench-line
# test, and the headline bench line at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/chunk_probe 10 > gpurun_out/chunk_probe.txt 2>&1 || { cat gpurun_out/chunk_probe.txt; exit 1; }
cat gpurun_out/chunk_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread -k "bench_line_reports" > gpurun_out/rccl_test.log 2>&1 || { tail -40 gpurun_out/rccl_test.log; exit 1; }
tail -2 gpurun_out/rccl_test.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --north-star-bases 0 --no-cpu-baseline > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || { tail -20 gpurun_out/bench_head.err; exit 1; }
cat gpurun_out/bench_head.json
