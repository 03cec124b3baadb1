# device-input tests, then the 10 GB north-star workloads (synthetic genome of 1.5 Gbase chromosomes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "device_input" > gpurun_out/di_tests.log 2>&1 || { tail -30 gpurun_out/di_tests.log; exit 1; }
tail -1 gpurun_out/di_tests.log
timeout -k 10 300 python bench.py --bases 10000000000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b10_k6.log 2>&1 || { tail -5 gpurun_out/b10_k6.log; exit 1; }
tail -1 gpurun_out/b10_k6.log
timeout -k 10 300 python bench.py --bases 10000000000 --k 11 --fasta-line 80 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b10_k11.log 2>&1 || { tail -5 gpurun_out/b10_k11.log; exit 1; }
tail -1 gpurun_out/b10_k11.log
timeout -k 10 300 python bench.py --bases 10000000000 --chrom 0 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b10_k6_onerun.log 2>&1 || { tail -5 gpurun_out/b10_k6_onerun.log; exit 1; }
tail -1 gpurun_out/b10_k6_onerun.log
