# skewed partition tests + 10 GB k=11 FASTA genome with the pairs path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "skewed" > gpurun_out/skew_tests.log 2>&1 || { tail -40 gpurun_out/skew_tests.log; exit 1; }
tail -1 gpurun_out/skew_tests.log
timeout -k 10 300 python bench.py --bases 10000000000 --k 11 --fasta-line 80 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b10_k11.log 2>&1 || { tail -5 gpurun_out/b10_k11.log; exit 1; }
tail -1 gpurun_out/b10_k11.log
