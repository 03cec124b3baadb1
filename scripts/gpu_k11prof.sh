# full GPU suite, then the k=11 FASTA kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k11p -o run -- python3 bench.py --k 11 --fasta-line 80 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/k11p.log 2>&1 || { tail -5 gpurun_out/k11p.log; exit 1; }
grep '"metric"' gpurun_out/k11p.log
