# kernel + memory-copy timeline of the world-1 sharded step (fast exchange)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29514 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ftrace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ftrace.log 2>&1 || { tail -20 gpurun_out/ftrace.log; exit 1; }
grep '^{' gpurun_out/ftrace.log | cut -c1-300
ls gpurun_out/ftrace
