# two ranks sharing cuda:0 over gloo: dist tests, then phase timing at 1 GB per rank
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -30 gpurun_out/dist_tests.log; exit 1; }
tail -1 gpurun_out/dist_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29777 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo --no-cpu-baseline > gpurun_out/dist2.log 2>&1 || { tail -20 gpurun_out/dist2.log; exit 1; }
grep '"metric"' gpurun_out/dist2.log
