# one-collective shard exchange: GPU dist tests (gloo ranks sharing cuda:0,
# RCCL world 1), then the k_tail timeline probe and the host step timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -60 gpurun_out/dist_tests.log; exit 1; }
tail -15 gpurun_out/dist_tests.log
timeout -k 10 120 python tools/tailprof.py 6 > gpurun_out/tailprof.log 2>&1 || { tail -20 gpurun_out/tailprof.log; exit 1; }
timeout -k 10 120 python tools/host_step_timing.py > gpurun_out/hoststep.log 2>&1 || { tail -20 gpurun_out/hoststep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tailprof.log gpurun_out/hoststep.log
