# native stitched exchange: GPU dist tests, then k=11 and k=6 sharded steps at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -60 gpurun_out/dist_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/dist_tests.log; tail -1 gpurun_out/dist_tests.log
bash scripts/gpu_k11_sharded.sh || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29514 bench.py --steps 50 --no-cpu-baseline > gpurun_out/b_native.log 2>&1 || { tail -20 gpurun_out/b_native.log; exit 1; }
echo "== k6 native $(grep '^{' gpurun_out/b_native.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('exchange'), d.get('transport'))")"
