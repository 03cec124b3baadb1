# the plain k=6 1 GB step vs the sharded step at world 1 over RCCL: native
# one-collective exchange (library communicator), the same through
# torch.distributed, and the stitched exchange; then the GPU dist tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/b_plain.log 2>&1 || { tail -20 gpurun_out/b_plain.log; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29510 bench.py --steps 50 --no-cpu-baseline > gpurun_out/b_native.log 2>&1 || { tail -20 gpurun_out/b_native.log; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 50 --no-cpu-baseline --torch-exchange > gpurun_out/b_fast.log 2>&1 || { tail -20 gpurun_out/b_fast.log; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 50 --no-cpu-baseline --stitched > gpurun_out/b_stitched.log 2>&1 || { tail -20 gpurun_out/b_stitched.log; exit 1; }
for f in plain native fast stitched; do echo "== $f"; grep '^{' gpurun_out/b_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('exchange'), d.get('transport'), d.get('phase_ms_per_step'))"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -60 gpurun_out/dist_tests.log; exit 1; }
tail -3 gpurun_out/dist_tests.log
