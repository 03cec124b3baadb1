# whole GPU suite + smoke, then the plain / sharded (world 1) step costs
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/b_plain.log 2>&1 || { tail -20 gpurun_out/b_plain.log; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29510 bench.py --steps 50 --no-cpu-baseline > gpurun_out/b_native.log 2>&1 || { tail -20 gpurun_out/b_native.log; exit 1; }
for f in plain native; do echo "== $f $(grep '^{' gpurun_out/b_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('exchange'), d.get('transport'))")"; done
