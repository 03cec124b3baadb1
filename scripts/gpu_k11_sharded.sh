# k=11 FASTA: plain step vs the sharded step at world 1 over RCCL (stitched exchange)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --k 11 --fasta-line 80 --steps 20 --no-cpu-baseline > gpurun_out/k11_plain.log 2>&1 || { tail -20 gpurun_out/k11_plain.log; exit 1; }
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --k 11 --fasta-line 80 --steps 20 --no-cpu-baseline > gpurun_out/k11_sh.log 2>&1 || { tail -20 gpurun_out/k11_sh.log; exit 1; }
for f in plain sh; do echo "== $f $(grep '^{' gpurun_out/k11_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('exchange'), d.get('phase_ms_per_step'))")"; done
