# the sharded step at world 1 over RCCL (torchrun, one rank): the exchange's
# per-phase times for k = 6 (one all-reduce), k = 11 (stitched) and k = 16
# (the table sharded by its top index bits: reduce-scatter of 16 GiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "6 10000000000 0" "11 10000000000 80" "16 1000000000 80"; do
  set -- $cfg
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --k $1 --bases $2 --fasta-line $3 --steps 10 --warmup 3 --no-cpu-baseline --north-star-bases 0 \
    > gpurun_out/rccl1_k$1.json 2> gpurun_out/rccl1_k$1.err || { tail -20 gpurun_out/rccl1_k$1.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rccl1_k$1.json').read().strip().splitlines()[-1])
print('k=$1', 'step %.3f ms' % d['ms_per_step'], d.get('exchange'), d.get('transport'), d.get('rccl'), {k: round(v, 3) for k, v in d.get('phase_ms_per_step', {}).items()})"
done
