# the sharded step at world 1 over RCCL (torchrun, one rank): the exchange's
# per-phase times.  CONFIGS="k:bases:line[:tune] ..." (default: k = 6, one
# all-reduce; k = 11, stitched; k = 16, the table sharded by its top index
# bits -- routed blobs, and with tune route=0 the 16 GiB reduce-scatter)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CONFIGS:-6:10000000000:0 11:10000000000:80 16:1000000000:80 16:1000000000:80:route=0}; do
  IFS=: read k n l tune <<< "$cfg"
  tag=k${k}_${tune:-default}
  FINDKMER_TUNE=$tune timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --k $k --bases $n --fasta-line $l --steps 10 --warmup 3 --no-cpu-baseline \
    --north-star-bases 0 --weak-bases 0 > gpurun_out/rccl1_$tag.json 2> gpurun_out/rccl1_$tag.err \
    || { tail -20 gpurun_out/rccl1_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rccl1_$tag.json').read().strip().splitlines()[-1])
print('$tag', 'step %.3f ms' % d['ms_per_step'], d.get('exchange'), d.get('transport'), d.get('rccl'), {k: round(v, 3) for k, v in d.get('phase_ms_per_step', {}).items()})"
done
