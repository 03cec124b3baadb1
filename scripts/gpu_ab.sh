# A/B of experiment builds (tools/exp_variant.py) against the product on one
# box, interleaved: VARIANTS="a b" [ARGS="bench.py args"] [ROUNDS=n]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 10 --warmup 3 --north-star-bases 0 --no-cpu-baseline"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in product $VARIANTS; do
    if [ $v = product ]; then lib=""; else lib=build/exp/libfk_$v.so; fi
    FINDKMER_LIB=$lib timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v failed"; tail -20 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']
print('%-12s step %.3f ms  %s %.3f ms' % ('$v', d['ms_per_step'], r['kernel'], r['kernel_ms']))"
  done
done
