# A/B of experiment builds (tools/exp_variant.py, exp_rev.py)
# against the product on one box, interleaved: VARIANTS="a b" [ROUNDS=n]
# [WORK="k:line:bases ..."] (default: the bench's headline, configs[2])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WORK=${WORK:-11:80:10000000000}
for w in $WORK; do
  IFS=: read k l n <<< "$w"
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in product $VARIANTS; do
      if [ $v = product ]; then lib=""; else lib=build/exp/libfk_$v.so; fi
      FINDKMER_LIB=$lib timeout -k 10 240 python bench.py --k $k --fasta-line $l --bases $n --steps ${STEPS:-10} --warmup 3 \
        --north-star-bases 0 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err \
        || { echo "$v failed"; tail -20 gpurun_out/ab_$v.err; exit 1; }
      python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']
print('k=%-2s n=%-11s %-8s step %.3f ms  %s %.3f ms' % ('$k', '$n', '$v', d['ms_per_step'], r['kernel'], r['kernel_ms']))"
    done
  done
done
