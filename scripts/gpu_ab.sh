# A/B of experiment builds (tools/exp_variant.py) against the product library
# on one bench workload, interleaved: VARIANTS="nt ntread", K, L, BASES
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${K:-11}; L=${L:-80}; BASES=${BASES:-10000000000}
one() {   # one <label> <lib or empty>
  if [ -n "$2" ]; then export FINDKMER_LIB=$2; else unset FINDKMER_LIB; fi
  timeout -k 10 240 python3 bench.py --k $K --fasta-line $L --bases $BASES --steps ${STEPS:-10} --warmup 2 \
    --no-cpu-baseline --north-star-bases 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['ms_per_step'],3), 'ms/step', r['kernel'], round(r['kernel_ms'],3), 'ms')"
}
for rep in 1 2; do
  one product ""
  for v in $VARIANTS; do one $v build/exp/libfk_$v.so; done
done
