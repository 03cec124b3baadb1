# A/B of FINDKMER_TUNE knob settings against the defaults on bench workloads,
# interleaved: KNOBS="part_pipe=0 ..." (one setting per word), WORK="k:line:bases ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WORK=${WORK:-11:80:10000000000}
one() {   # one <label> <knobs or empty> <k> <line> <bases>
  if [ -n "$2" ]; then export FINDKMER_TUNE=$2; else unset FINDKMER_TUNE; fi
  timeout -k 10 240 python3 bench.py --k $3 --fasta-line $4 --bases $5 --steps ${STEPS:-10} --warmup 2 \
    --no-cpu-baseline --north-star-bases 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('k=$3 L=$4 n=$5 $1', round(d['ms_per_step'],3), 'ms/step', r['kernel'], round(r['kernel_ms'],3), 'ms')"
}
for w in $WORK; do
  IFS=: read k l n <<< "$w"
  for rep in 1 2; do
    one default "" $k $l $n || exit 1
    for v in $KNOBS; do one $v $v $k $l $n || exit 1; done
  done
done
