set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-prod e9}; do
  if [ $v = prod ]; then L=""; else L=$PWD/build/exp/libfk_$v.so; fi
  FINDKMER_LIB=$L timeout -k 10 120 python bench.py --k ${K:-6} --fasta-line ${FL:-80} --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/expf_$v.log 2>&1 || { tail -5 gpurun_out/expf_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/expf_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms']*1000,1), 'us main kernel', round(d['ms_per_step']*1000,1), 'us/step')"
done
