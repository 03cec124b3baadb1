# A/B of engine library variants on the k=6 1 GB bench (interleaved runs)
# usage: LIBS="default build/exp/libfk_d4.so" bash scripts/gpu_ab_lib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${K:-6}; L=${L:-0}
for rep in 1 2; do
  for lib in $LIBS; do
    tag=$(basename $lib .so)_$rep
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --k $K --fasta-line $L --steps 40 --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
    else
      FINDKMER_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --k $K --fasta-line $L --steps 40 --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
    fi
    echo "$tag $(grep '^{' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['kernel_ms']*1000,1))")"
  done
done
