# k_bucket16 heavy-walk shapes (FINDKMER_TUNE b16s) at k = 14, 13, 12 (1 G bases)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 14 13 12; do
  for r in 1 2; do
    for s in 0 1 2 3; do
      FINDKMER_TUNE=b16s=$s timeout -k 10 240 python bench.py --k $k --fasta-line 80 --bases 1000000000 --steps 10 --warmup 3 \
        --north-star-bases 0 --no-cpu-baseline > gpurun_out/s.json 2> gpurun_out/s.err \
        || { echo "$k $s failed"; tail -20 gpurun_out/s.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/s.json'))
print('k=$k shape $s step %.3f ms' % d['ms_per_step'])"
    done
  done
done
echo done
