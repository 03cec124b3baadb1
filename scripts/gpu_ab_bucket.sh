# A/B of an engine library variant (build/exp/libfk_$V.so) on the FASTA
# steps of the partitioned path, then a kernel trace of each at k=11
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-bo1}
for rep in 1 2; do
for K in ${KS:-11 8 12}; do
for lib in "" build/exp/libfk_$V.so; do
FINDKMER_LIB=$lib timeout -k 10 120 python bench.py --k $K --fasta-line 80 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "k=$K lib=${lib:-product} $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'ms/step')")"
done
done
done
for lib in "" build/exp/libfk_$V.so; do
rm -rf gpurun_out/prof_ab
FINDKMER_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o run -- python3 bench.py --k 11 --fasta-line 80 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ab.log 2>&1 || { tail -20 gpurun_out/prof_ab.log; exit 1; }
echo "lib=${lib:-product}"
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof_ab/*kernel_stats.csv')[0])):
    if 'bucket' in r['Name'] or 'k_part' in r['Name']: print(' ', r['Name'][:32], r['Calls'], round(float(r['AverageNs'])/1000,1))
"
done
