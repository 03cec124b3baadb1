# k_part block size per k: FK_PART_WAVES=8 vs 16 on 1 GB 80-column FASTA, k = 9..12
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 9 10 11 12; do
for w in 8 16; do
FK_PART_WAVES=$w timeout -k 10 200 python bench.py --k $k --fasta-line 80 --steps 20 --no-cpu-baseline > gpurun_out/pw_${k}_$w.log 2>&1 || { tail -20 gpurun_out/pw_${k}_$w.log; exit 1; }
echo "k=$k W=$w $(grep '^{' gpurun_out/pw_${k}_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['kernel_ms']*1000,1))")"
done; done
