# k=11 80-column FASTA: FK_PART_WAVES=8 vs 16, interleaved, 3 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for w in 8 16; do
FK_PART_WAVES=$w timeout -k 10 200 python bench.py --k 11 --fasta-line 80 --steps 30 --no-cpu-baseline > gpurun_out/pw11_$w.log 2>&1 || { tail -20 gpurun_out/pw11_$w.log; exit 1; }
echo "rep=$rep W=$w $(grep '^{' gpurun_out/pw11_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['kernel_ms']*1000,1))")"
done; done
