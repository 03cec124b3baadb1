# one-run streams past the int32 seqSize zone (SURVEY cfg 3 taken literally: one header, 1e10 bases)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --bases 3000000000 --k 11 --fasta-line 80 --chrom 0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/or_k11.log 2>&1 || { tail -5 gpurun_out/or_k11.log; exit 1; }
grep '^{' gpurun_out/or_k11.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k11 3e9 one run', d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --bases 3000000000 --k 11 --fasta-line 80 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/or_k11c.log 2>&1 || { tail -5 gpurun_out/or_k11c.log; exit 1; }
grep '^{' gpurun_out/or_k11c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k11 3e9 chromosomes', d['ms_per_step'], d['roofline']['kernel_ms'])"
