# A/B: product build vs build/exp/libfk_head.so (k=6 pure, k=6 FASTA, header-dense k=6)
set -o pipefail
cd $GRAFT_REPO_ROOT
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
for rep in 1 2; do
for lib in "" build/exp/libfk_head.so; do
for L in 0 80; do
FINDKMER_LIB=$lib timeout -k 10 300 python bench.py --k 6 --fasta-line $L --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "lib=${lib:-product} L=$L $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
done
done
