# k=6 at 10 GB (north-star size), k=6 FASTA and k=11 FASTA/pure at 1 GB:
# one bench line each, main kernel and step times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/size_$tag.log 2>&1 || { tail -5 gpurun_out/size_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/size_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', r['kernel'], round(r['kernel_ms']*1000,1), 'us', round(r['achieved']), 'GB/s', round(r['frac'],3), '| step', round(d['ms_per_step']*1000,1), 'us', '%.4g' % d['value'], 'bases/s')"
}
run k6_10G --k 6 --bases 10000000000 --steps 10 --warmup 2 || exit 1
run k6_fasta --k 6 --fasta-line 80 --steps 20 --warmup 3 || exit 1
run k11_fasta --k 11 --fasta-line 80 --steps 10 --warmup 2 || exit 1
run k11_pure --k 11 --steps 10 --warmup 2 || exit 1
run k7 --k 7 --steps 20 --warmup 3 || exit 1
