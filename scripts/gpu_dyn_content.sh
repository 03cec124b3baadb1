#!/bin/bash
# dynamic tail vs static ranges on content-dependent inputs: 1 GB 80-col
# FASTA (newline path) and a 1 GB upstream-like FASTA (a header every
# ~1 KB: general tiles), k=6 and k=7
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pct in 100 90 75; do
  FK_STATIC_PCT=$pct timeout -k 10 120 python bench.py --no-cpu-baseline --fasta-line 80 --steps 30 --warmup 5 --timing-every 1 > gpurun_out/f_$pct.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/f_$pct.json').read().strip().splitlines()[-1]);print('fasta80 pct $pct', 'k_count_ms %.4f' % d['roofline']['kernel_ms'], 'step %.4f' % d['ms_per_step'])"
done
timeout -k 10 300 python tools/make_upstream.py /tmp/up1g.fa 1000000000 > /dev/null || exit 1
for pct in 100 90 75; do
  echo "upstream pct $pct"
  FK_STATIC_PCT=$pct timeout -k 10 200 python tools/upstream_bench.py /tmp/up1g.fa 6 7 || exit 1
done
# timeline of the default bench (gaps between kernels and steps)
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/tr.log 2>&1 || exit 1
python tools/trace_report.py gpurun_out/tr | tail -14
