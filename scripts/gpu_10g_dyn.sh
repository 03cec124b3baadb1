#!/bin/bash
# 10 GB k=6 genome: static ranges vs dynamic tail (FK_STATIC_PCT)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pct in 100 95 90 80; do
  FK_STATIC_PCT=$pct timeout -k 10 200 python bench.py --no-cpu-baseline --bases 10000000000 --steps 10 --warmup 3 --timing-every 1 > gpurun_out/g10_$pct.json 2>/dev/null || { echo "$pct failed"; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/g10_$pct.json').read().strip().splitlines()[-1]);print('$pct', 'k_count_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'step %.4f' % d['ms_per_step'])"
done
