#!/bin/bash
# k_count static shares per wave class (FK_CLASS_W) x static percentage
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --timing-every 1 > gpurun_out/c_$label.json 2>/dev/null || { echo "$label failed"; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c_$label.json').read().strip().splitlines()[-1]);print('$label', 'k_count_ms %.4f' % d['roofline']['kernel_ms'], 'step %.4f' % d['ms_per_step'])"
}
run static FK_STATIC_PCT=100
for pct in 97 93 90 85; do
  run w1_$pct FK_STATIC_PCT=$pct FK_CLASS_W=1168,1048,957,825
  run w2_$pct FK_STATIC_PCT=$pct FK_CLASS_W=1250,1080,930,740
  run w0_$pct FK_STATIC_PCT=$pct
done
FK_STATIC_PCT=90 FK_CLASS_W=1168,1048,957,825 FINDKMER_LIB=build/exp/libfk_wt.so timeout -k 10 120 python tools/wave_times.py 1e9 6 gpurun_out/wt_w1.npy 2>&1 | grep waves > gpurun_out/wt_w1.json
