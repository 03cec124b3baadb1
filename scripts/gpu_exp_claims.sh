#!/bin/bash
# k_count dynamic-range claim experiments (tools/exp.sh 40 41): kernel time
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --timing-every 1 > gpurun_out/x_$label.json 2>/dev/null || { echo "$label failed"; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/x_$label.json').read().strip().splitlines()[-1]);print('$label', 'k_count_ms %.4f' % d['roofline']['kernel_ms'], 'step %.4f' % d['ms_per_step'])"
}
run static FK_STATIC_PCT=100
run pool75 FK_STATIC_PCT=75
run priv_atomic75 FK_STATIC_PCT=75 FINDKMER_LIB=build/exp/libfk_e40.so
run priv_plain75 FK_STATIC_PCT=75 FINDKMER_LIB=build/exp/libfk_e41.so
run priv_plain90 FK_STATIC_PCT=90 FINDKMER_LIB=build/exp/libfk_e41.so
run priv_plain50 FK_STATIC_PCT=50 FINDKMER_LIB=build/exp/libfk_e41.so
