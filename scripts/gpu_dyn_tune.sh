#!/bin/bash
# k_count dynamic ranges: parity tests, then the bench's kernel time over the
# static share, and the per-wave finish spread (tools/wave_times.py)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "${1:-}" = tests ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "dynamic or eof_byte or onepass or shards or mixed_random" > gpurun_out/dyn_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dyn_tests.log; exit 1; }
tail -2 gpurun_out/dyn_tests.log
fi
for pct in 100 90 80 75 65 50; do
  FK_STATIC_PCT=$pct timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --timing-every 1 > gpurun_out/b_$pct.json 2>/dev/null || exit 1
  python - "$pct" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("pct", sys.argv[1], "step_ms %.4f" % d["ms_per_step"], "k_count_ms %.4f" % d["roofline"]["kernel_ms"], "frac %.3f" % d["roofline"]["frac"])
PY
done
FINDKMER_LIB=build/exp/libfk_wt.so timeout -k 10 120 python tools/wave_times.py > gpurun_out/wt_dyn.json 2>&1 && tail -c 1500 gpurun_out/wt_dyn.json
FK_STATIC_PCT=100 FINDKMER_LIB=build/exp/libfk_wt.so timeout -k 10 120 python tools/wave_times.py > gpurun_out/wt_static.json 2>&1 && tail -c 1500 gpurun_out/wt_static.json
