# HIP API + kernel trace of a short bench run: host-side cost of each runtime
# call in the last steps (no counters in this run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/apitrace
mkdir -p $OUT
B="bench.py --k ${K:-6} --fasta-line ${L:-0} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT -o run -- python3 $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
python3 tools/api_report.py $OUT
