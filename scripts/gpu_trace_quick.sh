# kernel trace of short bench runs (one-pass on/off), per-kernel stats printed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tq}
mkdir -p $OUT
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline ${BARGS}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/a -o run -- python3 $B > $OUT/a.log 2>&1 || { tail -20 $OUT/a.log; exit 1; }
f=$(find $OUT/a -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
f=$(find $OUT/a -name "*kernel_trace.csv" | head -1); cp $f $OUT/a_trace.csv
FK_NO_ONEPASS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b -o run -- python3 $B > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
f=$(find $OUT/b -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
f=$(find $OUT/b -name "*kernel_trace.csv" | head -1); cp $f $OUT/b_trace.csv
