# rocprofv3 kernel trace of a short bench run: per-kernel stats and the
# kernel/memset timeline of the last step (gaps between launches included)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/trace
mkdir -p $OUT
B="bench.py --k ${K:-6} --fasta-line ${L:-0} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT -o run -- python3 $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
python3 tools/trace_report.py $OUT
