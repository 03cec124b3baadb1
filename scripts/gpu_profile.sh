# rocprofv3 kernel trace + PMC passes of one bench.py workload (separate runs:
# --pmc never together with a trace domain).  Then
#   python3 tools/profile_summary.py $OUT <tag> --k K --fasta-line L --input-bytes B
# K, L, BASES, SEED select the workload (default: the bench's headline,
# configs[2]: k=11 over 10 G bases of 80-column FASTA).  SQ=1 adds two SQ
# counter passes (LDS / VALU / wait cycles); TRACE_ONLY=1 skips the PMC passes.
# FINDKMER_LIB=build/exp/libfk_<name>.so profiles an experiment build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
K=${K:-11}; L=${L:-80}; BASES=${BASES:-10000000000}; SEED=${SEED:-2}
B="bench.py --k $K --fasta-line $L --bases $BASES --seed $SEED --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --north-star-bases 0"
run() {   # run <dir> <rocprofv3 options...>
  d=$1; shift
  timeout -k 10 ${TLIM:-240} rocprofv3 "$@" --output-format csv -d $OUT/$d -o run -- python3 $B > $OUT/$d.log 2>&1 \
    || { tail -20 $OUT/$d.log; exit 1; }
}
run trace --kernel-trace --stats
tail -1 $OUT/trace.log
[ "${TRACE_ONLY:-0}" = 1 ] && { echo profile-done; exit 0; }
run pmc1 --pmc FETCH_SIZE
run pmc2 --pmc WRITE_SIZE
if [ "${SQ:-0}" = 1 ]; then
  run pmc3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
  run pmc4 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
fi
echo profile-done
