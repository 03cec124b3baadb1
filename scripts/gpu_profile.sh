# rocprofv3 kernel trace + PMC passes (separate runs, no sys-trace with pmc)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
K=${K:-6}; L=${L:-0}
B="bench.py --k $K --fasta-line $L --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 $B > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 $B > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc3 -o run -- python3 $B > $OUT/pmc3.log 2>&1 || { tail -20 $OUT/pmc3.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc4 -o run -- python3 $B > $OUT/pmc4.log 2>&1 || { tail -20 $OUT/pmc4.log; exit 1; }
find $OUT -name "*.csv" | head -20
