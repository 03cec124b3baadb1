# PMC counters for k_count (separate passes, no tracing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
B="bench.py --k ${K:-6} --fasta-line ${L:-0} --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $OUT/p1 -o run -- python3 $B > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 $B > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d $OUT/p3 -o run -- python3 $B > $OUT/p3.log 2>&1 || { tail -5 $OUT/p3.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob, os
for f in sorted(glob.glob('gpurun_out/pmc/p*/run_counter_collection.csv')):
    agg=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if os.environ.get('KERNEL', 'k_count') in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k,v in sorted(agg.items()):
        print(k, '%.4g' % (sum(v)/len(v)))
PY
