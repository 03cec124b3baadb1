# PMC of k_resume / k_count on the header-dense FASTA (k=6)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/uppmc -o run -- python3 tools/upstream_bench.py /tmp/up1g.fas 6 > gpurun_out/uppmc.log 2>&1 || { tail -5 gpurun_out/uppmc.log; exit 1; }
echo done
