# config-5 header-dense FASTA: kernel breakdown (k=6, 11) and k_resume PMC (k=6)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/upprof -o run -- python3 tools/upstream_bench.py /tmp/up1g.fas 6 11 > gpurun_out/upprof.log 2>&1 || { tail -5 gpurun_out/upprof.log; exit 1; }
tail -1 gpurun_out/upprof.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/uppmc -o run -- python3 tools/upstream_bench.py /tmp/up1g.fas 6 > gpurun_out/uppmc.log 2>&1 || { tail -5 gpurun_out/uppmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d gpurun_out/uppmc2 -o run -- python3 tools/upstream_bench.py /tmp/up1g.fas 6 > gpurun_out/uppmc2.log 2>&1 || { tail -5 gpurun_out/uppmc2.log; exit 1; }
for g in 1 2; do echo "general_tiles=$g $(FK_GENERAL_TILES=$g timeout -k 10 120 python tools/upstream_bench.py /tmp/up1g.fas 6 11 2>/dev/null | tail -1)"; done
find gpurun_out/upprof gpurun_out/uppmc gpurun_out/uppmc2 -name "*.csv" | head
