# config 5 engine time on a device-resident 1 GB upstream-like FASTA, general-tile budgets
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
for gt in default 32 128; do
if [ $gt = default ]; then unset FK_GENERAL_TILES; else export FK_GENERAL_TILES=$gt; fi
echo "general_tiles=$gt $(timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 7 9 11 2>/dev/null | tail -1)"
done
