# DPP scans (k_part batch scan, mixed tiles): parity suite, then A/B against
# the previous library on k=11 FASTA and the header-dense upstream-like FASTA
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
K=11 L=80 LIBS="default build/exp/libfk_prev.so" bash scripts/gpu_ab_lib.sh || exit 1
python tools/make_upstream.py /tmp/up1g.fas 1e9 3 > /dev/null
for rep in 1 2; do
echo "new  $(timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 11 2>/dev/null | tail -1)"
echo "prev $(FINDKMER_LIB=$GRAFT_REPO_ROOT/build/exp/libfk_prev.so timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 11 2>/dev/null | tail -1)"
done
