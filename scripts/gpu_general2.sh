# general-path change: GPU parity subset (general-heavy), header-dense FASTA timing
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
echo "upstream $(timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 2>/dev/null | tail -1)"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "k6 $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
echo "head upstream $(FINDKMER_LIB=build/exp/libfk_head.so timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 2>/dev/null | tail -1)"
for lib in "" build/exp/libfk_head.so; do
FINDKMER_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "lib=${lib:-product} k6 $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
