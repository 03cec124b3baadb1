# kernel breakdown of the config-5 (upstream-like FASTA) engine pass, k=6 and k=11
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/upprof -o run -- python3 tools/upstream_bench.py /tmp/up1g.fas 6 11 > gpurun_out/upprof.log 2>&1 || { tail -5 gpurun_out/upprof.log; exit 1; }
grep k6_ms gpurun_out/upprof.log
