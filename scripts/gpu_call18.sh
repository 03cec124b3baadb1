# round-6 end (r06d): the whole -m gpu suite + smoke, the default bench line,
# and traces of k = 15, 16 (1 G bases) and k = 17, 20 (10 G) after the
# one-pass k_repart
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_suite.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r06d_bench.json 2> gpurun_out/r06d_bench.err || { tail -20 gpurun_out/r06d_bench.err; exit 1; }
tail -1 gpurun_out/r06d_bench.json | cut -c1-200
for k in 15 16; do
  OUT=gpurun_out/r06d_k$k K=$k BASES=1000000000 TRACE_ONLY=1 bash scripts/gpu_profile.sh || exit 1
done
for k in 17 20; do
  OUT=gpurun_out/r06d_k$k K=$k STEPS=3 TRACE_ONLY=1 TLIM=300 bash scripts/gpu_profile.sh || exit 1
done
echo final-done
