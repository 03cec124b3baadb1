# round 3, first GPU pass: the full-size config tests, the bench line, the
# headline profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_shards_summaries_take_both_paths" \
  "tests/test_gpu_parity.py::test_baseline_genome_10g_vs_oracle" \
  "tests/test_gpu_dist.py::test_configs3_eight_ranks_full_size" > gpurun_out/r03a_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03a_tests.log; exit 1; }
tail -5 gpurun_out/r03a_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/r03a_bench.log 2>&1 || { tail -20 gpurun_out/r03a_bench.log; exit 1; }
tail -1 gpurun_out/r03a_bench.log
OUT=gpurun_out/prof_k11 bash scripts/gpu_profile.sh
