# Round deliverables on the GPU box: profiles for k=6 (configs[1]) and k=11
# FASTA, then the default bench line (with the CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=6 L=0 OUT=gpurun_out/prof_k6 bash scripts/gpu_profile.sh > gpurun_out/prof_k6.log 2>&1 || { tail -20 gpurun_out/prof_k6.log; exit 1; }
K=11 L=80 STEPS=3 OUT=gpurun_out/prof_k11 bash scripts/gpu_profile.sh > gpurun_out/prof_k11.log 2>&1 || { tail -20 gpurun_out/prof_k11.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
