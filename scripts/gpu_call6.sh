# kernel traces of the sparse k = 17 step (10 G bases) for the product and the k_kp_count ablations
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="product build/exp/libfk_kpx_nolb.so build/exp/libfk_kpx_noout.so build/exp/libfk_kpx_nocnt.so" STEPS=3 \
  BARGS="--k 17 --fasta-line 80 --bases 10000000000" bash scripts/gpu_trace.sh 2>&1 | grep -v "^Traceback\|^  File\|^    \|JSONDecodeError"
