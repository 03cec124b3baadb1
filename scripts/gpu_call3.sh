# kernel traces (1 G bases) for the product and experiment builds, per k
set -o pipefail
cd $GRAFT_REPO_ROOT
for k in ${KS:-16 15}; do
  echo "#### k=$k"
  LIBS="${LIBS:-product build/exp/libfk_old.so}" STEPS=4 BARGS="--k $k --fasta-line 80 --bases 1000000000" \
    bash scripts/gpu_trace.sh 2>&1 | grep -v "^Traceback\|^  File\|^    \|JSONDecodeError" || exit 1
  mkdir -p gpurun_out/k$k && cp -r gpurun_out/tr_* gpurun_out/k$k/ 2>/dev/null
done
