# end-to-end ./findKmer at k=11 without a z filter (4M-row CSV) on a 1 GB upstream-like FASTA
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e11
python tools/make_upstream.py /tmp/e2e11/up.fas 1e9 3
cd /tmp/e2e11
$GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -p up.fas > /dev/null 2>&1
for k in 11 6; do
s=$(date +%s.%N); timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k $k -p up.fas > out.txt 2>&1 || { tail -5 out.txt; exit 1; }; e=$(date +%s.%N)
echo "k=$k $(echo "$e - $s" | python3 -c 'import sys; print(eval(sys.stdin.read()))') s $(ls -la ${k}mer_Historam_Of_up.fas.csv | awk '{print $5}') bytes"
done
nproc
