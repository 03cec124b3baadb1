# -q 0 (per-record progress lines) cost on an upstream-like FASTA
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/q0
python tools/make_upstream.py /tmp/q0/up.fas 2e7 3
cd /tmp/q0
for q in 1 0; do
s=$(date +%s.%N); timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q $q -k 6 -p up.fas > out_q$q.txt 2>&1 || { tail -5 out_q$q.txt; exit 1; }; e=$(date +%s.%N)
echo "q=$q $(echo "$e - $s" | python3 -c 'import sys; print(eval(sys.stdin.read()))') s"
done
