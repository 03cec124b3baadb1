# BASELINE configs[4] at its size: ./findKmer --sweep (k = 6..11, -q 1 -z 100,
# as k6thru11fullANDupstream.sh runs each k) on a 10 GB upstream-like FASTA
# (five 2 GB tools/make_upstream.py parts, seeds 3..7), then plain -k 6 and -k 11
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e
export TMPDIR=/tmp
df -h /tmp | tail -1
for s in 3 4 5 6 7; do python tools/make_upstream.py /tmp/e2e/part$s 2e9 $s > /dev/null || exit 1; echo "part $s written"; done
cat /tmp/e2e/part3 /tmp/e2e/part4 /tmp/e2e/part5 /tmp/e2e/part6 /tmp/e2e/part7 > /tmp/e2e/up10.fas && rm -f /tmp/e2e/part*
ls -la /tmp/e2e/up10.fas
cd /tmp/e2e
timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p up10.fas > /dev/null 2> /dev/null || exit 1
for run in 1 2; do
s=$(date +%s.%N); FINDKMER_TIMES=1 timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 --sweep 11 -p up10.fas > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/sweep10_times.txt || exit 1; e=$(date +%s.%N)
echo "sweep 6..11 wall $(python3 -c "print(round($e-$s,3))") s"; cat $GRAFT_REPO_ROOT/gpurun_out/sweep10_times.txt
done
for k in 6 11; do
s=$(date +%s.%N); FINDKMER_TIMES=1 timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k $k -z 100 -p up10.fas > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/k${k}_10_times.txt || exit 1; e=$(date +%s.%N)
echo "k=$k wall $(python3 -c "print(round($e-$s,3))") s"; cat $GRAFT_REPO_ROOT/gpurun_out/k${k}_10_times.txt
done
