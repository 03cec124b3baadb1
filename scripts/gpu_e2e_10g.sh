# BASELINE configs[4] at its size: ./findKmer --sweep (k = 6..11, -q 1 -z 100,
# as k6thru11fullANDupstream.sh runs each k) on a 10 GB upstream-like FASTA
# (tools/write_upstream.py: fk_synth_upstream_device's records, the bytes
# tests/test_gpu_scale.py checks against the oracle), then plain -k 6 and -k 11
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e
export TMPDIR=/tmp
df -h /tmp | tail -1
timeout -k 10 300 python3 tools/write_upstream.py /tmp/e2e/up10.fas 1e10 3 || exit 1
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
sha256sum 6mer_Historam_Of_up10.faszScoreFiltered.csv 11mer_Historam_Of_up10.faszScoreFiltered.csv 2>/dev/null | cut -c1-16
