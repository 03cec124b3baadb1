# end-to-end CLI phase times (FINDKMER_TIMES=1) on a 2 GB upstream-like FASTA: --sweep 11 and a k=11 run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e
export TMPDIR=/tmp
python tools/make_upstream.py /tmp/e2e/up.fas 2e9 > /dev/null
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
cd /tmp/e2e
timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p up.fas > /dev/null 2> /dev/null || exit 1
s=$(date +%s.%N); FINDKMER_TIMES=1 timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 --sweep 11 -p up.fas > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/sweep_times.txt || exit 1; e=$(date +%s.%N)
echo "sweep wall $(python3 -c "print(round($e-$s,3))") s"; cat $GRAFT_REPO_ROOT/gpurun_out/sweep_times.txt
s=$(date +%s.%N); FINDKMER_TIMES=1 timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 11 -p up.fas > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/k11_times.txt || exit 1; e=$(date +%s.%N)
echo "k11 (no -z) wall $(python3 -c "print(round($e-$s,3))") s"; cat $GRAFT_REPO_ROOT/gpurun_out/k11_times.txt
