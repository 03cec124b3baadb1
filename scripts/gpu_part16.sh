# 16-wave k_part blocks: parity suite, then k = 8, 11, 12 FASTA steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
for k in 8 11 12; do
timeout -k 10 200 python bench.py --k $k --fasta-line 80 --steps 20 --no-cpu-baseline > gpurun_out/p16_$k.log 2>&1 || { tail -20 gpurun_out/p16_$k.log; exit 1; }
echo "k=$k $(grep '^{' gpurun_out/p16_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['kernel_ms']*1000,1))")"
done
