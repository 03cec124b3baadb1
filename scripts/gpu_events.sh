# cost of the timing events: host step split and bench with/without them
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/host_step_timing.py 2>&1 | grep -v amdgpu.ids
FK_NO_EVENTS=1 timeout -k 10 120 python tools/host_step_timing.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('events', d['ms_per_step'])"
FK_NO_EVENTS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('noevents', d['ms_per_step'])"
done
export TMPDIR=/tmp
FK_NO_EVENTS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tq/c -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/tq/c.log 2>&1
f=$(find gpurun_out/tq/c -name "*kernel_trace.csv" | head -1); cp $f gpurun_out/tq/c_trace.csv
