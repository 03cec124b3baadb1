# kernel trace of the routed k = 16 exchange at world 1 (one rank over RCCL,
# WORLD_SIZE=1 in the environment: bench.py joins the process group itself,
# no launcher under the profiler); TUNE=route=2 routes, route=0 reduce-scatters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/route}
mkdir -p $OUT
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29561}
for t in ${TUNES:-route=2 route=0}; do
  FINDKMER_TUNE=$t timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$t -o run -- \
    python3 bench.py --gpus 1 --k 16 --bases ${BASES:-1000000000} --fasta-line 80 --steps 10 --warmup 3 \
    --no-cpu-baseline --north-star-bases 0 --weak-bases 0 > $OUT/$t.log 2>&1 || { tail -20 $OUT/$t.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $OUT/$t.log
done
echo route-prof-done
