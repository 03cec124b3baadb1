cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 -k "k16_dense" > gpurun_out/dbg.log 2>&1
tail -30 gpurun_out/dbg.log
