# ingest threads for a 2 GB page-cache-resident file (FINDKMER_INGEST_THREADS)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e
python tools/make_upstream.py /tmp/e2e/up.fas 2e9 > /dev/null
cd /tmp/e2e
timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p up.fas > /dev/null 2> /dev/null || exit 1
for rep in 1 2; do for t in 8 16 24 32; do
FINDKMER_INGEST_THREADS=$t FINDKMER_TIMES=1 timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p up.fas 2>&1 > /dev/null | grep fk_input_load
done; done
