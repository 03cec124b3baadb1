# fk_input_load thread / chunk shape on 2 GB and 10 GB upstream-like files
# (page cache): FINDKMER_TIMES=1 read + copy rates of ./findKmer -k 6 -z 100
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/e2e
export TMPDIR=/tmp
for s in 3 4 5 6 7; do python tools/make_upstream.py /tmp/e2e/part$s 2e9 $s > /dev/null || exit 1; echo "part $s written"; done
cp /tmp/e2e/part3 /tmp/e2e/up2.fas
cat /tmp/e2e/part3 /tmp/e2e/part4 /tmp/e2e/part5 /tmp/e2e/part6 /tmp/e2e/part7 > /tmp/e2e/up10.fas && rm -f /tmp/e2e/part*
cd /tmp/e2e
timeout -k 10 300 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p up10.fas > /dev/null 2> /dev/null || exit 1
for rep in 1 2; do
for f in up2.fas up10.fas; do
for shape in 4:2 8:2 12:2 16:2 8:4; do
T=${shape%:*}; C=${shape#*:}
s=$(date +%s.%N)
FINDKMER_INGEST_THREADS=$T FINDKMER_INGEST_CHUNK_MB=$C FINDKMER_TIMES=1 timeout -k 10 120 $GRAFT_REPO_ROOT/findKmer -q 1 -k 6 -z 100 -p $f > /dev/null 2> /tmp/e2e/t.txt || exit 1
e=$(date +%s.%N)
echo "$f T=$T C=$C wall $(python3 -c "print(round($e-$s,3))") s | $(grep 'read + copy' /tmp/e2e/t.txt)"
done
done
done
