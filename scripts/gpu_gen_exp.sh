# tile_general experiments on the upstream-like file (k=6): product, unrolled loops (e30), no window adds (e31)
set -o pipefail
cd $GRAFT_REPO_ROOT
python tools/make_upstream.py /tmp/up1g.fas 1e9 3
for lib in "" build/exp/libfk_e30.so build/exp/libfk_e31.so; do
echo "lib=${lib:-product} $(FINDKMER_LIB=$lib timeout -k 10 300 python tools/upstream_bench.py /tmp/up1g.fas 6 2>/dev/null | tail -1)"
done
