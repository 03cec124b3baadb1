"""GPU parity at BASELINE.json's full sizes (10 GB inputs) against the CPU
oracle, bit-exact: the whole table (or, for 17 <= k <= 20, key ranges of it)
and every scalar the reference's outputs depend on.

The oracle runs the reference's scan (findKmer/src/findKmer.cpp:962-1069)
over the same bytes, copied back from the device, on the box's host threads
(fko_count_dense_par / fko_count_sparse_range: the stream in pieces, each
from its exact entering state).  Each 10 GB input is made once per module and
shared by the tests that read it.
"""
import numpy as np
import pytest

import findkmer_amd as fk
import oracle

pytestmark = pytest.mark.gpu

N10G = 10_000_000_000


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if fk.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")


@pytest.fixture(scope="module")
def genome10g():
    """configs[2]'s input: 10 G bases of 80-column FASTA, 1.5-Gbase
    chromosomes (bench.make_genome, seed 2) on the device, and its bytes on
    the host"""
    import torch
    import bench
    buf, size = bench.make_genome(N10G, 80, 2, bench.CHROM)
    torch.cuda.synchronize()
    host = buf[:size].cpu().numpy()
    yield buf, size, host
    del buf, host
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def upstream10g():
    """configs[4]'s input: a 10 GB upstream-regions-like FASTA (">ENST%011u"
    records of 1001 bases, 1 % of them with a 50-base N run;
    fk_synth_upstream_device, seed 3) on the device, and its bytes on the
    host"""
    import torch
    nrec = N10G // fk.FK_UPSTREAM_REC
    size = nrec * fk.FK_UPSTREAM_REC
    buf = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    assert fk.synth_upstream_device(buf.data_ptr(), size, nrec, 3) == size
    torch.cuda.synchronize()
    host = buf[:size].cpu().numpy()
    yield buf, size, host
    del buf, host
    torch.cuda.empty_cache()


def _engine_dense(k, ptr, size):
    with fk.Engine(k, want_nodes=True, collect_unknown=True) as e:
        e.feed_device(ptr, size)
        rc, r = e.finish()
        t = e.table()
        ub = e.unknown_bytes()
    return rc, r, t, ub


def _assert_dense_equal(k, host, rc, r_g, t_g, ub_g):
    assert rc == fk.FK_OK
    t_o, r_o, ub_o = oracle.count_dense(host, k, unknown_cap=1 << 16, threads=oracle.host_threads())
    bad = np.nonzero(t_o != t_g)[0]
    assert len(bad) == 0, f"k={k}: {len(bad)} bins differ, first {bad[:8]} oracle={t_o[bad[:8]]} gpu={t_g[bad[:8]]}"
    assert list(r_g.base_count) == list(r_o.base_count)
    assert (r_g.valid_bases, r_g.windows, r_g.distinct, r_g.nodes) == \
        (r_o.valid_bases, r_o.windows, r_o.distinct, r_o.nodes)
    assert list(r_g.depth1) == list(r_o.depth1)
    assert (r_g.unknown_chars, r_g.scanned_bytes, r_g.hit_eof_byte, r_g.unterminated_header) == \
        (r_o.unknown_chars, r_o.scanned_bytes, r_o.hit_eof_byte, r_o.unterminated_header)
    assert ub_g == ub_o
    return r_o


@pytest.mark.parametrize("k", [11, 12, 13])
def test_genome_10g_dense_vs_oracle(genome10g, k):
    """BASELINE.json configs[2] at its size (k = 11: the bench's headline)
    and the k > 11 paths north_star singles out on the same genome: k = 12
    (pairs mode, 2048 slices) and k = 13 (single windows, 2048 slices, the
    scan shared by all waves) -- whole tables against the oracle"""
    import bench
    buf, size, host = genome10g
    rc, r_g, t_g, ub_g = _engine_dense(k, buf.data_ptr(), size)
    assert r_g.windows == bench.expected_windows(N10G, k, bench.CHROM)
    _assert_dense_equal(k, host, rc, r_g, t_g, ub_g)


def _slices(k, width):
    """key ranges around 1/4, 1/3, 1/2, 2/3, 3/4 of the index space (where a
    key-range pass boundary falls for 2, 3 or 4 passes) and at both ends"""
    top = 1 << (2 * k)
    cs = [top // 4, top // 3, top // 2, 2 * top // 3, 3 * top // 4]
    out = [(0, width // 2)] + [(c - width // 2, c + width // 2) for c in cs] + [(top - width // 2, top)]
    return out


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_genome_10g_key_ranges_vs_oracle(genome10g, k):
    """17 <= k <= 20 at the configs' size: the 10 G-base genome through the
    key-range passes (several of them: the finished k = 17 table alone is
    ~90 GB); seven key ranges of the engine's table -- both ends of the index
    space and the points where 2, 3 or 4 passes meet -- key by key against
    the oracle's counts of the same ranges, plus every stream counter and
    the total distinct k-mers against the occupancy expectation"""
    import math
    import bench
    buf, size, host = genome10g
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), size)
        rc, r = e.finish()
        assert rc == fk.FK_OK
        width = 1 << 23
        ranges = _slices(k, width)
        got = [e.sparse_range(lo, hi) for lo, hi in ranges]
    keys_g = np.concatenate([g[0] for g in got])
    cnts_g = np.concatenate([g[1] for g in got])
    keys_o, cnts_o, r_o = oracle.count_sparse_range(host, k, ranges, threads=oracle.host_threads())
    assert len(keys_g) == len(keys_o) > 0
    assert np.array_equal(keys_g, keys_o)
    assert np.array_equal(cnts_g, cnts_o)
    assert r.windows == r_o.windows == bench.expected_windows(N10G, k, bench.CHROM)
    assert (r.valid_bases, list(r.base_count), list(r.depth1), r.scanned_bytes) == \
        (r_o.valid_bases, list(r_o.base_count), list(r_o.depth1), r_o.scanned_bytes)
    bins = float(1 << (2 * k))
    want = bins * -math.expm1(-r.windows / bins)
    assert abs(r.distinct - want) < 1e-3 * want, (r.distinct, want)


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_segmented_feeds_equal_one_feed(genome10g, k):
    """the fused first-base walks over many segments (every feed is one; a
    walk launch per segment, their rows and listed tiles shared) against one
    feed of the same 3 G bases: uneven device feeds, misaligned ones staged
    (retained copies) and aligned ones borrowed -- the same statistics and
    the same runs in seven key ranges"""
    buf, size, host = genome10g
    n = 3_000_000_000 + 12_345
    cuts = [0, 1 << 20, (1 << 20) + 17, 700_000_001, 700_000_001 + 4096, 1_900_000_000, n]
    ranges = _slices(k, 1 << 22)
    res = []
    for split, borrow in ((False, False), (True, True)):
        with fk.Engine(k, want_nodes=True, borrow_input=borrow) as e:
            if split:
                for a, b in zip(cuts[:-1], cuts[1:]):
                    e.feed_device(buf.data_ptr() + a, b - a)
            else:
                e.feed_device(buf.data_ptr(), n)
            rc, r = e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))
            got = [e.sparse_range(lo, hi) for lo, hi in ranges]
        res.append((r, got))
    (r1, g1), (r2, g2) = res
    assert (r1.windows, r1.distinct, r1.nodes, r1.valid_bases, list(r1.base_count), list(r1.depth1)) == \
        (r2.windows, r2.distinct, r2.nodes, r2.valid_bases, list(r2.base_count), list(r2.depth1))
    for (k1, c1), (k2, c2) in zip(g1, g2):
        assert np.array_equal(k1, k2) and np.array_equal(c1, c2)
    assert sum(len(x[0]) for x in g1) > 0


@pytest.mark.parametrize("k", [14, 15, 16])
def test_genome_1g_table_range_vs_oracle(k):
    """k = 14 (4096 slices of 2^16 bins, k_bucket16), k = 15 and k = 16 (the
    second partition level, k_repart + k_count_parts: 16 parts per coarse
    slice at k = 15, 64 at k = 16; a 4 / 16 GiB table) over 1 G bases
    of the 80-column genome: table ranges against the oracle's counts of the
    same key ranges"""
    import torch
    import bench
    n = 1_000_000_000
    buf, size = bench.make_genome(n, 80, 2, 0)
    torch.cuda.synchronize()
    host = buf[:size].cpu().numpy()
    width = 1 << 22
    ranges = _slices(k, width)
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), size)
        rc, r = e.finish()
        assert rc == fk.FK_OK
        parts = [e.table_range(lo, hi - lo) for lo, hi in ranges]
    del buf
    torch.cuda.empty_cache()
    keys_g = np.concatenate([np.nonzero(p)[0].astype(np.uint64) + lo for p, (lo, hi) in zip(parts, ranges)])
    cnts_g = np.concatenate([p[p != 0] for p in parts])
    keys_o, cnts_o, r_o = oracle.count_sparse_range(host, k, ranges, threads=oracle.host_threads())
    assert len(keys_o) > 0
    assert np.array_equal(keys_g, keys_o) and np.array_equal(cnts_g, cnts_o)
    assert (r.windows, r.valid_bases, list(r.base_count), list(r.depth1)) == \
        (r_o.windows, r_o.valid_bases, list(r_o.base_count), list(r_o.depth1))


def test_north_star_genome_10g_vs_oracle():
    """The north-star gate's workload: k = 6 over 10 G pure-ACGT bases
    (1.5-Gbase chromosomes, seed 1), whole table against the oracle"""
    import torch
    import bench
    buf, size = bench.make_genome(N10G, 0, 1, bench.CHROM)
    torch.cuda.synchronize()
    rc, r_g, t_g, ub_g = _engine_dense(6, buf.data_ptr(), size)
    host = buf[:size].cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    assert r_g.windows == bench.expected_windows(N10G, 6, bench.CHROM)
    _assert_dense_equal(6, host, rc, r_g, t_g, ub_g)


@pytest.mark.parametrize("k", [6, 7, 8, 9, 10, 11])
def test_upstream_10g_sweep_vs_oracle(upstream10g, k):
    """BASELINE.json configs[4] at its size: the k = 6..11 sweep of
    k6thru11fullANDupstream.sh:16-24 over one device-resident 10 GB
    upstream-like FASTA (as ./findKmer --sweep counts it: one copy, one
    engine per k) -- a '>' line every 1019 bytes, so the header-dense paths
    (k_count's general tiles + k_resume's mixed tiles for k <= 7, k_part's
    second region k_part<RES> for k >= 8) at full size"""
    buf, size, host = upstream10g
    rc, r_g, t_g, ub_g = _engine_dense(k, buf.data_ptr(), size)
    r_o = _assert_dense_equal(k, host, rc, r_g, t_g, ub_g)
    assert r_o.windows > 0.98 * (N10G // fk.FK_UPSTREAM_REC) * (1001 - k + 1) * 0.99


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_low_complexity_2g_vs_oracle(k):
    """17 <= k <= 20 on skewed input: a 2 G-base
    low-complexity stream -- 1 G bases of poly-A, then 1 G bases of an
    (ACGTT)n repeat -- puts ~half of all windows on one key and the rest on
    five, so one sparse part holds a billion windows of one k-mer (k = 17:
    k_kp_count's 16-bit bins wrap and the part is counted again in 32-bit
    halves, while the chained scan's later parts wait on it; k = 20: the part
    is past k_kp_sort's LDS and the pass takes the library sort).  The
    distinct keys come from the oracle over a short stream with the same
    junction; their counts over the whole stream from the oracle's threaded
    scan (fko_count_sparse_range) -- the engine's whole table must equal them
    key for key, with every counter."""
    import torch
    half = 1_000_000_000
    dev = torch.device("cuda", 0)
    buf = torch.empty(2 * half + 64, dtype=torch.uint8, device=dev)
    buf[:half] = ord("A")
    buf[half:2 * half] = torch.tensor(list(b"ACGTT"), dtype=torch.uint8, device=dev).repeat(half // 5)
    torch.cuda.synchronize()
    size = 2 * half
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), size)
        rc, r = e.finish()
        assert rc == fk.FK_OK
        keys_g, cnts_g = e.sparse()
    host = buf[:size].cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    small = b"A" * 1000 + b"ACGTT" * 200
    keys_s, _, r_s = oracle.count_sparse(small, k)
    ranges = [(int(x), int(x) + 1) for x in sorted(keys_s)]
    got = [oracle.count_sparse_range(host, k, ranges[i:i + 8], threads=oracle.host_threads())
           for i in range(0, len(ranges), 8)]   # (the oracle takes 8 ranges a scan)
    keys_o = np.concatenate([g[0] for g in got])
    cnts_o = np.concatenate([g[1] for g in got])
    r_o = got[0][2]
    assert len(keys_o) == len(keys_s) == r.distinct
    assert np.array_equal(np.asarray(keys_g, dtype=np.uint64), keys_o)
    assert np.array_equal(np.asarray(cnts_g, dtype=np.uint32), cnts_o)
    assert int(cnts_o.max()) > half - k   # the poly-A k-mer
    assert (r.windows, r.valid_bases, list(r.base_count), list(r.depth1), r.scanned_bytes) == \
        (r_o.windows, r_o.valid_bases, list(r_o.base_count), list(r_o.depth1), r_o.scanned_bytes)
