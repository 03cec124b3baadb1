"""GPU parity: the HIP engine (through the C-ABI) vs the CPU oracle, bit-exact.

Every comparison covers the full count table and every scalar the reference's
outputs depend on (base counts, baseCounter, windows, distinct, depth-1 trie
frequencies, nodeCounter, unknown bytes in order, bytes scanned).
"""
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

import findkmer_amd as fk
import oracle
from conftest import REPO, case_k, case_z, golden_file, golden_input

pytestmark = pytest.mark.gpu


def assert_same(data, k, want_nodes=True, feeds=None, ngpu_shards=None):
    t_o, r_o, ub_o = oracle.count_dense(data, k, unknown_cap=1 << 20)
    if ngpu_shards:
        t_g, r_g, ub_g, rc = shard_count(data, k, ngpu_shards)
    else:
        with fk.Engine(k, want_nodes=want_nodes, collect_unknown=True) as e:
            arr = np.frombuffer(bytes(data), dtype=np.uint8)
            if feeds is None:
                feeds = [len(arr)]
            pos = 0
            for n in feeds:
                if n:
                    e.feed(np.ascontiguousarray(arr[pos:pos + n]))
                pos += n
            assert pos == len(arr)
            rc, r_g = e.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER, fk.FK_E_ROLLOVER))
            t_g = e.table()
            ub_g = e.unknown_bytes()
    bad = np.nonzero(t_o != t_g)[0]
    assert len(bad) == 0, f"k={k}: {len(bad)} bins differ, first {bad[:8]} oracle={t_o[bad[:8]]} gpu={t_g[bad[:8]]}"
    assert list(r_g.base_count) == list(r_o.base_count)
    assert r_g.valid_bases == r_o.valid_bases
    assert r_g.windows == r_o.windows
    assert r_g.distinct == r_o.distinct
    assert list(r_g.depth1) == list(r_o.depth1)
    assert r_g.unknown_chars == r_o.unknown_chars
    assert ub_g == ub_o
    assert r_g.hit_eof_byte == r_o.hit_eof_byte
    assert r_g.unterminated_header == r_o.unterminated_header
    assert r_g.scanned_bytes == r_o.scanned_bytes
    if want_nodes and not ngpu_shards:
        assert r_g.nodes == r_o.nodes
    return r_g


def shard_count(data, k, nshards, summaries=False):
    """Exercise the multi-GPU shard protocol with several engines (on the one
    GPU of the test box): guess-from-halo, summaries, resolve, merge.
    summaries=True stitches as findkmer_amd/dist.py does: compose every
    shard's (compact) summary in order, and on FK_E_SUMMARY the full ones."""
    import torch
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    n = len(arr)
    chunk = 65536
    per = max(chunk, (n // nshards) // chunk * chunk)
    bounds = [min(i * per, n) for i in range(nshards)] + [n]
    dev = torch.from_numpy(arr.copy()).cuda() if n else torch.zeros(16, dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    engines = []
    for i in range(nshards):
        e = fk.Engine(k, collect_unknown=True)
        lo, hi = bounds[i], bounds[i + 1]
        halo = min(256, lo) // 16 * 16
        e.feed_shard_device(dev.data_ptr() + lo, hi - lo, halo)
        engines.append(e)
    if summaries:
        def chain(sums):
            st, ent = fk.FkState(), []
            for sm in sums:
                ent.append(st)
                st = fk.summary_apply(sm, st)
            return ent
        try:
            entering = chain([e.summary() for e in engines])
            shard_count.compact_ok += 1
        except fk.FindKmerError as err:
            assert err.code == fk.FK_E_SUMMARY
            entering = chain([e.summary_full() for e in engines])
            shard_count.compact_failed += 1
        for e, st in zip(engines, entering):
            e.resolve(st)
        # a full summary does not know where the stream ends: as dist.py
        # does, the shards after the first one that ended contribute nothing
        ends = [i for i, e in enumerate(engines) if e.state().ended]
        if ends:
            for e in engines[ends[0] + 1:]:
                e.reset()
    else:
        st = fk.FkState()
        for e in engines:
            e.resolve(st)
            st = e.state()
    base = engines[0]
    for e in engines[1:]:
        assert fk.lib().fk_engine_merge_from(base.h, e.h) == 0
    # table and counters are complete after the merge; end-of-stream fields
    # (short-run nodes, unterminated header) belong to the last shard
    rc, r = base.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER, fk.FK_E_ROLLOVER))
    t = base.table()
    ub = base.unknown_bytes()
    for e in engines:
        e.close()
    return t, r, ub, rc


shard_count.compact_ok = shard_count.compact_failed = 0


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if fk.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")


GOLDEN_INPUTS = ["test.txt", "edge.txt", "rand120k.fa", "missing.txt", "ffbyte.bin", "shortruns.txt"]


@pytest.mark.parametrize("name", GOLDEN_INPUTS)
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8, 11, 12])
def test_golden_inputs(name, k):
    assert_same(golden_input(name), k)


def random_text(rng, n, alphabet, weights):
    return bytes(rng.choices(alphabet, weights=weights, k=n))


def mixed_input(seed, n):
    """Random bytes with every class the scan distinguishes, long runs, lines
    of varying width and headers that cross chunk (64 KiB) boundaries."""
    rng = random.Random(seed)
    parts = []
    size = 0
    while size < n:
        r = rng.random()
        if r < 0.45:
            L = rng.randint(1, 5000)
            seq = random_text(rng, L, b"ACGT", [1, 1, 1, 1])
            w = rng.choice([0, 60, 80, 7, 1000])
            if w:
                seq = b"\n".join(seq[i:i + w] for i in range(0, len(seq), w))
            parts.append(seq)
        elif r < 0.55:
            parts.append(b">" + random_text(rng, rng.randint(0, 300), b"ACGTN >xyz\xff\r", [5, 5, 5, 5, 1, 2, 1, 1, 1, 1, 1, 1]) + b"\n")
        elif r < 0.60:
            parts.append(b">" + b"A" * rng.randint(60000, 140000) + b"\n")   # long header over a chunk edge
        elif r < 0.75:
            parts.append(random_text(rng, rng.randint(1, 40), b"ACGTNn\r\n\x00acgt1>", [3, 3, 3, 3, 2, 1, 1, 3, 1, 1, 1, 1, 1, 1, 1]))
        elif r < 0.80:
            parts.append(b"\n" * rng.randint(1, 3000))
        else:
            parts.append(random_text(rng, rng.randint(10000, 200000), b"ACGT", [4, 1, 1, 4]))
        size += len(parts[-1])
    return b"".join(parts)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("k", [2, 5, 6, 7, 9, 11, 13])
def test_mixed_random(seed, k):
    data = mixed_input(1000 + 2 * seed, 1_500_000 + 600_000 * seed)
    assert_same(data, k)


@pytest.mark.parametrize("k", [3, 6, 11])
def test_streaming_feeds_equal_one_shot(k):
    data = mixed_input(77, 2_000_000)
    rng = random.Random(5)
    feeds = []
    left = len(data)
    while left:
        n = min(left, rng.choice([1, 2, 15, 16, 17, 1000, 65536, 65537, 300000]))
        feeds.append(n)
        left -= n
    assert_same(data, k, feeds=feeds)


@pytest.mark.parametrize("k", [4, 6, 11])
@pytest.mark.parametrize("nshards", [2, 3, 5])
def test_shards_match_single(k, nshards):
    data = mixed_input(4242 + nshards, 1_200_000)
    # drop 0xFF and make sure it ends outside a header for the shard check
    data = data.replace(b"\xff", b"Z") + b"\nACGT"
    t_o, r_o, _ = oracle.count_dense(data, k)
    t_g, r_g, ub, rc = shard_count(data, k, nshards)
    assert np.array_equal(t_o, t_g)
    assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
    assert list(r_g.base_count) == list(r_o.base_count)


@pytest.mark.parametrize("k", [1, 6, 11, 16])
def test_edge_sizes(k):
    for data in [b"", b"A", b"ACGT" * 3, b">", b">abc", b"ACGT>x\n", b"\xff", b"AC\xffGT",
                 b"A" * 65535, b"A" * 65536, b"A" * 65537, b"C" * (3 * 65536 + 17)]:
        if k > 12:
            continue
        assert_same(data, k)


def test_k16_dense_table():
    """k=16: 4^16 u32 bins (16 GiB) in HBM; sampled bins vs the sparse oracle."""
    data = mixed_input(9, 800_000)
    codes, cnts, r = oracle.count_sparse(data, 16)
    with fk.Engine(16) as e:
        e.feed(np.frombuffer(data, dtype=np.uint8).copy())
        rc, rg = e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))
        # stream the 16 GiB table through host in 256 Mi-bin pieces
        step = 1 << 28
        seen = 0
        for first in range(0, 1 << 32, step):
            part = e.table_range(first, step)
            nz = np.nonzero(part)[0]
            sel = (codes >= first) & (codes < first + step)
            assert np.array_equal(nz.astype(np.uint64) + first, codes[sel])
            assert np.array_equal(part[nz], cnts[sel])
            seen += len(nz)
        assert seen == len(codes)
    assert rg.windows == r.windows and rg.distinct == r.distinct
    assert list(rg.base_count) == list(r.base_count)


def test_int32_seqsize_wrap():
    """A run longer than 2^31-1 bases: the reference stops counting windows
    when its int seqSize wraps (verified on the real binary: 'ACGTN' + A*(2^31+100)
    at k=2 gives AA=2147483646, AC=CG=GT=1, baseCounter 2147483651)."""
    import torch
    L = 2 ** 31 + 100
    buf = torch.full((5 + L,), ord("A"), dtype=torch.uint8, device="cuda")
    buf[:5] = torch.tensor(list(b"ACGTN"), dtype=torch.uint8)
    torch.cuda.synchronize()
    with fk.Engine(2) as e:
        e.feed_device(buf.data_ptr(), 5 + L)
        rc, r = e.finish()
        t = e.table()
    assert t[0] == 2147483646
    assert t[1] == 1 and t[6] == 1 and t[11] == 1
    assert int(t.sum()) == 2147483646 + 3
    assert r.valid_bases == 2147483651
    assert list(r.base_count) == [2147483648, 1, 1, 1]


def test_int32_seqsize_two_zones():
    """Run of 2^32 + 2^31 + 50 'A' at k=3: windows count for R in [3, 2^31-1]
    and again for R in [2^32+3, 2^32+2^31-1] (int32 seqSize climbs back to k)."""
    import torch
    L = 2 ** 32 + 2 ** 31 + 50
    k = 3
    buf = torch.full((L,), ord("A"), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), L)
        rc, r = e.finish(allow=(fk.FK_OK, fk.FK_E_ROLLOVER))
        t = e.table()
    z1 = (2 ** 31 - 1) - k + 1
    z2 = (2 ** 32 + 2 ** 31 - 1) - (2 ** 32 + k) + 1
    assert int(t[0]) == z1 + z2
    assert r.windows == z1 + z2
    # first windows of both zones add k bases each
    assert r.valid_bases == (z1 - 1 + k) + (z2 - 1 + k)
    del buf


@pytest.mark.parametrize("k,split,extra", [(11, 0, 1 << 22), (11, 0, 1 << 28), (11, 1 << 20, 1 << 28),
                                           (12, 0, 1 << 28), (8, 1 << 20, 1 << 28), (14, 0, 1 << 28),
                                           (15, 1 << 20, 1 << 28)])
def test_int32_zone_partitioned(k, split, extra):
    """8 <= k <= 15 on one run of random bases past 2^31-1 (the reference's
    int32 seqSize turns negative, findKmer.cpp:977): no windows in the zone,
    so the table is the table of the run's first 2^31-1 bases.  Most range
    guesses are wrong there, and the partitioned path recounts the segment
    from the exact states (resolve_and_fetch); split > 0 feeds the first
    `split` bytes separately, so that the table is not clean when the long
    segment starts (its snapshot is restored before the recount).  extra:
    bases past 2^31 (4 Mi: a few wrong ranges, cancelled by k_redo; 256 Mi:
    over 1/16 of the ranges, recounted)."""
    import torch
    L = 2 ** 31 + extra
    buf = torch.empty(L + 64, dtype=torch.uint8, device="cuda")
    assert fk.synth_device(buf.data_ptr(), L, L, 7, 0) == L
    torch.cuda.synchronize()
    with fk.Engine(k) as e:
        if split:
            e.feed_device(buf.data_ptr(), split)
        e.feed_device(buf.data_ptr() + split, L - split)
        rc, r = e.finish()
        t = e.table()
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), 2 ** 31 - 1)
        rc2, r2 = e.finish()
        t2 = e.table()
    del buf
    assert rc == rc2 == fk.FK_OK
    assert r.windows == r2.windows == 2 ** 31 - 1 - k + 1
    assert np.array_equal(t, t2)
    assert list(r.base_count) == list(r2.base_count) and r.valid_bases == r2.valid_bases
    assert list(r.depth1) == list(r2.depth1)


@pytest.mark.parametrize("k", [6, 11])
def test_full_size_properties(k):
    """BASELINE config sizes (1 GB stream, 1 GB of 80-col FASTA): exact
    totals, the oracle on a 64 MiB prefix, and a checksum of checksums."""
    import torch
    n = 1_000_000_000
    fasta = 80 if k == 11 else 0
    tot = fk.synth_size(n, fasta)
    buf = torch.empty(tot + 16, dtype=torch.uint8, device="cuda")
    w = fk.synth_device(buf.data_ptr(), tot, n, 1 if k == 6 else 2, fasta)
    assert w == tot
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), tot)
        rc, r = e.finish()
        t = e.table()
    assert r.windows == n - k + 1
    assert int(t.sum(dtype=np.uint64)) == r.windows
    assert r.valid_bases == n
    assert sum(r.base_count) == n
    # prefix parity with the oracle (synthetic bytes are identical on CPU)
    m = 64 << 20
    host = oracle.synth(m, 1 if k == 6 else 2, fasta)
    dev_prefix = buf[: len(host)].cpu().numpy()
    assert np.array_equal(host, dev_prefix)
    assert_same(host.tobytes(), k)


GOLD_CLI = ["test_k6", "test_k1", "test_k11", "test_k6_q0", "test_k0_default7", "test_k6_export",
            "test_k6_badopt", "edge_k3", "rand_k5", "rand_k6_z3", "rand_k8", "rand_k4_z2",
            "rand_k11", "missing_k3", "ffbyte_k3", "shortruns_k5", "empty_k3",
            "test_k15", "test_k20", "rand_k17", "rand_k19_z4", "shortruns_k18", "edge_k20", "ffbyte_k17",
            "up_k6", "up_k11_z3", "up_k7_q0"]


@pytest.mark.parametrize("case", GOLD_CLI)
def test_cli_matches_reference(case, manifest, tmp_path):
    """./findKmer (GPU) vs the golden outputs of the reference binary."""
    entry = manifest[case]
    shutil.copy(os.path.join(REPO, "tests", "golden", "inputs", entry["input"]), tmp_path / entry["input"])
    p = subprocess.run([os.path.join(REPO, "findKmer")] + entry["args"], cwd=tmp_path,
                       capture_output=True, timeout=300)
    ref_exit = entry["exit"]
    if ref_exit in (-11, -6, 134, 139):
        assert p.returncode == 0, p.stderr.decode()
    else:
        assert p.returncode == ref_exit
    import hashlib
    for kind, rec in entry["files"].items():
        got = open(tmp_path / rec["name"], "rb").read()
        assert hashlib.sha256(got).hexdigest() == rec["sha256"], (kind, got[:300])
    # stdout identical (the reference's own stdout ends where it crashes)
    assert p.stdout == golden_file(case, "stdout")
    # the reference dies in free() (findKmer.cpp:1370): drop glibc's abort line
    import re
    gerr = re.sub(rb"(?m)^[a-z_]+\(\): invalid pointer\n", b"", golden_file(case, "stderr"))
    assert p.stderr == gerr


def _run_cli(args, cwd, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    return subprocess.run([os.path.join(REPO, "findKmer")] + args, cwd=cwd, capture_output=True, timeout=300,
                          env=env)


@pytest.mark.parametrize("case", ["test_k6", "rand_k5", "rand_k6_z3", "rand_k11", "ffbyte_k3", "rand_k17"])
def test_cli_stream_ingest_matches_reference(case, manifest, tmp_path):
    """-q 1 runs load the file into HBM (fk_input_load); the streamed path
    (FINDKMER_INGEST=stream, 256 MiB host pieces) must give the same bytes"""
    entry = manifest[case]
    shutil.copy(os.path.join(REPO, "tests", "golden", "inputs", entry["input"]), tmp_path / entry["input"])
    p = _run_cli(entry["args"], tmp_path, {"FINDKMER_INGEST": "stream"})
    assert p.returncode == 0 or p.returncode == entry["exit"], p.stderr.decode()
    import hashlib
    for kind, rec in entry["files"].items():
        got = open(tmp_path / rec["name"], "rb").read()
        assert hashlib.sha256(got).hexdigest() == rec["sha256"], (kind, got[:300])
    assert p.stdout == golden_file(case, "stdout")


def test_cli_sweep_matches_reference_goldens(manifest, tmp_path):
    """config 5: `-k 6 -z 3 --sweep 11` over the upstream-like FASTA writes,
    for every k, the CSV and stats files the reference wrote in six runs"""
    import hashlib
    name = "upstream1m.fas"
    shutil.copy(os.path.join(REPO, "tests", "golden", "inputs", name), tmp_path / name)
    p = _run_cli(["-q", "1", "-k", "6", "-z", "3", "--sweep", "11", "-p", name], tmp_path)
    assert p.returncode == 0, p.stderr.decode()
    want_stdout = b""
    for k in range(6, 12):
        entry = manifest[f"up_k{k}_z3"]
        for kind, rec in entry["files"].items():
            got = open(tmp_path / rec["name"], "rb").read()
            assert hashlib.sha256(got).hexdigest() == rec["sha256"], (k, kind)
        want_stdout += golden_file(f"up_k{k}_z3", "stdout")
    assert p.stdout == want_stdout


@pytest.mark.parametrize("k", [3, 7, 11])
def test_device_input_matches_oracle(k, tmp_path):
    """fk_input_load (Python DeviceInput) -> one device feed == the oracle"""
    data = _long_header_input(21 + k, (40 << 20) + 12345)   # > one 32 MiB ingest chunk, ragged
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    t_o, r_o, ub_o = oracle.count_dense(data, k, unknown_cap=1 << 24)
    with fk.DeviceInput(str(path)) as inp, fk.Engine(k, collect_unknown=True) as e:
        assert inp.len == len(data)
        e.feed_device(inp.ptr, inp.len)
        rc, r = e.finish()
        t = e.table()
        ub = e.unknown_bytes()
    assert rc == fk.FK_OK
    assert np.array_equal(t, t_o)
    assert r.windows == r_o.windows and list(r.base_count) == list(r_o.base_count)
    assert ub == ub_o


def _header_mix(seed, n):
    """many short records, '>' inside header lines, N runs, runs shorter
    than k, lines of several widths, headers across 4 KiB chunk edges"""
    rng = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        out += b">" + bytes(rng.choices(b"ACGTN> x", k=rng.randint(0, 5000 if rng.random() < 0.05 else 60))) + b"\n"
        for _ in range(rng.randint(0, 4)):
            seq = bytes(rng.choices(b"ACGT", k=rng.choice([1, 3, 6, 7, 50, 900, 6000])))
            w = rng.choice([0, 60, 13])
            if w:
                seq = b"\n".join(seq[i:i + w] for i in range(0, len(seq), w))
            out += seq + rng.choice([b"", b"N", b"NNN", b"\n", b"q"])
    return bytes(out)


def _progress_model(data, k):
    """test-only model of the reference's -q 0 progress numbers
    (findKmer.cpp:996-1002, :1040-1057): baseCounter at every '>' that
    starts a comment line"""
    out, bc, run, hdr = [], 0, 0, False
    for i, c in enumerate(data):
        if hdr:
            if c == 10:
                hdr = False
            continue
        if c in b"ACGT":
            run += 1
            bc += k if run == k else (1 if run > k else 0)
        elif c == 10:
            continue
        else:
            run = 0
            if c == 62:
                out.append((i, bc))
                hdr = True
    return out


@pytest.mark.parametrize("k", [2, 6, 11])
def test_input_headers_match_model(k, tmp_path):
    """fk_input_headers (k_hdr_traj / k_hdr_list) == a byte loop, on records
    with '>' inside header lines, N runs and runs shorter than k, with
    headers across 4 KiB chunk edges; a 0xFF byte outside a header is
    refused (FK_E_STATE: the streamed path prints those files)"""
    data = _header_mix(200 + k, 300_000)
    path = tmp_path / "h.fa"
    path.write_bytes(data)
    want = _progress_model(data, k)
    with fk.DeviceInput(str(path)) as inp:
        pos, bases = inp.headers(k)
    assert len(want) > 50
    assert [int(p) for p in pos] == [p for p, _ in want]
    assert [int(b) for b in bases] == [b for _, b in want]
    path2 = tmp_path / "ff.fa"
    path2.write_bytes(data[:100_000] + b"ACGT\xffACGT" + data[100_000:])
    with fk.DeviceInput(str(path2)) as inp:
        with pytest.raises(fk.FindKmerError) as ei:
            inp.headers(k)
        assert ei.value.code == fk.FK_E_STATE


@pytest.mark.parametrize("k", [1, 6, 7, 11])
def test_cli_q0_progress_device_vs_stream(k, tmp_path):
    """-q 0 progress lines: device path (fk_input_headers) == streamed path
    (feeds split at every header, fk_engine_progress)"""
    data = _header_mix(100 + k, 2_000_000)
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    (a / "h.fa").write_bytes(data)
    (b / "h.fa").write_bytes(data)
    pa = _run_cli(["-q", "0", "-k", str(k), "-p", "h.fa"], a)
    pb = _run_cli(["-q", "0", "-k", str(k), "-p", "h.fa"], b, {"FINDKMER_INGEST": "stream"})
    assert pa.returncode == 0 and pb.returncode == 0, (pa.stderr[-500:], pb.stderr[-500:])
    assert pa.stdout.count(b"Read ") > 500
    assert pa.stdout == pb.stdout
    assert pa.stderr == pb.stderr
    for f in sorted(x.name for x in a.iterdir()):
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def _unknown_positions(data):
    """stream offsets of the bytes the reference warns about (:582-584): not
    A/C/G/T/N/'\n', outside '>' lines, before the first 0xFF outside one (:988)"""
    out, hdr = [], False
    for i, c in enumerate(data):
        if hdr:
            hdr = c != 10
            continue
        if c == 0x3E:
            hdr = True
        elif c == 0xFF:
            break
        elif c not in b"ACGTN\n":
            out.append(i)
    return out


def _unknown_records(seed, nrec):
    """FASTA records with soft-masked and stray bytes (warnings in most records)"""
    rng = random.Random(seed)
    recs = []
    for i in range(nrec):
        body = bytes(rng.choices(b"ACGTNacgxy*", weights=[20, 20, 20, 20, 2, 1, 1, 1, 1, 1, 1],
                                 k=rng.randint(0, 400)))
        recs.append(b">rec%d %s\n" % (i, bytes(rng.choices(b"abc xyz", k=rng.randint(0, 30)))) +
                    b"\n".join(body[j:j + 60] for j in range(0, len(body), 60)) + b"\n")
    return b"ACGTqACGT\n" + b"".join(recs) + b"ACGzTT\n"


@pytest.mark.parametrize("k", [4, 11, 17])
def test_unknown_positions(k):
    """collect_unknown=2: every unknown byte's stream offset, in order, over
    several feeds (what the CLI interleaves with the -q 0 progress lines)"""
    data = _unknown_records(5150 + k, 5000) + mixed_input(5150 + k, 300_000)
    want = _unknown_positions(data)
    arr = np.frombuffer(data, dtype=np.uint8)
    with fk.Engine(k, collect_unknown=2) as e:
        for a, b in ((0, 100_003), (100_003, 100_020), (100_020, 700_000), (700_000, len(arr))):
            e.feed(np.ascontiguousarray(arr[a:b]))
        e.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER))
        got = e.unknown_positions()
        ub = e.unknown_bytes()
    assert len(want) > 1000
    assert got.tolist() == want
    assert ub == bytes(data[i] for i in want)


def _run_merged(cmd, cwd, env_extra=None):
    """run cmd with stdout and stderr on one pipe (stdout fully buffered,
    stderr not); returns (combined output, exit code)"""
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run(cmd, cwd=cwd, stdin=subprocess.DEVNULL, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       env=env, timeout=300)
    return p.stdout, p.returncode


@pytest.mark.parametrize("ingest", ["device", "stream"])
def test_cli_q0_warnings_interleave_like_reference(ingest, tmp_path):
    """-q 0 with unknown characters: the reference prints each "Unknown
    character" warning (stderr, unbuffered, :582-584) during its scan, while
    its progress lines (stdout, :997) sit in stdio's buffer until a block
    fills.  With both streams on one pipe, the CLI's combined output must
    equal the reference binary's (oracle/_ref, compiled from the reference
    source) -- except that the reference's crash in free() at exit loses its
    last unflushed stdout block, so its output is a prefix of ours"""
    assert os.path.exists(oracle.REF_BIN), "oracle/_ref/findKmer_ref missing (make -C oracle)"
    data = _unknown_records(9, 300)
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    (a / "u.fa").write_bytes(data)
    (b / "u.fa").write_bytes(data)
    args = ["-q", "0", "-k", "4", "-p", "u.fa"]
    env = {"FINDKMER_INGEST": "stream"} if ingest == "stream" else None
    ours, rc = _run_merged([os.path.join(REPO, "findKmer")] + args, a, env)
    ref, _ = _run_merged([oracle.REF_BIN] + args, b)
    assert rc == 0, ours[-500:]
    assert ref.count(b"Unknown character") > 100 and ref.count(b"Read ") > 100
    # the reference's crash in free() at exit (:1370) may leave glibc's fatal
    # message at the end of its stderr (when there is no terminal to write it
    # to): it is no part of the program's output
    for tag in (b"free(): ", b"double free", b"munmap_chunk(): ", b"malloc(): ", b"corrupted "):
        cut = ref.rfind(tag)
        if cut >= 0 and len(ref) - cut < 256:
            ref = ref[:cut]
    i = next((i for i in range(min(len(ref), len(ours))) if ours[i] != ref[i]), None)
    assert ours.startswith(ref), (i, ref[max(0, (i or 0) - 80):(i or 0) + 80], ours[max(0, (i or 0) - 80):(i or 0) + 80])
    assert len(ours) - len(ref) <= 4096   # the reference's lost stdout block at most
    # what the reference lost is the end of our stdout alone (every warning
    # precedes it): run ours again with the streams apart and check the tail
    # byte for byte, so the final progress and "histogram creation" lines
    # are verified in merged mode too
    tail = ours[len(ref):]
    if tail:
        c = tmp_path / "c"
        c.mkdir()
        (c / "u.fa").write_bytes(data)
        p = _run_cli(args, c, env)
        assert p.returncode == 0
        assert p.stdout.endswith(tail), (tail[-200:], p.stdout[-200:])
        assert b"Unknown character" not in tail


@pytest.mark.parametrize("k0,k1", [(5, 9), (16, 17)])
def test_cli_sweep_matches_separate_runs(k0, k1, tmp_path):
    """--sweep k0..k1 over one device-resident read == separate runs
    (stdout concatenated, the same CSV and stats files per k); 16..17
    crosses from the dense table to the sparse one"""
    name = "mix.fa"
    data = _long_header_input(11, 3 << 20)
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    (a / name).write_bytes(data)
    (b / name).write_bytes(data)
    outs = []
    for k in range(k0, k1 + 1):
        p = _run_cli(["-q", "1", "-k", str(k), "-z", "2", "-p", name], a)
        assert p.returncode == 0, p.stderr.decode()
        outs.append(p)
    p = _run_cli(["-q", "1", "-k", str(k0), "-z", "2", "--sweep", str(k1), "-p", name], b)
    assert p.returncode == 0, p.stderr.decode()
    assert p.stdout == b"".join(o.stdout for o in outs)
    assert p.stderr == b"".join(o.stderr for o in outs)
    files = sorted(f.name for f in a.iterdir())
    assert files == sorted(f.name for f in b.iterdir()) and len(files) == 1 + 2 * (k1 - k0 + 1)
    for f in files:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def test_cli_device_ingest_large(tmp_path):
    """a 300 MB FASTA (several 32 MiB ingest chunks, ragged end): the
    device-resident path and the streamed path write identical files"""
    seq = oracle.synth(300_000_000, 5, 60)
    name = "big.fa"
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    raw = seq.tobytes() + b"ACGTN\n>tail\nGATTACA"
    (a / name).write_bytes(raw)
    (b / name).write_bytes(raw)
    pa = _run_cli(["-q", "1", "-k", "7", "-p", name], a)
    pb = _run_cli(["-q", "1", "-k", "7", "-p", name], b, {"FINDKMER_INGEST": "stream"})
    assert pa.returncode == 0 and pb.returncode == 0, (pa.stderr.decode(), pb.stderr.decode())
    assert pa.stdout == pb.stdout
    for f in sorted(x.name for x in a.iterdir()):
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


@pytest.mark.parametrize("k", [8, 10, 11, 12])
@pytest.mark.parametrize("kind", ["polyA", "period7", "fasta_polyA", "polyA_C"])
def test_partition_skewed(k, kind):
    """8 <= k <= 12 on inputs whose windows all fall in one or a few table
    slices: k_part batches of one run of up to 64 K entries (the 16-bit
    count field holds count - 1), k_bucket_count's
    long-run loop, pair and single slices (FASTA halves with a newline).
    polyA_C (A^30 C) puts hundreds of thousands of counts into two adjacent
    bins (kernel codes 0 and 1: ...A and ...C), each past 2^16"""
    n = 24 << 20
    if kind == "polyA":
        data = b"A" * n
    elif kind == "polyA_C":
        data = ((b"A" * 30 + b"C") * (n // 31 + 1))[:n]
    elif kind == "period7":
        data = (b"ACGTTGC" * (n // 7 + 1))[:n]
    else:
        line = b"A" * 60 + b"\n"
        data = b">x\n" + line * (n // len(line))
    assert_same(data, k, want_nodes=False)


@pytest.mark.parametrize("kind", ["mixed", "dense_records", "polyA", "fasta_polyA", "polyA_C", "acgt_feeds"])
def test_partition_k14(kind):
    """k = 14 through the partition: 4096 slices of 16-bit codes whose run
    cursors are packed two per LDS word, each slice counted by two
    k_bucket_count blocks (one per half of its 2^16 bins).  A poly-A batch
    puts all 64 K entries into slice 0 (the packed cursor reaching 2^16 at
    the batch's end), polyA_C two adjacent bins past 2^16 counts; headers
    every few hundred bytes send ranges to k_part<RES>; 1 GiB of oracle
    table, compared whole"""
    n = 12 << 20
    feeds = None
    if kind == "mixed":
        data = mixed_input(1414, n)
    elif kind == "dense_records":
        data = _dense_records(1415, n)
    elif kind == "polyA":
        data = b"A" * n
    elif kind == "polyA_C":
        data = ((b"A" * 30 + b"C") * (n // 31 + 1))[:n]
    elif kind == "fasta_polyA":
        line = b"A" * 60 + b"\n"
        data = b">x\n" + line * (n // len(line))
    else:
        data = oracle.synth(n, 14, 80).tobytes()
        feeds = [1_000_003, 17, 65_536, len(data) - 1_065_556]
    assert_same(data, 14, want_nodes=kind != "polyA", feeds=feeds)


def _assert_same_sparse_view(data, k, feeds=None, want_nodes=True):
    """14 <= k <= 16 (dense table): the table's nonzero bins, read in 2^28-bin
    ranges, and every scalar vs the sparse oracle"""
    codes, cnts, r = oracle.count_sparse(data, k, cap=len(data) + 16)
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    with fk.Engine(k, want_nodes=want_nodes, collect_unknown=True) as e:
        pos = 0
        for n in (feeds or [len(arr)]):
            e.feed(np.ascontiguousarray(arr[pos:pos + n]))
            pos += n
        assert pos == len(arr)
        rc, rg = e.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER))
        step = 1 << 28
        got_c, got_n = [], []
        for first in range(0, 1 << (2 * k), step):
            part = e.table_range(first, min(step, (1 << (2 * k)) - first))
            nz = np.nonzero(part)[0]
            got_c.append(nz.astype(np.uint64) + first)
            got_n.append(part[nz])
        ub = e.unknown_bytes()
    assert np.array_equal(np.concatenate(got_c), codes)
    assert np.array_equal(np.concatenate(got_n), cnts)
    assert (rg.windows, rg.distinct, rg.valid_bases) == (r.windows, r.distinct, r.valid_bases)
    assert list(rg.base_count) == list(r.base_count)
    assert list(rg.depth1) == list(r.depth1)
    assert (rg.unknown_chars, rg.scanned_bytes, rg.hit_eof_byte) == (r.unknown_chars, r.scanned_bytes, r.hit_eof_byte)
    if want_nodes:
        assert rg.nodes == r.nodes
    return rg


@pytest.mark.parametrize("k,tune", [(15, "glist_cap=1"), (16, "glist_cap=4096"), (15, "no_mixed=1"),
                                    (15, "part_general=5"), (12, "glist_cap=1"), (13, "glist_cap=1"),
                                    (14, "part_general=5")])
def test_fresh_table_window_list_never_truncates(k, tune, monkeypatch):
    """k = 12..16 right after a reset: k_count_parts / k_bucket16 (k_pair_fold
    at k = 12) write every bin (no zeroing) and the general tiles' windows go
    to a list added afterwards.
    A list forced tiny (glist_cap) overflows on header-dense input: the
    overflow is flagged on the device (FK_FAULT_LIST) and the segment counted
    again from its exact range states, never truncated.
    no_mixed (no fresh table) and a larger part_general budget (the list's
    capacity follows it) count exactly too"""
    data = _dense_records(1717 + k, 3 << 20)
    base = None
    if tune.startswith("glist_cap"):
        with fk.Engine(k) as e:   # the same feed with the list's own capacity
            e.feed(np.frombuffer(data, dtype=np.uint8).copy())
            base = e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))[1].redo_chunks
    monkeypatch.setenv("FINDKMER_TUNE", tune)
    rg = _assert_same_sparse_view(data, k)
    if base is not None:
        assert rg.redo_chunks > base   # the whole segment was counted again


@pytest.mark.parametrize("k,kind", [(15, "mixed"), (15, "dense_records"), (15, "polyA"), (15, "fasta_polyA"),
                                    (15, "acgt_feeds"), (16, "fasta_polyA"), (16, "acgt_feeds")])
def test_partition_k15_and_k16(k, kind):
    """k = 15, 16 through the two-level partition: k_part's 2048 coarse
    slices of 32-bit codes, k_repart splitting each into 16 / 64 contiguous
    16-bit part streams, k_count_parts counting each part in 2^15 LDS bins;
    poly-A puts every entry into coarse slice 0 and part 0 (one k_repart
    block takes the whole input); header-dense records send ranges to
    k_part<RES>"""
    n = 6 << 20
    feeds = None
    if kind == "mixed":
        data = mixed_input(1515 + k, n)
    elif kind == "dense_records":
        data = _dense_records(1516 + k, n)
    elif kind == "polyA":
        data = b"A" * n
    elif kind == "fasta_polyA":
        line = b"A" * 60 + b"\n"
        data = b">x\n" + line * (n // len(line))
    else:
        data = oracle.synth(n, k, 80).tobytes()
        feeds = [1_000_003, 17, 65_536, len(data) - 1_065_556]
    _assert_same_sparse_view(data, k, feeds, want_nodes=kind != "polyA")


def _long_header_input(seed, n):
    """ACGT runs with '>' lines longer than the 256-byte halo, so ranges
    start inside a header their halo cannot see the start of (the one-pass
    k_count's redo path), plus short lines and N runs"""
    rng = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        r = rng.random()
        if r < 0.5:
            seq = bytes(rng.choices(b"ACGT", k=rng.randint(1000, 30000)))
            w = rng.choice([0, 60, 80])
            if w:
                seq = b"\n".join(seq[i:i + w] for i in range(0, len(seq), w))
            out += seq
        elif r < 0.7:
            out += b">" + bytes(rng.choices(b"ACGTN x", k=rng.randint(300, 40000))) + b"\n"
        else:
            out += b"N" * rng.randint(1, 600)
    return bytes(out[:n]) + b"\n"


@pytest.mark.parametrize("k", [2, 5, 6, 7])
@pytest.mark.parametrize("want_nodes", [False, True])
def test_onepass_long_headers(k, want_nodes):
    data = _long_header_input(1000 + k, 600_000)
    assert_same(data, k, want_nodes=want_nodes)


@pytest.mark.parametrize("k", [3, 6, 7])
def test_onepass_reset_reuse(k):
    """the bench's cycle on one engine: reset, feed, finish, several times over
    different inputs (the one-pass k_count does the pending reset itself)"""
    inputs = [_long_header_input(7 + i, 150_000 + 40_000 * i) for i in range(3)]
    inputs.append(bytes(random.Random(5).choices(b"ACGT", k=300_000)))
    with fk.Engine(k) as e:
        for rep in range(2):
            for data in inputs:
                e.reset()
                e.feed(np.frombuffer(data, dtype=np.uint8).copy())
                rc, r_g = e.finish(allow=(fk.FK_OK,))
                t_g = e.table()
                t_o, r_o, _ = oracle.count_dense(data, k)
                assert np.array_equal(t_g, t_o)
                assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
                assert list(r_g.base_count) == list(r_o.base_count)
                assert r_g.distinct == r_o.distinct


@pytest.mark.parametrize("k", [4, 6, 7])
def test_onepass_many_headers_no_nodes(k):
    """headers every few hundred bytes: ranges run out of general tiles (the
    one-pass k_count's resume fallback), without nodeCounter (fresh reset)"""
    rng = random.Random(77 + k)
    out = bytearray()
    while len(out) < 400_000:
        out += b">" + bytes(rng.choices(b"ACGT xyz", k=rng.randint(5, 60))) + b"\n"
        out += bytes(rng.choices(b"ACGT", k=rng.randint(20, 300))) + b"\n"
    assert_same(bytes(out), k, want_nodes=False)


@pytest.mark.parametrize("k", [4, 6, 7, 11])
@pytest.mark.parametrize("nshards", [2, 3])
@pytest.mark.parametrize("kind", ["mixed", "long_headers", "acgt"])
def test_shards_summaries(k, nshards, kind):
    """dist.py's stitch on one GPU: compact summaries of one-pass shards,
    composed in order; the full transfer functions where one does not apply
    (a shard starting inside a header longer than the halo)"""
    if kind == "mixed":
        data = mixed_input(77 + nshards, 900_000).replace(b"\xff", b"Z") + b"\nACGT"
    elif kind == "long_headers":
        data = _long_header_input(500 + nshards, 900_000)
    else:
        data = bytes(random.Random(k).choices(b"ACGT", k=800_000))
    t_o, r_o, _ = oracle.count_dense(data, k)
    t_g, r_g, ub, rc = shard_count(data, k, nshards, summaries=True)
    assert np.array_equal(t_o, t_g)
    assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
    assert list(r_g.base_count) == list(r_o.base_count)


@pytest.mark.parametrize("k", [4, 6, 7])
def test_shards_summaries_take_both_paths(k):
    """dist.py's stitch takes both paths, on inputs built for each: pure ACGT
    shards (every compact summary applies), and a shard that starts inside a
    comment line longer than its 256-byte halo, made of bases only, so the
    halo looks like a run: the guess is wrong, the compact summary refuses
    the true entering state (FK_E_SUMMARY) and the full transfer functions
    are exchanged instead"""
    rng = random.Random(90 + k)
    ok0, failed0 = shard_count.compact_ok, shard_count.compact_failed
    acgt = random_text(rng, 600_000, b"ACGT", [1, 1, 1, 1])
    t_o, r_o, _ = oracle.count_dense(acgt, k)
    t_g, r_g, _, _ = shard_count(acgt, k, 2, summaries=True)
    assert np.array_equal(t_o, t_g) and r_g.windows == r_o.windows
    assert shard_count.compact_ok == ok0 + 1 and shard_count.compact_failed == failed0
    # shard_count cuts 600000 bytes into two shards at 262144 (4 x 64 KiB)
    cut = 262144
    data = bytearray(acgt)
    data[cut - 1000:cut + 2000] = b">" + random_text(rng, 2998, b"ACGT", [1, 1, 1, 1]) + b"\n"
    data = bytes(data)
    t_o, r_o, _ = oracle.count_dense(data, k)
    t_g, r_g, _, _ = shard_count(data, k, 2, summaries=True)
    assert np.array_equal(t_o, t_g)
    assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
    assert list(r_g.base_count) == list(r_o.base_count)
    assert shard_count.compact_failed == failed0 + 1, "the shard inside a long comment must refuse its compact summary"


def assert_same_sparse(data, k, feeds=None, borrow=False):
    """17 <= k <= 20: the engine's sparse table and scalars vs the oracle's.
    borrow: the feeds are slices of one device buffer and the engine re-reads
    them at finish instead of keeping a copy (fk_opts.borrow_input)"""
    keys_o, cnt_o, r_o = oracle.count_sparse(data, k, cap=max(16, len(data) + 16))
    dev = None
    if borrow:
        import torch
        dev = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
        dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        torch.cuda.synchronize()
    with fk.Engine(k, want_nodes=True, collect_unknown=True, borrow_input=borrow) as e:
        arr = np.frombuffer(bytes(data), dtype=np.uint8)
        if feeds is None:
            feeds = [len(arr)]
        pos = 0
        for n in feeds:
            if n and dev is not None:
                e.feed_device(dev.data_ptr() + pos, n)
            elif n:
                e.feed(np.ascontiguousarray(arr[pos:pos + n]))
            pos += n
        assert pos == len(arr)
        rc, r_g = e.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER, fk.FK_E_ROLLOVER))
        keys_g, cnt_g = e.sparse()
        ub_g = e.unknown_bytes()
    _, _, ub_o = oracle.count_dense(data, 3, unknown_cap=1 << 20)   # unknown bytes do not depend on k
    assert np.array_equal(keys_g, keys_o), (len(keys_g), len(keys_o))
    assert np.array_equal(cnt_g, cnt_o)
    assert list(r_g.base_count) == list(r_o.base_count)
    assert r_g.valid_bases == r_o.valid_bases and r_g.windows == r_o.windows
    assert r_g.distinct == r_o.distinct == len(keys_o)
    assert list(r_g.depth1) == list(r_o.depth1)
    assert r_g.nodes == r_o.nodes
    assert r_g.unknown_chars == r_o.unknown_chars and ub_g == ub_o
    assert r_g.hit_eof_byte == r_o.hit_eof_byte and r_g.scanned_bytes == r_o.scanned_bytes
    assert r_g.unterminated_header == r_o.unterminated_header


@pytest.mark.parametrize("name", GOLDEN_INPUTS)
@pytest.mark.parametrize("k", [17, 18, 20])
def test_sparse_golden_inputs(name, k):
    assert_same_sparse(golden_input(name), k)


@pytest.mark.parametrize("k", [17, 19, 20])
def test_sparse_mixed_and_streaming(k):
    data = mixed_input(900 + k, 400_000)
    assert_same_sparse(data, k)
    rng = random.Random(k)
    feeds, left = [], len(data)
    while left:
        n = min(left, rng.choice([1, 31, 4096, 70001, 150000]))
        feeds.append(n)
        left -= n
    assert_same_sparse(data, k, feeds=feeds)


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_borrowed_device_feeds(k):
    """fk_opts.borrow_input: device feeds (16-B aligned pieces of one buffer,
    one piece too short for the device path and one misaligned, which the
    engine stages and copies) re-read at finish from the caller's buffer"""
    data = mixed_input(1300 + k, 600_000)
    feeds = [4096, 160_000, 16, 7, 200_009, len(data) - 4096 - 160_000 - 16 - 7 - 200_009]
    assert_same_sparse(data, k, feeds=feeds, borrow=True)


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_long_headers_and_acgt(k):
    assert_same_sparse(_long_header_input(33 + k, 500_000), k)
    assert_same_sparse(bytes(random.Random(k).choices(b"ACGT", k=700_000)), k)


@pytest.mark.parametrize("k", [17, 20])
def test_sparse_key_range_passes(k, monkeypatch):
    """the sparse table built in many key-range passes: FINDKMER_TUNE sp_pass=N
    caps a sorted pass at N window keys (merged buckets), and a bucket with
    more windows than that is counted in a dense table (a poly-A stretch puts
    ~200k windows into bucket 0); boundaries between passes must not change
    the table, the statistics or nodeCounter"""
    monkeypatch.setenv("FINDKMER_TUNE", "sp_pass=5000")
    rng = random.Random(k)
    body = bytes(rng.choices(b"ACGT", k=150_000)) + b"A" * 200_000 + b"NN" + bytes(rng.choices(b"ACGTN", k=80_000))
    lines = b"\n".join(body[i:i + 70] for i in range(0, len(body), 70))
    assert_same_sparse(b">chr1\n" + lines + b"\n>chr2 x\nACGTAC\nGT\n", k)
    assert_same_sparse(mixed_input(1300 + k, 300_000), k)


@pytest.mark.parametrize("k", [17])
def test_sparse_count_bins_wrap_and_top_key(k):
    """k_kp_count's 16-bit bins: a 70 K-base poly-A stretch puts ~70 K windows
    into one bin of part 0 (the halves' sum falls short: the part is counted
    again in 32-bit halves), and a 70 K-base poly-T stretch ~70 K windows of
    the top key 4^k - 1, which k_kpart counts apart and the last part adds"""
    rng = random.Random(k)
    body = b"A" * 70_000 + bytes(rng.choices(b"ACGT", k=300_000)) + b"T" * 70_000
    lines = b"\n".join(body[i:i + 60] for i in range(0, len(body), 60))
    assert_same_sparse(b">w\n" + lines + b"\n", k)


@pytest.mark.parametrize("tune", ["sp_walk=0", "sp_walk_rows=1", "sp_walk_glist=1", "sp_walk_dbg=1"])
@pytest.mark.parametrize("k", [17, 20])
def test_sparse_walk_fallbacks(k, tune, monkeypatch):
    """the fused walks (k_sp_wpart) against the key-list passes: sp_walk=0
    takes the key lists; a row or general-tile list capacity of 1 overflows
    in the first walk and the finish restarts by the key lists; sp_walk_dbg=1
    sends every tile through k_sp_gtiles' list"""
    monkeypatch.setenv("FINDKMER_TUNE", tune)
    assert_same_sparse(mixed_input(1717 + k, 300_000), k)


def test_sparse_k17_walk_rows_split():
    """a batch of the fused walk with more windows of its pass than a row
    holds (poly-A: every window is key 0, 16 x 4 x 2048 of them a batch) is
    written as several rows; poly-T puts them all into the last pass"""
    body = b"A" * 400_000 + b"C" * 5 + b"T" * 300_000
    lines = b"\n".join(body[i:i + 61] for i in range(0, len(body), 61))
    assert_same_sparse(b">s\n" + lines + b"\n", 17)


def test_sparse_shared_walk_falls_back_alone(monkeypatch):
    """k=20, sp_pass=300000: ~4 wide passes share one emit walk; the first
    holds a poly-A stretch (100k windows of key 0, one part past k_kp_sort's
    LDS), takes the library sort and the walk is redone one pass at a time"""
    monkeypatch.setenv("FINDKMER_TUNE", "sp_pass=300000")
    rng = random.Random(20)
    body = b"A" * 100_000 + bytes(rng.choices(b"ACGT", k=1_000_000))
    lines = b"\n".join(body[i:i + 60] for i in range(0, len(body), 60))
    assert_same_sparse(b">p\n" + lines + b"\n", 20)


def test_sparse_every_bucket_dense(monkeypatch):
    """sp_pass=1: every nonempty bucket takes the dense path (k=17: 2^22 u64
    per bucket), golden inputs"""
    monkeypatch.setenv("FINDKMER_TUNE", "sp_pass=1")
    for name in ("edge.txt", "ffbyte.bin"):
        assert_same_sparse(golden_input(name), 17)


def test_sparse_dense_entry_points_refuse():
    """the dense-table calls answer FK_E_INVALID / FK_E_K_UNSUPPORTED for k > 16"""
    with fk.Engine(17) as e:
        e.feed(np.frombuffer(b"ACGT" * 100, dtype=np.uint8).copy())
        e.finish()
        with pytest.raises(fk.FindKmerError):
            e.table_range(0, 16)
    rc, _, _ = (None, None, None)
    assert fk.lib().fk_count(None, 0, 17, None, None, None) == fk.FK_E_K_UNSUPPORTED


# ---- k_count's dynamic ranges (k <= 7): static ranges, then claims --------
# static_pct < 100 turns them on (the product default is 100: static
# ranges only, measured as fast on plain streams) and dyn_min_chunks=1 for
# inputs of any size (else only segments of >= 8 chunks per wave slot), so
# the claim path, k_tail's per-range chain items and the multi-launch
# fallbacks over dynamic ranges all meet the oracle here.

@pytest.fixture
def dyn_env(monkeypatch):
    monkeypatch.setenv("FINDKMER_TUNE", "dyn_min_chunks=1,static_pct=75")
    yield


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("k", [2, 5, 6, 7])
def test_dynamic_ranges_mixed(dyn_env, seed, k):
    data = mixed_input(3000 + seed, 2_000_000 + 700_000 * seed)
    assert_same(data, k)
    assert_same(data, k, want_nodes=False)


@pytest.mark.parametrize("k", [3, 6, 7])
def test_dynamic_ranges_headers_and_resume(dyn_env, k):
    assert_same(_long_header_input(900 + k, 3_000_000), k, want_nodes=False)
    rng = random.Random(78 + k)
    out = bytearray()
    while len(out) < 2_000_000:
        out += b">" + bytes(rng.choices(b"ACGT xyz", k=rng.randint(5, 60))) + b"\n"
        out += bytes(rng.choices(b"ACGT", k=rng.randint(20, 300))) + b"\n"
    assert_same(bytes(out), k, want_nodes=False)


@pytest.mark.parametrize("k", [4, 6, 7])
def test_dynamic_ranges_acgt_and_streaming(dyn_env, k):
    data = bytes(random.Random(k).choices(b"ACGT", k=6_000_001))
    assert_same(data, k, want_nodes=False)
    mixed = mixed_input(99, 3_000_000)
    assert_same(mixed, k, feeds=[1_000_000, 17, 65536, len(mixed) - 1_065_553])


@pytest.mark.parametrize("k", [5, 6])
@pytest.mark.parametrize("pct", ["1", "50", "99"])
def test_dynamic_ranges_static_share(dyn_env, monkeypatch, k, pct):
    """from almost all dynamic to almost all static"""
    monkeypatch.setenv("FINDKMER_TUNE", f"dyn_min_chunks=1,static_pct={pct}")
    data = mixed_input(4000 + int(pct), 2_500_000)
    assert_same(data, k, want_nodes=False)


@pytest.mark.parametrize("k", [6, 7])
@pytest.mark.parametrize("nshards", [2, 3])
def test_dynamic_ranges_shards(dyn_env, k, nshards):
    data = mixed_input(55 + nshards, 3_000_000).replace(b"\xff", b"Z") + b"\nACGT"
    t_o, r_o, _ = oracle.count_dense(data, k)
    t_g, r_g, ub, rc = shard_count(data, k, nshards, summaries=True)
    assert np.array_equal(t_o, t_g)
    assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
    assert list(r_g.base_count) == list(r_o.base_count)


@pytest.mark.parametrize("k", [6, 11])
@pytest.mark.parametrize("summaries", [False, True])
def test_shards_with_eof_byte(k, summaries):
    """a 0xFF outside a header in the second of three shards ends the stream
    there: the chained state is `ended` and the third shard counts nothing"""
    base = mixed_input(808, 3 * 400_000).replace(b"\xff", b"Z")
    data = bytearray(base)
    at = len(data) // 2
    data[at - 2:at + 1] = b"\nA\xff"
    data = bytes(data)
    t_o, r_o, _ = oracle.count_dense(data, k)
    assert r_o.hit_eof_byte
    t_g, r_g, ub, rc = shard_count(data, k, 3, summaries=summaries)
    assert np.array_equal(t_o, t_g)
    assert r_g.windows == r_o.windows and r_g.valid_bases == r_o.valid_bases
    assert list(r_g.base_count) == list(r_o.base_count)


@pytest.mark.parametrize("k", [4, 6, 7, 11])
@pytest.mark.parametrize("kind", ["mixed", "acgt"])
def test_shard_exit_states_match_stream(k, kind):
    """after resolve, a shard engine's state is the stream's state at the
    shard's end (one engine fed the prefix): the compact path of
    fk_engine_resolve must apply the shard's own summary"""
    if kind == "mixed":
        data = mixed_input(31 + k, 1_500_000).replace(b"\xff", b"Z")
    else:
        data = bytes(random.Random(k).choices(b"ACGT", k=1_200_000))
    import torch
    arr = np.frombuffer(data, dtype=np.uint8)
    n = len(arr)
    per = (n // 3) // 65536 * 65536
    bounds = [0, per, 2 * per, n]
    dev = torch.from_numpy(arr.copy()).cuda()
    torch.cuda.synchronize()
    want = []
    with fk.Engine(k) as e:
        for i in range(3):
            e.feed(np.ascontiguousarray(arr[bounds[i]:bounds[i + 1]]))
            s = e.state()
            want.append((s.hdr, s.run, s.code & ((1 << (2 * min(s.run, 31))) - 1) if not s.hdr else 0))
    st = fk.FkState()
    for i in range(3):
        with fk.Engine(k) as e:
            lo, hi = bounds[i], bounds[i + 1]
            e.feed_shard_device(dev.data_ptr() + lo, hi - lo, min(256, lo))
            e.resolve(st)
            st = e.state()
            got = (st.hdr, st.run, st.code & ((1 << (2 * min(st.run, 31))) - 1) if not st.hdr else 0)
            assert got == want[i], (i, got, want[i])


def _dense_records(seed, n, min_len=1, max_len=3000):
    """Header-dense FASTA: every tile holds comment lines, run breaks and
    newlines in every arrangement, so nearly every tile takes the mixed path
    (tile_mixed): upstream-like records, records shorter than k, N blocks,
    soft-masked bases, empty lines, '\\r', headers made of bases only, headers
    back to back, unknown and 0xFF bytes inside comments."""
    rng = random.Random(seed)
    parts, size, rec = [], 0, 0
    while size < n:
        r = rng.random()
        if r < 0.08:
            head = b">" + random_text(rng, rng.randint(0, 40), b"ACGT", [1, 1, 1, 1]) + b"\n"
        elif r < 0.12:
            head = b">" + random_text(rng, rng.randint(0, 30), b"AC>x\xff\rN", [3, 3, 1, 1, 1, 1, 1]) + b"\n"
        else:
            head = b">ENST%011d\n" % rec
        rec += 1
        L = rng.randint(min_len, max_len) if rng.random() < 0.8 else rng.randint(0, 20)
        seq = bytearray(random_text(rng, L, b"ACGT", [1, 1, 1, 1]))
        for _ in range(rng.choice([0, 0, 0, 1, 3])):
            if seq:
                a = rng.randrange(len(seq))
                b = min(len(seq), a + rng.randint(1, 60))
                seq[a:b] = rng.choice([b"N", b"n", b"a", b"\r", b"x"]) * (b - a)
        w = rng.choice([0, 0, 0, 60, 80, 13, 1, 16])
        if w:
            seq = b"\n".join(bytes(seq[i:i + w]) for i in range(0, len(seq), w))
        tail = b"\n" * rng.choice([1, 1, 1, 0, 2, 5])
        parts.append(head + bytes(seq) + tail)
        size += len(parts[-1])
    return b"".join(parts)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("k", [1, 2, 3, 5, 6, 7, 8, 9, 11, 12, 13])
def test_mixed_tiles_header_dense(seed, k):
    data = _dense_records(4000 + seed, 700_000 + 200_000 * seed)
    assert_same(data, k)


@pytest.mark.parametrize("k", [14, 15, 16])
def test_mixed_tiles_header_dense_large_k(k):
    """k = 14..16 (global atomics, dense table): nonzero bins vs the sparse oracle."""
    data = _dense_records(4050 + k, 500_000)
    codes, cnts, r = oracle.count_sparse(data, k)
    with fk.Engine(k, want_nodes=True) as e:
        e.feed(np.frombuffer(data, dtype=np.uint8).copy())
        rc, rg = e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))
        step = 1 << 28
        got_c, got_n = [], []
        for first in range(0, 1 << (2 * k), step):
            part = e.table_range(first, min(step, (1 << (2 * k)) - first))
            nz = np.nonzero(part)[0]
            got_c.append(nz.astype(np.uint64) + first)
            got_n.append(part[nz])
    assert np.array_equal(np.concatenate(got_c), codes)
    assert np.array_equal(np.concatenate(got_n), cnts)
    assert (rg.windows, rg.distinct, rg.valid_bases) == (r.windows, r.distinct, r.valid_bases)
    assert list(rg.base_count) == list(r.base_count)
    assert list(rg.depth1) == list(r.depth1)
    assert rg.nodes == r.nodes


@pytest.mark.parametrize("k", [2, 6, 7, 10, 13])
def test_mixed_tiles_short_records(k):
    # records around k long: short runs (nodeCounter), first windows and
    # depth-1 touches in nearly every lane
    data = _dense_records(4100 + k, 600_000, min_len=1, max_len=3 * k)
    assert_same(data, k)


@pytest.mark.parametrize("k", [3, 6, 11, 13])
def test_mixed_tiles_ff_outside_comment(k):
    data = bytearray(_dense_records(4200 + k, 400_000))
    cut = 300_001
    while data[cut] in b">\n":
        cut += 1
    # the first 0xFF outside a comment ends the reference's scan (:988)
    j = data.rfind(b">", 0, cut)
    if j >= 0 and data.find(b"\n", j, cut) < 0:
        cut = data.find(b"\n", j) + 1
    data[cut] = 0xFF
    r = assert_same(bytes(data), k)
    assert r.hit_eof_byte


@pytest.mark.parametrize("k", [4, 6, 7, 11, 12])
def test_mixed_tiles_match_general_path(k, monkeypatch):
    # the same header-dense input with mixed tiles switched off (no_mixed:
    # the byte walk of tile_general) counts identically
    data = _dense_records(4300 + k, 500_000)
    r1 = assert_same(data, k)
    monkeypatch.setenv("FINDKMER_TUNE", "no_mixed=1")
    r2 = assert_same(data, k)
    assert (r1.windows, r1.valid_bases, r1.nodes) == (r2.windows, r2.valid_bases, r2.nodes)


@pytest.mark.parametrize("k", [8, 11, 12])
@pytest.mark.parametrize("budget", ["0", "1", "3"])
def test_part_resume_budgets(k, budget, monkeypatch):
    # k_part stops a range after `budget` general tiles and k_part<RES> counts
    # the rest (mixed tiles into region 2 of the partition); ranges that stop
    # and ranges that do not in one feed
    monkeypatch.setenv("FINDKMER_TUNE", f"part_general={budget}")
    rng = random.Random(77 + k)
    data = _dense_records(4400 + k, 300_000) + random_text(rng, 900_000, b"ACGT", [1, 1, 1, 1]) + \
        _dense_records(4500 + k, 200_000)
    assert_same(data, k)


@pytest.mark.parametrize("k", [5, 11, 13])
def test_device_feed_segments(k, monkeypatch):
    """a device feed cut into segments (the HBM budget of segment_budget when
    other processes share the GPU; forced small here with seg_kb) counts
    exactly as one segment: the scan state carries across the cuts"""
    import torch
    data = mixed_input(606 + k, 3_000_000).replace(b"\xff", b"Z")
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    t_o, r_o, ub_o = oracle.count_dense(data, k, unknown_cap=1 << 20)
    monkeypatch.setenv("FINDKMER_TUNE", "seg_kb=272")
    with fk.Engine(k, want_nodes=True, collect_unknown=True) as e:
        e.feed_device(dev.data_ptr(), len(data))
        rc, r = e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))
        t = e.table()
        ub = e.unknown_bytes()
    assert np.array_equal(t, t_o)
    assert (r.windows, r.valid_bases, r.distinct, r.nodes) == (r_o.windows, r_o.valid_bases, r_o.distinct, r_o.nodes)
    assert list(r.base_count) == list(r_o.base_count) and list(r.depth1) == list(r_o.depth1)
    assert ub == ub_o


def test_cli_concurrent_fanout_matches_goldens(manifest, tmp_path):
    """k6thru11fullANDupstream.sh:16-24 on one node: ./Debug/findKmer and
    ./findKmer for each k = 6..11 started together in one directory
    (fk_device_select spreads them over the GPUs; here the box has one), the
    outputs equal the reference's separate runs"""
    import hashlib
    name = "upstream1m.fas"
    shutil.copy(os.path.join(REPO, "tests", "golden", "inputs", name), tmp_path / name)
    procs = []
    for k in range(6, 12):
        for exe in ("Debug/findKmer", "findKmer"):
            procs.append(subprocess.Popen([os.path.join(REPO, exe), "-q", "1", "-k", str(k), "-z", "3", "-p", name],
                                          cwd=tmp_path, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    for p in procs:
        _, err = p.communicate(timeout=300)
        assert p.returncode == 0, err.decode()[-500:]
    for k in range(6, 12):
        for kind, rec in manifest[f"up_k{k}_z3"]["files"].items():
            got = open(tmp_path / rec["name"], "rb").read()
            assert hashlib.sha256(got).hexdigest() == rec["sha256"], (k, kind)


@pytest.mark.parametrize("k,tune", [(8, ""), (9, ""), (10, ""), (11, ""), (12, ""), (13, ""), (12, "pairs_kmax=11")])
def test_partition_batches(k, tune, monkeypatch):
    # k_part's pipelined batches (pairs for k <= 12, single windows for
    # k = 13 and, with pairs_kmax=11, k = 12): FASTA lines, a '\n' in every
    # 16-byte half now and then, a comment line, a poly-A stretch (one slice
    # takes a whole batch) and a ragged end
    monkeypatch.setenv("FINDKMER_TUNE", tune)
    rng = random.Random(91 + k)
    body = random_text(rng, 1_500_000, b"ACGT", [1, 1, 1, 1])
    lines = b"\n".join(body[i:i + 61] for i in range(0, len(body), 61))
    data = b">chr1\n" + lines + b"\n" + b"A" * 300_000 + b"\n>chr2 x\n" + lines[:400_003]
    assert_same(data, k)
