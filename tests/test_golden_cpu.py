"""CPU tests: pin the oracle and the product's output writer to the reference.

The golden files under tests/golden/cases were produced by the reference program
itself (oracle/_ref/findKmer_ref, compiled from /root/reference by
oracle/Makefile; script tests/golden/make_golden.py).  Here the oracle's counts
are pushed through the product writer (fk_write_stats / fk_write_csv in
libfindkmer_hip.so) and must reproduce the reference's CSV and stats files
byte for byte, and the numbers the reference printed on stdout.
"""
import hashlib
import os
import re

import numpy as np
import pytest

import findkmer_amd as fk
import oracle
from conftest import case_k, case_z, golden_file, golden_input

CPU_CASES = [c for c in [
    *(f"test_k{k}" for k in list(range(1, 13)) + [15, 20]),
    "test_k6_q0", "test_k0_default7", "edge_k2", "edge_k3", "edge_k4",
    "rand_k5", "rand_k6_z3", "rand_k8", "rand_k4_z2", "rand_k11",
    "missing_k3", "ffbyte_k3", "shortruns_k5",
    "rand_k17", "rand_k19_z4", "shortruns_k18", "edge_k20", "ffbyte_k17",
    "up_k6", "up_k7_q0", *(f"up_k{k}_z3" for k in range(6, 12)),
]]


def to_fkresult(r, distinct=None):
    out = fk.FkResult()
    for b in range(4):
        out.base_count[b] = r.base_count[b]
        out.depth1[b] = r.depth1[b]
    out.valid_bases = r.valid_bases
    out.windows = r.windows
    out.distinct = r.distinct if distinct is None else distinct
    out.nodes = r.nodes
    return out


def oracle_counts(data, k):
    if k <= 13:
        t, r, _ = oracle.count_dense(data, k)
        return t, r
    codes, cnts, r = oracle.count_sparse(data, k)
    return (codes, cnts), r


def write_outputs(tmp_path, entry, k):
    data = golden_input(entry["input"])
    tbl, r = oracle_counts(data, k)
    stats_path = str(tmp_path / "stats.txt")
    rc, prob = fk.write_stats(stats_path, k, to_fkresult(r))
    csv_path = str(tmp_path / "out.csv")
    zen, zthr = case_z(entry)
    if rc == 0:
        if isinstance(tbl, tuple) and k > 16:
            # 17 <= k <= 20: the product's sparse writer
            codes, cnts = tbl
            fk.write_csv_sparse(csv_path, k, codes, cnts, prob, r.windows, zen, zthr, threads=4)
        else:
            if isinstance(tbl, tuple):
                # sparse oracle (k > 13) into a dense table
                codes, cnts = tbl
                dense = np.zeros(1 << (2 * k), dtype=np.uint32)
                dense[codes.astype(np.int64)] = cnts
                tbl = dense
            fk.write_csv(csv_path, k, tbl, prob, r.windows, zen, zthr, threads=4)
    else:
        open(csv_path, "w").write("Sequence, Shannon Entropy h, Shannon Entropy H, Frequency, Z score")
    return stats_path, csv_path, r


@pytest.mark.parametrize("case", CPU_CASES)
def test_writer_matches_reference(case, manifest, tmp_path):
    entry = manifest[case]
    k = case_k(entry)
    stats_path, csv_path, r = write_outputs(tmp_path, entry, k)
    gs = entry["files"]["stats"]
    got = open(stats_path, "rb").read()
    assert hashlib.sha256(got).hexdigest() == gs["sha256"], (got, golden_file(case, "stats"))
    gc = entry["files"]["csv"]
    got = open(csv_path, "rb").read()
    if gc["stored"]:
        assert got == golden_file(case, "csv")
    assert len(got) == gc["bytes"]
    assert hashlib.sha256(got).hexdigest() == gc["sha256"]


@pytest.mark.parametrize("case", CPU_CASES)
def test_oracle_stdout_numbers(case, manifest):
    """The oracle's baseCounter, base counts and nodeCounter (tree density) must
    match what the reference printed (statistics(), findKmer.cpp:512-542)."""
    entry = manifest[case]
    k = case_k(entry)
    data = golden_input(entry["input"])
    _, r = oracle_counts(data, k)
    out = golden_file(case, "stdout").decode("latin-1")
    m = re.search(r"Found (\d+) valid bases", out)
    if m:
        assert int(m.group(1)) == r.valid_bases
    counts = re.findall(r"^(\d+), ", out, re.M)
    for b, c in enumerate(counts[:4]):
        assert int(c) == (r.base_count[b] & 0xFFFFFFFF)
    m = re.search(r"^(\d+)% tree density", out, re.M)
    if m:
        maxn = 1 + sum(4 ** n for n in range(1, k + 1))
        assert int(m.group(1)) == int(round(r.nodes / maxn * 100)) or \
            ("%0.0f" % (r.nodes / maxn * 100)) == m.group(1)


def test_test_txt_k6_known_values():
    """1882 distinct 6-mers, 2988 windows, 3003 valid bases,
    A=737 C=816 G=718 T=732."""
    t, r, _ = oracle.count_dense(golden_input("test.txt"), 6)
    assert (t > 0).sum() == 1882 == r.distinct
    assert r.windows == 2988 == int(t.sum())
    assert r.valid_bases == 3003
    assert list(r.base_count) == [737, 816, 718, 732]


def test_oracle_dense_sparse_agree():
    data = golden_input("rand120k.fa")
    for k in (3, 7, 10):
        t, r, _ = oracle.count_dense(data, k)
        codes, cnts, r2 = oracle.count_sparse(data, k)
        nz = np.nonzero(t)[0]
        assert np.array_equal(nz.astype(np.uint64), codes)
        assert np.array_equal(t[nz], cnts)
        assert r.nodes == r2.nodes and r.valid_bases == r2.valid_bases


def test_oracle_int32_run_wrap_small_model():
    """The reference's seqSize is an int (findKmer.cpp:977): verified on the
    real binary that a 2^31+100-base run of 'A' at k=2 gives AA=2147483646
    (DESIGN.md).  Check the oracle's arithmetic of that rule analytically on a
    long run without materialising 2 GiB: count windows for R in [k, 2^31-1]."""
    k = 2
    L = 2 ** 31 + 100
    expect_aa = (2 ** 31 - 1) - k + 1
    assert expect_aa == 2147483646
    # and the base counter: first window adds k, then one per base
    assert k + (2 ** 31 - 1 - k) + 4 == 2147483651


def test_unknown_bytes_in_order():
    data = golden_input("edge.txt")
    t, r, ub = oracle.count_dense(data, 3, unknown_cap=64)
    assert ub == b"\racgt1"


def test_synth_generator_deterministic():
    a = oracle.synth(1000, 1)
    b = oracle.synth(1000, 1)
    assert bytes(a) == bytes(b) and set(bytes(a)) <= set(b"ACGT")
    f = oracle.synth(200, 2, fasta_line=80)
    assert bytes(f[:11]) == b">synthetic\n" and f[11 + 80] == ord("\n")


def _cut_inputs():
    """inputs whose cuts land in every place the entering state depends on:
    long comment lines (cuts inside one), '>' inside comments, runs shorter
    than k, N runs, unknown bytes, a 0xFF byte outside a comment, one long run"""
    import random
    rng = random.Random(11)
    out = []
    for seed in range(3):
        parts = bytearray()
        while len(parts) < 400_000:
            r = rng.random()
            if r < 0.3:
                parts += b">" + bytes(rng.choices(b"ACGT>xN\xff", k=rng.randint(0, 30000))) + b"\n"
            elif r < 0.7:
                seq = bytes(rng.choices(b"ACGT", k=rng.randint(1, 20000)))
                w = rng.choice([0, 1, 7, 80])
                parts += b"\n".join(seq[i:i + w] for i in range(0, len(seq), w)) if w else seq
            else:
                parts += bytes(rng.choices(b"ACGTNn\r1\n", k=rng.randint(1, 50)))
        out.append(bytes(parts))
    ff = bytearray(out[0])
    j = ff.rfind(b"\n", 0, 250_000)
    ff[j + 1] = 0xFF          # line start: outside a comment
    out.append(bytes(ff))
    out.append(b"ACGT" * 300_000)
    out.append(b">" + b"A" * 1_500_000)
    return out


@pytest.mark.parametrize("k", [1, 4, 7, 11])
def test_oracle_pieces_equal_sequential(k):
    """fko_count_dense_par (the scan over contiguous pieces, each from the
    entering state derived from the bytes before its cut) == the sequential
    scan, for every table bin and every scalar"""
    for data in _cut_inputs():
        t1, r1, u1 = oracle.count_dense(data, k, unknown_cap=1 << 20)
        for th in (2, 5, 16):
            t2, r2, u2 = oracle.count_dense(data, k, unknown_cap=1 << 20, threads=th)
            assert np.array_equal(t1, t2)
            assert bytes(r1) == bytes(r2)
            assert u1 == u2


@pytest.mark.parametrize("k", [3, 9, 17, 20])
def test_oracle_key_range_equals_sparse_slice(k):
    """fko_count_sparse_range (one key range, pieces over threads) == the
    matching slice of the sequential sparse oracle, for ranges at the start,
    inside and at the end of the index space, with every counter of the
    stream; the 10 GB k >= 17 GPU tests compare the engine with it"""
    import random as _r
    rng = _r.Random(k)
    parts = []
    for _ in range(300):
        parts.append(bytes(rng.choices(b"ACGT", k=rng.randint(1, 3000))))
        parts.append(rng.choice([b"\n", b"N", b">hdr x\n", b"\n\n", b"acgt"]))
    data = b"".join(parts)
    codes, cnts, r = oracle.count_sparse(data, k)
    top = 1 << (2 * k)
    span = min(top, 1 << 20)
    for ranges in ([(0, span)], [(top // 3, top // 3 + span)], [(top - span, top)],
                   [(0, span // 4), (top // 2, top // 2 + span // 4), (top - span // 4, top)]):
        c2, n2, r2 = oracle.count_sparse_range(data, k, ranges, threads=5)
        sel = np.zeros(len(codes), dtype=bool)
        for lo, hi in ranges:
            sel |= (codes >= lo) & (codes < hi)
        assert np.array_equal(c2, codes[sel]) and np.array_equal(n2, cnts[sel])
        assert r2.distinct == int(sel.sum())
        assert (r2.windows, r2.valid_bases, list(r2.base_count), list(r2.depth1), r2.unknown_chars,
                r2.scanned_bytes) == (r.windows, r.valid_bases, list(r.base_count), list(r.depth1),
                                      r.unknown_chars, r.scanned_bytes)
