"""CPU tests of the drop-in boundary: the C-ABI library loads without a GPU,
exports every function include/findkmer.h declares, and fails loudly (no CPU
fallback) when no device is present."""
import ctypes
import os
import re
import subprocess

import pytest

import findkmer_amd as fk
from conftest import REPO

HEADER = os.path.join(REPO, "include", "findkmer.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(fk_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_the_engine_api():
    names = declared_functions()
    for must in ["fk_engine_create", "fk_engine_feed", "fk_engine_finish", "fk_engine_table",
                 "fk_count", "fk_count_multi", "fk_write_stats", "fk_write_rows",
                 "fk_engine_feed_shard", "fk_engine_resolve", "fk_summary_apply"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(fk.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", fk.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (fk_[a-z0-9_]+)$", out, re.M))
    assert set(declared_functions()) <= exported


def test_python_binding_covers_the_header():
    bound = {n for n, _, _ in fk.SIGNATURES}
    assert set(declared_functions()) == bound


def test_abi_version_and_strerror():
    L = fk.lib()
    assert L.fk_abi_version() == 2
    assert L.fk_strerror(fk.FK_E_EMPTY) == b"Sequence File Is Empty, Ending Program"
    assert L.fk_strerror(fk.FK_E_ROLLOVER) == b"COUNTER ROLLOVER DETECTED"


def test_no_gpu_fails_loudly():
    if fk.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(fk.FindKmerError) as ei:
        fk.Engine(6)
    assert ei.value.code == fk.FK_E_NO_DEVICE
    with pytest.raises(fk.FindKmerError):
        fk.count(b"ACGTACGT", 3)


def test_summary_apply_is_host_only():
    """Shard stitching math (fk_summary_apply) needs no device: identity summary."""
    s = fk.FkSummary()
    # identity transfer function: c1 = (hdr=1,R=0), f0 = shift by 0
    words = [0] * 12
    words[2] = 1          # c1.hdr
    for i, w in enumerate(words):
        s.w[i] = w
    st = fk.FkState()
    st.run = 1234
    st.code = 0xABC
    out = fk.summary_apply(s, st)
    assert (out.run, out.code, out.hdr) == (1234, 0xABC, 0)


def test_drop_in_binary_is_built():
    exe = os.path.join(REPO, "findKmer")
    assert os.access(exe, os.X_OK)
    dbg = os.path.join(REPO, "Debug", "findKmer")
    assert os.access(dbg, os.X_OK)   # k6thru11fullANDupstream.sh also runs ./Debug/findKmer
    # -h prints the reference usage and exits 1 (findKmer.cpp:402-403)
    p = subprocess.run([exe, "-h"], capture_output=True, text=True)
    assert p.returncode == 1 and "Usage: findKmer [options]" in p.stdout


def test_cli_k_out_of_range_message():
    p = subprocess.run([os.path.join(REPO, "findKmer"), "-k", "21"], capture_output=True, text=True)
    assert p.returncode == 1
    assert "21 is not a valid value for k.\nPlease select a number greater than zero and less than 21\n" in p.stderr


COMPACT = 0x434F4D50414354   # "COMPACT" tag of a one-pass shard summary (fk_engine.hip)


def _compact(g_run, g_code, g_hdr, nvb0, c_run, c_code, c_hdr, absorb, nv, shard_len, k):
    """a compact shard summary in the C-ABI's 12 words; codes in the engine's
    internal order (the C-ABI converts fk_state codes with sigma)"""
    s = fk.FkSummary()
    w = [g_code, g_run | (g_hdr << 32), nvb0, c_run, c_code, c_hdr | (absorb << 32), nv, shard_len, k, 0, 0, COMPACT]
    for i, v in enumerate(w):
        s.w[i] = v
    return s


def _sigma(x):
    return x ^ ((x >> 1) & 0x5555555555555555)


def test_compact_summary_apply():
    """fk_summary_apply on compact summaries (host-only arithmetic): a shift
    for a state equivalent to the shard's guess, the constant exit for an
    absorbing shard, FK_E_SUMMARY for a state that would count the shard's
    first range differently or could reach the int32 wrap"""
    k = 6
    mask = (1 << (2 * (k - 1))) - 1
    # shard guessed deep in a run (R=256, last bases 0x0ABC), 1000 bases, no break
    s = _compact(256, 0x0ABC, 0, 16384, 0, 0x3F3F, 0, 0, 1000, 16384, k)
    st = fk.FkState(run=5000, code=_sigma(0x1230ABC & ((1 << 64) - 1)), hdr=0)
    out = fk.summary_apply(s, st)
    assert out.run == 6000 and out.hdr == 0
    assert _sigma(out.code) & ((1 << 64) - 1) == 0x3F3F   # 1000 >= 32 new bases
    # a state whose last k-1 bases differ from the guess: not equivalent
    bad = fk.FkState(run=5000, code=_sigma(0x0ABD), hdr=0)
    with pytest.raises(fk.FindKmerError) as e:
        fk.summary_apply(s, bad)
    assert e.value.code == fk.FK_E_SUMMARY
    # a short run (R < k) is not equivalent to a deep guess
    with pytest.raises(fk.FindKmerError):
        fk.summary_apply(s, fk.FkState(run=3, code=_sigma(0x0ABC & mask), hdr=0))
    # near the int32 wrap: the shard's local checks do not cover it
    with pytest.raises(fk.FindKmerError):
        fk.summary_apply(s, fk.FkState(run=(1 << 31) - 20000, code=_sigma(0x0ABC), hdr=0))
    # an absorbing shard (run break inside): constant exit
    a = _compact(256, 0x0ABC, 0, 16384, 77, 0x155, 0, 1, 0, 16384, k)
    out = fk.summary_apply(a, fk.FkState(run=9999, code=_sigma(0x0ABC), hdr=0))
    assert out.run == 77 and _sigma(out.code) == 0x155 and out.hdr == 0
    # header status must match the guess
    with pytest.raises(fk.FindKmerError):
        fk.summary_apply(a, fk.FkState(run=0, code=0, hdr=1))


def _rows(summaries, valid=None):
    """pack rows (fk_engine_shard_pack's layout) of compact summaries"""
    import numpy as np
    rows = np.zeros(len(summaries) * fk.FK_PACK_ROW_WORDS, dtype=np.uint32)
    for r, s in enumerate(summaries):
        base = r * fk.FK_PACK_ROW_WORDS
        for j in range(12):
            rows[base + 2 * j] = s.w[j] & 0xFFFFFFFF
            rows[base + 2 * j + 1] = s.w[j] >> 32
        rows[base + 24] = 1 if valid is None or valid[r] else 0
    return rows


def test_shard_rows_compose():
    """fk_shard_rows_compose (host-only): the entering state of each rank
    from the gathered pack rows, None when a row is invalid or a guess does
    not hold (every rank then falls back to the stitched exchange)"""
    k = 6
    # rank 0 from the stream start (guess R=0), 1000 bases, ends deep in a
    # run with last bases 0x0ABC; rank 1 guessed deep with those bases
    s0 = _compact(0, 0, 0, 16384, 0, 0x0ABC, 0, 0, 1000, 16384, k)
    s1 = _compact(256, 0x0ABC, 0, 16384, 77, 0x155, 0, 1, 0, 16384, k)
    s2 = _compact(50, 0x155, 0, 16384, 0, 0x3F3F, 0, 0, 500, 16384, k)
    rows = _rows([s0, s1, s2])
    st0 = fk.shard_rows_compose(rows.ctypes.data, 3, 0)
    assert (st0.run, st0.code, st0.hdr, st0.ended) == (0, 0, 0, 0)
    st1 = fk.shard_rows_compose(rows.ctypes.data, 3, 1)
    assert st1.run == 1000 and _sigma(st1.code) == 0x0ABC and st1.hdr == 0
    st2 = fk.shard_rows_compose(rows.ctypes.data, 3, 2)
    assert st2.run == 77 and _sigma(st2.code) == 0x155
    # rank 2 guessed R=50 where the true run is 77 bases: both deep, same bases
    # -> equivalent; a guess of a different header flag is not
    bad = _compact(0, 0, 1, 16384, 0, 0, 0, 1, 0, 16384, k)
    assert fk.shard_rows_compose(_rows([s0, s1, bad]).ctypes.data, 3, 0) is None
    # an invalid pack anywhere: every rank falls back
    assert fk.shard_rows_compose(_rows([s0, s1, s2], valid=[1, 0, 1]).ctypes.data, 3, 2) is None
    # a shard that ends the stream (0xFF) is never packed as valid
    eof = _compact(0, 0, 0, 16384, 0, 0x0ABC, 0, 0, 1000, 16384, k)
    eof.w[9] = 1
    assert fk.shard_rows_compose(_rows([eof, s1]).ctypes.data, 2, 1) is None


def test_device_policy_spreads_processes():
    """fk_device_policy (host-only rule behind fk_device_select): devices
    with room for the run take processes round-robin by salt (the pid), a
    full device is skipped, and with no room anywhere the emptiest wins"""
    import ctypes
    L = fk.lib()
    G = 1 << 30
    free = (ctypes.c_uint64 * 8)(*[200 * G] * 8)
    picks = [L.fk_device_policy(8, free, 20 * G, salt) for salt in range(1000, 1024)]
    assert sorted(set(picks)) == list(range(8)) and all(picks.count(d) == 3 for d in range(8))
    free[3] = 5 * G
    picks = {L.fk_device_policy(8, free, 20 * G, salt) for salt in range(64)}
    assert picks == set(range(8)) - {3}
    small = (ctypes.c_uint64 * 3)(1 * G, 7 * G, 2 * G)
    assert L.fk_device_policy(3, small, 20 * G, 5) == 1
    assert L.fk_device_policy(0, small, 1, 0) == fk.FK_E_INVALID
