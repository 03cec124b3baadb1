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
    assert L.fk_abi_version() == 1
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
