"""Test-side loader of the CPU oracle (oracle/liboracle.so) — the CHECKER only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this.
"""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
REF_BIN = os.path.join(REPO, "oracle", "_ref", "findKmer_ref")


class FkoResult(ctypes.Structure):
    _fields_ = [("base_count", ctypes.c_uint64 * 4),
                ("valid_bases", ctypes.c_uint64),
                ("windows", ctypes.c_uint64),
                ("distinct", ctypes.c_uint64),
                ("depth1", ctypes.c_uint64 * 4),
                ("nodes", ctypes.c_uint64),
                ("unknown_chars", ctypes.c_uint64),
                ("scanned_bytes", ctypes.c_uint64),
                ("hit_eof_byte", ctypes.c_int32),
                ("unterminated_header", ctypes.c_int32),
                ("rollover", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


_L = None


def olib():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "liboracle.so"], check=True,
                           capture_output=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.fko_count_dense.restype = ctypes.c_int
        L.fko_count_dense.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.POINTER(FkoResult),
                                      ctypes.c_void_p, ctypes.c_uint64]
        L.fko_count_dense_par.restype = ctypes.c_int
        L.fko_count_dense_par.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.POINTER(FkoResult),
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
        L.fko_count_sparse.restype = ctypes.c_int
        L.fko_count_sparse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(FkoResult)]
        L.fko_count_sparse_range.restype = ctypes.c_int
        L.fko_count_sparse_range.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(FkoResult), ctypes.c_int]
        L.fko_synth.restype = ctypes.c_uint64
        L.fko_synth.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_int]
        _L = L
    return _L


def _buf(data):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    if len(a) == 0:
        a = np.zeros(1, dtype=np.uint8)
        return a, 0
    return a, len(a)


def host_threads():
    """Threads for the oracle on this host, measured: the CPUs this process
    may run on (sched_getaffinity), capped by the cgroup's CPU quota
    (cpu.max, cgroup v2; cpu.cfs_quota_us / cfs_period_us, v1) where one is
    set -- os.cpu_count() shows the whole machine's CPUs on the GPU box."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def count_dense(data, k, unknown_cap=0, threads=1):
    """Oracle counts: (table uint32[4^k], result, unknown_bytes).  threads > 1:
    fko_count_dense_par (the same scan over contiguous pieces, each from its
    exact entering state)."""
    a, n = _buf(data)
    t = np.zeros(1 << (2 * k), dtype=np.uint32)
    r = FkoResult()
    ub = np.zeros(max(1, unknown_cap), dtype=np.uint8)
    if threads > 1:
        rc = olib().fko_count_dense_par(a.ctypes.data, n, k, t.ctypes.data, ctypes.byref(r),
                                        ub.ctypes.data if unknown_cap else None, unknown_cap, threads)
    else:
        rc = olib().fko_count_dense(a.ctypes.data, n, k, t.ctypes.data, ctypes.byref(r),
                                    ub.ctypes.data if unknown_cap else None, unknown_cap)
    assert rc == 0
    return t, r, bytes(ub[: min(unknown_cap, r.unknown_chars)])


def count_sparse(data, k, cap=1 << 22):
    a, n = _buf(data)
    codes = np.zeros(cap, dtype=np.uint64)
    cnts = np.zeros(cap, dtype=np.uint32)
    nu = ctypes.c_uint64()
    r = FkoResult()
    rc = olib().fko_count_sparse(a.ctypes.data, n, k, codes.ctypes.data, cnts.ctypes.data, cap,
                                 ctypes.byref(nu), ctypes.byref(r))
    assert rc == 0
    return codes[: nu.value], cnts[: nu.value], r


def count_sparse_range(data, k, ranges, threads=1):
    """ranges: ascending disjoint (lo, hi) key ranges.  Returns (distinct
    indices inside them ascending, their counts, result with the whole
    stream's counters; result.distinct = the ranges')"""
    a, n = _buf(data)
    lo = np.array([r[0] for r in ranges], dtype=np.uint64)
    hi = np.array([r[1] for r in ranges], dtype=np.uint64)
    cap = max(1, int((hi - lo).sum()))
    codes = np.zeros(cap, dtype=np.uint64)
    cnts = np.zeros(cap, dtype=np.uint32)
    nu = ctypes.c_uint64()
    r = FkoResult()
    rc = olib().fko_count_sparse_range(a.ctypes.data, n, k, lo.ctypes.data, hi.ctypes.data, len(ranges),
                                       codes.ctypes.data, cnts.ctypes.data, cap, ctypes.byref(nu), ctypes.byref(r),
                                       threads)
    assert rc == 0
    return codes[: nu.value], cnts[: nu.value], r


def synth(n_bases, seed, fasta_line=0):
    cap = n_bases + (n_bases // fasta_line + 11 if fasta_line > 0 else 0)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    w = olib().fko_synth(out.ctypes.data, cap, n_bases, seed, fasta_line)
    return out[:w]
