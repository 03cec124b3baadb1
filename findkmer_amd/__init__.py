"""findkmer_amd — Python binding of the MI355X k-mer engine C-ABI (include/findkmer.h).

The product is the native library ``findkmer_amd/lib/libfindkmer_hip.so`` (HIP
kernels for gfx950 + the byte-identical writer) and the drop-in ``./findKmer``
program.  This module is a thin ctypes layer over that library for tests and
``bench.py``; it never falls back to a CPU implementation: if the library is
missing or no GPU is visible, calls raise.

Reference interface mirrored: the scan ``findKmer()`` of
findKmer/src/findKmer.cpp:962-1069 (counts + base statistics), ``statistics()``
(:491-565) and ``histo_recursive()`` (:699-942).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FINDKMER_LIB selects another build of the same library (e.g. a variant
# compiled for an experiment); the default is the in-tree build.
LIB_PATH = os.environ.get("FINDKMER_LIB") or os.path.join(_HERE, "lib", "libfindkmer_hip.so")

FK_OK = 0
FK_E_INVALID = -1
FK_E_K_UNSUPPORTED = -2
FK_E_NO_DEVICE = -3
FK_E_HIP = -4
FK_E_OOM = -5
FK_E_EMPTY = -6
FK_E_UNTERMINATED_HEADER = -7
FK_E_ROLLOVER = -8
FK_E_STATE = -9
FK_E_IO = -10
FK_E_RCCL = -11
FK_E_SUMMARY = -12
FK_E_INTERNAL = -13
FK_K_MAX_DENSE = 16
FK_PACK_COUNTERS = 14     # include/findkmer.h: fk_engine_shard_pack's counters
FK_PACK_ROW_WORDS = 32    # ... and its rows (uint32 words)
FK_PACK_STATS = 8         # a sharded table's (total, distinct) as limbs
FK_XCHG_FAST = 1          # fk_engine_shard_exchange flags (info[0])
FK_XCHG_SHARD_TABLE = 2
FK_ROUTE_KMIN = 15        # routed sharded tables from this k (include/findkmer.h)
FK_XCHG_TEST_INVALID = 4
FK_COMM_ID_BYTES = 128
FK_UPSTREAM_REC = 1019    # fk_synth_upstream_device's record: ">ENST%011u\n" + 1001 bases + "\n"


class FkState(ctypes.Structure):
    _fields_ = [("run", ctypes.c_uint64), ("code", ctypes.c_uint64),
                ("hdr", ctypes.c_uint32), ("ended", ctypes.c_uint32)]


class FkResult(ctypes.Structure):
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
                ("nodes_valid", ctypes.c_int32),
                ("chunks", ctypes.c_uint64),
                ("redo_chunks", ctypes.c_uint64),
                ("device_ms", ctypes.c_double),
                ("main_kernel_ms", ctypes.c_double), ("timed_kernels", ctypes.c_uint64)]

    def as_dict(self):
        d = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            d[name] = list(v) if isinstance(v, ctypes.Array) else v
        return d


class FkOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("want_nodes", ctypes.c_int32),
                ("stream", ctypes.c_void_p), ("collect_unknown", ctypes.c_int32),
                ("timing_every", ctypes.c_int32), ("borrow_input", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 5)]


class FkSummary(ctypes.Structure):
    _fields_ = [("w", ctypes.c_uint64 * 12)]


# (name, restype, argtypes) for every symbol declared in include/findkmer.h
_P = ctypes.c_void_p
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)
SIGNATURES = [
    ("fk_abi_version", ctypes.c_int, []),
    ("fk_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("fk_device_count", ctypes.c_int, []),
    ("fk_engine_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(FkOpts), ctypes.POINTER(_P)]),
    ("fk_engine_destroy", None, [_P]),
    ("fk_engine_reset", ctypes.c_int, [_P]),
    ("fk_engine_feed", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int]),
    ("fk_engine_feed_shard", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
    ("fk_engine_summary", ctypes.c_int, [_P, ctypes.POINTER(FkSummary)]),
    ("fk_engine_summary_full", ctypes.c_int, [_P, ctypes.POINTER(FkSummary)]),
    ("fk_summary_apply", ctypes.c_int, [ctypes.POINTER(FkSummary), ctypes.POINTER(FkState), ctypes.POINTER(FkState)]),
    ("fk_summary_is_full", ctypes.c_int, [ctypes.POINTER(FkSummary)]),
    ("fk_engine_resolve", ctypes.c_int, [_P, ctypes.POINTER(FkState)]),
    ("fk_engine_shard_pack", ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("fk_engine_stream", ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    ("fk_comm_id", ctypes.c_int, [_P]),
    ("fk_comm_create", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    ("fk_comm_destroy", None, [_P]),
    ("fk_engine_shard_exchange", ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_int32)]),
    ("fk_merge_layout", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _U64P, _U64P]),
    ("fk_engine_route_pack", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _U64P]),
    ("fk_engine_route_copy", ctypes.c_int, [_P, _P]),
    ("fk_engine_route_absorb", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _P, _U64P, _P]),
    ("fk_comm_available", ctypes.c_int, [ctypes.c_int]),
    ("fk_comm_info", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]),
    ("fk_shard_rows_compose", ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(FkState)]),
    ("fk_engine_finish", ctypes.c_int, [_P, ctypes.POINTER(FkResult)]),
    ("fk_engine_table", ctypes.c_int, [_P, _U32P]),
    ("fk_engine_table_device", ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    ("fk_engine_table_range", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, _U32P]),
    ("fk_engine_table_to_device", ctypes.c_int, [_P, _P]),
    ("fk_engine_table_from_device", ctypes.c_int, [_P, _P]),
    ("fk_engine_state", ctypes.c_int, [_P, ctypes.POINTER(FkState)]),
    ("fk_engine_progress", ctypes.c_int, [_P, _U64P, _U64P]),
    ("fk_engine_merge_from", ctypes.c_int, [_P, _P]),
    ("fk_engine_unknown", ctypes.c_int, [_P, _U8P, ctypes.c_uint64, _U64P]),
    ("fk_engine_unknown_since", ctypes.c_int, [_P, ctypes.c_uint64, _U8P, _U64P, ctypes.c_uint64, _U64P]),
    ("fk_engine_sparse", ctypes.c_int, [_P, _U64P, _U32P, ctypes.c_uint64, _U64P]),
    ("fk_engine_sparse_device", ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, _U64P]),
    ("fk_engine_sparse_range", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, _U64P, _U32P, ctypes.c_uint64,
                                              _U64P]),
    ("fk_engine_sparse_split", ctypes.c_int, [_P, ctypes.c_int, _U64P]),
    ("fk_engine_sparse_adopt", ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, _U64P]),
    ("fk_engine_sparse_exchange", ctypes.c_int, [_P, _P, ctypes.c_int, _P, _U64P]),
    ("fk_count", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(FkOpts), _U32P, ctypes.POINTER(FkResult)]),
    ("fk_count_multi", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(FkOpts), _U32P, ctypes.POINTER(FkResult)]),
    ("fk_synth_device", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, _P, _U64P]),
    ("fk_synth_upstream_device", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint64, _P, _U64P]),
    ("fk_input_load", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    ("fk_input_info", ctypes.c_int, [_P, ctypes.POINTER(_P), _U64P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]),
    ("fk_input_destroy", None, [_P]),
    ("fk_input_headers", ctypes.c_int, [_P, ctypes.c_int, _U64P, _U64P, ctypes.c_uint64, _U64P]),
    ("fk_device_select", ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]),
    ("fk_device_policy", ctypes.c_int, [ctypes.c_int, _U64P, ctypes.c_uint64, ctypes.c_uint32]),
    ("fk_write_stats", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(FkResult), _P, ctypes.POINTER(ctypes.c_double)]),
    ("fk_write_rows", ctypes.c_int, [_P, ctypes.c_int, _U32P, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_int]),
    ("fk_write_rows_sparse", ctypes.c_int, [_P, ctypes.c_int, _U64P, _U32P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_int]),
    ("fk_write_csv_sparse", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _U64P, _U32P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_int]),
    ("fk_write_csv", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _U32P, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_int]),
]

_lib = None


class FindKmerError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib().fk_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def lib():
    """Load the native library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        # PyTorch-ROCm bundles its own HIP runtime.  Two runtimes share the
        # process's GPU address space only if torch initialises first, so when
        # torch is in use, bring it up before this library touches HIP.
        import sys
        if "torch" in sys.modules:
            try:
                sys.modules["torch"].cuda.is_available()
            except Exception:
                pass
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc, what, ok=(FK_OK,)):
    if rc not in ok:
        raise FindKmerError(rc, what)
    return rc


def device_count():
    return lib().fk_device_count()


def _ptr(obj):
    """Address of a bytes-like host buffer, numpy array or torch tensor."""
    if hasattr(obj, "data_ptr"):
        return obj.data_ptr()
    if hasattr(obj, "ctypes"):
        return obj.ctypes.data
    if isinstance(obj, (bytes, bytearray, memoryview)):
        mv = memoryview(obj)
        if mv.readonly:
            buf = (ctypes.c_char * len(mv)).from_buffer_copy(mv)
            _ptr.keep = buf
            return ctypes.addressof(buf)
        return ctypes.addressof((ctypes.c_char * len(mv)).from_buffer(mv))
    raise TypeError(type(obj))


class Engine:
    """One k-mer engine on one GPU (mirrors the findKmer() scan, :962-1069)."""

    def __init__(self, k, device=-1, want_nodes=False, collect_unknown=False, stream=None, timing_every=1,
                 borrow_input=False):
        L = lib()
        self.k = k
        o = FkOpts()
        o.device = device
        o.want_nodes = 1 if want_nodes else 0
        # collect_unknown: True/1 = the bytes, 2 = also their stream offsets (unknown_positions)
        o.collect_unknown = int(collect_unknown) if collect_unknown else 0
        o.stream = stream
        o.timing_every = int(timing_every)
        # 17 <= k <= 20: finish re-reads the caller's device feeds (kept unchanged
        # until finish) instead of a copy (fk_opts.borrow_input)
        o.borrow_input = 1 if borrow_input else 0
        h = ctypes.c_void_p()
        _check(L.fk_engine_create(k, ctypes.byref(o), ctypes.byref(h)), "fk_engine_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().fk_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reset(self):
        _check(lib().fk_engine_reset(self.h), "reset")

    def feed(self, buf, nbytes=None, on_device=False):
        n = len(buf) if nbytes is None else nbytes
        _check(lib().fk_engine_feed(self.h, _ptr(buf), n, 1 if on_device else 0), "feed")

    def feed_device(self, ptr, nbytes):
        _check(lib().fk_engine_feed(self.h, ptr, nbytes, 1), "feed")

    def feed_shard_device(self, ptr, nbytes, halo):
        _check(lib().fk_engine_feed_shard(self.h, ptr, nbytes, halo, 1), "feed_shard")

    def summary(self):
        s = FkSummary()
        _check(lib().fk_engine_summary(self.h, ctypes.byref(s)), "summary")
        return s

    def summary_full(self):
        s = FkSummary()
        _check(lib().fk_engine_summary_full(self.h, ctypes.byref(s)), "summary_full")
        return s

    def resolve(self, state):
        _check(lib().fk_engine_resolve(self.h, ctypes.byref(state)), "resolve")

    def shard_pack(self, table_ptr, counters_ptr, rows_ptr, nrows=1, slot=0, is_last=False):
        """Enqueue the pending shard's one-pass result (table, counter limbs,
        pack rows) into device buffers on the engine's stream (no wait)."""
        _check(lib().fk_engine_shard_pack(self.h, table_ptr, counters_ptr, rows_ptr, nrows, slot,
                                          1 if is_last else 0), "shard_pack")

    def shard_exchange(self, comm, merge_ptr, fast=True, shard_table=False, test_invalid=False):
        """fk_engine_shard_exchange: the whole exchange of a pending shard over
        `comm` (a Comm) on the engine's stream, into the device merge buffer.
        Returns (one_collective, first_end): one_collective = every rank's
        buffer holds the merged table (else rank 0's does, or with
        shard_table each rank its slice); first_end = the rank whose shard
        ends the stream (a 0xFF byte) or None."""
        flags = (FK_XCHG_FAST if fast else 0) | (FK_XCHG_SHARD_TABLE if shard_table else 0) | \
            (FK_XCHG_TEST_INVALID if test_invalid else 0)
        info = (ctypes.c_int32 * 2)(flags, -1)
        _check(lib().fk_engine_shard_exchange(self.h, comm.h, merge_ptr, info), "shard_exchange")
        return bool(info[0]), (info[1] if info[1] >= 0 else None)

    def route_pack(self, world, counting=True):
        """fk_engine_route_pack: the finished table's blobs for owners
        0..world-1 (routed sharded table, k >= FK_ROUTE_KMIN); returns their
        sizes in int32 words (fk_engine_route_copy fetches them)."""
        words = (ctypes.c_uint64 * world)()
        _check(lib().fk_engine_route_pack(self.h, world, 1 if counting else 0, words), "route_pack")
        return [int(w) for w in words]

    def route_copy(self, ptr):
        _check(lib().fk_engine_route_copy(self.h, ptr), "route_copy")

    def route_absorb(self, world, rank, recv_ptr, words, slice_ptr):
        """fk_engine_route_absorb: the blobs received from every source
        (words[s] int32 each, side by side at recv_ptr) into this rank's
        slice of the merged table (device int32 at slice_ptr)."""
        w = (ctypes.c_uint64 * world)(*words)
        _check(lib().fk_engine_route_absorb(self.h, world, rank, recv_ptr, w, slice_ptr), "route_absorb")

    def stream(self):
        """The engine's hipStream_t (as an int)."""
        p = ctypes.c_void_p()
        _check(lib().fk_engine_stream(self.h, ctypes.byref(p)), "stream")
        return p.value or 0

    def state(self):
        s = FkState()
        _check(lib().fk_engine_state(self.h, ctypes.byref(s)), "state")
        return s

    def finish(self, allow=(FK_OK,)):
        r = FkResult()
        rc = lib().fk_engine_finish(self.h, ctypes.byref(r))
        _check(rc, "finish", ok=tuple(allow))
        return rc, r

    def table(self):
        import numpy as np
        t = np.zeros(1 << (2 * self.k), dtype=np.uint32)
        _check(lib().fk_engine_table(self.h, t.ctypes.data_as(_U32P)), "table")
        return t

    def table_range(self, first, n):
        import numpy as np
        t = np.zeros(n, dtype=np.uint32)
        _check(lib().fk_engine_table_range(self.h, first, n, t.ctypes.data_as(_U32P)), "table_range")
        return t

    def table_device_ptr(self):
        p = ctypes.c_void_p()
        _check(lib().fk_engine_table_device(self.h, ctypes.byref(p)), "table_device")
        return p.value

    def table_to_device(self, ptr):
        _check(lib().fk_engine_table_to_device(self.h, ptr), "table_to_device")

    def table_from_device(self, ptr):
        _check(lib().fk_engine_table_from_device(self.h, ptr), "table_from_device")

    def sparse(self):
        """17 <= k <= 20, after finish(): (distinct k-mer indices uint64
        ascending, their uint32 counts)"""
        import numpy as np
        n = ctypes.c_uint64()
        _check(lib().fk_engine_sparse(self.h, None, None, 0, ctypes.byref(n)), "sparse")
        keys = np.zeros(max(1, n.value), dtype=np.uint64)
        cnts = np.zeros(max(1, n.value), dtype=np.uint32)
        _check(lib().fk_engine_sparse(self.h, keys.ctypes.data_as(_U64P), cnts.ctypes.data_as(_U32P), n.value,
                                      ctypes.byref(n)), "sparse")
        return keys[: n.value], cnts[: n.value]

    def sparse_range(self, key_lo, key_hi):
        """17 <= k <= 20, after finish(): the runs with keys in [key_lo,
        key_hi) (uint64 keys ascending, uint32 counts)"""
        import numpy as np
        n = ctypes.c_uint64()
        _check(lib().fk_engine_sparse_range(self.h, key_lo, key_hi, None, None, 0, ctypes.byref(n)), "sparse_range")
        keys = np.zeros(max(1, n.value), dtype=np.uint64)
        cnts = np.zeros(max(1, n.value), dtype=np.uint32)
        _check(lib().fk_engine_sparse_range(self.h, key_lo, key_hi, keys.ctypes.data_as(_U64P),
                                            cnts.ctypes.data_as(_U32P), n.value, ctypes.byref(n)), "sparse_range")
        return keys[: n.value], cnts[: n.value]

    @property
    def sparse_table(self):
        """17 <= k <= 20: the table is sparse (sparse(), the sparse_* merge)"""
        return self.k > 16

    def sparse_split(self, world):
        """after finish(): the table's run count per owner rank (owner of index
        x: x // ceil(4^k / world))"""
        out = (ctypes.c_uint64 * world)()
        _check(lib().fk_engine_sparse_split(self.h, world, out), "sparse_split")
        return [int(v) for v in out]

    def sparse_device(self, keys_ptr, counts_ptr, cap):
        """the sparse table into device buffers (uint64 keys, uint32 counts);
        returns the run count"""
        n = ctypes.c_uint64()
        _check(lib().fk_engine_sparse_device(self.h, keys_ptr, counts_ptr, cap, ctypes.byref(n)), "sparse_device")
        return n.value

    def sparse_exchange(self, comm, counting, limbs_ptr):
        """fk_engine_sparse_exchange: the sparse tables merged to their
        owners over `comm` (a Comm), the counter limbs at limbs_ptr (device
        int32) completed with this slice's (total, distinct) and all-reduced.
        Returns (distinct, total) of this rank's slice."""
        st = (ctypes.c_uint64 * 2)()
        _check(lib().fk_engine_sparse_exchange(self.h, comm.h, 1 if counting else 0, limbs_ptr, st),
               "sparse_exchange")
        return int(st[0]), int(st[1])

    def sparse_adopt(self, keys_ptr, counts_ptr, n):
        """replace the sparse table by the runs received in the exchange
        (device pointers); returns (distinct, sum of u32 counts)"""
        st = (ctypes.c_uint64 * 2)()
        _check(lib().fk_engine_sparse_adopt(self.h, keys_ptr, counts_ptr, n, st), "sparse_adopt")
        return int(st[0]), int(st[1])

    def unknown_positions(self):
        """collect_unknown=2: the stream offset of every unknown byte, in order"""
        import numpy as np
        n = ctypes.c_uint64()
        _check(lib().fk_engine_unknown_since(self.h, 0, None, None, 0, ctypes.byref(n)), "unknown_since")
        pos = np.zeros(max(1, n.value), dtype=np.uint64)
        _check(lib().fk_engine_unknown_since(self.h, 0, None, pos.ctypes.data_as(_U64P), n.value, ctypes.byref(n)),
               "unknown_since")
        return pos[: n.value]

    def unknown_bytes(self):
        n = ctypes.c_uint64()
        _check(lib().fk_engine_unknown(self.h, None, 0, ctypes.byref(n)), "unknown")
        out = (ctypes.c_uint8 * max(1, n.value))()
        _check(lib().fk_engine_unknown(self.h, out, n.value, ctypes.byref(n)), "unknown")
        return bytes(out[: n.value])


def summary_apply(summary, state):
    out = FkState()
    _check(lib().fk_summary_apply(ctypes.byref(summary), ctypes.byref(state), ctypes.byref(out)), "summary_apply")
    return out


def comm_id():
    """A fresh RCCL unique id (FK_COMM_ID_BYTES bytes) for Comm: made by one
    rank, handed to the others by the caller."""
    b = (ctypes.c_uint8 * FK_COMM_ID_BYTES)()
    _check(lib().fk_comm_id(b), "comm_id")
    return bytes(b)


class Comm:
    """The library's own RCCL communicator (fk_comm): every rank constructs
    it with the same id (collective)."""

    def __init__(self, uid, world, rank, device):
        b = (ctypes.c_uint8 * FK_COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _check(lib().fk_comm_create(b, world, rank, device, ctypes.byref(h)), "comm_create")
        self.h = h
        self.world, self.rank, self.device = world, rank, device

    def info(self):
        """(rank count, rank, device) as RCCL reports them (fk_comm_info;
        -1 where this RCCL lacks the query)"""
        n, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().fk_comm_info(self.h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)), "comm_info")
        return n.value, r.value, d.value

    def close(self):
        if getattr(self, "h", None):
            lib().fk_comm_destroy(self.h)
            self.h = None


def shard_rows_compose(rows_ptr, world, rank):
    """Compose `world` gathered pack rows (host memory, uint32) in rank
    order: the FkState entering `rank`'s shard, or None if some row is not
    a valid pack or a compact summary does not apply (every rank gets the
    same answer)."""
    out = FkState()
    rc = lib().fk_shard_rows_compose(rows_ptr, world, rank, ctypes.byref(out))
    if rc == FK_E_SUMMARY:
        return None
    _check(rc, "shard_rows_compose")
    return out


def summary_is_full(summary):
    """1 for a full transfer function, 0 for a compact summary"""
    rc = lib().fk_summary_is_full(ctypes.byref(summary))
    if rc < 0:
        raise FindKmerError(rc, "summary_is_full")
    return rc == 1


def count(data, k, ngpu=1, want_nodes=False):
    """Count k-mers of a host byte buffer on the GPU(s).  Returns (rc, table, result)."""
    import numpy as np
    L = lib()
    t = np.zeros(1 << (2 * k), dtype=np.uint32)
    r = FkResult()
    o = FkOpts()
    o.device = -1
    o.want_nodes = 1 if want_nodes else 0
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not hasattr(data, "ctypes") else data
    if len(buf) == 0:
        buf = np.zeros(1, dtype=np.uint8)
        n = 0
    else:
        n = len(buf)
    if ngpu > 1:
        rc = L.fk_count_multi(buf.ctypes.data, n, k, ngpu, ctypes.byref(o), t.ctypes.data_as(_U32P), ctypes.byref(r))
    else:
        rc = L.fk_count(buf.ctypes.data, n, k, ctypes.byref(o), t.ctypes.data_as(_U32P), ctypes.byref(r))
    if rc not in (FK_OK, FK_E_EMPTY, FK_E_UNTERMINATED_HEADER, FK_E_ROLLOVER):
        raise FindKmerError(rc, "fk_count")
    return rc, t, r


def synth_device(ptr, cap, n_bases, seed, fasta_line=0, stream=None):
    w = ctypes.c_uint64()
    _check(lib().fk_synth_device(ptr, cap, n_bases, seed, fasta_line, stream, ctypes.byref(w)), "synth")
    return w.value


def synth_upstream_device(ptr, cap, n_records, seed, first_rec=0, stream=None):
    """fk_synth_upstream_device: records [first_rec, first_rec + n_records)
    of the upstream-like FASTA (BASELINE.json configs[4]) into a device
    buffer; returns the bytes written"""
    w = ctypes.c_uint64()
    _check(lib().fk_synth_upstream_device(ptr, cap, first_rec, n_records, seed, stream, ctypes.byref(w)),
           "synth_upstream")
    return w.value


class DeviceInput:
    """A file made device-resident by fk_input_load (parallel pread into
    pinned buffers, async H2D); feed it with Engine.feed_device(ptr, len)."""

    def __init__(self, path, device=-1, threads=0):
        self.h = _P()
        _check(lib().fk_input_load(os.fsencode(path), device, threads, ctypes.byref(self.h)), "input_load")
        ptr, n, dev, sec = _P(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_double()
        _check(lib().fk_input_info(self.h, ctypes.byref(ptr), ctypes.byref(n), ctypes.byref(dev),
                                   ctypes.byref(sec)), "input_info")
        self.ptr, self.len, self.device, self.seconds = ptr.value or 0, n.value, dev.value, sec.value

    def headers(self, k):
        """(offsets of the '>' that start comment lines, baseCounter at each)
        as numpy uint64 arrays; raises FindKmerError(FK_E_STATE) when the
        file needs the streamed path"""
        import numpy as np
        n = ctypes.c_uint64()
        _check(lib().fk_input_headers(self.h, k, None, None, 0, ctypes.byref(n)), "input_headers")
        pos = np.zeros(max(1, n.value), dtype=np.uint64)
        bases = np.zeros(max(1, n.value), dtype=np.uint64)
        _check(lib().fk_input_headers(self.h, k, pos.ctypes.data_as(_U64P), bases.ctypes.data_as(_U64P), n.value,
                                      ctypes.byref(n)), "input_headers")
        return pos[:n.value], bases[:n.value]

    def close(self):
        if self.h:
            lib().fk_input_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_size(n_bases, fasta_line=0):
    if fasta_line > 0:
        return 11 + n_bases + n_bases // fasta_line
    if fasta_line < 0:
        return n_bases + n_bases // (-fasta_line)
    return n_bases


def write_stats(path, k, result, prob_out=True):
    import numpy as np
    p = (ctypes.c_double * 4)()
    rc = lib().fk_write_stats(path.encode(), k, ctypes.byref(result), None, p)
    return rc, [p[i] for i in range(4)]


def write_csv(path, k, counts, prob, windows, z_enable=0, z_threshold=0.0, threads=0):
    import numpy as np
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    p = (ctypes.c_double * 4)(*prob)
    _check(lib().fk_write_csv(path.encode(), k, c.ctypes.data_as(_U32P), p, windows, z_enable,
                              float(z_threshold), threads), "write_csv")


def write_csv_sparse(path, k, keys, counts, prob, windows, z_enable=0, z_threshold=0.0, threads=0):
    """CSV of a sparse table (17 <= k <= 20): distinct k-mer indices ascending + counts"""
    import numpy as np
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    if len(kk) == 0:
        kk = np.zeros(1, dtype=np.uint64)
        c = np.zeros(1, dtype=np.uint32)
        n = 0
    else:
        n = len(kk)
    p = (ctypes.c_double * 4)(*prob)
    _check(lib().fk_write_csv_sparse(path.encode(), k, kk.ctypes.data_as(_U64P), c.ctypes.data_as(_U32P), n, p,
                                     windows, z_enable, float(z_threshold), threads), "write_csv_sparse")
