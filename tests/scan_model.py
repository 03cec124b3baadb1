"""TEST INFRASTRUCTURE ONLY — a small pure-Python model of the reference scan
(findKmer/src/findKmer.cpp:962-1069) over (hdr, R, code) states, used by the
CPU multi-process tests to stand in for the GPU engine: it builds a shard's
transfer function in the engine's fk_summary layout (fk_device.h, struct TF)
and counts a shard from a given entering state.  Small inputs only.

States use the engine's internal base codes A0 C1 T2 G3 ((byte>>1)&3); the
C-ABI (fk_summary_apply, fk_state) converts codes to the reference's
A0 C1 G2 T3 (base2int :567-589) with fk_sigma.
"""
import numpy as np

SYM = {ord("A"): 0, ord("C"): 1, ord("T"): 2, ord("G"): 3}
M64 = (1 << 64) - 1


def sigma(x):
    """internal <-> reference digit map (swap 2 and 3), an involution"""
    return x ^ ((x >> 1) & 0x5555555555555555)


def advance(data, hdr, R, code):
    """Scan `data` from state (hdr, R, code).  Returns (hdr, R, code,
    any_reset, nv): any_reset = a run break outside a header ('>' :991, or a
    non-ACGT non-'\\n' byte :1063), nv = bases seen (meaningful without a
    reset).  0xFF bytes are not modelled (they end the reference's scan)."""
    any_reset = False
    nv = 0
    for c in data:
        if hdr:
            if c == 10:
                hdr = 0
            continue
        if c == ord(">"):
            hdr, R, any_reset = 1, 0, True
            continue
        if c == 10:
            continue
        s = SYM.get(c)
        if s is None:
            R, any_reset = 0, True
            continue
        code = ((code << 2) | s) & M64
        R += 1
        nv += 1
    return hdr, R, code, any_reset, nv


def summary_words(data):
    """The span's transfer function as the 12 u64 words of fk_summary:
    c1 (entering inside a header), then c0 if the span breaks a run outside a
    header (f0_const), else a shift by nv bases whose last bases are cs."""
    h1, r1, k1, _, _ = advance(data, 1, 0, 0)
    h0, r0, k0, reset, nv = advance(data, 0, 0, 0)
    w = [0] * 12
    w[0], w[1], w[2] = r1, k1, h1                     # c1 {R, code, hdr}
    if reset:
        w[3], w[4], w[5] = r0, k0, h0                 # c0
        w[8] = 1                                      # f0_const
    else:
        w[6], w[7] = nv, k0                           # nv, cs
    return w


def count_from(data, k, hdr, R, code, table):
    """Windows of `data` counted from the entering state (reference rules
    :1035-1057; int32 seqSize), added to `table` (reference index order)."""
    mask = (1 << (2 * k)) - 1
    for c in data:
        if hdr:
            if c == 10:
                hdr = 0
            continue
        if c == ord(">"):
            hdr, R = 1, 0
            continue
        if c == 10:
            continue
        s = SYM.get(c)
        if s is None:
            R = 0
            continue
        code = ((code << 2) | s) & M64
        R += 1
        seq = np.int64(R & 0xFFFFFFFF).astype(np.int32)
        if seq >= k:
            table[sigma(code & mask)] += 1
    return hdr, R, code


FK_SUMMARY_COMPACT = 0x434F4D50414354   # fk_engine.hip: tag of a compact summary (w[11])


class _Res:
    """the fk_result fields count_sharded reads"""

    def __init__(self):
        self.windows = self.valid_bases = self.unknown_chars = self.scanned_bytes = 0
        self.base_count = [0, 0, 0, 0]
        self.depth1 = [0, 0, 0, 0]
        self.hit_eof_byte = self.unterminated_header = 0


class ModelEngine:
    """Stands in for findkmer_amd.Engine in the CPU multi-process tests of
    findkmer_amd/dist.py: the same shard calls, computed with the reference
    rules (findKmer.cpp:962-1069, 0xFF = EOF at :988) on a host shard.
    guess = None: full transfer-function summaries (as for 8 <= k <= 12);
    else the (hdr, R, internal code) the shard's count is guessed from, and
    summary() returns a compact summary valid for equivalent states."""

    REF = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}

    def __init__(self, k, shard, guess=None):
        self.k = k
        self.data = bytes(shard)
        self.guess = guess
        self.entering = None
        self.tab = np.zeros(1 << (2 * k), dtype=np.uint32)

    def feed_shard_device(self, ptr, nbytes, halo):
        assert nbytes == len(self.data)

    def summary_full(self):
        from findkmer_amd import FkSummary
        s = FkSummary()
        for i, v in enumerate(summary_words(self.data)):
            s.w[i] = v % (1 << 64)
        return s

    def summary(self):
        if self.guess is None:
            return self.summary_full()
        from findkmer_amd import FkSummary
        hdr, R, code = self.guess
        h, r, c, ended = hdr, R, code, 0
        absorb, nv = 0, 0
        for ch in self.data:
            if h:
                if ch == 10:
                    h = 0
                continue
            if ch == ord(">"):
                h, r, absorb = 1, 0, 1
                continue
            if ch == 10:
                continue
            s = SYM.get(ch)
            if s is None:
                if ch == 0xFF:
                    ended = 1
                r, absorb = 0, 1
                continue
            c = ((c << 2) | s) & M64
            r += 1
            nv += 1
        if hdr and not absorb:
            absorb = 1   # a guessed header span: the state after it is fixed
        s = FkSummary()
        w = [code, R | (hdr << 32), len(self.data), r, c, h | (absorb << 32), nv, len(self.data), self.k,
             ended, 0, FK_SUMMARY_COMPACT]
        for i, v in enumerate(w):
            s.w[i] = v % (1 << 64)
        return s

    def resolve(self, state):
        self.entering = (state.hdr, state.run, sigma(state.code), state.ended)

    # fk_engine_shard_pack writes device buffers; this model writes host ones
    host_pack = True

    def shard_pack(self, table_ptr, counters_ptr, rows_ptr, nrows=1, slot=0, is_last=False):
        """fk_engine_shard_pack on host memory: the shard counted from its
        guess, its counters as 16-bit limbs, its compact summary in row
        `slot` (word 24 = 1 when valid: a compact guess and no 0xFF)."""
        import ctypes
        from findkmer_amd import FK_PACK_ROW_WORDS
        nb = 1 << (2 * self.k)
        tab = np.ctypeslib.as_array((ctypes.c_uint32 * nb).from_address(table_ptr))
        cnt = np.ctypeslib.as_array((ctypes.c_int32 * 56).from_address(counters_ptr))
        rows = np.ctypeslib.as_array((ctypes.c_uint32 * (nrows * FK_PACK_ROW_WORDS)).from_address(rows_ptr))
        rows[:] = 0
        cnt[:] = 0
        if self.guess is None:
            return
        hdr, R, code = self.guess
        saved = self.entering
        self.entering = (hdr, R, code, 0)
        _, res = self.finish()
        self.entering = saved
        if res.hit_eof_byte:
            return
        tab[:] = self.tab
        vals = [res.windows, res.valid_bases, *res.base_count, *res.depth1, res.unknown_chars,
                res.scanned_bytes, 0, res.unterminated_header if is_last else 0]
        for i, v in enumerate(vals):
            for j in range(4):
                cnt[4 * i + j] = (v >> (16 * j)) & 0xFFFF
        w = [int(x) for x in self.summary().w]
        row = rows[slot * FK_PACK_ROW_WORDS:(slot + 1) * FK_PACK_ROW_WORDS]
        for j, v in enumerate(w):
            row[2 * j] = v & 0xFFFFFFFF
            row[2 * j + 1] = v >> 32
        row[24] = 1

    def finish(self, allow=None):
        hdr, R, code, ended = self.entering
        k = self.k
        res = _Res()
        self.tab[:] = 0
        if ended:
            res.hit_eof_byte = 1
            return 0, res
        mask = (1 << (2 * k)) - 1
        # the reference's kmer[] window in reference codes, rebuilt from the
        # entering code (internal A0 C1 T2 G3 -> reference A0 C1 G2 T3)
        rcode = sigma(code)
        for pos, ch in enumerate(self.data):
            if hdr:
                if ch == 10:
                    hdr = 0
                continue
            if ch == ord(">"):
                hdr, R = 1, 0
                continue
            if ch == 10:
                continue
            b = self.REF.get(ch)
            if b is None:
                if ch == 0xFF:
                    res.hit_eof_byte = 1
                    res.scanned_bytes = pos
                    return 0, res
                if ch != ord("N"):
                    res.unknown_chars += 1
                R = 0
                continue
            rcode = ((rcode << 2) | b) & M64
            R += 1
            seq = int(np.int64(R & 0xFFFFFFFF).astype(np.int32))
            if seq >= k:
                idx = rcode & mask
                self.tab[idx] += 1
                res.windows += 1
                res.depth1[idx >> (2 * k - 2)] += 1
                if seq > k:
                    res.valid_bases += 1
                    res.base_count[b] += 1
                else:
                    res.valid_bases += k
                    for j in range(k):
                        res.base_count[(idx >> (2 * (k - 1 - j))) & 3] += 1
            elif seq >= 1:
                res.depth1[(rcode >> (2 * seq - 2)) & 3] += 1
        res.scanned_bytes = len(self.data)
        res.unterminated_header = hdr
        return 0, res

    def table(self):
        return self.tab.copy()


class SparseModelEngine(ModelEngine):
    """ModelEngine with the sparse table interface of 17 <= k <= 20
    (fk_engine_sparse / _split / _device / _adopt) on host buffers, so the
    gloo tests drive dist.py's all-to-all merge (dist._sparse_merge) at a
    small k."""

    device_str = "cpu"
    sparse_table = True

    def __init__(self, k, shard, guess=None):
        super().__init__(k, shard, guess)
        self.runs = None

    def finish(self, allow=None):
        rc, res = super().finish(allow)
        nz = np.nonzero(self.tab)[0]
        self.runs = (nz.astype(np.uint64), self.tab[nz].astype(np.uint32))
        return rc, res

    def sparse(self):
        return self.runs[0].copy(), self.runs[1].copy()

    def sparse_split(self, world):
        S = ((1 << (2 * self.k)) + world - 1) // world
        owner = (self.runs[0] // np.uint64(S)).astype(np.int64)
        return [int(v) for v in np.bincount(owner, minlength=world)[:world]]

    def sparse_device(self, keys_ptr, counts_ptr, cap):
        import ctypes
        n = len(self.runs[0])
        assert cap >= n
        ctypes.memmove(keys_ptr, self.runs[0].ctypes.data, 8 * n)
        ctypes.memmove(counts_ptr, self.runs[1].ctypes.data, 4 * n)
        return n

    def sparse_adopt(self, keys_ptr, counts_ptr, n):
        import ctypes
        keys = np.ctypeslib.as_array((ctypes.c_uint64 * max(1, n)).from_address(keys_ptr))[:n].copy()
        cnts = np.ctypeslib.as_array((ctypes.c_uint32 * max(1, n)).from_address(counts_ptr))[:n].astype(np.uint64)
        uk, inv = np.unique(keys, return_inverse=True)
        sums = np.zeros(len(uk), dtype=np.uint64)
        np.add.at(sums, inv, cnts)
        self.runs = (uk, (sums & 0xFFFFFFFF).astype(np.uint32))
        return len(uk), int(self.runs[1].astype(np.uint64).sum())
