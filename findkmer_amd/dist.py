"""Multi-GPU orchestration of one sharded stream.

One process per GPU.  Each rank owns a contiguous byte range of the stream
(plus up to 256 bytes of halo before it) and counts it with guessed entry
states (fk_engine_feed_shard).  The path has two exchange steps, plus a third
only when a shard may end the stream:

1. state stitch: all-gather the 96-byte shard summaries (fk_engine_summary:
   for a shard counted in one pass, a compact summary valid for entering
   states equivalent to the shard's guessed entry; else the full transfer
   function) and compose them in rank order (fk_summary_apply) -> the exact
   entering state, handed to fk_engine_resolve, which recounts only what the
   guess got wrong (nothing, when the compact summaries applied).  If one
   does not apply, all ranks exchange the full summaries in a second round.
   A compact summary also says whether its shard ends the stream (a 0xFF
   byte outside a header: the reference's signed-char EOF, findKmer.cpp:988),
   and the composed state of every later shard is then `ended`: those ranks
   count nothing.  A full transfer function does not know where the stream
   ends, so when any rank's summary is full (always for 8 <= k <= 12), the
   ranks all-gather their exact end flags after the resolve (8 bytes each);
2. table merge: one reduce of the 4^k count tables to rank 0 (the rank that
   writes the outputs).  Counts are u32 in the reference (findKmer.cpp:110);
   int32 sums are bitwise identical.  The reduced buffer carries, after the
   table, every rank's scalar counters (windows, bases, composition, depth-1
   counts, ...) split into 16-bit limbs, so rank 0 gets their exact u64 sums
   from the same collective and checks the merged table for the reference's
   rollover exit (a u32 trie counter reaching 2^32, :642-648): a merged bin
   that wrapped makes the table total fall short of the window count.
   For k >= SHARD_KMIN (4^k >= 16 Mi bins: 64 MiB to 16 GiB) the table is
   sharded instead: a reduce-scatter leaves rank r the bins
   [r*S, (r+1)*S) of the sum -- the k-mers whose first bases fall in r's
   range, a contiguous run of the CSV's rows (findKmer.cpp:719-724) -- and
   one small all-reduce gives every rank the counters plus every slice's
   total and distinct bins (the rollover check needs the whole table's sum).
   ShardedResult.table_full() gathers the slices onto rank 0 when one
   process writes the CSV.
   For 17 <= k <= 20 the tables are sparse (fk_engine_sparse: sorted
   distinct indices + u32 counts) and the same ownership holds without a
   dense buffer: each rank cuts its finished table at the owners' bounds
   (fk_engine_sparse_split), one all-to-all sends every run to its owner,
   and the owner sums repeated keys (fk_engine_sparse_adopt, on the GPU):
   SparseShardedResult.

The library's own RCCL communicator (backend nccl, native_comm) runs the
whole exchange inside fk_engine_shard_exchange on the engine's stream: the
one-collective path below when it applies, else steps 1-2 with
all-reduces of rows standing in for the all-gathers (one host wait each).
torch.distributed carries the same protocol for gloo rehearsals.

One-collective fast path (k <= 7, shards counted in one pass): before any
host round trip, every rank packs what its shard would report if its guessed
entering state holds -- table, counter limbs, and its compact summary in its
own row of a rows region (fk_engine_shard_pack, on the engine's stream) --
and ONE all-reduce merges the tables and counters and, since the other
ranks' rows are zero, all-gathers the summaries.  Each rank then composes
the rows on the host (fk_shard_rows_compose); when every guess held (the
normal case: a 256-byte halo fixes the state deep in a run) the merged
buffer is already exact and the shard is resolved without further device
work.  Otherwise every rank sees the same failure and runs steps 1-2 above.

The same functions run over RCCL (backend "nccl", device tensors, bench.py)
and over gloo on the CPU (tests/test_dist_cpu.py, with a model engine).
"""
import os
import torch
import torch.distributed as dist

from . import FK_E_EMPTY, FK_E_ROLLOVER, FK_E_SUMMARY, FK_E_UNTERMINATED_HEADER, FK_OK, FK_ROUTE_KMIN
from . import FK_PACK_COUNTERS, FK_PACK_ROW_WORDS, FK_PACK_STATS
from . import Comm, FindKmerError, FkState, FkSummary, comm_id, lib, shard_rows_compose, summary_apply, summary_is_full

SUMMARY_WORDS = 12
GATHER_WORDS = SUMMARY_WORDS + 1      # + "my summary is full" flag
_U64 = 1 << 64

# scalar counters merged with the table (u64 each, 4 x 16-bit limbs)
COUNTERS = ("windows", "valid_bases", "base0", "base1", "base2", "base3",
            "depth1_0", "depth1_1", "depth1_2", "depth1_3", "unknown_chars",
            "scanned_bytes", "ended", "unterminated_header")
LIMBS = 4
COUNTER_SLOTS = len(COUNTERS) * LIMBS
assert len(COUNTERS) == FK_PACK_COUNTERS   # the order fk_engine_shard_pack writes them in
ROW_WORDS = FK_PACK_ROW_WORDS
STAT_SLOTS = FK_PACK_STATS              # a sharded table's (total, distinct) as 4 limbs each
FAST_KMAX = 7                          # shards counted in one pass (k_count + k_tail)
SHARD_KMIN = 12                        # from here on the merged table is sharded over the ranks
SPARSE_KMIN = 17                       # from here on the tables are sparse (fk_engine_sparse)


def _to_i64(v):
    return v - _U64 if v >= 1 << 63 else v


def table_words(k, world):
    """4^k rounded up to a multiple of world (fk_merge_layout)"""
    nb = 1 << (2 * k)
    return (nb + world - 1) // world * world


def merge_buffer(k, device, world=None):
    """The int32 buffer count_sharded merges (include/findkmer.h,
    fk_merge_layout): the table padded to a multiple of the world size, the
    counter limbs, the slice statistics, then one pack row per rank (the fast
    path's all-gather)."""
    if world is None:
        world = dist.get_world_size() if dist.is_initialized() else 1
    return torch.zeros(table_words(k, world) + COUNTER_SLOTS + STAT_SLOTS + world * ROW_WORDS, dtype=torch.int32,
                       device=device)


def _regions(buf, k, world):
    """(4^k, padded table words, table + counters + stats, rows)"""
    nb, tw = 1 << (2 * k), table_words(k, world)
    end = tw + COUNTER_SLOTS + STAT_SLOTS
    assert buf.numel() >= end + world * ROW_WORDS, "merge_buffer(k, device, world)"
    return nb, tw, buf[:end], buf[end:end + world * ROW_WORDS]


def _compose(words, world, rank):
    """Compose the gathered summaries in rank order from the stream's initial
    state.  Returns (entering state of `rank`, first rank whose shard ends the
    stream as far as the compact summaries tell, any full summary) or None if
    a compact summary does not apply."""
    state = FkState()
    entering, first_end, any_full = None, None, False
    for r in range(world):
        if r == rank:
            entering = state
        row = words[r * GATHER_WORDS:(r + 1) * GATHER_WORDS]
        s = FkSummary()
        for i, v in enumerate(row[:SUMMARY_WORDS]):
            s.w[i] = v % _U64
        any_full = any_full or bool(row[SUMMARY_WORDS])
        was_ended = bool(state.ended)
        try:
            state = summary_apply(s, state)
        except FindKmerError as err:
            if err.code != FK_E_SUMMARY:
                raise
            return None
        if state.ended and not was_ended:
            first_end = r
    return entering, first_end, any_full


def _gather_rows(row, group, device):
    world = dist.get_world_size(group)
    mine = torch.tensor([_to_i64(int(v) % _U64) for v in row], dtype=torch.int64, device=device)
    # one gather into one tensor and one copy to the host (not one
    # synchronising copy per rank: at 1 GB per GPU a step is ~0.2 ms)
    everyone = torch.empty(world * len(row), dtype=torch.int64, device=mine.device)
    dist.all_gather_into_tensor(everyone, mine, group=group)
    return everyone.tolist()


def stitch_entry_state(summary, group=None, device=None, full=None):
    """All-gather every rank's shard summary (fk_summary, or its 12 u64
    words) and compose them in rank order.  Returns (entering FkState of this
    rank's shard, first ending rank per the compact summaries or None, any
    rank's summary is full), or None when some rank's compact summary does
    not apply to the state entering it (every rank sees the same failure and
    the caller exchanges the full summaries instead)."""
    words = list(summary.w) if isinstance(summary, FkSummary) else list(summary)
    if full is None:
        s = summary if isinstance(summary, FkSummary) else _as_summary(words)
        full = summary_is_full(s)
    rows = _gather_rows(words + [1 if full else 0], group, device)
    return _compose(rows, dist.get_world_size(group), dist.get_rank(group))


def _as_summary(words):
    s = FkSummary()
    for i, v in enumerate(words):
        s.w[i] = int(v) % _U64
    return s


def sum_tables(table, group=None, everywhere=False):
    """Sum the ranks' int32 buffers into rank 0's (the rank that writes the
    CSV): one reduce, half the bytes of an all-reduce over the xGMI ring
    (16 MiB per GPU at k=11).  everywhere=True: all-reduce."""
    if everywhere:
        dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.reduce(table, dst=0, op=dist.ReduceOp.SUM, group=group)
    return table


def _limbs_value(limbs):
    v = 0
    for j, x in enumerate(limbs):
        v += int(x) << (16 * j)
    return v % _U64


class ShardedResult:
    """The merged result of one sharded pass.  Complete on rank 0 (the reduce
    destination), on every rank after the one-collective path, and with a
    sharded table (`sharded`) each rank holds the slice [lo, hi) of the
    merged table (`table`) and every merged counter.  Counter fields mirror
    fk_result (include/findkmer.h); they are decoded from the buffer on
    first access (one device-to-host copy)."""

    def __init__(self, buf, k, rank, first_end, local=None, path="stitched", transport="torch", world=1,
                 sharded=False, group=None):
        self.local = local          # this rank's own fk_result (timings)
        self.path = path            # "fast": one all-reduce; "stitched": summary exchange + reduce
        self.transport = transport  # "rccl-native": the library's own communicator; "torch": torch.distributed
        self.buf = buf
        self.k = k
        self.rank = rank
        self.world = world
        self.group = group
        self.first_end = first_end
        self.sharded = sharded and path == "stitched"
        self.nb = 1 << (2 * k)
        self.tw = table_words(k, world)
        if self.sharded:
            S = self.tw // world
            self.lo, self.hi = min(rank * S, self.nb), min((rank + 1) * S, self.nb)
        else:
            self.lo, self.hi = 0, self.nb
        self.table = buf[self.lo:self.hi]
        self._vals = None
        self._tsum = self._distinct = None

    def _table_stats(self):
        """The merged table's u64 total (int32 sum + 2^32 per negative bin)
        and its distinct k-mers, computed on first use (like `table`, valid
        until the buffer is merged into again); a sharded table's come from
        the all-reduced slice statistics."""
        if self._tsum is None:
            if self.sharded:
                st = self.buf[self.tw + COUNTER_SLOTS:self.tw + COUNTER_SLOTS + STAT_SLOTS].tolist()
                self._tsum, self._distinct = _limbs_value(st[:4]), _limbs_value(st[4:])
            else:
                assert self.rank == 0 or self.path == "fast", "the merged table lives on rank 0"
                t = self.table
                self._tsum = int((t.sum(dtype=torch.int64) + (t < 0).sum(dtype=torch.int64) * (1 << 32)).item())
                self._distinct = int((t != 0).sum(dtype=torch.int64).item())
        return self._tsum, self._distinct

    def table_full(self, dst=0):
        """The whole merged table (int32 view of the u32 counts) on rank
        `dst`, None on the others; a collective for a sharded table (every
        rank calls it), a view of the buffer otherwise."""
        if not self.sharded:
            return self.buf[:self.nb] if self.rank == dst or self.path == "fast" else None
        S = self.tw // self.world
        mine = self.buf[self.rank * S:(self.rank + 1) * S].contiguous()
        parts = [torch.empty_like(mine) for _ in range(self.world)] if self.rank == dst else None
        dist.gather(mine, parts, dst=dist.get_global_rank(self.group, dst) if self.group is not None else dst,
                    group=self.group)
        return torch.cat(parts)[:self.nb] if parts is not None else None

    def _decode(self):
        if self._vals is None:
            limbs = self.buf[self.tw:self.tw + COUNTER_SLOTS].tolist()
            self._vals = {name: _limbs_value(limbs[i * LIMBS:(i + 1) * LIMBS]) for i, name in enumerate(COUNTERS)}
        return self._vals

    def __getattr__(self, name):
        if name.startswith("_") or name in ("buf", "k", "rank", "first_end", "table", "local", "nb", "path",
                                                     "transport", "world", "group", "sharded", "tw", "lo", "hi"):
            raise AttributeError(name)
        v = self._decode()
        if name == "base_count":
            return [v[f"base{b}"] for b in range(4)]
        if name == "depth1":
            return [v[f"depth1_{b}"] for b in range(4)]
        if name == "hit_eof_byte":
            return v["ended"]
        if name in v:
            return v[name]
        raise AttributeError(name)

    @property
    def distinct(self):
        return self._table_stats()[1]

    @property
    def rollover(self):
        """The reference's COUNTER ROLLOVER exit (:642-648): a merged bin or
        a depth-1 trie counter reached 2^32."""
        tsum, _ = self._table_stats()
        v = self._decode()
        if tsum != v["windows"]:
            return True
        return any(v[f"depth1_{b}"] >= 1 << 32 for b in range(4))

    def status(self):
        """fk_engine_finish's status for the whole stream (rank 0)."""
        if self.rollover:
            return FK_E_ROLLOVER
        if self.unterminated_header:
            return FK_E_UNTERMINATED_HEADER
        return FK_OK


class SparseShardedResult(ShardedResult):
    """The merged result of a sharded pass for 17 <= k <= 20: this rank owns
    the k-mer indices [lo, hi) of the merged sparse table (`keys`, `counts`,
    numpy, ascending = CSV row order); the counters, total and distinct
    k-mers are merged over all ranks (one all-reduce of limbs)."""

    def __init__(self, buf, k, rank, first_end, local, world, group, engine):
        super().__init__(buf, k, rank, first_end, local, path="stitched", transport="torch", world=world,
                         sharded=True, group=group)
        self.tw = 0                     # the buffer holds counters and slice statistics only
        S = ((1 << (2 * k)) + world - 1) // world
        self.lo, self.hi = min(rank * S, self.nb), min((rank + 1) * S, self.nb)
        self.table = None
        self.keys, self.counts = engine.sparse()

    def _table_stats(self):
        if self._tsum is None:
            st = self.buf[COUNTER_SLOTS:COUNTER_SLOTS + STAT_SLOTS].tolist()
            self._tsum, self._distinct = _limbs_value(st[:4]), _limbs_value(st[4:])
        return self._tsum, self._distinct

    def _decode(self):
        if self._vals is None:
            limbs = self.buf[:COUNTER_SLOTS].tolist()
            self._vals = {name: _limbs_value(limbs[i * LIMBS:(i + 1) * LIMBS]) for i, name in enumerate(COUNTERS)}
        return self._vals

    def table_full(self, dst=0):
        """(keys, counts) of the whole merged table on rank `dst` (a
        collective: every rank calls it), None on the others.  Only `dst`
        receives the other ranks' runs (point-to-point, exact sizes): no rank
        but dst ever holds more than its own slice."""
        import numpy as np
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"
        n = torch.tensor([len(self.keys)], dtype=torch.int64, device=dev)
        sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        sizes = [int(v.item()) for v in sizes]
        g = (lambda r: dist.get_global_rank(self.group, r)) if self.group is not None else (lambda r: r)
        if self.rank != dst:
            if sizes[self.rank]:
                kp = torch.from_numpy(self.keys.view(np.int64)).to(dev)
                cp = torch.from_numpy(self.counts.view(np.int32)).to(dev)
                dist.send(kp, g(dst), group=self.group)
                dist.send(cp, g(dst), group=self.group)
            return None
        keys, cnts = [], []
        for r in range(self.world):
            if r == self.rank:
                keys.append(self.keys)
                cnts.append(self.counts)
            elif sizes[r]:
                kp = torch.empty(sizes[r], dtype=torch.int64, device=dev)
                cp = torch.empty(sizes[r], dtype=torch.int32, device=dev)
                dist.recv(kp, g(r), group=self.group)
                dist.recv(cp, g(r), group=self.group)
                keys.append(kp.cpu().numpy().view(np.uint64))
                cnts.append(cp.cpu().numpy().view(np.uint32))
        return (np.concatenate(keys) if keys else np.zeros(0, np.uint64),
                np.concatenate(cnts) if cnts else np.zeros(0, np.uint32))


def _sparse_merge(engine, vals, counting, rank, world, group, first_end, r):
    """17 <= k <= 20: every rank's runs to their owners (one all-to-all of
    keys and one of counts, after one of the run counts), the owner's sum
    (fk_engine_sparse_adopt), then one all-reduce of the counter and slice
    statistic limbs."""
    nccl = dist.get_backend(group) == "nccl"
    coll = "cuda" if nccl else "cpu"
    edev = getattr(engine, "device_str", "cuda")   # where the engine's buffers live
    counts = engine.sparse_split(world) if counting else [0] * world
    n = sum(counts)
    keys = torch.empty(max(1, n), dtype=torch.int64, device=edev)
    cnts = torch.empty(max(1, n), dtype=torch.int32, device=edev)
    if n:
        got = engine.sparse_device(keys.data_ptr(), cnts.data_ptr(), n)
        assert got == n, (got, n)
    send = torch.tensor(counts, dtype=torch.int64, device=coll)
    recv = torch.empty(world, dtype=torch.int64, device=coll)
    dist.all_to_all_single(recv, send, group=group)
    rsizes = [int(v) for v in recv.tolist()]
    m = sum(rsizes)
    k_out = torch.empty(max(1, m), dtype=torch.int64, device=coll)
    c_out = torch.empty(max(1, m), dtype=torch.int32, device=coll)
    dist.all_to_all_single(k_out[:m], keys[:n].to(coll), rsizes, counts, group=group)
    dist.all_to_all_single(c_out[:m], cnts[:n].to(coll), rsizes, counts, group=group)
    k_in, c_in = k_out.to(edev), c_out.to(edev)
    if edev != "cpu":
        torch.cuda.synchronize()
    distinct, total = engine.sparse_adopt(k_in.data_ptr(), c_in.data_ptr(), m)
    buf = torch.zeros(COUNTER_SLOTS + STAT_SLOTS, dtype=torch.int32, device=coll)
    _put_counters(buf, vals, None, 0)
    buf[COUNTER_SLOTS:].copy_(torch.tensor([(v >> (16 * j)) & 0xFFFF for v in (total, distinct) for j in range(LIMBS)],
                                           dtype=torch.int32))
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return SparseShardedResult(buf.cpu(), engine.k, rank, first_end, r, world, group, engine)


def _put_counters(buf, values, pinned, nb=None):
    """Write the u64 counters into the buffer's limb slots (host -> buffer),
    after the nb table words (default: the last COUNTER_SLOTS entries)."""
    limbs = []
    for v in values:
        v = int(v) % _U64
        limbs.extend((v >> (16 * j)) & 0xFFFF for j in range(LIMBS))
    dst = buf[nb:nb + COUNTER_SLOTS] if nb is not None else buf[-COUNTER_SLOTS:]
    if pinned is not None:
        pinned.copy_(torch.tensor(limbs, dtype=torch.int32))
        dst.copy_(pinned, non_blocking=True)
    else:
        dst.copy_(torch.tensor(limbs, dtype=torch.int32))


_comms = {}


def native_comm(group=None):
    """The library's own RCCL communicator (findkmer_amd.Comm) over the
    ranks of `group` (backend nccl), made on first use: group rank 0 creates
    the id, one broadcast hands it over, every rank joins.  None when RCCL
    could not be set up on some rank (every rank then learns it from one
    more all-reduce and uses the torch.distributed path instead)."""
    key = group   # None: the default group (process groups hash by identity)
    if key in _comms:
        return _comms[key]
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    # every rank checks what fk_comm_create needs before its collective init
    # (RCCL loadable, the device usable), and all agree first: a rank that
    # cannot join must not leave the others blocked inside the init
    ok = lib().fk_comm_available(torch.cuda.current_device()) == FK_OK
    t = torch.zeros(130, dtype=torch.uint8, device="cuda")
    t[129] = 0 if ok else 1
    dist.all_reduce(t[129:], group=group)
    if int(t[129].item()):
        _comms[key] = None
        return None
    if rank == 0:
        try:
            t[:128].copy_(torch.frombuffer(bytearray(comm_id()), dtype=torch.uint8))
        except FindKmerError:
            t[128] = 1
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(t[:129], src=src, group=group)
    c, failed = None, bool(t[128].item())
    if not failed:
        try:
            c = Comm(bytes(t[:128].cpu().tolist()), world, rank, torch.cuda.current_device())
        except FindKmerError:
            failed = True
    bad = torch.tensor([1 if failed else 0], dtype=torch.int32, device="cuda")
    dist.all_reduce(bad, group=group)
    if int(bad.item()):
        if c is not None:
            c.close()
        c = None
    _comms[key] = c
    return c


def close_native_comms():
    for c in _comms.values():
        if c is not None:
            c.close()
    _comms.clear()


class _FastPath:
    """Per-engine scratch of the one-collective path: the engine's stream as
    a torch stream, a pinned host copy of the rows, and (gloo rehearsal of a
    GPU engine) a device staging buffer for the pack."""

    def __init__(self, engine, buf, world):
        self.host_pack = getattr(engine, "host_pack", False)
        self.world = world
        self.rows_h = None
        self.stage = None
        self.ext = None
        if not self.host_pack:
            self.ext = torch.cuda.ExternalStream(engine.stream())
            self.rows_h = torch.empty(world * ROW_WORDS, dtype=torch.int32, pin_memory=True)
            if not buf.is_cuda:
                self.stage = torch.empty(buf.numel(), dtype=torch.int32, device="cuda")


def _fast_exchange(engine, buf, rank, world, group, times, t0):
    """The one-collective path (see the module docstring).  Returns a
    ShardedResult, or None when some rank's pack is not valid or its compact
    summary does not apply (all ranks return None together; the shard is
    still pending)."""
    import time
    fp = getattr(engine, "_fk_fast", None)
    if fp is None or fp.world != world or (fp.stage is None) != (buf.is_cuda or fp.host_pack):
        fp = _FastPath(engine, buf, world)
        engine._fk_fast = fp
    k = engine.k
    nb, tw, merged, rows = _regions(buf, k, world)
    n = tw + COUNTER_SLOTS + STAT_SLOTS + world * ROW_WORDS
    dst = fp.stage if fp.stage is not None else buf
    if not fp.host_pack:
        # the pack writes into the buffer after whatever torch's stream still
        # has pending on it (a previous pass's collective or copy)
        fp.ext.wait_stream(torch.cuda.current_stream())
    if tw > nb or STAT_SLOTS:
        dst[nb:tw].zero_()
        dst[tw + COUNTER_SLOTS:tw + COUNTER_SLOTS + STAT_SLOTS].zero_()
        if not fp.host_pack:
            fp.ext.wait_stream(torch.cuda.current_stream())
    engine.shard_pack(dst.data_ptr(), dst.data_ptr() + 4 * tw, dst.data_ptr() + 4 * (tw + COUNTER_SLOTS + STAT_SLOTS),
                      world, rank, rank == world - 1)
    if not fp.host_pack:
        # the copy or the collective runs after the pack (engine stream ->
        # torch's current stream)
        torch.cuda.current_stream().wait_stream(fp.ext)
    if fp.stage is not None:
        # gloo rehearsal of a GPU engine: the host buffer gets the pack
        buf[:n].copy_(fp.stage[:n].cpu())
    t1 = time.perf_counter()
    dist.all_reduce(buf[:n], op=dist.ReduceOp.SUM, group=group)
    if buf.is_cuda:
        fp.rows_h.copy_(rows, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        rows_ptr = fp.rows_h.data_ptr()
    else:
        rows_ptr = rows.data_ptr()
    state = shard_rows_compose(rows_ptr, world, rank)
    t2 = time.perf_counter()
    if state is None:
        return None
    engine.resolve(state)
    _, r = engine.finish(allow=(FK_OK, FK_E_ROLLOVER, FK_E_UNTERMINATED_HEADER, FK_E_EMPTY))
    if times is not None:
        times["count"] = times.get("count", 0.0) + (t1 - t0)
        times["exchange"] = times.get("exchange", 0.0) + (t2 - t1)
        times["resolve"] = times.get("resolve", 0.0) + (time.perf_counter() - t2)
    return ShardedResult(buf, k, rank, None, r, path="fast", world=world, group=group)


def count_sharded(engine, ptr, nbytes, halo, buf, group=None, times=None, pinned=None, fast=True,
                  native=True, shard_table=None, test_invalid=False):
    """One sharded pass on this rank's GPU: count the shard, stitch the entry
    state, recount what the guess got wrong, and merge the tables and
    counters into `buf` (merge_buffer(k, device, world): on the GPU for RCCL,
    on the host for a gloo rehearsal; the sum lands on rank 0, and on every
    rank when the one-collective path applies).  Returns a ShardedResult.
    `pinned` (optional): a pinned host int32 tensor of COUNTER_SLOTS entries
    for an asynchronous counter upload.  fast=False: always the stitched
    exchange (steps 1-2).  native: over RCCL (backend nccl, device buffer)
    the whole exchange -- one collective or stitched -- runs inside the
    library on the engine's stream (fk_engine_shard_exchange with its own
    communicator, native_comm) instead of through torch.distributed; the
    buffer is complete when this returns.

    `engine` is a findkmer_amd.Engine (or, in the CPU tests, a model with the
    same feed_shard_device / summary / summary_full / resolve / finish /
    table_to_device / shard_pack methods).

    17 <= k <= 20: `buf` is unused (may be None); the sparse tables are
    merged by an all-to-all to their owners (SparseShardedResult).

    shard_table: the stitched path reduce-scatters the table (each rank
    keeps its slice of the merged table) instead of reducing it onto rank 0;
    None = for k >= SHARD_KMIN.  test_invalid (native path, tests): this
    rank's pack row reads as invalid, forcing the fallback after the
    one-collective all-reduce."""
    import time
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = buf.device if buf is not None else None
    k = engine.k
    if shard_table is None:
        shard_table = k >= SHARD_KMIN
    t0 = time.perf_counter()
    engine.feed_shard_device(ptr, nbytes, halo)
    comm = None
    sparse = bool(getattr(engine, "sparse_table", k >= SPARSE_KMIN))
    if native and not sparse and buf is not None and buf.is_cuda and hasattr(engine, "shard_exchange") \
            and dist.get_backend(group) == "nccl":
        comm = native_comm(group)
    if comm is not None:
        # the whole exchange inside the library, on the engine's stream: one
        # all-reduce when every guess held (k <= 7), else the stitched
        # exchange (fk_engine_shard_exchange)
        one, first_end = engine.shard_exchange(comm, buf.data_ptr(), fast=fast and k <= FAST_KMAX,
                                               shard_table=shard_table, test_invalid=test_invalid)
        t1 = time.perf_counter()
        _, r = engine.finish(allow=(FK_OK, FK_E_ROLLOVER, FK_E_UNTERMINATED_HEADER, FK_E_EMPTY))
        if times is not None:
            times["exchange"] = times.get("exchange", 0.0) + (t1 - t0)
            times["finish"] = times.get("finish", 0.0) + (time.perf_counter() - t1)
        return ShardedResult(buf, k, rank, first_end, r, path="fast" if one else "stitched",
                             transport="rccl-native", world=world, sharded=shard_table, group=group)
    if fast and not sparse and engine.k <= FAST_KMAX and hasattr(engine, "shard_pack"):
        got = _fast_exchange(engine, buf, rank, world, group, times, t0)
        if got is not None:
            return got
    t1 = time.perf_counter()
    sdev = dev if buf is not None else ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
    got = stitch_entry_state(engine.summary(), group, sdev)
    if got is None:
        # a compact summary did not apply somewhere: the full transfer
        # functions (every rank takes this branch together)
        got = stitch_entry_state(engine.summary_full(), group, sdev, full=True)
    state, first_end, any_full = got
    engine.resolve(state)
    rc, r = engine.finish(allow=(FK_OK, FK_E_ROLLOVER, FK_E_UNTERMINATED_HEADER, FK_E_EMPTY))
    if any_full:
        # where the stream ends is exact only after the resolve: one more
        # small all-gather of the ranks' end flags
        ends = _gather_rows([1 if (r.hit_eof_byte and not state.ended) else 0], group, sdev)
        first_end = next((i for i, f in enumerate(ends) if f), None)
    t2 = time.perf_counter()
    counting = first_end is None or rank <= first_end
    last = first_end if first_end is not None else world - 1
    if sparse:
        vals = [0] * len(COUNTERS)
        if counting:
            vals = [r.windows, r.valid_bases, *r.base_count, *r.depth1, r.unknown_chars, r.scanned_bytes,
                    1 if rank == first_end else 0, r.unterminated_header if rank == last else 0]
        scomm = None
        if native and hasattr(engine, "sparse_exchange") and dist.get_backend(group) == "nccl":
            scomm = native_comm(group)
        if scomm is not None:
            # over RCCL: the all-to-all of runs, their merge and the counter
            # all-reduce inside the library, on the engine's stream
            limbs = torch.zeros(COUNTER_SLOTS + STAT_SLOTS, dtype=torch.int32, device="cuda")
            _put_counters(limbs, vals, None, 0)
            engine.sparse_exchange(scomm, counting, limbs.data_ptr())
            res = SparseShardedResult(limbs.cpu(), engine.k, rank, first_end, r, world, group, engine)
            res.transport = "rccl-native"
        else:
            res = _sparse_merge(engine, vals, counting, rank, world, group, first_end, r)
        if times is not None:
            times["count"] = times.get("count", 0.0) + (t1 - t0)
            times["stitch"] = times.get("stitch", 0.0) + (t2 - t1)
            times["merge"] = times.get("merge", 0.0) + (time.perf_counter() - t2)
        return res
    nb, tw, merged, _ = _regions(buf, k, world)
    # k >= FK_ROUTE_KMIN over gloo: each owner gets only the nonzero bins of
    # its slice (fk_engine_route_*), not the whole table
    route = shard_table and k >= FK_ROUTE_KMIN and hasattr(engine, "route_pack") and \
        dist.get_backend(group) != "nccl" and torch.cuda.is_available() and route_mode() >= 1
    if counting:
        if route:
            pass
        elif buf.is_cuda:
            engine.table_to_device(buf.data_ptr())
        else:
            buf[:nb].copy_(torch.from_numpy(engine.table().view("int32")))
        vals = [r.windows, r.valid_bases, *r.base_count, *r.depth1, r.unknown_chars, r.scanned_bytes,
                1 if rank == first_end else 0,
                r.unterminated_header if rank == last else 0]
    else:
        if not route:
            buf[:nb].zero_()
        vals = [0] * len(COUNTERS)
    if not route:
        buf[nb:tw].zero_()
    buf[tw + COUNTER_SLOTS:tw + COUNTER_SLOTS + STAT_SLOTS].zero_()
    _put_counters(buf, vals, pinned, tw)
    if shard_table:
        _scatter_tables(buf, k, rank, world, group, engine=engine if route else None, counting=counting)
    else:
        sum_tables(merged, group)
    if times is not None:
        # host wall time per phase: count (the feed returns when the shard's
        # kernels are done), stitch + resolve, table merge (enqueued)
        times["count"] = times.get("count", 0.0) + (t1 - t0)
        times["stitch"] = times.get("stitch", 0.0) + (t2 - t1)
        times["merge"] = times.get("merge", 0.0) + (time.perf_counter() - t2)
    return ShardedResult(buf, k, rank, first_end, r, world=world, sharded=shard_table, group=group)


def route_mode():
    """FINDKMER_TUNE route (the library's knob, fk_engine_create): 0 (the
    default) = the sharded table is reduce-scattered, 1 / 2 = routed (the
    nonzero bins of each owner's slice) -- so the gloo rehearsal takes the
    path the library's RCCL exchange takes."""
    for item in os.environ.get("FINDKMER_TUNE", "").split(","):
        name, _, val = item.partition("=")
        if name == "route" and val.isdigit():
            return min(int(val), 2)
    return 0


def _route_tables(engine, buf, k, rank, world, group, counting):
    """The routed sharded merge over torch.distributed (gloo): every rank's
    blobs (fk_engine_route_pack: the nonzero bins of each owner's slice) go
    to their owners by all_to_all_single, and the owner counts what it got
    into its slice (fk_engine_route_absorb), then copies the slice to `buf`."""
    nb, tw = 1 << (2 * k), table_words(k, world)
    S = tw // world
    dev = torch.device("cuda", torch.cuda.current_device())
    words = engine.route_pack(world, counting)
    send = torch.empty(max(1, sum(words)), dtype=torch.int32, device=dev)
    engine.route_copy(send.data_ptr())
    coll = buf.device
    rsz = torch.empty(world, dtype=torch.int64, device=coll)
    dist.all_to_all_single(rsz, torch.tensor(words, dtype=torch.int64, device=coll), group=group)
    rwords = [int(v) for v in rsz.tolist()]
    recv = torch.empty(sum(rwords), dtype=torch.int32, device=coll)
    at = 0
    for w in rwords:   # each blob's trailer must arrive with it (fk_engine_route_absorb checks it)
        at += w
        recv[max(0, at - 2):at] = 0
    dist.all_to_all_single(recv, send[:sum(words)].to(coll), rwords, words, group=group)
    lo = rank * S
    n = max(0, min(S, nb - lo))
    mine = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    recv_d = recv.to(dev)
    engine.route_absorb(world, rank, recv_d.data_ptr(), rwords, mine.data_ptr())
    if n:
        buf[lo:lo + n].copy_(mine[:n])


def _scatter_tables(buf, k, rank, world, group, engine=None, counting=True):
    """The sharded merge through torch.distributed: rank r gets bins
    [r*S, (r+1)*S) of the summed table (a reduce-scatter over RCCL; gloo has
    none, so an all-reduce whose other slices are then ignored), then the
    counters and each slice's (total, distinct) limbs are all-reduced."""
    nb, tw = 1 << (2 * k), table_words(k, world)
    S = tw // world
    table = buf[:tw]
    if engine is not None:
        _route_tables(engine, buf, k, rank, world, group, counting)
    elif dist.get_backend(group) == "nccl":
        mine = torch.empty(S, dtype=buf.dtype, device=buf.device)
        dist.reduce_scatter_tensor(mine, table, op=dist.ReduceOp.SUM, group=group)
        buf[rank * S:(rank + 1) * S].copy_(mine)
    else:
        dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)
    sl = buf[min(rank * S, nb):min((rank + 1) * S, nb)]
    tot = int((sl.sum(dtype=torch.int64) + (sl < 0).sum(dtype=torch.int64) * (1 << 32)).item())
    nz = int((sl != 0).sum(dtype=torch.int64).item())
    limbs = [(v >> (16 * j)) & 0xFFFF for v in (tot, nz) for j in range(LIMBS)]
    buf[tw + COUNTER_SLOTS:tw + COUNTER_SLOTS + STAT_SLOTS].copy_(torch.tensor(limbs, dtype=torch.int32))
    dist.all_reduce(buf[tw:tw + COUNTER_SLOTS + STAT_SLOTS], op=dist.ReduceOp.SUM, group=group)
