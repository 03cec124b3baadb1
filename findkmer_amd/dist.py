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

The same functions run over RCCL (backend "nccl", device tensors, bench.py)
and over gloo on the CPU (tests/test_dist_cpu.py, with a model engine).
"""
import torch
import torch.distributed as dist

from . import FK_E_EMPTY, FK_E_ROLLOVER, FK_E_SUMMARY, FK_E_UNTERMINATED_HEADER, FK_OK
from . import FindKmerError, FkState, FkSummary, summary_apply, summary_is_full

SUMMARY_WORDS = 12
GATHER_WORDS = SUMMARY_WORDS + 1      # + "my summary is full" flag
_U64 = 1 << 64

# scalar counters merged with the table (u64 each, 4 x 16-bit limbs)
COUNTERS = ("windows", "valid_bases", "base0", "base1", "base2", "base3",
            "depth1_0", "depth1_1", "depth1_2", "depth1_3", "unknown_chars",
            "scanned_bytes", "ended", "unterminated_header")
LIMBS = 4
COUNTER_SLOTS = len(COUNTERS) * LIMBS


def _to_i64(v):
    return v - _U64 if v >= 1 << 63 else v


def merge_buffer(k, device):
    """The int32 buffer count_sharded reduces: the 4^k table, then the
    counter limbs."""
    return torch.zeros((1 << (2 * k)) + COUNTER_SLOTS, dtype=torch.int32, device=device)


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


class ShardedResult:
    """The merged result of one sharded pass.  Complete on rank 0 (the reduce
    destination); other ranks hold only their own contribution.  Counter
    fields mirror fk_result (include/findkmer.h); they are decoded from the
    reduced buffer on first access (one device-to-host copy)."""

    def __init__(self, buf, k, rank, first_end, local=None):
        self.local = local          # this rank's own fk_result (timings)
        self.buf = buf
        self.k = k
        self.rank = rank
        self.first_end = first_end
        nb = 1 << (2 * k)
        self.table = buf[:nb]
        self._vals = None
        if rank == 0:
            # on the device, enqueued behind the reduce (no host wait here):
            # the merged table's u64 total (int32 sum + 2^32 per negative
            # bin) and its distinct k-mers
            t = self.table
            self._tsum = t.sum(dtype=torch.int64) + (t < 0).sum(dtype=torch.int64) * (1 << 32)
            self._distinct = (t != 0).sum(dtype=torch.int64)

    def _decode(self):
        if self._vals is None:
            limbs = self.buf[-COUNTER_SLOTS:].tolist()
            vals = {}
            for i, name in enumerate(COUNTERS):
                v = 0
                for j in range(LIMBS):
                    v += int(limbs[i * LIMBS + j]) << (16 * j)
                vals[name] = v % _U64
            self._vals = vals
        return self._vals

    def __getattr__(self, name):
        if name.startswith("_") or name in ("buf", "k", "rank", "first_end", "table", "local"):
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
        assert self.rank == 0, "the merged table lives on rank 0"
        return int(self._distinct.item())

    @property
    def rollover(self):
        """The reference's COUNTER ROLLOVER exit (:642-648): a merged bin or
        a depth-1 trie counter reached 2^32."""
        assert self.rank == 0, "the merged table lives on rank 0"
        v = self._decode()
        if int(self._tsum.item()) != v["windows"]:
            return True
        return any(v[f"depth1_{b}"] >= 1 << 32 for b in range(4))

    def status(self):
        """fk_engine_finish's status for the whole stream (rank 0)."""
        if self.rollover:
            return FK_E_ROLLOVER
        if self.unterminated_header:
            return FK_E_UNTERMINATED_HEADER
        return FK_OK


def _put_counters(buf, values, pinned):
    """Write the u64 counters into the buffer's limb slots (host -> buffer)."""
    limbs = []
    for v in values:
        v = int(v) % _U64
        limbs.extend((v >> (16 * j)) & 0xFFFF for j in range(LIMBS))
    if pinned is not None:
        pinned.copy_(torch.tensor(limbs, dtype=torch.int32))
        buf[-COUNTER_SLOTS:].copy_(pinned, non_blocking=True)
    else:
        buf[-COUNTER_SLOTS:].copy_(torch.tensor(limbs, dtype=torch.int32))


def count_sharded(engine, ptr, nbytes, halo, buf, group=None, times=None, pinned=None):
    """One sharded pass on this rank's GPU: count the shard, stitch the entry
    state, recount what the guess got wrong, and merge the tables and
    counters into `buf` (merge_buffer(k, device): on the GPU for RCCL, on the
    host for a gloo rehearsal; the sum lands on rank 0).  Returns a
    ShardedResult.  `pinned` (optional): a pinned host int32 tensor of
    COUNTER_SLOTS entries for an asynchronous counter upload.

    `engine` is a findkmer_amd.Engine (or, in the CPU tests, a model with the
    same feed_shard_device / summary / summary_full / resolve / finish /
    table_to_device methods)."""
    import time
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = buf.device
    t0 = time.perf_counter()
    engine.feed_shard_device(ptr, nbytes, halo)
    t1 = time.perf_counter()
    got = stitch_entry_state(engine.summary(), group, dev)
    if got is None:
        # a compact summary did not apply somewhere: the full transfer
        # functions (every rank takes this branch together)
        got = stitch_entry_state(engine.summary_full(), group, dev, full=True)
    state, first_end, any_full = got
    engine.resolve(state)
    rc, r = engine.finish(allow=(FK_OK, FK_E_ROLLOVER, FK_E_UNTERMINATED_HEADER, FK_E_EMPTY))
    if any_full:
        # where the stream ends is exact only after the resolve: one more
        # small all-gather of the ranks' end flags
        ends = _gather_rows([1 if (r.hit_eof_byte and not state.ended) else 0], group, dev)
        first_end = next((i for i, f in enumerate(ends) if f), None)
    t2 = time.perf_counter()
    counting = first_end is None or rank <= first_end
    last = first_end if first_end is not None else world - 1
    nb = 1 << (2 * engine.k)
    if counting:
        if buf.is_cuda:
            engine.table_to_device(buf.data_ptr())
        else:
            buf[:nb].copy_(torch.from_numpy(engine.table().view("int32")))
        vals = [r.windows, r.valid_bases, *r.base_count, *r.depth1, r.unknown_chars, r.scanned_bytes,
                1 if rank == first_end else 0,
                r.unterminated_header if rank == last else 0]
    else:
        buf[:nb].zero_()
        vals = [0] * len(COUNTERS)
    _put_counters(buf, vals, pinned)
    sum_tables(buf, group)
    if times is not None:
        # host wall time per phase: count (the feed returns when the shard's
        # kernels are done), stitch + resolve, table merge (enqueued)
        times["count"] = times.get("count", 0.0) + (t1 - t0)
        times["stitch"] = times.get("stitch", 0.0) + (t2 - t1)
        times["merge"] = times.get("merge", 0.0) + (time.perf_counter() - t2)
    return ShardedResult(buf, engine.k, rank, first_end, r)
