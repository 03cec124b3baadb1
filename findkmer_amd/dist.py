"""Multi-GPU orchestration of one sharded stream.

One process per GPU.  Each rank owns a contiguous byte range of the stream
(plus up to 256 bytes of halo before it) and counts it with guessed entry
states (fk_engine_feed_shard).  The path has exactly two exchange steps:

1. state stitch: all-gather the 96-byte shard summaries (fk_engine_summary:
   for a shard counted in one pass, a compact summary valid for entering
   states equivalent to the shard's guessed entry; else the full transfer
   function) and compose them in rank order (fk_summary_apply) -> the exact
   entering state, handed to fk_engine_resolve, which recounts only what the
   guess got wrong (nothing, when the compact summaries applied).  If one
   does not apply, all ranks exchange the full summaries in a second round;
2. table merge: one reduce of the 4^k count tables to rank 0 (the rank that
   writes the outputs).  Counts are u32 in the reference (findKmer.cpp:110);
   int32 sums are bitwise identical.

The same functions run over RCCL (backend "nccl", device tensors, bench.py)
and over gloo on the CPU (tests/test_dist_cpu.py).
"""
import torch
import torch.distributed as dist

from . import FK_E_SUMMARY, FindKmerError, FkState, FkSummary, summary_apply

SUMMARY_WORDS = 12
_U64 = 1 << 64


def _to_i64(v):
    return v - _U64 if v >= 1 << 63 else v


def stitch_entry_state(summary_words, group=None, device=None):
    """All-gather every rank's shard summary (12 u64 words) and compose them
    in rank order from the stream's initial state.  Returns the exact
    entering state (FkState) of this rank's shard, or None when some rank's
    compact summary does not apply to the state entering it (its shard's
    guessed entry would count differently): then every rank sees the same
    failure and the caller exchanges the full summaries instead."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    mine = torch.tensor([_to_i64(int(w)) for w in summary_words], dtype=torch.int64, device=device)
    # one gather into one tensor and one copy to the host (not one
    # synchronising copy per rank: at 1 GB per GPU a step is ~0.2 ms)
    everyone = torch.empty(world * SUMMARY_WORDS, dtype=torch.int64, device=mine.device)
    dist.all_gather_into_tensor(everyone, mine, group=group)
    words = everyone.tolist()
    state = FkState()
    entering = None
    for r in range(world):
        if r == rank:
            entering = state
        s = FkSummary()
        for i, v in enumerate(words[r * SUMMARY_WORDS:(r + 1) * SUMMARY_WORDS]):
            s.w[i] = v % _U64
        try:
            state = summary_apply(s, state)
        except FindKmerError as err:
            if err.code != FK_E_SUMMARY:
                raise
            return None
    return entering


def sum_tables(table, group=None, everywhere=False):
    """Sum the ranks' count tables (int32 tensor = u32 counts) into rank 0's
    `table` (the rank that writes the CSV): one reduce, half the bytes of an
    all-reduce over the xGMI ring (16 MiB per GPU at k=11).  everywhere=True:
    all-reduce, every rank gets the sum."""
    if everywhere:
        dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.reduce(table, dst=0, op=dist.ReduceOp.SUM, group=group)
    return table


def count_sharded(engine, ptr, nbytes, halo, table, group=None, times=None):
    """One sharded pass on this rank's GPU: count the shard, stitch the entry
    state, recount what the guess got wrong, and merge the tables into
    `table` (int32 tensor of 4^k entries = u32 counts, the sum on rank 0
    afterwards; on the GPU for RCCL, on the host for a gloo rehearsal).  The
    engine keeps its own shard's table and counters: finish() reports this
    shard's windows and bases (additive across ranks); distinct k-mers and
    the CSV come from the merged table."""
    import time
    t0 = time.perf_counter()
    engine.feed_shard_device(ptr, nbytes, halo)
    t1 = time.perf_counter()
    state = stitch_entry_state(list(engine.summary().w), group, table.device)
    if state is None:
        # a compact summary did not apply somewhere: the full transfer
        # functions (every rank takes this branch together)
        state = stitch_entry_state(list(engine.summary_full().w), group, table.device)
    engine.resolve(state)
    t2 = time.perf_counter()
    if table.is_cuda:
        engine.table_to_device(table.data_ptr())
    else:
        dev = torch.empty(table.numel(), dtype=torch.int32, device="cuda")
        engine.table_to_device(dev.data_ptr())
        table.copy_(dev.cpu())
    out = sum_tables(table, group)
    if times is not None:
        # host wall time per phase: count (the feed returns when the shard's
        # kernels are done), stitch + resolve, table merge (enqueued)
        times["count"] = times.get("count", 0.0) + (t1 - t0)
        times["stitch"] = times.get("stitch", 0.0) + (t2 - t1)
        times["merge"] = times.get("merge", 0.0) + (time.perf_counter() - t2)
    return out
