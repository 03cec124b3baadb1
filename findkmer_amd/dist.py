"""Multi-GPU orchestration of one sharded stream.

One process per GPU.  Each rank owns a contiguous byte range of the stream
(plus up to 256 bytes of halo before it) and counts it with guessed entry
states (fk_engine_feed_shard).  The path has exactly two exchange steps:

1. state stitch: all-gather the 96-byte shard summaries (the shard's scan
   transfer function, fk_engine_summary) and compose those of the ranks
   before this one (fk_summary_apply) -> the exact entering state, handed to
   fk_engine_resolve, which recounts only what the guess got wrong;
2. table merge: one all-reduce of the 4^k count tables.  Counts are u32 in
   the reference (findKmer.cpp:110); int32 sums are bitwise identical.

The same functions run over RCCL (backend "nccl", device tensors, bench.py)
and over gloo on the CPU (tests/test_dist_cpu.py).
"""
import torch
import torch.distributed as dist

from . import FkState, FkSummary, summary_apply

SUMMARY_WORDS = 12
_U64 = 1 << 64


def _to_i64(v):
    return v - _U64 if v >= 1 << 63 else v


def stitch_entry_state(summary_words, group=None, device=None):
    """All-gather every rank's shard summary (12 u64 words) and compose the
    summaries of the ranks before this one, starting from the stream's
    initial state.  Returns the exact entering state (FkState) of this rank's
    shard."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    mine = torch.tensor([_to_i64(int(w)) for w in summary_words], dtype=torch.int64, device=device)
    everyone = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(everyone, mine, group=group)
    state = FkState()
    for r in range(rank):
        s = FkSummary()
        for i, v in enumerate(everyone[r].tolist()):
            s.w[i] = v % _U64
        state = summary_apply(s, state)
    return state


def sum_tables(table, group=None):
    """Sum the ranks' count tables in place (int32 tensor = u32 counts)."""
    dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)
    return table


def count_sharded(engine, ptr, nbytes, halo, table, group=None):
    """One sharded pass on this rank's GPU: count the shard, stitch the entry
    state, recount what the guess got wrong, and merge the tables into
    `table` (int32 tensor of 4^k entries = u32 counts, identical on every rank
    afterwards; on the GPU for RCCL, on the host for a gloo rehearsal).  The
    engine keeps its own shard's table and counters: finish() reports this
    shard's windows and bases (additive across ranks); distinct k-mers and
    the CSV come from the merged table."""
    engine.feed_shard_device(ptr, nbytes, halo)
    state = stitch_entry_state(list(engine.summary().w), group, table.device)
    engine.resolve(state)
    if table.is_cuda:
        engine.table_to_device(table.data_ptr())
    else:
        dev = torch.empty(table.numel(), dtype=torch.int32, device="cuda")
        engine.table_to_device(dev.data_ptr())
        table.copy_(dev.cpu())
    return sum_tables(table, group)
