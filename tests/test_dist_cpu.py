"""Multi-process shard stitching on the CPU (world_size 2, 3 and 8, gloo).

Runs the real orchestration of findkmer_amd/dist.py (all-gather of shard
summaries, composition with the C-ABI fk_summary_apply, the end-flag
exchange, the reduce of tables + counter limbs) with
tests/scan_model.ModelEngine standing in for the GPU engine.  Checks the
stitched entering state of every shard against a direct scan of the prefix,
and the merged table and counters against the oracle on the whole input --
including inputs whose stream ends at a 0xFF byte in a middle shard (the
reference's signed-char EOF, findKmer.cpp:988).
"""
import os
import random
import socket

import numpy as np
import pytest

import oracle
import scan_model

K = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _input(seed, n):
    """headers, N runs, unknown bytes, newlines of several widths; no 0xFF"""
    rng = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        r = rng.random()
        if r < 0.6:
            seq = bytes(rng.choices(b"ACGT", k=rng.randint(1, 900)))
            w = rng.choice([0, 60, 7])
            if w:
                seq = b"\n".join(seq[i:i + w] for i in range(0, len(seq), w))
            out += seq
        elif r < 0.75:
            out += b">" + bytes(rng.choices(b"ACGTN xyz", k=rng.randint(0, 120))) + b"\n"
        elif r < 0.85:
            out += b"N" * rng.randint(1, 40)
        elif r < 0.9:
            out += bytes(rng.choices(b"acgtRY*", k=rng.randint(1, 5)))
        else:
            out += b"\n"
    return bytes(out[:n])


def _worker(rank, world, port, data, bounds, mode, results, shard=False, sparse=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import findkmer_amd.dist as fkdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bounds[rank], bounds[rank + 1]
        shard_table = shard
        shard = data[lo:hi]
        hdr, R, code, _, _ = scan_model.advance(data[:lo], 0, 0, 0)
        if mode == "state":
            # the stitched state is the state a direct scan of the prefix reaches
            state, _, _ = fkdist.stitch_entry_state(scan_model.summary_words(shard), full=True)
            assert state.hdr == hdr and state.run == R, (rank, state.hdr, hdr, state.run, R)
            if not hdr:
                nb = min(R, 32)
                m = (1 << (2 * nb)) - 1
                assert (state.code & m) == (scan_model.sigma(code) & m)
            return
        guess = None
        if mode == "compact":
            guess = (hdr, R, code)                 # every guess right: no full round
        elif mode == "compact_miss" and rank == 1:
            guess = (1 - hdr, 0, 0)                # rank 1 guessed wrong: full summaries
        elif mode == "compact_miss":
            guess = (hdr, R, code)
        if sparse:
            # the sparse tables' all-to-all merge (17 <= k <= 20 on the GPU)
            eng = scan_model.SparseModelEngine(K, shard, guess)
            res = fkdist.count_sharded(eng, 0, len(shard), 0, None)
            got = res.table_full()
            S = ((1 << (2 * K)) + world - 1) // world
            assert res.lo == min(rank * S, 1 << (2 * K)) and res.hi == min((rank + 1) * S, 1 << (2 * K))
            assert all(res.lo <= int(x) < res.hi for x in res.keys), "a key outside the owner's range"
            full = None
            if rank == 0:
                full = np.zeros(1 << (2 * K), dtype=np.uint32)
                full[got[0].astype(np.int64)] = got[1]
                full = __import__("torch").from_numpy(full.view(np.int32))
        else:
            eng = scan_model.ModelEngine(K, shard, guess)
            buf = fkdist.merge_buffer(K, "cpu")
            res = fkdist.count_sharded(eng, 0, len(shard), 0, buf, shard_table=bool(shard_table))
            full = res.table_full()   # a collective when the table is sharded
        if res.sharded and not sparse:
            # this rank's slice: the first bases' range [lo, hi) of the table
            want_lo = min(rank * (fkdist.table_words(K, world) // world), 1 << (2 * K))
            assert res.lo == want_lo and res.table.numel() == res.hi - res.lo
            assert np.array_equal(res.table.numpy(), buf[res.lo:res.hi].numpy())
        if rank == 0:
            out = {n: getattr(res, n) for n in ("windows", "valid_bases", "base_count", "depth1",
                                                 "unknown_chars", "scanned_bytes", "hit_eof_byte",
                                                 "unterminated_header", "distinct", "rollover")}
            out["first_end"] = res.first_end
            out["path"] = res.path
            out["sharded"] = res.sharded
            results.put((full.numpy().astype(np.uint32).tobytes(), out))
    finally:
        dist.destroy_process_group()


def _run(world, data, bounds, mode, shard=False, sparse=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    results = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), data, bounds, mode, results, shard, sparse),
                       nprocs=world, join=True, start_method="spawn")
    return None if mode == "state" else results.get()


def _bounds(n, world):
    return [0] + [n * i // world // 16 * 16 for i in range(1, world)] + [n]


@pytest.mark.parametrize("world", [2, 3])
def test_stitched_states_gloo(world):
    data = _input(world, 24000)
    _run(world, data, _bounds(len(data), world), "state")


def _check(data, world, mode, bounds=None, shard=False, sparse=False):
    bounds = bounds or _bounds(len(data), world)
    table, got = _run(world, data, bounds, mode, shard, sparse)
    want, r, _ = oracle.count_dense(data, K)
    assert np.array_equal(np.frombuffer(table, dtype=np.uint32), want)
    assert got["windows"] == r.windows
    assert got["valid_bases"] == r.valid_bases
    assert got["base_count"] == list(r.base_count)
    assert got["depth1"] == list(r.depth1)
    assert got["unknown_chars"] == r.unknown_chars
    assert got["scanned_bytes"] == r.scanned_bytes
    assert got["hit_eof_byte"] == r.hit_eof_byte
    assert got["unterminated_header"] == r.unterminated_header
    assert got["distinct"] == r.distinct
    assert not got["rollover"]
    return got


@pytest.mark.parametrize("world,mode", [(2, "full"), (3, "full"), (3, "compact"), (3, "compact_miss"),
                                        (8, "full"), (8, "compact"), (8, "compact_miss")])
def test_merge_gloo(world, mode):
    got = _check(_input(world + 7, 24000), world, mode)
    assert got["first_end"] is None
    # every guess right: one all-reduce; a wrong guess or full summaries:
    # the stitched exchange
    assert got["path"] == ("fast" if mode == "compact" else "stitched")


@pytest.mark.parametrize("mode", ["full", "compact", "compact_miss"])
def test_eof_byte_in_middle_shard_gloo(mode):
    """A 0xFF outside a header in rank 1's shard ends the stream there:
    rank 2 (and rank 1's bytes after it) must count nothing."""
    data = bytearray(_input(11, 24000))
    n = len(data)
    b = _bounds(n, 3)
    # a 0xFF in the middle of rank 1's shard, outside any header
    at = (b[1] + b[2]) // 2
    data[at - 2:at + 1] = b"\nA\xff"
    data = bytes(data)
    _, r, _ = oracle.count_dense(data, K)
    assert r.hit_eof_byte and r.scanned_bytes == at
    got = _check(data, 3, mode, b)
    assert got["first_end"] == 1


def test_eof_byte_in_header_is_not_the_end_gloo():
    """A 0xFF inside a '>' line is skipped with the header (:999-1005)."""
    data = bytearray(_input(12, 24000))
    b = _bounds(len(data), 3)
    at = (b[1] + b[2]) // 2
    data[at - 3:at + 3] = b"\n>\xff\xffx\n"
    got = _check(bytes(data), 3, "full", b)
    assert got["first_end"] is None and not got["hit_eof_byte"]


def test_merged_rollover_detection():
    """Rank 0's checks on the reduced buffer: a merged bin that wrapped past
    2^32 (table total short of the window count), or a depth-1 counter
    reaching 2^32, is the reference's COUNTER ROLLOVER exit (:642-648)."""
    import torch
    import findkmer_amd as fk
    import findkmer_amd.dist as fkdist

    def result(table_vals, windows, depth1=(0, 0, 0, 0)):
        buf = fkdist.merge_buffer(2, "cpu")
        buf[:16] = torch.tensor(np.array(table_vals, dtype=np.uint32).view(np.int32))
        vals = [windows, 0, 0, 0, 0, 0, *depth1, 0, 0, 0, 0]
        fkdist._put_counters(buf, vals, None, 16)
        return fkdist.ShardedResult(buf, 2, 0, None)

    ok = result([3] * 15 + [0xFFFFFFFF], 45 + 0xFFFFFFFF)
    assert not ok.rollover and ok.status() == fk.FK_OK and ok.distinct == 16
    wrapped = result([3] * 15 + [4], 45 + (1 << 32) + 4)          # bin 15 reached 2^32 + 4
    assert wrapped.rollover and wrapped.status() == fk.FK_E_ROLLOVER
    deep = result([1] * 16, 16, depth1=(1 << 32, 0, 0, 0))
    assert deep.rollover


@pytest.mark.parametrize("world,mode", [(2, "full"), (3, "full"), (8, "compact_miss"), (3, "compact")])
def test_sharded_table_gloo(world, mode):
    """the table sharded over the ranks (reduce-scatter semantics: rank r
    keeps bins [r*S, (r+1)*S), world 3 pads 4^5 to 1026 words): the slices
    gathered in rank order are the oracle's table, and every rank's merged
    counters, total and distinct bins are exact (the one-collective path,
    "compact", leaves every rank the whole table instead)"""
    got = _check(_input(world + 40, 24000), world, mode, shard=True)
    assert got["sharded"] == (mode != "compact")
    assert got["path"] == ("fast" if mode == "compact" else "stitched")


def test_sharded_table_eof_in_middle_gloo():
    data = bytearray(_input(41, 24000))
    b = _bounds(len(data), 3)
    at = (b[1] + b[2]) // 2
    data[at - 2:at + 1] = b"\nA\xff"
    got = _check(bytes(data), 3, "full", b, shard=True)
    assert got["first_end"] == 1 and got["sharded"]


@pytest.mark.parametrize("world,mode", [(2, "full"), (3, "compact_miss"), (8, "full")])
def test_sparse_tables_all_to_all_gloo(world, mode):
    """17 <= k <= 20's merge (dist._sparse_merge): every rank cuts its sparse
    table at the owners' bounds, one all-to-all sends the runs to their
    owners, each owner sums repeated keys; the owners' slices in rank order
    are the oracle's table, the merged counters, total and distinct exact"""
    got = _check(_input(world + 60, 24000), world, mode, sparse=True)
    assert got["sharded"] and got["path"] == "stitched"


def test_sparse_tables_eof_in_middle_gloo():
    data = bytearray(_input(61, 24000))
    b = _bounds(len(data), 3)
    at = (b[1] + b[2]) // 2
    data[at - 2:at + 1] = b"\nA\xff"
    got = _check(bytes(data), 3, "full", b, sparse=True)
    assert got["first_end"] == 1
