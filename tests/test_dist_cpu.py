"""Multi-process shard stitching on the CPU (world_size 2 and 3, gloo).

Runs the real orchestration of findkmer_amd/dist.py (all-gather of shard
summaries, composition with the C-ABI fk_summary_apply, all-reduce of the
tables) with tests/scan_model.py standing in for the GPU engine.  Checks the
stitched entering state of every shard against a direct scan of the prefix,
and the merged table against the oracle on the whole input.
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


def _worker(rank, world, port, data, bounds, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import findkmer_amd.dist as fkdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bounds[rank], bounds[rank + 1]
        shard = data[lo:hi]
        state = fkdist.stitch_entry_state(scan_model.summary_words(shard))
        # the stitched state is the state a direct scan of the prefix reaches
        hdr, R, code, _, _ = scan_model.advance(data[:lo], 0, 0, 0)
        assert state.hdr == hdr and state.run == R, (rank, state.hdr, hdr, state.run, R)
        if not hdr:
            nb = min(R, 32)
            m = (1 << (2 * nb)) - 1
            assert (state.code & m) == (scan_model.sigma(code) & m)
        table = torch.zeros(1 << (2 * K), dtype=torch.int32)
        t = table.numpy()
        scan_model.count_from(shard, K, state.hdr, state.run, scan_model.sigma(state.code), t)
        fkdist.sum_tables(table)
        if rank == 0:
            results.put(table.numpy().astype(np.uint32).tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_stitch_and_merge_gloo(world):
    import torch.multiprocessing as mp
    data = _input(world, 24000)
    n = len(data)
    bounds = [0] + [n * i // world // 16 * 16 for i in range(1, world)] + [n]
    ctx = mp.get_context("spawn")
    results = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), data, bounds, results), nprocs=world,
                       join=True, start_method="spawn")
    merged = np.frombuffer(results.get(), dtype=np.uint32)
    want, res, _ = oracle.count_dense(data, K)
    assert np.array_equal(merged, want)
    assert int(merged.sum()) == res.windows
