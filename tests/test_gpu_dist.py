"""Sharded multi-process path on the GPU box, two, three or eight ranks sharing
cuda:0 with host-side (gloo) collectives: the real engine's feed_shard /
summary / resolve and findkmer_amd/dist.py's stitch, end-flag exchange and
table + counter merge.  (RCCL itself needs one GPU per rank: the driver's
multi-GPU bench covers it.)"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(nproc, port, script, args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), script] + args
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.gpu
@pytest.mark.parametrize("k,fasta,chrom", [(6, 0, 1_500_000_000), (11, 80, 1_500_000_000), (6, 0, 20_000_000),
                                           (7, 0, 12_799_900)])
def test_two_rank_shards_gloo(k, fasta, chrom):
    """bench.py under torchrun: chrom < 25.6M puts an 'N' run break inside
    rank 1's shard (20M), or in its 256-byte halo (12_799_900: 100 bases
    before the shard); bench.py asserts the merged windows and bases"""
    out = _torchrun(2, 29600 + k + chrom % 97, os.path.join(REPO, "bench.py"),
                    ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "gloo",
                     "--north-star-bases", "0",
                     "--k", str(k), "--fasta-line", str(fasta), "--bases", "25600000", "--chrom", str(chrom),
                     "--weak-bases", "0"])
    assert out["n_gpus"] == 2 and out["value"] > 0
    # pure ACGT shards with a halo that fixes the state: one all-reduce
    assert out["exchange"] == ("fast" if k <= 7 else "stitched")


@pytest.mark.gpu
@pytest.mark.parametrize("k,fasta", [(6, 0), (11, 80)])
def test_eight_rank_shards_gloo(k, fasta):
    """The world size of the driver's 8-GPU bench, rehearsed with eight
    ranks on cuda:0 over gloo: bench.py's shard layout (halos; pure ACGT:
    'N' chromosome breaks at 40M and 80M bases, inside ranks 3 and 6), the
    merged counts bench.py asserts, and both exchanges"""
    out = _torchrun(8, 29650 + k, os.path.join(REPO, "bench.py"),
                    ["--gpus", "8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "gloo",
                     "--north-star-bases", "0",
                     "--k", str(k), "--fasta-line", str(fasta), "--bases", "102400000", "--chrom", "40000000",
                     "--weak-bases", "0"])
    assert out["n_gpus"] == 8 and out["value"] > 0
    assert out["exchange"] in (("fast", "stitched") if k <= 7 else ("stitched",))


@pytest.mark.gpu
def test_bench_gpus_flag_launches_the_ranks():
    """`python bench.py --gpus 2` with no launcher (the driver's form): the
    bench starts torch.distributed.run itself as a child process, two ranks
    count the two halves of one stream (strong scaling), and the merged-count
    guard holds; the weak sub-record gives each rank a whole shard"""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--north-star-bases", "0",
           "--k", "11", "--fasta-line", "80", "--bases", "25600000", "--weak-bases", "12800000",
           "--chrom", "20000000"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["value"] > 0
    assert out["config"]["total_bases"] == 25_600_000 and out["config"]["bases_per_gpu"] == 12_800_000
    assert out["exchange"] == "stitched"
    w = out["weak_scaling"]
    assert w["scaling"] == "weak" and w["bases_per_gpu"] == 12_800_000 and w["value"] > 0


@pytest.mark.gpu
def test_configs3_eight_ranks_full_size():
    """BASELINE.json configs[3] at its size: k=11 over one 10 G-base genome
    (80-column FASTA, 1.5-Gbase chromosomes) cut into 8 shards of 1.25 G
    bases, eight ranks (gloo, all on cuda:0) through bench.py's sharded pass;
    rank 0 then counts the whole stream with one engine (--verify-single) and
    the merged table and every counter must equal it"""
    out = _torchrun(8, 29690, os.path.join(REPO, "bench.py"),
                    ["--gpus", "8", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dist-backend", "gloo",
                     "--north-star-bases", "0", "--k", "11", "--fasta-line", "80", "--bases", "10000000000",
                     "--weak-bases", "0", "--verify-single"])
    assert out["n_gpus"] == 8 and out["exchange"] == "stitched"
    assert out["scaling"] == "strong" and out["config"]["total_bases"] == 10_000_000_000
    assert out["config"]["bases_per_gpu"] == 1_250_000_000
    v = out["verify"]
    assert v["table_equal"] and v["status"] == 0
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert v[key][0] == v[key][1], (key, v[key])
    import bench
    assert v["windows"][0] == bench.expected_windows(10_000_000_000, 11, bench.CHROM)


@pytest.mark.gpu
@pytest.mark.parametrize("k,world,eof_in", [(6, 8, 5), (11, 8, -1), (6, 3, 1), (11, 3, 1), (11, 2, 0), (13, 3, 1)])
def test_sharded_mixed_input_against_oracle(k, world, eof_in):
    """headers, N runs, unknown bytes, ragged lines; eof_in >= 0: a 0xFF
    byte ends the stream inside that rank's shard, and the later ranks'
    counts must not reach the merged table"""
    out = _torchrun(world, 29700 + 7 * k + world + eof_in, os.path.join(REPO, "tests", "dist_worker.py"),
                    ["--k", str(k), "--eof-in", str(eof_in)])
    assert out["table_equal"]
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert out[key][0] == out[key][1], (key, out[key])
    assert not out["rollover"]
    assert out["first_end"] == (eof_in if eof_in >= 0 else None)
    if eof_in >= 0 or k > 7:
        assert out["path"] == "stitched"   # a 0xFF shard / k_part shards are never packed


@pytest.mark.gpu
@pytest.mark.parametrize("k,fast,eof_in,native", [(6, 1, -1, 1), (6, 1, -1, 0), (11, 1, 0, 1)])
def test_rccl_single_rank_merge(k, fast, eof_in, native):
    """The RCCL code path on a one-GPU box (world 1, backend nccl): the pack
    into the device merge buffer, the engine-stream -> collective ordering,
    the all-reduce and the pinned rows; a 0xFF (eof_in 0) or k >= 8 takes
    the stitched exchange over RCCL instead"""
    out = _torchrun(1, 29800 + 3 * k + fast + eof_in + 5 * native, os.path.join(REPO, "tests", "dist_worker.py"),
                    ["--k", str(k), "--backend", "nccl", "--fast", str(fast), "--eof-in", str(eof_in),
                     "--input", "fasta", "--native", str(native)])
    assert out["table_equal"]
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert out[key][0] == out[key][1], (key, out[key])
    assert out["path"] == ("fast" if fast and k <= 7 and eof_in < 0 else "stitched")
    # the library's own RCCL communicator on the engine's stream (both paths)
    assert out["transport"] == ("rccl-native" if native else "torch")
    if eof_in >= 0:
        assert out["first_end"] == eof_in


@pytest.mark.gpu
@pytest.mark.parametrize("k,world,eof_in,nbytes,route", [(12, 2, -1, 3_000_000, 0), (12, 8, 3, 3_000_000, 0),
                                                        (14, 8, -1, 3_000_000, 0), (15, 3, 1, 1_500_000, 1),
                                                        (16, 2, -1, 1_500_000, 1)])
def test_sharded_table_gloo_against_oracle(k, world, eof_in, nbytes, route, monkeypatch):
    """k > 11: the merged table sharded over the ranks by its top index bits
    (rank r owns bins [r*4^k/G, (r+1)*4^k/G): the north star's "table shards
    by top bits"), gathered in rank order on rank 0 == the oracle's table
    (k = 14, 16: its sparse form); the counters, total and distinct bins
    from the all-reduced limbs.  k = 14 over 8 ranks: k_bucket16's fresh
    tables reduced.  route = 1 (k = 15, 16; FINDKMER_TUNE route=1): the
    routed exchange end to end (fk_engine_route_pack, all_to_all_single,
    fk_engine_route_absorb with its trailer check) instead of the table
    reduction.  eof_in >= 0 at k = 15: the shards after the 0xFF byte were
    counted into fresh tables and are then discarded (the statistics that
    count left must not reach finish)"""
    if route:
        monkeypatch.setenv("FINDKMER_TUNE", f"route={route}")
    out = _torchrun(world, 29750 + k + world + eof_in, os.path.join(REPO, "tests", "dist_worker.py"),
                    ["--k", str(k), "--eof-in", str(eof_in), "--shard-table", "1", "--bytes", str(nbytes)])
    assert out["table_equal"] and out["sharded"]
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert out[key][0] == out[key][1], (key, out[key])
    assert not out["rollover"]
    assert out["first_end"] == (eof_in if eof_in >= 0 else None)


@pytest.mark.gpu
@pytest.mark.parametrize("k,shard,invalid", [(12, 1, 0), (6, 0, 1), (11, 1, 0), (15, 1, 0)])
def test_rccl_single_rank_sharded_and_fallback(k, shard, invalid, monkeypatch):
    """The native RCCL exchange (world 1): the reduce-scatter of the table
    with the slice statistics' all-reduce, and (invalid) a pack row forced
    invalid after the one-collective all-reduce, so that the fallback runs
    the stitched exchange over the merge buffer that collective already
    changed.  k = 15: the routed table (fk_engine_route_*: the
    nonzero bins packed per owner, one grouped ncclSend/ncclRecv, counted
    into the slice) instead of the reduce-scatter (FINDKMER_TUNE route=2: at
    world 1 too)"""
    if k >= 15:
        monkeypatch.setenv("FINDKMER_TUNE", "route=2")
    out = _torchrun(1, 29850 + 3 * k + shard + 7 * invalid, os.path.join(REPO, "tests", "dist_worker.py"),
                    ["--k", str(k), "--backend", "nccl", "--input", "fasta", "--shard-table", str(shard),
                     "--test-invalid", str(invalid)])
    assert out["table_equal"] and out["transport"] == "rccl-native"
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert out[key][0] == out[key][1], (key, out[key])
    assert out["path"] == "stitched"
    assert out["sharded"] == bool(shard)


@pytest.mark.gpu
@pytest.mark.parametrize("k,world,eof_in,backend", [(17, 8, 3, "gloo"), (20, 3, -1, "gloo"),
                                                    (18, 8, -1, "gloo"), (17, 1, -1, "nccl"), (20, 1, 0, "nccl")])
def test_sparse_tables_all_to_all_against_oracle(k, world, eof_in, backend):
    """17 <= k <= 20 over several ranks: each rank's sparse table (key-range
    passes over its shard, counted from the stitched exact state) cut at the
    owners' bounds, one all-to-all to the owners, the owner's sum on the GPU
    (fk_engine_sparse_adopt); the owners' slices gathered in rank order ==
    the oracle's sparse table, every merged counter exact.  nccl: world 1
    over RCCL through the library's communicator (fk_engine_sparse_exchange:
    the run counts, keys and counts by grouped send/recv, the merge, the
    counter all-reduce, on the engine's stream)"""
    out = _torchrun(world, 29900 + k + 3 * world + eof_in + (50 if backend == "nccl" else 0),
                    os.path.join(REPO, "tests", "dist_worker.py"),
                    ["--k", str(k), "--eof-in", str(eof_in), "--bytes", "2000000", "--backend", backend])
    assert out["table_equal"] and out["sharded"]
    assert out["transport"] == ("rccl-native" if backend == "nccl" else "torch")
    for key in ("windows", "valid_bases", "base_count", "depth1", "unknown_chars", "scanned_bytes",
                "hit_eof_byte", "unterminated_header", "distinct"):
        assert out[key][0] == out[key][1], (key, out[key])
    assert not out["rollover"]
    assert out["first_end"] == (eof_in if eof_in >= 0 else None)


@pytest.mark.gpu
@pytest.mark.parametrize("k,fasta", [(12, 80)])
def test_rccl_single_rank_bench_line_reports_the_world(k, fasta):
    """bench.py over RCCL (world 1, backend nccl, the library's communicator):
    the line carries what RCCL itself reports -- its rank count, every
    rank's rank and device (fk_comm_info: ncclCommCount / ncclCommUserRank /
    ncclCommCuDevice) -- with the exchange path, transport and per-phase
    host milliseconds, so that the driver's 8-GPU line proves its own world"""
    out = _torchrun(1, 29960 + k, os.path.join(REPO, "bench.py"),
                    ["--gpus", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "nccl",
                     "--north-star-bases", "0", "--k", str(k), "--fasta-line", str(fasta), "--bases", "64000000"])
    assert out["n_gpus"] == 1 and out["transport"] == "rccl-native"
    assert out["rccl"] == {"nranks": 1, "ranks": [0], "devices": [0], "local_ranks": [0]}
    assert out["exchange"] == ("fast" if k <= 7 else "stitched")
    assert set(out["phase_ms_per_step"]) >= {"exchange", "finish"}
    assert all(v >= 0 for v in out["phase_ms_per_step"].values())


@pytest.mark.gpu
@pytest.mark.parametrize("k,world", [(15, 3), (16, 2)])
def test_routed_table_blobs_against_the_summed_tables(k, world):
    """fk_engine_route_pack / _absorb in one process: `world` engines over
    different inputs pack their finished tables for `world` owners, each
    owner's blobs from every source are absorbed into its slice, and the
    slices side by side == the sum of the engines' tables.  world 3 puts
    owner boundaries inside 2^15-bin parts; a 300 K-base poly-A stretch
    gives one bin a count past the 2^17 - 1 an entry holds (the overflow
    pairs); the last source packs as a rank the stream never reached
    (counting = 0: empty blobs) and must not count."""
    import numpy as np
    import torch

    import findkmer_amd as fk
    from test_gpu_parity import mixed_input
    dev = torch.device("cuda", 0)
    nb = 1 << (2 * k)
    tw = (nb + world - 1) // world * world
    S = tw // world
    inputs = [b"A" * 300_000 + mixed_input(7 + k, 400_000), mixed_input(8 + k, 900_000)]
    inputs += [mixed_input(9 + k + s, 300_000) for s in range(world - len(inputs))]
    engines, blobs, words, want = [], [], [], torch.zeros(nb, dtype=torch.int32, device=dev)
    try:
        for s, data in enumerate(inputs[:world]):
            e = fk.Engine(k)
            engines.append(e)
            e.feed(np.frombuffer(data, dtype=np.uint8).copy())
            e.finish(allow=(fk.FK_OK, fk.FK_E_UNTERMINATED_HEADER))
            counting = s < world - 1 or world == 2
            w = e.route_pack(world, counting)
            b = torch.empty(max(1, sum(w)), dtype=torch.int32, device=dev)
            e.route_copy(b.data_ptr())
            blobs.append(b)
            words.append(w)
            if counting:
                t = torch.empty(nb, dtype=torch.int32, device=dev)
                e.table_to_device(t.data_ptr())
                want += t
                del t
        assert words[0][0] > 4 + (S >> 15)   # entries were packed
        got = torch.empty(tw, dtype=torch.int32, device=dev)
        for r in range(world):
            parts, rw = [], []
            for s in range(world):
                off = sum(words[s][:r])
                parts.append(blobs[s][off:off + words[s][r]])
                rw.append(words[s][r])
            recv = torch.cat(parts)
            engines[r].route_absorb(world, r, recv.data_ptr(), rw, got[r * S:].data_ptr())
        assert torch.equal(got[:nb], want)
        assert int(want.max()) >= (1 << 17)   # an overflow pair was needed
        # a blob that arrives short (its trailer cleared, as the exchange
        # clears the receive buffer's) or with one word changed is refused
        for damage in ("short", "word"):
            parts, rw = [], []
            for s in range(world):
                off = sum(words[s][:0])
                parts.append(blobs[s][off:off + words[s][0]].clone())
                rw.append(words[s][0])
            if damage == "short":
                parts[0][-2:] = 0
            else:
                parts[0][4 + (S >> 15) // 2] += 1
            recv = torch.cat(parts)
            with pytest.raises(fk.FindKmerError) as ei:
                engines[0].route_absorb(world, 0, recv.data_ptr(), rw, got.data_ptr())
            assert ei.value.code == fk.FK_E_RCCL, damage
    finally:
        for e in engines:
            e.close()
