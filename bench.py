#!/usr/bin/env python3
"""bench.py — k-mer scan throughput on MI355X (BASELINE.json metric).

Headline workload (BASELINE.json configs[2], the largest single-GPU config):
k=11 over a 10 G-base synthetic genome — 80-column FASTA (one
">synthetic" header, ≈1.0125e10 bytes), an 'N' run break every 1.5 Gbases
(chromosomes), generated in HBM before the timed region.  One step = one pass
of the hot path over the batch: reset, the engine's feed (k_part +
k_bucket_count + k_pair_fold + the statistics kernels for 8 <= k <= 12) and
fk_engine_finish.

The same line carries the north-star gate as a sub-record ("north_star"):
k=6 over a 10 G-base pure-ACGT genome (1.5-Gbase chromosomes), with its own
value, ms_per_step and roofline (k_count).

With --gpus N (one process per GPU, torch.distributed over RCCL; without a
launcher `python bench.py --gpus N` starts torch.distributed.run itself as a
child process) the headline is BASELINE.json configs[3]: the same 10 G-base
genome cut into N shards (strong scaling).  Each shard's entry state is
stitched and the count tables merged inside the library
(findkmer_amd/dist.py, fk_engine_shard_exchange) -- the path's real exchange
steps.  A "weak_scaling" sub-record gives every rank a whole 10 G-base shard
of an N x 10 G-base stream.

Prints ONE JSON line on rank 0 (contract in the task statement): value =
bases/s over all ranks, "roofline" for the dominant kernel (HIP events on the
engine's stream, recorded inside the launch), "cpu_baseline" (the reference
binary on a bounded sample, rank 0 at N=1 only) and "cpu_baseline_multicore"
(the oracle's dense scan over 16 host threads, the "fast CPU" of BASELINE.md).
"""
import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "bases/sec scanned at fixed k; achieved HBM GB/s vs roofline, 1/2/4/8 GPUs"
CHROM = 1_500_000_000    # an 'N' run break every CHROM bases (synthetic chromosomes)
HEADER = 11              # len(">synthetic\n"), fk_synth_device with fasta_line > 0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=11)
    ap.add_argument("--bases", type=int, default=10_000_000_000,
                    help="bases of the headline stream, split over the --gpus ranks (strong scaling)")
    ap.add_argument("--weak-bases", type=int, default=10_000_000_000,
                    help="N > 1 sub-record: this many bases per GPU (weak scaling; 0 = skip)")
    ap.add_argument("--fasta-line", type=int, default=80, help="80 = FASTA (configs[2]); 0 = pure ACGT stream")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--chrom", type=int, default=CHROM,
                    help="an 'N' run break at every base index that is a multiple of this (0 = one run)")
    ap.add_argument("--north-star-bases", type=int, default=10_000_000_000,
                    help="sub-record: k=6 over this many pure-ACGT bases per GPU (0 = skip)")
    ap.add_argument("--cpu-sample-bytes", type=int, default=0, help="0 = auto (~10-20 s of reference CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="time the count kernel with HIP events on every Nth step")
    ap.add_argument("--stitched", action="store_true",
                    help="sharded pass: always the summary all-gather + reduce (no one-collective path)")
    ap.add_argument("--torch-exchange", action="store_true",
                    help="exchange through torch.distributed instead of the library's RCCL communicator")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = host-side rehearsal")
    ap.add_argument("--verify-single", action="store_true",
                    help="rank 0 also counts the whole stream with one engine and compares the merged "
                         "table and counters with it (configs[3] parity)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- the stream

def base_offset(b, first, fasta_line, rank0):
    """Byte offset of stream base b in a buffer that starts at base `first`
    (plus the header on rank 0 of a FASTA stream)."""
    rel = b - first
    if fasta_line <= 0:
        return rel
    return (HEADER if rank0 else 0) + rel + rel // fasta_line


def make_genome(n, fasta_line, seed, chrom, first=0, rank0=True, device="cuda"):
    """The synthetic genome's bases [first, first + n) in a fresh device
    buffer (+64 bytes of slack): fk_synth_device's splitmix64 ACGT (the same
    bytes as the oracle's fko_synth), FASTA framing when fasta_line > 0 (the
    header only on the stream's first shard), and an 'N' at every base index
    j*chrom (j >= 1).  Returns (buffer, size in bytes)."""
    import torch
    import findkmer_amd as fk
    assert first % 32 == 0 and (fasta_line <= 0 or first % fasta_line == 0)
    frame = (fasta_line if rank0 else -fasta_line) if fasta_line > 0 else 0
    size = fk.synth_size(n, frame)
    buf = torch.empty(size + 64, dtype=torch.uint8, device=device)
    w = fk.synth_device(buf.data_ptr(), size, n, seed + first // 32, frame)
    assert w == size
    if chrom > 0:
        for b in range((first // chrom + 1) * chrom, first + n, chrom):
            off = base_offset(b, first, fasta_line, rank0)
            assert chr(buf[off].item()) in "ACGT", (b, off)
            buf[off] = ord("N")
    return buf, size


def run_windows(n, k):
    """Windows the reference counts in one run of n bases: those where its
    `int seqSize` (findKmer.cpp:977) is >= k, i.e. R mod 2^32 in
    [k, 2^31 - 1] for R = 1..n (a run longer than 2^31 - 1 bases stops
    counting until the int32 wraps back to positive values)."""
    period, hi = 1 << 32, (1 << 31) - 1
    full, rem = divmod(n, period)
    return full * (hi - k + 1) + max(0, min(rem, hi) - k + 1)


def _runs(total, chrom):
    if not chrom:
        return [total]
    out, start = [], 0
    for b in range(chrom, total, chrom):
        out.append(b - start)
        start = b + 1
    return out + [total - start]


def expected_windows(total, k, chrom):
    """Windows in a stream of `total` bases with 'N' at j*chrom (j >= 1)"""
    return sum(run_windows(r, k) for r in _runs(total, chrom))


def want_valid(total, k, chrom):
    """baseCounter of the same stream when no run reaches 2^31 bases: every
    base of a run of >= k bases (findKmer.cpp:1040, :1056)"""
    return sum(r for r in _runs(total, chrom) if r >= k)


# ---------------------------------------------------------------- baselines

def cpu_baseline(k, seed, fasta_line, n_sample):
    """The reference CPU loop (oracle/_ref/findKmer_ref, the reference
    program compiled from its source) on a bounded prefix of the same stream."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle   # checker / baseline only
    data = oracle.synth(n_sample, seed, fasta_line)
    ref = oracle.REF_BIN
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "sample.fa")
            data.tofile(p)
            t0 = time.perf_counter()
            subprocess.run([ref, "-q", "1", "-k", str(k), "-p", "sample.fa"], cwd=td,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
        kind = "reference"
        what = (f"oracle/_ref/findKmer_ref (reference findKmer.cpp, g++ -O3, single thread) "
                f"end-to-end on the first {n_sample} bases of the same stream, k={k}")
    else:
        t0 = time.perf_counter()
        oracle.count_dense(data, k)
        dt = time.perf_counter() - t0
        kind = "port"
        what = f"oracle port (fk_oracle.c, 1 thread) on the first {n_sample} bases, k={k}"
    return {"value": n_sample / dt, "unit": "bases/s", "cores": 1, "kind": kind,
            "sample": what, "seconds": round(dt, 3)}


def cpu_baseline_multicore(k, seed, fasta_line, n_sample):
    """BASELINE.md's "fast CPU": the oracle's dense-table scan split over the
    host threads this process may use (fko_count_dense_par; oracle.host_threads:
    its CPU affinity capped by the cgroup quota), on a bounded prefix of the
    same stream, input in host memory."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle
    data = oracle.synth(n_sample, seed, fasta_line)
    th = oracle.host_threads()
    oracle.count_dense(data[: 1 << 20], k, threads=th)       # page in the library
    t0 = time.perf_counter()
    oracle.count_dense(data, k, threads=th)
    dt = time.perf_counter() - t0
    cpu = ""
    try:
        cpu = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        pass
    return {"value": n_sample / dt, "unit": "bases/s", "cores": th, "kind": "port",
            "sample": f"fko_count_dense_par (dense u32 table, {th} threads = this process's CPU affinity "
                      f"capped by its cgroup CPU quota) on the first {n_sample} bases "
                      f"of the same stream, k={k}; host CPU {cpu}, os.cpu_count()={os.cpu_count()}",
            "seconds": round(dt, 3)}


# ---------------------------------------------------------------- one workload

class Ctx:
    def __init__(self, args, world, rank, local, dist, coll_dev):
        self.args, self.world, self.rank, self.local, self.dist, self.coll_dev = \
            args, world, rank, local, dist, coll_dev


def measure(ctx, k, n, L, seed, chrom, steps, warmup, verify=False):
    """Time `steps` passes of the hot path over this rank's shard of the
    stream (n bases per rank).  Returns the record (rank 0's view)."""
    import torch
    import findkmer_amd as fk
    import findkmer_amd.dist as fkdist
    args, world, rank, dist = ctx.args, ctx.world, ctx.rank, ctx.dist
    sharded = dist is not None
    assert n % 32 == 0 and (L <= 0 or n % L == 0), \
        "--bases: a multiple of 32 (generator words) and of the FASTA line width"
    # this rank's shard: bases [rank*n, (rank+1)*n) plus the bytes just before
    # it (halo) so the engine can guess the entry state
    halo_bases = 0 if rank == 0 else (1280 if L > 0 else 256)
    first = rank * n - halo_bases
    chrom_on = chrom > 0 and world * n > chrom
    buf, size = make_genome(n + halo_bases, L, seed, chrom if chrom_on else 0, first, rank == 0)
    halo = base_offset(first + halo_bases, first, L, rank == 0) - (HEADER if (L > 0 and rank == 0) else 0)
    nbytes = size - halo
    torch.cuda.synchronize()

    # (17 <= k <= 20: finish re-reads the step's input from `buf`, which stays
    # unchanged, instead of a copy the engine keeps: fk_opts.borrow_input)
    eng = fk.Engine(k, device=ctx.local, timing_every=args.timing_every, borrow_input=True)
    # 17 <= k <= 20: sparse tables, merged by an all-to-all (no dense buffer)
    merge_t = fkdist.merge_buffer(k, ctx.coll_dev) if sharded and k < fkdist.SPARSE_KMIN else None
    pinned = torch.empty(fkdist.COUNTER_SLOTS, dtype=torch.int32, pin_memory=True) \
        if (sharded and ctx.coll_dev == "cuda") else None
    phase_s = {}

    def step():
        eng.reset()
        if sharded:
            res = fkdist.count_sharded(eng, buf.data_ptr() + halo, nbytes, halo, merge_t, times=phase_s,
                                       pinned=pinned, fast=not args.stitched, native=not args.torch_exchange)
            return res.local, res
        eng.feed_device(buf.data_ptr(), nbytes)
        # an ablation build (FINDKMER_LIB) may leave the table incomplete
        rc, r = eng.finish(allow=(fk.FK_OK, fk.FK_E_ROLLOVER) if os.environ.get("FINDKMER_LIB") else (fk.FK_OK,))
        return r, None

    for _ in range(warmup):
        step()
    phase_s.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = merged = None
    main_ms, timed = 0.0, 0
    for _ in range(steps):
        last, merged = step()
        main_ms += last.main_kernel_ms
        timed += last.timed_kernels
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = main_ms / timed if timed else 0.0   # mean over the timed launches of the timed region
    if dist:
        tt = torch.tensor([dt, kern_ms], dtype=torch.float64, device=ctx.coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, kern_ms = float(tt[0].item()), float(tt[1].item())

    # correctness guard on the measured pass (the merged result lives on rank 0)
    if not os.environ.get("FINDKMER_LIB") and rank == 0:
        total = merged.windows if merged is not None else last.windows
        if merged is not None:
            assert merged.status() == fk.FK_OK, ("merged table: rollover or unterminated header",
                                                 merged._table_stats(), merged.windows, merged.unterminated_header)
        valid = merged.valid_bases if merged is not None else last.valid_bases
        if chrom_on and chrom < (1 << 31):
            assert valid == want_valid(world * n, k, chrom), (valid, want_valid(world * n, k, chrom))
        want = expected_windows(world * n, k, chrom if chrom_on else 0)
        assert total == want, (total, want)

    # what RCCL itself reports for the communicator the exchange ran on, from
    # every rank: the world the line claims is the world that ran
    rccl = None
    if merged is not None and merged.transport == "rccl-native":
        comm = fkdist.native_comm(None)
        mine = torch.tensor(list(comm.info()) + [ctx.local], dtype=torch.int64, device=ctx.coll_dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        rows = [[int(x) for x in t.tolist()] for t in every]
        rccl = {"nranks": rows[0][0], "ranks": [r[1] for r in rows], "devices": [r[2] for r in rows],
                "local_ranks": [r[3] for r in rows]}

    check = None
    if verify:
        check = verify_single(ctx, k, n, L, seed, chrom if chrom_on else 0, merged, last)

    ms_step = dt / steps * 1e3
    algo_bytes = nbytes + 4 * (1 << (2 * k))       # input read once + u32 table written once
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0   # 0: events off (FINDKMER_TUNE events=0)
    step_gbs = algo_bytes / (ms_step * 1e-3) / 1e9
    main = "k_part" if 8 <= k <= 16 else "k_count"
    rec = {
        "value": world * n / (dt / steps),
        "ms_per_step": ms_step,
        "workload": (f"k={k} over a {world * n / 1e9:g} G-base synthetic "
                     + ("ACGT stream" if L == 0 else f"FASTA genome ({L}-col lines)")
                     + (f" cut into {world} shards of {n / 1e9:g} G bases, one per GPU" if world > 1 else "")
                     + (f", {args.chrom / 1e9:g} G-base chromosomes" if chrom_on else ", one run")),
        "k": k, "bases_per_gpu": n, "input_bytes_per_gpu": nbytes,
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_for(k, L, nbytes, main),
            "kernel": main, "kernel_ms": kern_ms, "timed_launches": timed,
            "algorithmic_bytes": algo_bytes,
            "step_achieved": step_gbs, "step_frac": step_gbs / HBM_PEAK_GBS,
            "step_traffic": traffic_for(k, L, nbytes, main, "hbm_bytes_per_step"),
        },
    }
    if phase_s:
        rec["phase_ms_per_step"] = {k_: v / steps * 1e3 for k_, v in phase_s.items()}
    if merged is not None:
        rec["exchange"] = merged.path
        rec["transport"] = merged.transport
    if rccl is not None:
        rec["rccl"] = rccl
    if check is not None:
        rec["verify"] = check
    eng.close()
    del buf, merge_t
    torch.cuda.empty_cache()
    return rec


def traffic_for(k, L, nbytes, main, what="hbm_bytes_per_launch"):
    """HBM bytes from the committed PMC profile of this exact workload
    (profiles/traffic_k<K>_L<L>_n<bytes>.json, written by
    tools/profile_summary.py), else None: per launch of the dominant kernel
    (`hbm_bytes_per_launch`), or per step, every kernel of the step summed
    (`hbm_bytes_per_step`)."""
    tf = os.path.join(REPO, "profiles", f"traffic_k{k}_L{L}_n{nbytes}.json")
    try:
        prof = json.load(open(tf))
    except Exception:
        return None
    if prof.get("input_bytes") == nbytes and prof.get("kernel") == main:
        return prof.get(what)
    return None


def verify_single(ctx, k, n, L, seed, chrom, merged, last):
    """configs[3] parity: rank 0 counts the whole world x n stream with one
    engine and compares it with the sharded pass's merged table and counters.
    Every rank takes part in gathering the merged table first (a collective
    when the table is sharded over the ranks: k >= 12, or sparse for k >= 17)."""
    import numpy as np
    import torch
    import findkmer_amd as fk
    if merged is None:
        raise SystemExit("--verify-single needs a sharded run (torchrun)")
    full = merged.table_full()          # collective; None except on rank 0
    if ctx.rank != 0:
        return None
    buf, size = make_genome(ctx.world * n, L, seed, chrom)
    torch.cuda.synchronize()
    with fk.Engine(k, device=ctx.local) as e:
        e.feed_device(buf.data_ptr(), size)
        rc, r = e.finish()
        if k > fk.FK_K_MAX_DENSE:
            keys, cnts = e.sparse()
            equal = bool(np.array_equal(full[0], keys) and np.array_equal(full[1], cnts))
        else:
            equal = bool(np.array_equal(full.cpu().numpy().view(np.uint32), e.table()))
    del buf
    torch.cuda.empty_cache()
    out = {"table_equal": equal, "status": rc}
    for key in ("windows", "valid_bases", "unknown_chars", "scanned_bytes", "hit_eof_byte",
                "unterminated_header", "distinct"):
        out[key] = [int(getattr(merged, key)), int(getattr(r, key))]
    out["base_count"] = [list(merged.base_count), list(r.base_count)]
    out["depth1"] = [list(merged.depth1), list(r.depth1)]
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(gpus, argv, port):
    """`python bench.py --gpus N` without a launcher: the torchrun command
    that runs this same script with the same arguments, one rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def world_check(gpus, env):
    """None when this process may run the bench as is; "spawn" when it must
    launch --gpus ranks itself (no WORLD_SIZE, N > 1); else the error text of
    a launcher world that is not the one --gpus asks for."""
    if "WORLD_SIZE" not in env:
        return "spawn" if gpus > 1 else None
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        return f"bench.py: WORLD_SIZE={world} but --gpus {gpus}: the line would claim a world that did not run"
    return None


def shard_bases(total, world, L):
    """Bases per rank when the `total`-base stream is cut into `world` equal
    shards (configs[3]: one 10 G-base genome split N ways).  A shard is a
    whole number of generator words (32 bases) and FASTA lines."""
    if world == 1:
        return total
    unit = 32 if L <= 0 else 32 * L // math.gcd(32, L)
    return total // world // unit * unit


def main():
    args = parse()
    chk = world_check(args.gpus, os.environ)
    if chk == "spawn":
        # before torch or any GPU call: this process only waits for the ranks
        # (a child process, never an exec, from a process that touched no GPU)
        p = subprocess.run(launcher_cmd(args.gpus, sys.argv[1:], free_port()))
        sys.exit(p.returncode)
    if chk is not None:
        print(chk, file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import findkmer_amd.dist as fkdist
    # a gloo rehearsal may put several ranks on one GPU
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    # under torch.distributed.run (WORLD_SIZE set, even to 1) the sharded
    # pass with its exchange runs; `python bench.py` at N=1 feeds directly
    if world > 1 or "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    ctx = Ctx(args, world, rank, local, dist, coll_dev)

    # the headline: one `args.bases`-base stream, cut into `world` shards
    # (strong scaling; at N > 1 this is configs[3]: the 10 G-base genome of
    # configs[2] split N ways, counted by N ranks, merged)
    n = shard_bases(args.bases, world, args.fasta_line)
    head = measure(ctx, args.k, n, args.fasta_line, args.seed, args.chrom, args.steps, args.warmup,
                   verify=args.verify_single)
    if head.get("transport") == "rccl-native":
        # the world this line claims is the world RCCL itself reports
        assert head["rccl"]["nranks"] == world, (head["rccl"], world)
    weak = None
    if world > 1 and args.weak_bases > 0:
        # sub-record: every rank a whole `weak_bases` shard of an N x as long
        # stream (per-GPU work fixed as N grows)
        weak = measure(ctx, args.k, shard_bases(args.weak_bases, 1, args.fasta_line), args.fasta_line, args.seed,
                       args.chrom, args.steps, args.warmup)
    ns = None
    if args.north_star_bases > 0:
        ns = measure(ctx, 6, args.north_star_bases, 0, 1, CHROM, args.steps, args.warmup)
        ns["gate"] = "k=6 over a 10 GB synthetic genome at >= 70% of single-GPU HBM-read roofline (BASELINE.json)"

    cfg_tag = {(11, 80, 10_000_000_000): " (BASELINE.json configs[2])",
               (6, 0, 1_000_000_000): " (BASELINE.json configs[1])"}.get((args.k, args.fasta_line, args.bases), "")
    if world > 1 and (args.k, args.fasta_line, args.bases) == (11, 80, 10_000_000_000):
        cfg_tag = f" (BASELINE.json configs[3]: the configs[2] genome split over {world} GPUs)"
    out = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "bases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        # the stream is the same `--bases` bases whatever N is
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 uniform ACGT genome, generated in HBM)",
        "config": {
            "workload": head["workload"] + cfg_tag,
            "k": args.k, "total_bases": n * world, "bases_per_gpu": n,
            "input_bytes_per_gpu": head["input_bytes_per_gpu"],
            "parallelism": f"shard{world}",
        },
        "roofline": head["roofline"],
    }
    for key in ("phase_ms_per_step", "exchange", "transport", "rccl", "verify"):
        if key in head:
            out[key] = head[key]
    if weak is not None:
        out["weak_scaling"] = {key: weak[key] for key in ("workload", "value", "ms_per_step", "bases_per_gpu",
                                                           "roofline", "exchange", "transport", "rccl",
                                                           "phase_ms_per_step") if key in weak}
        out["weak_scaling"]["scaling"] = "weak"
    if ns is not None:
        out["north_star"] = {key: ns[key] for key in ("workload", "gate", "value", "ms_per_step", "roofline",
                                                       "exchange", "transport") if key in ns}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # ~15 s of reference CPU work: ~76 Mbases/s at k=6, ~3 Mbases/s at k=11
        sample = args.cpu_sample_bytes or (1 << 30 if args.k <= 7 else 48 << 20)
        sample = min(sample, args.bases)
        out["cpu_baseline"] = cpu_baseline(args.k, args.seed, args.fasta_line, sample)
        out["cpu_baseline_multicore"] = cpu_baseline_multicore(args.k, args.seed, args.fasta_line,
                                                               min(1 << 30, args.bases))
        # the sample's rate applied to the whole configured workload (the
        # reference's loop is linear in the input: one fgetc and one trie walk
        # per byte, findKmer.cpp:988-1062)
        for key in ("cpu_baseline", "cpu_baseline_multicore"):
            out[key]["extrapolated_s_full_config"] = round(args.bases / out[key]["value"], 1)
            out[key]["extrapolation"] = (f"sample rate x {args.bases} bases (linear: the reference scans "
                                         f"once per byte, findKmer.cpp:988)")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        fkdist.close_native_comms()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
