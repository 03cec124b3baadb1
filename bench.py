#!/usr/bin/env python3
"""bench.py — k-mer scan throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): k=6 over a 1 GB synthetic ACGT stream per
GPU, input resident in HBM before the timed region.  One step = one pass of
the hot path over the batch: reset, k_count + k_tail (the engine's
fk_engine_feed: count, fold, check the guessed range states, publish), and the
result scalars (fk_engine_finish).  With
--gpus N (one process per GPU, torch.distributed over RCCL) each rank owns the
next 1 GB shard of one N GB stream (a synthetic genome with an 'N' run break
every 1.5 Gbases, so no run reaches the reference's int32 wrap; the N=1 stream
has none): the shard entry state is stitched by
all-gathering the 96-byte shard transfer functions, and the count tables are
summed with a reduce to rank 0 — the path's two real exchange steps.

Prints ONE JSON line on rank 0 (contract in the task statement): value =
bases/s over all ranks, plus "roofline" for the dominant kernel (k_count, HIP
events on the engine's stream) and "cpu_baseline" (the reference binary, or
the oracle port if it is absent, on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "bases/sec scanned at fixed k; achieved HBM GB/s vs roofline, 1/2/4/8 GPUs"
CHROM = 1_500_000_000   # multi-GPU stream: an 'N' run break every CHROM bases (synthetic chromosomes)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--bases", type=int, default=1_000_000_000, help="bases per GPU")
    ap.add_argument("--fasta-line", type=int, default=0, help="0 = pure ACGT stream (configs[1]); 80 = FASTA")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-sample-bytes", type=int, default=0, help="0 = auto (~10-20 s of reference CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chrom", type=int, default=CHROM,
                    help="streams longer than this (pure ACGT): an 'N' run break every this many bases, a genome of chromosomes (0 = one run)")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="time the count kernel with HIP events on every Nth step")
    ap.add_argument("--stitched", action="store_true",
                    help="sharded pass: always the summary all-gather + reduce (no one-collective path)")
    ap.add_argument("--torch-exchange", action="store_true",
                    help="one-collective path through torch.distributed instead of the library's RCCL communicator")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = host-side rehearsal")
    return ap.parse_args()


def cpu_baseline(args, n_sample):
    """The reference CPU loop on a bounded prefix of the same stream."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle   # checker / baseline only
    data = oracle.synth(n_sample, args.seed, args.fasta_line if args.fasta_line > 0 else 0)
    bases = n_sample
    ref = oracle.REF_BIN
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "sample.fa")
            data.tofile(p)
            t0 = time.perf_counter()
            subprocess.run([ref, "-q", "1", "-k", str(args.k), "-p", "sample.fa"], cwd=td,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
        kind = "reference"
        what = (f"oracle/_ref/findKmer_ref (reference findKmer.cpp, g++ -O3, single thread) "
                f"end-to-end on the first {bases} bases of the same stream, k={args.k}")
    else:
        t0 = time.perf_counter()
        oracle.count_dense(data.tobytes(), args.k)
        dt = time.perf_counter() - t0
        kind = "port"
        what = f"oracle port (fk_oracle.c, 1 thread) on the first {bases} bases, k={args.k}"
    return {"value": bases / dt, "unit": "bases/s", "cores": 1, "kind": kind,
            "sample": what, "seconds": round(dt, 3)}


def run_windows(n, k):
    """Windows the reference counts in one run of n bases: those where its
    `int seqSize` (findKmer.cpp:977) is >= k, i.e. R mod 2^32 in
    [k, 2^31 - 1] for R = 1..n (a run longer than 2^31 - 1 bases stops
    counting until the int32 wraps back to positive values)."""
    period, hi = 1 << 32, (1 << 31) - 1
    full, rem = divmod(n, period)
    return full * (hi - k + 1) + max(0, min(rem, hi) - k + 1)


def expected_windows(total, k, chrom):
    """Windows in a pure-ACGT stream of `total` positions whose positions
    j*chrom (j >= 1) hold 'N' run breaks: each run is shorter than 2^31, so
    the reference's int32 seqSize (findKmer.cpp:977) never wraps."""
    w, start = 0, 0
    for b in range(chrom, total, chrom):
        w += run_windows(b - start, k)
        start = b + 1
    return w + run_windows(total - start, k)


def want_valid(total, k, chrom):
    """baseCounter of the same stream: every base of a run of >= k bases
    (findKmer.cpp:1040, :1056; runs are shorter than 2^31 here)"""
    if not chrom:
        return total if total >= k else 0
    v, start = 0, 0
    for b in range(chrom, total, chrom):
        v += (b - start) if b - start >= k else 0
        start = b + 1
    return v + ((total - start) if total - start >= k else 0)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import findkmer_amd as fk
    import findkmer_amd.dist as fkdist
    # a gloo rehearsal may put several ranks on one GPU
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    # under torch.distributed.run (WORLD_SIZE set, even to 1) the sharded
    # pass with its exchange runs; `python bench.py` at N=1 feeds directly
    sharded = world > 1 or "WORLD_SIZE" in os.environ
    if sharded:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    k = args.k
    n = args.bases
    L = args.fasta_line
    assert n % 1280 == 0, "--bases must be a multiple of 1280 (32-base generator words, 80-col lines)"

    # this rank's shard of one stream: bases [rank*n, (rank+1)*n), plus the
    # bytes just before it (halo) so the engine can guess the entry state
    halo_bases = 0 if rank == 0 else (1280 if L > 0 else 256)
    first = rank * n - halo_bases
    if L > 0:
        halo = halo_bases + halo_bases // L
        frame = L if rank == 0 else -L
        size = fk.synth_size(n + halo_bases, frame)
    else:
        halo = halo_bases
        frame = 0
        size = n + halo_bases
    buf = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    w = fk.synth_device(buf.data_ptr(), size, n + halo_bases, args.seed + first // 32, frame)
    assert w == size
    nbytes = size - halo
    # one N-GB stream as a genome of CHROM-base chromosomes: an 'N' at every
    # base index that is a multiple of CHROM (as in real genomes, no run
    # reaches the reference's int32 seqSize wrap at 2^31 bases).  FASTA
    # framing: single-GPU streams only (base b sits at byte 11 + b + b // L).
    chrom_breaks = args.chrom > 0 and world * n > args.chrom and (L == 0 or world == 1)
    if chrom_breaks:
        for b in range((max(first, 0) // args.chrom + 1) * args.chrom, first + n + halo_bases, args.chrom):
            off = b - first if L == 0 else 11 + b + b // L
            assert chr(buf[off].item()) in "ACGT", (b, off)
            buf[off] = ord("N")
    torch.cuda.synchronize()

    # the count kernel's HIP events on every 4th step of the timed region
    # (recording them on every launch costs ~2% of the step)
    eng = fk.Engine(k, device=local, timing_every=args.timing_every)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    merge_t = fkdist.merge_buffer(k, coll_dev) if sharded else None
    pinned = torch.empty(fkdist.COUNTER_SLOTS, dtype=torch.int32, pin_memory=True) if coll_dev == "cuda" else None

    def step():
        eng.reset()
        if sharded:
            # shard, stitch entry states (all-gather of 96-B summaries), merge
            # tables + counters (reduce to rank 0): findkmer_amd/dist.py
            res = fkdist.count_sharded(eng, buf.data_ptr() + halo, nbytes, halo, merge_t, times=phase_s,
                                       pinned=pinned, fast=not args.stitched, native=not args.torch_exchange)
            return res.local, res
        eng.feed_device(buf.data_ptr(), nbytes)
        # an ablation build (FINDKMER_LIB) may leave the table incomplete
        rc, r = eng.finish(allow=(fk.FK_OK, fk.FK_E_ROLLOVER) if os.environ.get("FINDKMER_LIB") else (fk.FK_OK,))
        return r, None

    phase_s = {}
    for _ in range(args.warmup):
        step()
    phase_s.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = merged = None
    main_ms, timed = 0.0, 0
    for _ in range(args.steps):
        last, merged = step()
        main_ms += last.main_kernel_ms
        timed += last.timed_kernels
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # correctness guard on the measured pass: the synthetic stream (pure ACGT,
    # or FASTA whose '\n' are transparent) is one run, every window counts
    if not os.environ.get("FINDKMER_LIB") and rank == 0:
        # the merged counters and table live on rank 0 (dist.reduce)
        total = merged.windows if merged is not None else last.windows
        if merged is not None:
            assert merged.status() == fk.FK_OK, "merged table: rollover or unterminated header"
            if chrom_breaks or world * n < (1 << 31):   # no run reaches the int32 seqSize wrap
                assert merged.valid_bases == want_valid(world * n, k, args.chrom if chrom_breaks else 0)
        want = expected_windows(world * n, k, args.chrom) if chrom_breaks else run_windows(world * n, k)
        assert total == want, (total, want)

    ms_step = dt / args.steps * 1e3
    value = world * n / (dt / args.steps)
    kern_ms = main_ms / timed if timed else 0.0   # mean over the timed launches of the timed region
    algo_bytes = nbytes + 4 * (1 << (2 * k))       # input read once + u32 table written once
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0   # 0: events off (FK_NO_EVENTS)
    traffic = None
    tf = os.path.join(REPO, "profiles", f"traffic_k{k}_L{L}.json")
    if os.path.exists(tf):
        try:
            prof = json.load(open(tf))
            # only a profile of this exact workload size describes this launch
            if prof.get("input_bytes") == nbytes:
                traffic = prof.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "bases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 uniform ACGT, generated in HBM)",
        "config": {
            "workload": (f"k={k} over a {n / 1e9:g} G-base synthetic "
                         + ("ACGT stream" if L == 0 else f"FASTA ({L}-col lines)") + " per GPU"
                         + (f", one {world * n / 1e9:g} G-base genome of {args.chrom / 1e9:g} G-base chromosomes"
                            if chrom_breaks else "")
                         + (" (BASELINE.json configs[1])" if (k, L, n) == (6, 0, 1_000_000_000) else "")),
            "k": k, "bases_per_gpu": n, "input_bytes_per_gpu": nbytes,
            "parallelism": f"shard{world}",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "k_part" if 8 <= k <= 12 else "k_count", "kernel_ms": kern_ms, "timed_launches": timed,
            "algorithmic_bytes": algo_bytes,
        },
    }
    if phase_s:
        # rank 0's host time per step in each phase of the sharded pass
        out["phase_ms_per_step"] = {k_: v / args.steps * 1e3 for k_, v in phase_s.items()}
    if merged is not None:
        # "fast": one all-reduce of tables + counters + shard summaries;
        # "stitched": summary all-gather, then a reduce (findkmer_amd/dist.py)
        out["exchange"] = merged.path
        out["transport"] = merged.transport
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # ~15 s of reference CPU work: ~76 Mbases/s at k=6, ~3 Mbases/s at k=11
        sample = args.cpu_sample_bytes or (1 << 30 if k <= 7 else 48 << 20)
        sample = min(sample, n)
        out["cpu_baseline"] = cpu_baseline(args, sample)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        fkdist.close_native_comms()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
