"""TEST INFRASTRUCTURE: one rank of a sharded count on the GPU with the real
engine (findkmer_amd.Engine) and findkmer_amd/dist.py, launched by
tests/test_gpu_dist.py under torch.distributed.run (gloo; every rank on
cuda:0).  The input is a mixed FASTA-like stream (tests/test_dist_cpu._input)
of --bytes bytes; --eof-in R puts a 0xFF byte outside a header in the middle
of rank R's shard (the reference's signed-char EOF, findKmer.cpp:988).
Rank 0 checks the merged table and counters against the CPU oracle and
prints one JSON line."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--bytes", type=int, default=3_000_000)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--eof-in", type=int, default=-1)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"],
                    help="nccl: RCCL with a device merge buffer (one rank per GPU: world 1 on a 1-GPU box)")
    ap.add_argument("--fast", type=int, default=1, help="0: always the stitched exchange")
    ap.add_argument("--native", type=int, default=1, help="nccl: 0 = the one-collective path through torch.distributed")
    ap.add_argument("--input", default="mixed", choices=["mixed", "fasta"],
                    help="fasta: one header + 80-column ACGT lines (every k <= 7 shard counts in one pass)")
    ap.add_argument("--shard-table", default="auto", choices=["auto", "0", "1"],
                    help="1: the merged table reduce-scattered over the ranks (auto: k >= 12)")
    ap.add_argument("--test-invalid", type=int, default=0,
                    help="native path: mark this rank's pack row invalid (the fallback after the all-reduce)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import findkmer_amd as fk
    import findkmer_amd.dist as fkdist
    import oracle
    from test_dist_cpu import _input

    torch.cuda.set_device(0)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    if args.input == "fasta":
        rng = np.random.default_rng(args.seed)
        bases = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, args.bytes)]
        lines = bases[: len(bases) // 80 * 80].reshape(-1, 80)
        body = np.concatenate([lines, np.full((len(lines), 1), 10, dtype=np.uint8)], axis=1).tobytes()
        data = bytearray(b">synthetic\n" + body)
    else:
        data = bytearray(_input(args.seed, args.bytes))
    n = len(data)
    bounds = [0] + [n * i // world // 16 * 16 for i in range(1, world)] + [n]
    if args.eof_in >= 0:
        at = (bounds[args.eof_in] + bounds[args.eof_in + 1]) // 2
        data[at - 2:at + 1] = b"\nA\xff"
    data = bytes(data)
    lo, hi = bounds[rank], bounds[rank + 1]
    halo = min(256, lo)
    dev = torch.empty(hi - lo + halo + 64, dtype=torch.uint8, device="cuda")
    dev[: hi - lo + halo].copy_(torch.frombuffer(bytearray(data[lo - halo:hi]), dtype=torch.uint8))
    torch.cuda.synchronize()
    eng = fk.Engine(args.k, device=0)
    sparse = args.k >= fkdist.SPARSE_KMIN   # sparse tables: no merge buffer, an all-to-all to the owners
    buf = None if sparse else fkdist.merge_buffer(args.k, "cuda" if args.backend == "nccl" else "cpu")
    # twice: the second pass reuses the engine, the buffer and the fast
    # path's scratch (stale rows from the first must not leak into it)
    shard = None if args.shard_table == "auto" else bool(int(args.shard_table))
    for _ in range(2 if args.k < 16 else 1):   # (k = 16: a 16 GiB table a pass)
        eng.reset()
        res = fkdist.count_sharded(eng, dev.data_ptr() + halo, hi - lo, halo, buf, fast=bool(args.fast),
                                   native=bool(args.native), shard_table=shard, test_invalid=bool(args.test_invalid))
    full = res.table_full()   # every rank (a gather when the table is sharded)
    out = {"rank": rank}
    if sparse:
        # every rank owns a contiguous key range of the merged table
        assert len(res.keys) == 0 or (int(res.keys.min()) >= res.lo and int(res.keys.max()) < res.hi), \
            "a key outside the owner's range"
    if rank == 0 and sparse:
        keys, cnts, r = oracle.count_sparse(data, args.k, cap=len(data) + 16)
        equal = bool(np.array_equal(full[0], keys) and np.array_equal(full[1], cnts))
    elif rank == 0:
        got = full.cpu().numpy().view(np.uint32)
        if args.k <= 13:
            want, r, _ = oracle.count_dense(data, args.k)
            equal = bool(np.array_equal(got, want))
        else:
            keys, cnts, r = oracle.count_sparse(data, args.k, cap=len(data) + 16)
            nz = np.nonzero(got)[0]
            equal = bool(np.array_equal(nz.astype(np.uint64), keys) and np.array_equal(got[nz], cnts))
    if rank == 0:
        out.update({
            "table_equal": equal,
            "sharded": res.sharded,
            "windows": [res.windows, r.windows],
            "valid_bases": [res.valid_bases, r.valid_bases],
            "base_count": [res.base_count, list(r.base_count)],
            "depth1": [res.depth1, list(r.depth1)],
            "unknown_chars": [res.unknown_chars, r.unknown_chars],
            "scanned_bytes": [res.scanned_bytes, r.scanned_bytes],
            "hit_eof_byte": [res.hit_eof_byte, r.hit_eof_byte],
            "unterminated_header": [res.unterminated_header, r.unterminated_header],
            "distinct": [res.distinct, r.distinct],
            "rollover": res.rollover,
            "first_end": res.first_end,
            "path": res.path,
            "transport": res.transport,
        })
        print(json.dumps(out), flush=True)
    eng.close()
    fkdist.close_native_comms()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
