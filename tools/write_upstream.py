"""Write BASELINE.json configs[4]'s input to a file: an upstream-regions-like
FASTA (">ENST%011u" records of 1001 bases, 1 % with a 50-base N run) made
on the GPU by fk_synth_upstream_device -- the bytes tests/test_gpu_scale.py
checks against the oracle -- in 1 GiB pieces.

usage: python3 tools/write_upstream.py OUT BYTES [SEED]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import findkmer_amd as fk
    out, nbytes = sys.argv[1], int(float(sys.argv[2]))
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    nrec = max(1, nbytes // fk.FK_UPSTREAM_REC)
    per = (1 << 30) // fk.FK_UPSTREAM_REC
    buf = torch.empty(per * fk.FK_UPSTREAM_REC + 64, dtype=torch.uint8, device="cuda")
    with open(out, "wb") as f:
        for r0 in range(0, nrec, per):
            n = min(per, nrec - r0)
            w = fk.synth_upstream_device(buf.data_ptr(), n * fk.FK_UPSTREAM_REC, n, seed, first_rec=r0)
            torch.cuda.synchronize()
            f.write(buf[:w].cpu().numpy().tobytes())
    print(out, nrec * fk.FK_UPSTREAM_REC, "bytes")


if __name__ == "__main__":
    main()
