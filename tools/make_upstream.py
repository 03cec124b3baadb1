"""Upstream-regions-like FASTA (SURVEY.md §8(d) cfg 5): records
">ENST%011u\\n" + 1001 bases + "\\n", bases uniform ACGT, and a seeded 1 %
chance per record of a 50-base N block (run breaks).  Deterministic for a
seed.  Usage: python tools/make_upstream.py OUT BYTES [SEED]"""
import sys

import numpy as np

REC_BASES = 1001
HDR = 17                      # ">ENST" + 11 digits + "\n"
REC = HDR + REC_BASES + 1


def main():
    out, nbytes = sys.argv[1], int(float(sys.argv[2]))
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rng = np.random.default_rng(seed)
    nrec = max(1, nbytes // REC)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    with open(out, "wb") as f:
        for r0 in range(0, nrec, 65536):
            n = min(65536, nrec - r0)
            a = np.empty((n, REC), dtype=np.uint8)
            a[:, 0:5] = np.frombuffer(b">ENST", dtype=np.uint8)
            ids = np.arange(r0, r0 + n, dtype=np.int64)
            for d in range(11):
                a[:, 5 + 10 - d] = ord("0") + (ids // 10 ** d) % 10
            a[:, HDR - 1] = ord("\n")
            a[:, HDR:HDR + REC_BASES] = acgt[rng.integers(0, 4, size=(n, REC_BASES), dtype=np.uint8)]
            a[:, REC - 1] = ord("\n")
            nb = np.nonzero(rng.random(n) < 0.01)[0]
            starts = rng.integers(0, REC_BASES - 50, size=len(nb))
            for i, s0 in zip(nb, starts):
                a[i, HDR + s0:HDR + s0 + 50] = ord("N")
            f.write(a.tobytes())


if __name__ == "__main__":
    main()
