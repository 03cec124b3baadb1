"""TEST INFRASTRUCTURE ONLY — a small pure-Python model of the reference scan
(findKmer/src/findKmer.cpp:962-1069) over (hdr, R, code) states, used by the
CPU multi-process tests to stand in for the GPU engine: it builds a shard's
transfer function in the engine's fk_summary layout (fk_device.h, struct TF)
and counts a shard from a given entering state.  Small inputs only.

States use the engine's internal base codes A0 C1 T2 G3 ((byte>>1)&3); the
C-ABI (fk_summary_apply, fk_state) converts codes to the reference's
A0 C1 G2 T3 (base2int :567-589) with fk_sigma.
"""
import numpy as np

SYM = {ord("A"): 0, ord("C"): 1, ord("T"): 2, ord("G"): 3}
M64 = (1 << 64) - 1


def sigma(x):
    """internal <-> reference digit map (swap 2 and 3), an involution"""
    return x ^ ((x >> 1) & 0x5555555555555555)


def advance(data, hdr, R, code):
    """Scan `data` from state (hdr, R, code).  Returns (hdr, R, code,
    any_reset, nv): any_reset = a run break outside a header ('>' :991, or a
    non-ACGT non-'\\n' byte :1063), nv = bases seen (meaningful without a
    reset).  0xFF bytes are not modelled (they end the reference's scan)."""
    any_reset = False
    nv = 0
    for c in data:
        if hdr:
            if c == 10:
                hdr = 0
            continue
        if c == ord(">"):
            hdr, R, any_reset = 1, 0, True
            continue
        if c == 10:
            continue
        s = SYM.get(c)
        if s is None:
            R, any_reset = 0, True
            continue
        code = ((code << 2) | s) & M64
        R += 1
        nv += 1
    return hdr, R, code, any_reset, nv


def summary_words(data):
    """The span's transfer function as the 12 u64 words of fk_summary:
    c1 (entering inside a header), then c0 if the span breaks a run outside a
    header (f0_const), else a shift by nv bases whose last bases are cs."""
    h1, r1, k1, _, _ = advance(data, 1, 0, 0)
    h0, r0, k0, reset, nv = advance(data, 0, 0, 0)
    w = [0] * 12
    w[0], w[1], w[2] = r1, k1, h1                     # c1 {R, code, hdr}
    if reset:
        w[3], w[4], w[5] = r0, k0, h0                 # c0
        w[8] = 1                                      # f0_const
    else:
        w[6], w[7] = nv, k0                           # nv, cs
    return w


def count_from(data, k, hdr, R, code, table):
    """Windows of `data` counted from the entering state (reference rules
    :1035-1057; int32 seqSize), added to `table` (reference index order)."""
    mask = (1 << (2 * k)) - 1
    for c in data:
        if hdr:
            if c == 10:
                hdr = 0
            continue
        if c == ord(">"):
            hdr, R = 1, 0
            continue
        if c == 10:
            continue
        s = SYM.get(c)
        if s is None:
            R = 0
            continue
        code = ((code << 2) | s) & M64
        R += 1
        seq = np.int64(R & 0xFFFFFFFF).astype(np.int32)
        if seq >= k:
            table[sigma(code & mask)] += 1
    return hdr, R, code
