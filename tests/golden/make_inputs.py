"""Regenerates the synthetic golden inputs (committed alongside; kept for provenance).

test.txt is the reference's own sample input (findKmer/test.txt), copied as data.
"""
import random, os
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "inputs")

def main():
    rng = random.Random(20141)
    out, n, rec = [], 0, 0
    while n < 120000:                      # upstream-like records, 60-col lines
        out.append('>ENST%011d\n' % rec); rec += 1
        L = rng.randint(200, 3000)
        seq = [rng.choice('ACGT') for _ in range(L)]
        if rng.random() < 0.3:             # occasional N block breaks runs
            s = rng.randint(0, L - 20); e = s + rng.randint(1, 15)
            for i in range(s, e): seq[i] = 'N'
        seq = ''.join(seq)
        for i in range(0, L, 60):
            out.append(seq[i:i + 60] + '\n')
        n += L
    open(os.path.join(HERE, 'rand120k.fa'), 'w').write(''.join(out))
    # 0xFF ends the scan outside a header (signed char == EOF) but not inside one
    open(os.path.join(HERE, 'ffbyte.bin'), 'wb').write(
        b'>hdr\xffx\nACGTTGCA\x00ACGGT\nTTAC\xffGGGGCCCC\n')
    # no run reaches k=5: baseCounter == 0 -> NaN probabilities
    open(os.path.join(HERE, 'shortruns.txt'), 'w').write('ACGNTTNACGTN\nGA\n')
    open(os.path.join(HERE, 'edge.txt'), 'wb').write(
        b'ACGTACGTTGCA\r\nacgtACGTNNACG>comment ACGT\nTTGACCA1GGTAC\n>h\nAAAACCCCGGGGTTTT\nGATTACA')
    open(os.path.join(HERE, 'missing.txt'), 'w').write('AAAACCCCGGGG\n')
    open(os.path.join(HERE, 'empty.txt'), 'w').write('')

if __name__ == '__main__':
    main()
