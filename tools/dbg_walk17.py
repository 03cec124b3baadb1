"""debug: the fused k = 17 walks vs the key-list passes on the borrowed-feeds
test's input (feeds as in test_sparse_borrowed_device_feeds), host vs device"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import findkmer_amd as fk
from test_gpu_parity import mixed_input

data = mixed_input(1300 + 17, 600_000)
FEEDS = [4096, 160_000, 16, 7, 200_009, len(data) - 4096 - 160_000 - 16 - 7 - 200_009]


def run(tune, feeds, borrow):
    os.environ["FINDKMER_TUNE"] = tune
    dev = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    torch.cuda.synchronize()
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    with fk.Engine(17, want_nodes=True, borrow_input=borrow) as e:
        pos = 0
        for n in feeds:
            if borrow:
                e.feed_device(dev.data_ptr() + pos, n)
            else:
                e.feed(np.ascontiguousarray(arr[pos:pos + n]))
            pos += n
        e.finish(allow=(fk.FK_OK, fk.FK_E_EMPTY, fk.FK_E_UNTERMINATED_HEADER, fk.FK_E_ROLLOVER))
        return e.sparse()


ref = run("sp_walk=0", [len(data)], False)
for name, tune, feeds, borrow in [("one host feed", "", [len(data)], False), ("again", "", [len(data)], False),
                                  ("again", "", [len(data)], False), ("all general", "sp_walk_dbg=1", [len(data)], False),
                                  ("borrowed", "", FEEDS, True), ("again", "", FEEDS, True)]:
    k, c = run(tune, feeds, borrow)
    same = np.array_equal(k, ref[0]) and np.array_equal(c, ref[1])
    print(name, "same" if same else "DIFF", len(k), len(ref[0]))
    if not same:
        a = dict(zip(ref[0].tolist(), ref[1].tolist()))
        b = dict(zip(k.tolist(), c.tolist()))
        bad = sorted(set(a) ^ set(b) | {x for x in a if x in b and a[x] != b[x]})
        for x in bad[:12]:
            print("  key %d (first base %d) ref %s got %s" % (x, x >> 32, a.get(x), b.get(x)))
        print("  total windows ref", sum(a.values()), "got", sum(b.values()))
