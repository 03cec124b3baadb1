import sys, os, random
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
import findkmer_amd as fk, oracle
from test_gpu_parity import mixed_input
k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
base = mixed_input(808, 3 * 400_000).replace(b"\xff", b"Z")
data = bytearray(base); at = len(data) // 2; data[at - 2:at + 1] = b"\nA\xff"; data = bytes(data)
t_o, r_o, _ = oracle.count_dense(data, k)
arr = np.frombuffer(data, dtype=np.uint8); n = len(arr)
per = (n // 3) // 65536 * 65536
bounds = [0, per, 2 * per, n]
dev = torch.from_numpy(arr.copy()).cuda(); torch.cuda.synchronize()
for mode in ["seq", "sum"]:
    engs = []
    for i in range(3):
        e = fk.Engine(k, collect_unknown=True)
        lo, hi = bounds[i], bounds[i + 1]
        halo = min(256, lo) // 16 * 16
        e.feed_shard_device(dev.data_ptr() + lo, hi - lo, halo)
        engs.append(e)
    with fk.Engine(k) as e:
        e.feed(np.ascontiguousarray(arr[:bounds[1]])); st1 = e.state()
        e.feed(np.ascontiguousarray(arr[bounds[1]:bounds[2]])); st2 = e.state()
    print("true states", (st1.hdr, st1.run, st1.code), (st2.hdr, st2.run, st2.ended))
    if mode == "seq":
        st = fk.FkState()
        for e in engs:
            e.resolve(st); st = e.state()
            print("state", st.hdr, st.run, st.code, st.ended)
    else:
        st = fk.FkState(); ent = []
        for e in engs:
            ent.append(st); s = e.summary(); print("full", fk.summary_is_full(s))
            try:
                st = fk.summary_apply(s, st)
            except fk.FindKmerError as err:
                print("apply failed", err); st = fk.summary_apply(e.summary_full(), st)
            print("composed", st.hdr, st.run, st.code, st.ended)
        for e, s in zip(engs, ent): e.resolve(s)
    tabs = []
    for e in engs:
        rc, r = e.finish(allow=(0, -6, -7, -8))
        tabs.append(e.table().astype(np.int64))
        print(mode, "rc", rc, "win", r.windows, "eof", r.hit_eof_byte, "scanned", r.scanned_bytes)
    tot = sum(tabs)
    print(mode, "sum==oracle", np.array_equal(tot, t_o), "diff bins", int((tot != t_o).sum()), "delta", int(tot.sum() - t_o.sum()), "oracle windows", r_o.windows)
    # e0+e1 alone vs a single-engine count of the prefix
    with fk.Engine(k) as e:
        e.feed(np.ascontiguousarray(arr[:at]))
        e.finish(allow=(0, -6, -7, -8)); tp = e.table().astype(np.int64)
    print("single prefix == oracle", np.array_equal(tp, t_o))
    d = tabs[0] + tabs[1] - t_o
    print("e0+e1 - oracle nonzero", int((d != 0).sum()), "sum", int(d.sum()), "e2 sum", int(tabs[2].sum()))
    for e in engs: e.close()
