import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
torch.cuda.init()
import findkmer_amd as fk

def wrap():
    L = 2 ** 31 + 100
    buf = torch.full((5 + L,), ord("A"), dtype=torch.uint8, device="cuda")
    buf[:5] = torch.tensor(list(b"ACGTN"), dtype=torch.uint8)
    with fk.Engine(2) as e:
        e.feed_device(buf.data_ptr(), 5 + L)
        rc, r = e.finish()
        t = e.table()
    print("wrap t0", int(t[0]), "ok" if int(t[0]) == 2147483646 else "BAD", flush=True)

def zones(tag):
    L = 2 ** 32 + 2 ** 31 + 50
    k = 3
    buf = torch.full((L,), ord("A"), dtype=torch.uint8, device="cuda")
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), L)
        rc, r = e.finish(allow=(fk.FK_OK, fk.FK_E_ROLLOVER))
        t = e.table()
    z = 2 ** 31 - 3
    print(tag, "zones t0", int(t[0]), "diff", 2 * z - int(t[0]), "windows", r.windows, "redo", r.redo_chunks,
          "ptr", hex(buf.data_ptr()), flush=True)

zones("fresh")
wrap()
zones("after-wrap")
zones("again")
