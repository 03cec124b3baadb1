import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
torch.cuda.init()
import findkmer_amd as fk
L = 2 ** 32 + 2 ** 31 + 50
k = 3
buf = torch.full((L,), ord("A"), dtype=torch.uint8, device="cuda")
z = 2 ** 31 - 3
for it in range(4):
    with fk.Engine(k) as e:
        e.feed_device(buf.data_ptr(), L)
        rc, r = e.finish(allow=(fk.FK_OK, fk.FK_E_ROLLOVER))
        t = e.table()
    print(it, "t0", int(t[0]), "diff", 2 * z - int(t[0]), "windows", r.windows, "redo", r.redo_chunks, flush=True)
