"""Timeline of k_tail (one-pass feeds (experiment build FK_EXP=20:
build/exp/libfk_e20.so): per step, microseconds from the kernel's first
block entry to each probe point (max over blocks)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["FINDKMER_LIB"] = os.path.join(REPO, "build", "exp", "libfk_e20.so")
sys.path.insert(0, REPO)
import torch  # noqa: E402
import findkmer_amd as fk  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n = 1_000_000_000
lib = ctypes.CDLL(os.environ["FINDKMER_LIB"])
buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
fk.synth_device(buf.data_ptr(), n, n, 1, 0)
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 16)()
names = ["entry", "sliced", "last_go", "results", "published", "loaded", "synced", "", "entry_max", "shuffled", "xput_issued"]
with fk.Engine(k) as e:
    for step in range(8):
        lib.fk_debug_tailprof(None)
        e.reset()
        e.feed_device(buf.data_ptr(), n)
        e.finish()
        lib.fk_debug_tailprof(out)
        t0 = out[0]
        print(f"k={k} step {step}: " + " ".join(f"{names[i]}={(out[i] - t0) / 100.0:.1f}" for i in (8, 5, 6, 9, 10, 1, 2, 3, 4)), flush=True)
