"""Per-wave timing of k_count (experiment build tools/wave_times.sh, loaded
with FINDKMER_LIB=build/exp/libfk_wt.so): start, loop end and end of every
wave (s_memrealtime, 100 MHz) and its XCD, for one 1 G-base k=6 feed.
Prints the spread of start and end times and per-XCD loop durations."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import findkmer_amd as fk  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
fk.synth_device(buf.data_ptr(), n, n, 1, 0)
torch.cuda.synchronize()
eng = fk.Engine(k)
for _ in range(5):
    eng.reset()
    eng.feed_device(buf.data_ptr(), n)
    eng.finish()
L = fk.lib()
f = L.fk_debug_wave_times
f.restype = ctypes.c_int
out = np.zeros(32768 * 4, dtype=np.uint64)
assert f(out.ctypes.data_as(ctypes.c_void_p), 32768) == 0
w = out.reshape(-1, 4)
w = w[w[:, 0] > 0]
t0 = w[:, 0].min()
st, le, en, xcc = (w[:, 0] - t0) * 10e-3, (w[:, 1] - t0) * 10e-3, (w[:, 2] - t0) * 10e-3, w[:, 3]
res = {
    "waves": int(len(w)),
    "start_us": [float(np.percentile(st, p)) for p in (0, 50, 99, 100)],
    "loop_end_us": [float(np.percentile(le, p)) for p in (0, 1, 10, 50, 90, 99, 100)],
    "end_us": [float(np.percentile(en, p)) for p in (0, 50, 99, 100)],
    "mean_loop_us": float((le - st).mean()),
    "per_xcd_mean_loop_end_us": {int(x): float(le[xcc == x].mean()) for x in np.unique(xcc)},
    "per_xcd_max_loop_end_us": {int(x): float(le[xcc == x].max()) for x in np.unique(xcc)},
}
print(json.dumps(res))
