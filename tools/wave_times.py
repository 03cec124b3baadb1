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
out = np.zeros(32768 * 8, dtype=np.uint64)
assert f(out.ctypes.data_as(ctypes.c_void_p), 32768) == 0
w = out.reshape(-1, 8)
w = w[w[:, 0] > 0]
t0 = w[:, 0].min()
st, le, en, xcc = (w[:, 0] - t0) * 10e-3, (w[:, 1] - t0) * 10e-3, (w[:, 2] - t0) * 10e-3, w[:, 3] & 0xF
hwid = (w[:, 3] >> 32).astype(np.int64)
res = {
    "waves": int(len(w)),
    "start_us": [float(np.percentile(st, p)) for p in (0, 50, 99, 100)],
    "loop_end_us": [float(np.percentile(le, p)) for p in (0, 1, 10, 50, 90, 99, 100)],
    "end_us": [float(np.percentile(en, p)) for p in (0, 50, 99, 100)],
    "mean_loop_us": float((le - st).mean()),
    "per_xcd_mean_loop_end_us": {int(x): float(le[xcc == x].mean()) for x in np.unique(xcc)},
    "per_xcd_max_loop_end_us": {int(x): float(le[xcc == x].max()) for x in np.unique(xcc)},
    "static_end_us": [float(np.percentile((w[:, 4] - t0) * 10e-3, p)) for p in (0, 10, 50, 90, 100)],
    "dyn_ranges_per_wave": [float(np.percentile(w[:, 5], p)) for p in (0, 10, 50, 90, 100)],
    "claim_us_per_wave": [float(np.percentile(w[:, 6] * 10e-3, p)) for p in (0, 10, 50, 90, 100)],
    "dyn_kib_per_wave": [float(np.percentile(w[:, 7] / 1024, p)) for p in (0, 10, 50, 90, 100)],
    "dyn_rate_GBs": float(w[:, 7].sum() / max(1e-9, ((le.max() - np.percentile((w[:, 4] - t0) * 10e-3, 50)) * 1e-6)) / 1e9),
}
# where the spread lives: per CU (xcc, se, sh, cu from HW_REG_HW_ID), per
# block (8 waves), per SIMD
cu = (xcc.astype(np.int64) << 16) | ((hwid >> 8) & 0xF) | (((hwid >> 12) & 1) << 4) | (((hwid >> 13) & 7) << 5)
simd = (hwid >> 4) & 3
blk = np.nonzero(w[:, 0] > 0)[0] // 8 if False else None
def spread(keys):
    u, inv = np.unique(keys, return_inverse=True)
    means = np.array([le[inv == i].mean() for i in range(len(u))])
    within = np.sqrt(np.mean([le[inv == i].var() for i in range(len(u))]))
    return {"groups": int(len(u)), "std_of_group_means": float(means.std()), "mean_within_std": float(within),
            "group_mean_range": [float(means.min()), float(means.max())]}
res["by_cu"] = spread(cu)
res["by_cu_simd"] = spread(cu * 4 + simd)
res["by_xcc"] = spread(xcc)
res["overall_std"] = float(le.std())
print(json.dumps(res))
if len(sys.argv) > 3:
    np.save(sys.argv[3], np.stack([st, le, en, xcc.astype(np.float64), hwid.astype(np.float64)]))
