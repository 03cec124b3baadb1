"""Host-side cost of one engine step (reset / feed_device / finish) on a
1 GB device-resident synthetic stream: where the time between kernels goes."""
import time

import torch

import findkmer_amd as fk

n = 1 << 30
buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
fk.synth_device(buf.data_ptr(), n, n, 1, 0)
torch.cuda.synchronize()
eng = fk.Engine(6, device=0)
for _ in range(5):
    eng.reset(); eng.feed_device(buf.data_ptr(), n); eng.finish()
ts = {"reset": 0, "feed": 0, "finish": 0}
steps = 50
t0 = time.perf_counter_ns()
for _ in range(steps):
    a = time.perf_counter_ns(); eng.reset()
    b = time.perf_counter_ns(); eng.feed_device(buf.data_ptr(), n)
    c = time.perf_counter_ns(); eng.finish()
    d = time.perf_counter_ns()
    ts["reset"] += b - a; ts["feed"] += c - b; ts["finish"] += d - c
tot = (time.perf_counter_ns() - t0) / steps / 1e3
print("step %.1f us:" % tot, " ".join("%s %.1f" % (k, v / steps / 1e3) for k, v in ts.items()))
# raw ctypes call overhead
t = time.perf_counter_ns()
for _ in range(1000):
    fk.lib().fk_strerror(0)
print("ctypes call %.2f us" % ((time.perf_counter_ns() - t) / 1000 / 1e3))
