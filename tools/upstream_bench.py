"""Device-resident upstream-like FASTA (config 5, tools/make_upstream.py):
feed + finish time per k on the GPU, the step the CLI runs after ingest.
Usage: python tools/upstream_bench.py FILE [k ...]"""
import json
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import findkmer_amd as fk  # noqa: E402

path = sys.argv[1]
ks = [int(x) for x in sys.argv[2:]] or [6, 11]
out = {}
with fk.DeviceInput(path) as inp:
    for k in ks:
        with fk.Engine(k, collect_unknown=True) as e:
            ts = []
            for _ in range(4):
                e.reset()
                t0 = time.perf_counter()
                e.feed_device(inp.ptr, inp.len)
                rc, r = e.finish()
                ts.append(time.perf_counter() - t0)
            out[f"k{k}_ms"] = round(min(ts[1:]) * 1e3, 3)
            out[f"k{k}_bases_per_s"] = r.valid_bases / min(ts[1:])
out["bytes"] = inp.len
print(json.dumps(out))
