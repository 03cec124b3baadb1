"""Experiment build (never the product): the working tree's engine compiled
with extra -D macros (tuning constants guarded by #ifndef in fk_engine.hip),
as build/exp/libfk_<name>.so for an A/B run through FINDKMER_LIB
(scripts/gpu_ab.sh VARIANTS=<name>).

usage: python3 tools/exp_macro.py NAME -DMACRO=VALUE [...]    (run `make` first)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "build", "exp")
name, defs = sys.argv[1], sys.argv[2:]
assert all(d.startswith("-D") for d in defs), defs
os.makedirs(OUT, exist_ok=True)
inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "findkmer_amd", "csrc")]
flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-value"]
obj = os.path.join(OUT, f"{name}.o")
subprocess.run(["/opt/rocm/bin/hipcc", *flags, *inc, *defs, "-c", "-x", "hip",
                os.path.join(REPO, "findkmer_amd", "csrc", "fk_engine.hip"), "-o", obj], check=True)
b = os.path.join(REPO, "build")
lib = os.path.join(OUT, f"libfk_{name}.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, obj] +
               [os.path.join(b, f) for f in ("fk_sparse.o", "fk_ingest.o", "fk_comm.o", "fk_writer.o")] +
               ["-lpthread", "-ldl"], check=True)
print("built", lib)
