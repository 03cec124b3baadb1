"""Experiment build (never the product): the engine as of a git revision, as
build/exp/libfk_<name>.so, for an interleaved A/B against the working tree
through FINDKMER_LIB (scripts/gpu_ab.sh VARIANTS=<name>).

usage: python3 tools/exp_rev.py REV NAME    (run `make` first: the other
objects -- sparse, ingest, comm, writer -- come from the working tree)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "build", "exp")

rev, name = sys.argv[1], sys.argv[2]
os.makedirs(OUT, exist_ok=True)
src = subprocess.run(["git", "-C", REPO, "show", f"{rev}:findkmer_amd/csrc/fk_engine.hip"], check=True,
                     capture_output=True, text=True).stdout
dst = os.path.join(OUT, f"fk_engine_{name}.hip")
open(dst, "w").write(src)
inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "findkmer_amd", "csrc")]
flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-value"]
obj = os.path.join(OUT, f"{name}.o")
subprocess.run(["/opt/rocm/bin/hipcc", *flags, *inc, "-c", "-x", "hip", dst, "-o", obj], check=True)
b = os.path.join(REPO, "build")
lib = os.path.join(OUT, f"libfk_{name}.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, obj] +
               [os.path.join(b, f) for f in ("fk_sparse.o", "fk_ingest.o", "fk_comm.o", "fk_writer.o")] +
               ["-lpthread", "-ldl"], check=True)
print("built", lib)
