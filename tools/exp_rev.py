"""Experiment build (never the product): the engine as of a git revision, as
build/exp/libfk_<name>.so, for an interleaved A/B against the working tree
through FINDKMER_LIB (scripts/gpu_ab.sh VARIANTS=<name>).

usage: python3 tools/exp_rev.py REV NAME    (run `make` first: the other
objects -- sparse, ingest, comm, writer -- come from the working tree;
REV must hold the split engine sources, fk_engine_internal.h and its TUs)
"""
import subprocess
import sys

from exp_variant import build_tree

rev, name = sys.argv[1], sys.argv[2]
listing = subprocess.run(["git", "ls-tree", "--name-only", rev, "findkmer_amd/csrc/"], check=True,
                         capture_output=True, text=True).stdout.split()
files = {}
for path in listing:
    if path.endswith((".hip", ".h")):
        files[path.rsplit("/", 1)[1]] = subprocess.run(["git", "show", f"{rev}:{path}"], check=True,
                                                        capture_output=True, text=True).stdout
build_tree(name, files)
