import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    # torch bundles its own HIP runtime: it must initialise before
    # libfindkmer_hip.so does (see findkmer_amd.lib()).  Only when a GPU run
    # is requested: the CPU suite never touches HIP.
    if "not gpu" not in (config.getoption("-m") or ""):
        try:
            import torch
            torch.cuda.is_available()
        except Exception:
            pass


@pytest.fixture(scope="session")
def manifest():
    return json.load(open(os.path.join(GOLD, "manifest.json")))


def golden_input(name):
    return open(os.path.join(GOLD, "inputs", name), "rb").read()


def golden_file(case, kind):
    p = os.path.join(GOLD, "cases", case, kind)
    return open(p, "rb").read() if os.path.exists(p) else None


def case_k(entry):
    a = entry["args"]
    k = int(a[a.index("-k") + 1]) if "-k" in a else 0
    return k if k else 7   # k=0 selects DEFAULT_K_VALUE (findKmer.cpp:263-265)


def case_z(entry):
    a = entry["args"]
    return (1, float(int(a[a.index("-z") + 1]))) if "-z" in a else (0, 0.0)
