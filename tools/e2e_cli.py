"""End-to-end ./findKmer timings on an upstream-like FASTA (SURVEY.md §8(d)
cfg 5, k6thru11fullANDupstream.sh's `-q 1 -k K -z 100` runs): device-
resident ingest vs the streamed path, and `--sweep 11` vs six separate runs.
Usage: python tools/e2e_cli.py BYTES OUT.json"""
import json
import os
import shutil
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, cwd, env=None):
    e = dict(os.environ)
    e.update(env or {})
    t0 = time.perf_counter()
    p = subprocess.run([os.path.join(REPO, "findKmer")] + args, cwd=cwd, env=e,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=600)
    dt = time.perf_counter() - t0
    assert p.returncode == 0, p.stderr[-2000:]
    return dt


def main():
    nbytes = int(float(sys.argv[1]))
    out = sys.argv[2]
    work = os.path.join(os.environ.get("TMPDIR", "/tmp"), "fk_e2e")
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    name = "upstream.fas"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "make_upstream.py"),
                    os.path.join(work, name), str(nbytes)], check=True)
    size = os.path.getsize(os.path.join(work, name))
    res = {"input": f"upstream-like FASTA, {size} bytes (tools/make_upstream.py, page-cache resident)",
           "bytes": size}
    run(["-q", "1", "-k", "6", "-z", "100", "-p", name], work)   # warm (context, page cache)
    for k in (6, 11):
        res[f"k{k}_device_ingest_s"] = run(["-q", "1", "-k", str(k), "-z", "100", "-p", name], work)
        res[f"k{k}_stream_ingest_s"] = run(["-q", "1", "-k", str(k), "-z", "100", "-p", name], work,
                                           {"FINDKMER_INGEST": "stream"})
    res["sweep_6_11_s"] = run(["-q", "1", "-k", "6", "-z", "100", "--sweep", "11", "-p", name], work)
    res["separate_6_11_s"] = sum(run(["-q", "1", "-k", str(k), "-z", "100", "-p", name], work)
                                 for k in range(6, 12))
    shutil.rmtree(work, ignore_errors=True)
    print(json.dumps(res))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
