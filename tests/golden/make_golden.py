"""Generate golden outputs by running the REFERENCE program (oracle/_ref/findKmer_ref,
compiled from /root/reference/findKmer/src/findKmer.cpp by oracle/Makefile) on the
inputs in tests/golden/inputs.  Run in this container only (the GPU box has no
reference).  Outputs: tests/golden/cases/<case>/{csv|csv.sha256, stats, stdout,
stderr} and tests/golden/manifest.json.

stdout is captured through `stdbuf -oL`: the reference always dies in free() at
exit (findKmer.cpp:1370) and would otherwise lose its block-buffered stdout.
"""
import hashlib, json, os, shutil, subprocess, sys, tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "findKmer_ref")
INPUTS = os.path.join(HERE, "inputs")
CASES = os.path.join(HERE, "cases")
BIG = 200_000          # CSVs above this many bytes are stored as sha256 only

def cases():
    c = []
    for k in list(range(1, 13)) + [15, 20]:
        c.append((f"test_k{k}", "test.txt", ["-q", "1", "-k", str(k), "-p", "test.txt"]))
    c.append(("test_k6_q0", "test.txt", ["-q", "0", "-k", "6", "-p", "test.txt"]))
    c.append(("test_k0_default7", "test.txt", ["-q", "1", "-k", "0", "-p", "test.txt"]))
    c.append(("test_k6_export", "test.txt", ["-q", "1", "-k", "6", "-e", "myout.csv", "-p", "test.txt"]))
    c.append(("test_k6_badopt", "test.txt", ["-q", "1", "-x", "-k", "6", "-p", "test.txt"]))
    for k in (2, 3, 4):
        c.append((f"edge_k{k}", "edge.txt", ["-q", "1", "-k", str(k), "-p", "edge.txt"]))
    c.append(("rand_k5", "rand120k.fa", ["-q", "1", "-k", "5", "-p", "rand120k.fa"]))
    c.append(("rand_k6_z3", "rand120k.fa", ["-q", "1", "-k", "6", "-z", "3", "-p", "rand120k.fa"]))
    c.append(("rand_k8", "rand120k.fa", ["-q", "1", "-k", "8", "-p", "rand120k.fa"]))
    c.append(("rand_k4_z2", "rand120k.fa", ["-q", "1", "-k", "4", "-z", "2", "-p", "rand120k.fa"]))
    c.append(("rand_k11", "rand120k.fa", ["-q", "1", "-k", "11", "-p", "rand120k.fa"]))
    c.append(("missing_k3", "missing.txt", ["-q", "1", "-k", "3", "-p", "missing.txt"]))
    c.append(("ffbyte_k3", "ffbyte.bin", ["-q", "1", "-k", "3", "-p", "ffbyte.bin"]))
    c.append(("shortruns_k5", "shortruns.txt", ["-q", "1", "-k", "5", "-p", "shortruns.txt"]))
    c.append(("empty_k3", "empty.txt", ["-q", "1", "-k", "3", "-p", "empty.txt"]))
    # config 5 (k6thru11fullANDupstream.sh): an upstream-like FASTA
    # (tools/make_upstream.py upstream1m.fas 1e6 3), k = 6..11 with a z filter
    c.append(("up_k6", "upstream1m.fas", ["-q", "1", "-k", "6", "-p", "upstream1m.fas"]))
    c.append(("up_k7_q0", "upstream1m.fas", ["-q", "0", "-k", "7", "-p", "upstream1m.fas"]))
    for k in range(6, 12):
        c.append((f"up_k{k}_z3", "upstream1m.fas", ["-q", "1", "-k", str(k), "-z", "3", "-p", "upstream1m.fas"]))
    # 17 <= k <= 20: the sparse table
    c.append(("rand_k17", "rand120k.fa", ["-q", "1", "-k", "17", "-p", "rand120k.fa"]))
    c.append(("rand_k19_z4", "rand120k.fa", ["-q", "1", "-k", "19", "-z", "4", "-p", "rand120k.fa"]))
    c.append(("shortruns_k18", "shortruns.txt", ["-q", "1", "-k", "18", "-p", "shortruns.txt"]))
    c.append(("edge_k20", "edge.txt", ["-q", "1", "-k", "20", "-p", "edge.txt"]))
    c.append(("ffbyte_k17", "ffbyte.bin", ["-q", "1", "-k", "17", "-p", "ffbyte.bin"]))
    return c

def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    shutil.rmtree(CASES, ignore_errors=True)
    os.makedirs(CASES)
    manifest = {}
    for name, inp, args in cases():
        with tempfile.TemporaryDirectory() as td:
            shutil.copy(os.path.join(INPUTS, inp), os.path.join(td, inp))
            before = set(os.listdir(td))
            p = subprocess.run(["stdbuf", "-oL", REF] + args, cwd=td,
                               capture_output=True, timeout=300)
            produced = sorted(set(os.listdir(td)) - before)
            d = os.path.join(CASES, name)
            os.makedirs(d)
            entry = {"input": inp, "args": args, "exit": p.returncode, "files": {}}
            open(os.path.join(d, "stdout"), "wb").write(p.stdout)
            open(os.path.join(d, "stderr"), "wb").write(p.stderr)
            for f in produced:
                data = open(os.path.join(td, f), "rb").read()
                kind = "csv" if f.endswith(".csv") else "stats"
                rec = {"name": f, "bytes": len(data),
                       "sha256": hashlib.sha256(data).hexdigest()}
                if kind == "csv" and len(data) > BIG:
                    rec["stored"] = False
                else:
                    open(os.path.join(d, kind), "wb").write(data)
                    rec["stored"] = True
                entry["files"][kind] = rec
            manifest[name] = entry
            print(name, p.returncode, {k: v["bytes"] for k, v in entry["files"].items()})
    json.dump(manifest, open(os.path.join(HERE, "manifest.json"), "w"), indent=1, sort_keys=True)

if __name__ == "__main__":
    main()
