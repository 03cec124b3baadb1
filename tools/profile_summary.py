"""Turn one scripts/gpu_profile.sh run into the committed profile artefacts
under profiles/:

  profiles/<tag>_kernel_stats.csv          rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_summary.json              per-kernel average durations, the PMC
                                           HBM bytes of the dominant kernel per launch
  profiles/traffic_k<K>_L<L>_n<B>.json     what bench.py reports as roofline.traffic
                                           for the workload of B input bytes

The dominant kernel is matched by its exact template prefix: the main k_part
pass `k_part<true, false` (8 <= k <= 12) / `k_part<false, false` (k = 13;
not the k_part<.., true> resume launches) or `k_count<` (k <= 7 and
14 <= k <= 16).

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE
(KiB) is doubled on gfx950 for 16-B-per-lane streaming reads, WRITE_SIZE (KiB)
is taken as is; each comes from its own --pmc pass.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("src", nargs="?", default="gpurun_out/prof")
ap.add_argument("tag", nargs="?", default="r03_k11_L80")
ap.add_argument("--k", type=int, default=11)
ap.add_argument("--fasta-line", type=int, default=80)
ap.add_argument("--input-bytes", type=int, required=True, help="input bytes per launch (bench.py's input_bytes_per_gpu)")
ap.add_argument("--kernel", default=None, help="template prefix of the dominant kernel")
ap.add_argument("--stats-csv", default=None,
                help="a committed rocprofv3 kernel_stats.csv instead of <src>/trace (re-summarise an old profile)")
ap.add_argument("--steps", type=int, default=0,
                help="steps the trace covers (warmup included): adds per-step milliseconds per kernel")
ap.add_argument("--merge", default=None, help="keep the fields of this older summary JSON that this run does not set")
args = ap.parse_args()
src, tag, k, L = args.src, args.tag, args.k, args.fasta_line
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(repo, "profiles")
os.makedirs(out, exist_ok=True)

# k_part's template: <PAIRS, RES, W>; pairs mode for k <= 12, single windows for k = 13..16
main = args.kernel or ("k_part<true, false" if 8 <= k <= 12 else "k_part<false, false" if 13 <= k <= 16
                       else "k_count<")
main_short = main.split("<")[0]


def is_main(name):
    return name.replace("void ", "", 1).startswith(main)


def counter(pass_dir, name):
    vals = []
    for f in glob.glob(os.path.join(src, pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if is_main(r["Kernel_Name"]) and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


def counter_by_kernel(pass_dir, name):
    """{kernel name (no arguments): total counter value over its launches}"""
    tot = {}
    for f in glob.glob(os.path.join(src, pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                kn = r["Kernel_Name"].split("(")[0].replace("void ", "", 1)
                tot[kn] = tot.get(kn, 0.0) + float(r["Counter_Value"])
    return tot


def label(full):
    """A short readable name.  Not a key: C++ names hold parentheses inside
    their template arguments (rocPRIM's `(target_arch)950`, `(anonymous
    namespace)`), so cutting at the first '(' made different kernels collide
    (round-4 sparse summaries).  The key is the full name."""
    n = full.replace("void ", "", 1)
    if "rocprim" in n:
        for what in ("radix_sort_onesweep_iteration", "onesweep_histograms", "radix_sort_block_sort",
                     "radix_sort_onesweep", "radix_sort", "reduce_by_key_init", "reduce_by_key", "run_length_encode",
                     "trivial_runs", "merge_sort", "scan", "reduce", "transform"):
            if what in n:
                return "rocprim::" + what
        return "rocprim::" + n.split("<")[0].split("::")[-1]
    n = n.replace("(anonymous namespace)::", "")
    depth, out_ = 0, []
    for ch in n:   # cut at the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out_.append(ch)
    return "".join(out_)


stats = [args.stats_csv] if args.stats_csv else glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"),
                                                           recursive=True)
summary = {"tag": tag, "k": k, "fasta_line": L, "input_bytes": args.input_bytes, "main_kernel": main,
           "kernels": {}}
if stats:
    dst_csv = os.path.join(out, f"{tag}_kernel_stats.csv")
    if os.path.abspath(stats[0]) != os.path.abspath(dst_csv):
        shutil.copy(stats[0], dst_csv)
    total_ns = 0.0
    for r in csv.DictReader(open(stats[0])):
        full = r["Name"]
        assert full not in summary["kernels"], full
        rec = {"label": label(full), "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
               "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
               "total_ms": float(r["TotalDurationNs"]) / 1e6}
        total_ns += float(r["TotalDurationNs"])
        if args.steps:
            rec["ms_per_step"] = rec["total_ms"] / args.steps
        summary["kernels"][full] = rec
    summary["csv_total_ms"] = total_ns / 1e6
    by_label = {}
    for rec in summary["kernels"].values():
        by_label[rec["label"]] = by_label.get(rec["label"], 0.0) + rec["total_ms"]
    summary["total_ms_by_label"] = dict(sorted(by_label.items(), key=lambda kv: -kv[1]))
    if args.steps:
        summary["steps_traced"] = args.steps
        summary["ms_per_step_by_label"] = {n: v / args.steps for n, v in summary["total_ms_by_label"].items()}
    # the per-kernel totals must add up to the CSV's (no kernel lost to a key collision)
    assert abs(sum(r["total_ms"] for r in summary["kernels"].values()) - summary["csv_total_ms"]) \
        <= 0.05 * summary["csv_total_ms"] + 1e-9
fetch = counter("pmc1", "FETCH_SIZE")
write = counter("pmc2", "WRITE_SIZE")
if fetch and write:
    f_kib = statistics.mean(fetch)
    w_kib = statistics.mean(write)
    hbm = f_kib * 1024 * 2 + w_kib * 1024
    summary[main_short + "_pmc"] = {"launches": len(fetch), "fetch_size_kib": f_kib, "write_size_kib": w_kib,
                                    "hbm_bytes_per_launch": hbm}
    # the whole step: every kernel's bytes (the generator's excepted) per
    # launch of the main kernel (one per step)
    fk_, wk_ = counter_by_kernel("pmc1", "FETCH_SIZE"), counter_by_kernel("pmc2", "WRITE_SIZE")
    per_kernel = {}
    for kn in sorted(set(fk_) | set(wk_)):
        if kn.startswith("k_synth"):
            continue
        per_kernel[kn] = (fk_.get(kn, 0.0) * 2 + wk_.get(kn, 0.0)) * 1024 / len(fetch)
    step = sum(per_kernel.values())
    summary["step_pmc"] = {"hbm_bytes_per_step": step, "per_kernel_bytes_per_step": per_kernel}
    json.dump({"kernel": main_short, "kernel_template": main, "k": k, "fasta_line": L,
               "input_bytes": args.input_bytes, "hbm_bytes_per_launch": hbm,
               "hbm_bytes_per_step": step, "per_kernel_bytes_per_step": per_kernel,
               "fetch_size_kib": f_kib, "write_size_kib": w_kib, "launches": len(fetch),
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                         f"(k={k}, fasta_line={L}, {args.input_bytes} input bytes); bytes = 2*FETCH_SIZE*1024 "
                         "(gfx950 streaming-read correction, MI355X_MICROARCH.md) + WRITE_SIZE*1024, "
                         f"mean per launch of the kernels named {main}...",
               "source": tag},
              open(os.path.join(out, f"traffic_k{k}_L{L}_n{args.input_bytes}.json"), "w"), indent=1)
for p in ("pmc3", "pmc4", "pmc5"):
    for f in glob.glob(os.path.join(src, p, "**", "*counter_collection.csv"), recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if is_main(r["Kernel_Name"]):
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        summary.setdefault(main_short + "_sq", {}).update({n: statistics.mean(v) for n, v in agg.items()})
if args.merge:
    for key, v in json.load(open(args.merge)).items():
        if key not in summary and key not in ("kernels_ms_per_step", "calls"):
            summary[key] = v
json.dump(summary, open(os.path.join(out, f"{tag}_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1)[:3000])
