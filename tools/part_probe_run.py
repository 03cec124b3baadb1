"""Run the k_part phase probe (tools/exp_part_probe.py's build/exp/libfk_probe.so)
on the bench's genome and print where a batch's time goes.

usage: python3 tools/part_probe_run.py [k] [bases] [fasta_line]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FINDKMER_LIB", os.path.join(REPO, "build", "exp", "libfk_probe.so"))
sys.path.insert(0, REPO)


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10_000_000_000
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 80
    import torch
    import findkmer_amd as fk
    import bench
    torch.cuda.set_device(0)
    buf, size = bench.make_genome(n, L, 2, bench.CHROM if n > bench.CHROM else 0)
    torch.cuda.synchronize()
    L_ = fk.lib()
    L_.fk_debug_part_phases.argtypes = [ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 16)()
    with fk.Engine(k) as e:
        for _ in range(2):
            e.reset()
            e.feed_device(buf.data_ptr(), size)
            e.finish()
        L_.fk_debug_part_phases(out)   # reset
        reps = 3
        ms = 0.0
        for _ in range(reps):
            e.reset()
            e.feed_device(buf.data_ptr(), size)
            rc, r = e.finish()
            ms += r.main_kernel_ms
        L_.fk_debug_part_phases(out)
    names = ["tile", "hist", "bar1", "scan_a", "bar2", "scan_c", "bar3", "place", "bar4", "out"]
    v = [out[i] for i in range(12)]
    batches = v[10]
    tot = sum(v[:10])
    print(f"k={k} bases={n} L={L}: k_part {ms / reps:.3f} ms per launch; wave-batches {batches}")
    for i, nm in enumerate(names):
        print(f"  {nm:6s} {v[i] / max(1, batches):10.0f} cycles/batch  {100.0 * v[i] / max(1, tot):5.1f} %")
    print(f"  loop total (kt) {v[11] / max(1, batches):10.0f} cycles/batch")


if __name__ == "__main__":
    main()
