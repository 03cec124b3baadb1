"""Experiment builds (never the product): the engine with named source
patches, as build/exp/libfk_<name>.so for an A/B run through FINDKMER_LIB
(bench.py and findkmer_amd load it instead of the product library).

usage: python3 tools/exp_variant.py NAME [NAME ...]    (run `make` first)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "findkmer_amd", "csrc", "fk_engine.hip")
OUT = os.path.join(REPO, "build", "exp")

VARIANTS = {
    # k_part's batch write-out and k_bucket_count's code reads bypass the
    # caches' normal retention (the run-index lines stay in L2 longer)
    "nt": [
        ("    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W)) dst[i] = src[i];\n    return any_more;",
         "    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W))\n"
         "        __builtin_nontemporal_store(reinterpret_cast<const u32x4 *>(src)[i], reinterpret_cast<u32x4 *>(dst) + i);\n"
         "    return any_more;"),
    ],
    "ntread": [
        ("            for (int u = 0; u < BUCKET_U; u++) v[j][u] = q0 + 4 * u < q1 ? g4[q0 + 4 * u] : make_uint4(0, 0, 0, 0);",
         "            for (int u = 0; u < BUCKET_U; u++) { if (q0 + 4 * u < q1) { u32x4 t_ = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(g4) + q0 + 4 * u); v[j][u] = make_uint4(t_.x, t_.y, t_.z, t_.w); } else v[j][u] = make_uint4(0, 0, 0, 0); }"),
    ],
    # k_bucket_count: consecutive slices on one XCD (blocks b, b+8, .. share
    # an XCD), so the 128-B lines two neighbouring runs share hit its L2
    "xcd": [
        ("    const uint32_t b = blockIdx.x % pg.nslices, g = blockIdx.x / pg.nslices;\n    for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) slice[i] = 0;",
         "    const uint32_t b = groups == 1 && (pg.nslices & 7u) == 0 ? (blockIdx.x & 7u) * (pg.nslices >> 3) + (blockIdx.x >> 3)\n"
         "                                                       : blockIdx.x % pg.nslices;\n"
         "    const uint32_t g = blockIdx.x / pg.nslices;\n"
         "    for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) slice[i] = 0;"),
    ],
    # k_bucket_count's first loads per quad: rows x 16-B pieces per lane
    "u4r3": [("#define BUCKET_U 5", "#define BUCKET_U 4"), ("#define BUCKET_ROWS 2", "#define BUCKET_ROWS 3")],
    "u6": [("#define BUCKET_U 5", "#define BUCKET_U 6")],
    "u3r4": [("#define BUCKET_U 5", "#define BUCKET_U 3"), ("#define BUCKET_ROWS 2", "#define BUCKET_ROWS 4")],
    # k_bucket_count without the XCD-aware slice order
    "noxcd": [
        ("    const uint32_t b = groups == 1 && (pg.nslices & 7u) == 0 ? (bx & 7u) * (pg.nslices >> 3) + (bx >> 3)\n"
         "                                                           : bx % pg.nslices;",
         "    const uint32_t b = bx % pg.nslices;"),
    ],
}


def build(name):
    src = open(SRC).read()
    for part in name.split("+"):
        for old, new in VARIANTS[part]:
            assert src.count(old) == 1, (part, old[:80])
            src = src.replace(old, new)
    os.makedirs(OUT, exist_ok=True)
    dst = os.path.join(OUT, f"fk_engine_{name}.hip")
    open(dst, "w").write(src)
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "findkmer_amd", "csrc")]
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics"]
    obj = os.path.join(OUT, f"{name}.o")
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, *inc, "-c", "-x", "hip", dst, "-o", obj], check=True)
    b = os.path.join(REPO, "build")
    lib = os.path.join(OUT, f"libfk_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, obj] +
                   [os.path.join(b, f) for f in ("fk_sparse.o", "fk_ingest.o", "fk_comm.o", "fk_writer.o")] +
                   ["-lpthread", "-ldl"], check=True)
    print("built", lib)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
