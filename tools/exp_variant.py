"""Experiment builds (never the product): the engine with named source
patches, as build/exp/libfk_<name>.so for an A/B run through FINDKMER_LIB
(bench.py and findkmer_amd load it instead of the product library).  Each
patch applies to whichever source file of findkmer_amd/csrc holds its text.
The ablations of the sparse passes (round 5: no key stores, no counting, no
look-back, no output, no sort) live here, not as #ifdefs in the product.

usage: python3 tools/exp_variant.py NAME [NAME ...]    (run `make` first)

Each variant's patches target the source as it was when that experiment ran
(DESIGN.md records the outcomes); later edits can make an old one fail to
apply, which the build reports.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "findkmer_amd", "csrc")
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
    "u4": [("#define BUCKET_U 5", "#define BUCKET_U 4")],
    "u3": [("#define BUCKET_U 5", "#define BUCKET_U 3")],
    "r1": [("#define BUCKET_ROWS 2", "#define BUCKET_ROWS 1")],
    "r1u8": [("#define BUCKET_U 5", "#define BUCKET_U 8"), ("#define BUCKET_ROWS 2", "#define BUCKET_ROWS 1")],
    "u3r4": [("#define BUCKET_U 5", "#define BUCKET_U 3"), ("#define BUCKET_ROWS 2", "#define BUCKET_ROWS 4")],
    # k_bucket_count without the XCD-aware slice order
    "noxcd": [
        ("    const uint32_t b = groups == 1 && (pg.nslices & 7u) == 0 ? (bx & 7u) * (pg.nslices >> 3) + (bx >> 3)\n"
         "                                                           : bx % pg.nslices;",
         "    const uint32_t b = bx % pg.nslices;"),
    ],
    # k_bucket_count: the run bounds of a 16-B piece as an 8-bit mask (32-bit
    # arithmetic once per piece instead of two 64-bit compares per code)
    "mask8": [
        ("""        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const uint64_t at = q * 8 + h;
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            if (SPLIT) {   /* k = 14: this block's half of the slice */
                if (at >= s0 && at < s1 && (c >> binsh) == half) atomicAdd(&slice[c & (nb - 1u)], 1u);
            } else {
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if (at >= s0 && at < s1) atomicAdd(&slice[a], 1u);
            }
        }""",
         """        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const uint64_t q8 = q * 8;
        const uint32_t lo = s0 > q8 ? (uint32_t)min(s0 - q8, (uint64_t)8) : 0u;
        const uint32_t hi = s1 > q8 ? (uint32_t)min(s1 - q8, (uint64_t)8) : 0u;
        const uint32_t m = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            const bool in = (m >> h) & 1u;
            if (SPLIT) {   /* k = 14: this block's half of the slice */
                if (in && (c >> binsh) == half) atomicAdd(&slice[c & (nb - 1u)], 1u);
            } else {
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if (in) atomicAdd(&slice[a], 1u);
            }
        }"""),
    ],
    # k_part: four tiles in flight per wave instead of three (the batch's
    # barriers wait on the slowest wave's loads)
    "pre4": [
        ("    uint32_t A[8] = {}, B[8] = {}, C[8] = {};\n    asm volatile(\"\" ::: \"memory\");\n    FK_LOADP(A, t);",
         "    uint32_t A[8] = {}, B[8] = {}, C[8] = {}, D[8] = {};\n    asm volatile(\"\" ::: \"memory\");\n    FK_LOADP(A, t);"),
        ("    FK_LOADP(C, t + 2);\n    /* entering state: the known stream state for chunk 0, else a guess from\n       the halo (k_scan checks it",
         "    FK_LOADP(C, t + 2);\n    asm volatile(\"\" ::: \"memory\");\n    FK_LOADP(D, t + 3);\n    /* entering state: the known stream state for chunk 0, else a guess from\n       the halo (k_scan checks it"),
        ("        FK_LOADP(X, t + 2);                                                          \\\n        {   /* static stash slots",
         "        FK_LOADP(X, t + 3);                                                          \\\n        {   /* static stash slots"),
        ("        FK_ROUND(A);\n        FK_ROUND(B);\n        FK_ROUND(C);\n    }\n#undef FK_ROUND\n#undef FK_LOADP\n    /* rows the block",
         "        FK_ROUND(A);\n        FK_ROUND(B);\n        FK_ROUND(C);\n        FK_ROUND(D);\n    }\n#undef FK_ROUND\n#undef FK_LOADP\n    /* rows the block"),
    ],
    # ablations of the pipelined k_part (timing only: the counts are wrong):
    # no placement of the stashed batch, no histogram atomics, no write-out
    "noplace": [
        ("            if (hold_) part_entries<PAIRS, false>(old_, mk, m1, pg.sh, lowm, pg.npair, place); \\\n",
         "            if (hold_) keep(old_.AC ^ old_.A2 ^ old_.BC ^ old_.B2);                  \\\n"),
    ],
    "nohist": [
        ("            if (have) part_entries<PAIRS, false>(em, mk, m1, pg.sh, lowm, pg.npair,   \\\n"
         "                                                 [&](uint32_t b_, uint32_t) { atomicAdd(&hist[b_], 1u); }); \\\n",
         "            if (have) keep(em.AC ^ em.A2 ^ em.BC ^ em.B2);                          \\\n"),
    ],
    "noout": [
        ("    for (uint32_t i = t0; i < n8; i += nt) dst[i] = src[i];\n}",
         "    if (total == 0xFFFFFFFFu) for (uint32_t i = t0; i < n8; i += nt) dst[i] = src[i];\n}"),
    ],
    # k_bucket_count without its LDS atomics (timing only): what the run
    # reads alone cost
    "bk_noadd": [
        ("                if (at >= s0 && at < s1) atomicAdd(&slice[a], 1u);",
         "                if (at >= s0 && at < s1) sink ^= a;"),
        ("    constexpr uint32_t QL = 4u;   /* lanes per run */",
         "    uint32_t sink = 0;\n    constexpr uint32_t QL = 4u;   /* lanes per run */"),
        ("    __syncthreads();\n    if (pg.pairs) {\n        /* pairs mode: the slice's bins",
         "    if (sink == 0x12345u) slice[0] = sink;\n    __syncthreads();\n    if (pg.pairs) {\n        /* pairs mode: the slice's bins"),
    ],
    # k = 11 through smaller k_part blocks (2 x 8 or 4 x 4 waves per CU, 512
    # slices each): fewer waves per barrier, shorter runs for k_bucket_count
    "k11w8": [
        ("static uint32_t part_waves_of(const fk_engine *e) { return e->k >= 11 ? 16u : 8u; }",
         "static uint32_t part_waves_of(const fk_engine *e) { return e->k == 11 ? 8u : e->k >= 11 ? 16u : 8u; }"),
        ("    if (e->part) max_waves = (uint64_t)e->cus * part_waves_of(e) * (part_waves_of(e) >= 16u ? 1u : 2u);",
         "    if (e->part) max_waves = (uint64_t)e->cus * 16u;"),
        ("                            : (pairs ? k_part<true, false, 8u, PART_SM(8u), false, true>",
         "                            : (pairs ? (k == 11 ? k_part<true, false, 8u, 512u, false, true, 11u> : k_part<true, false, 8u, PART_SM(8u), false, true>)"),
        ("                               : (pairs ? k_part<true, true, 8u> : k_part<false, true, 8u>);",
         "                               : (pairs ? (k == 11 ? k_part<true, true, 8u, 512u> : k_part<true, true, 8u>) : k_part<false, true, 8u>);"),
    ],
    "k11w4": [
        ("static uint32_t part_waves_of(const fk_engine *e) { return e->k >= 11 ? 16u : 8u; }",
         "static uint32_t part_waves_of(const fk_engine *e) { return e->k == 11 ? 4u : e->k >= 11 ? 16u : 8u; }"),
        ("    if (e->part) max_waves = (uint64_t)e->cus * part_waves_of(e) * (part_waves_of(e) >= 16u ? 1u : 2u);",
         "    if (e->part) max_waves = (uint64_t)e->cus * 16u;"),
        ("    auto kmain = c32 ? k_part<false, false, 16u, PART_SM(16u), true>",
         "    auto kmain = W == 4u ? k_part<true, false, 4u, 512u, false, true, 11u> : c32 ? k_part<false, false, 16u, PART_SM(16u), true>"),
        ("        auto kres = c32 ? k_part<false, true, 16u, PART_SM(16u), true>",
         "        auto kres = W == 4u ? k_part<true, true, 4u, 512u> : c32 ? k_part<false, true, 16u, PART_SM(16u), true>"),
    ],
    # chunked codes: the write-out without its global stores (timing only)
    "ch_nostore": [
        ("                    codes[p < n1 ? (uint64_t)d1 + p : (uint64_t)d2 + (p - n1)] = x;",
         "                    if (x.x == 0x12345678u && x.y == 0x9abcdef0u) codes[p < n1 ? (uint64_t)d1 + p : (uint64_t)d2 + (p - n1)] = x;"),
    ],
    # sparse passes (round 5 ablations, timing only): k_sp_emit without its
    # key stores; k_kp_count without counting; the chained scan's look-back
    # skipped; no run output; k_kp_sort without sorting
    "spx_nostore": [
        ("            if (at < em.ps[i].cap) {", "            if (at < em.ps[i].cap && v == ~0ull - 1) {"),
        ("                if (at < ps.cap) {", "                if (at < ps.cap && v == ~0ull - 1) {"),
    ],
    "kpx_nocnt": [
        ("            if (hsel < 0) atomicAdd(&bins[b >> 1], 1u << ((b & 1u) << 4));",
         "            if (hsel < -1) atomicAdd(&bins[b >> 1], 1u << ((b & 1u) << 4));"),
        ("        if (sa != (unsigned long long)m.n) {", "        if (sa == ~0ull) {"),
    ],
    "kpx_nolb": [
        ("        const unsigned long long pre = chain_prefix(flags, blk, total, err);\n        if (lane == 0) {\n            bprefix = pre;\n            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;\n        }\n    }\n    /* the nearest",
         "        const unsigned long long pre = 0;\n        if (lane == 0) {\n            bprefix = pre;\n            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;\n        }\n    }\n    /* the nearest"),
    ],
    "kpx_noout": [
        ("        for (uint32_t i = t; i < nr; i += 1024u) {\n            __builtin_nontemporal_store(",
         "        for (uint32_t i = t; i < nr && total == ~0u; i += 1024u) {\n            __builtin_nontemporal_store("),
    ],
    "kpx_nosort": [
        ("        if (nb > 1u && nb <= 16u) {", "        if (nb > 1u && nb <= 16u && nb == 99u) {"),
        ("        if (nb <= 64) wave_sort_bucket<1>(keys + b0, nb);", "        if (nb != 99u) continue;\n        if (nb <= 64) wave_sort_bucket<1>(keys + b0, nb);"),
    ],
    # k_repart (round 6, span-streamed; timing only): no pass B; pass B
    # without its write-out
    "rp_nob": [
        ("    /* pass B: each round counted by part,",
         "    if (nrows != 0xFFFFFFFFu) return;\n    /* pass B: each round counted by part,"),
    ],
    "rp_noout": [
        ("                    for (uint32_t j = lane; j < n; j += 64u) dst[j] = rbuf[o + j];",
         "                    for (uint32_t j = lane; j < n && n == 0xFFFFFFFFu; j += 64u) dst[j] = rbuf[o + j];"),
    ],
    "rpa_noatom": [
        ("                        if (rn) atomicAdd(&cnt[rp], rn);", "                        if (rn == 0xFFFFFFu) atomicAdd(&cnt[rp], rn);"),
        ("                if (rn) atomicAdd(&cnt[rp], rn);\n            }\n        }",
         "                if (rn == 0xFFFFFFu) atomicAdd(&cnt[rp], rn);\n            }\n        }"),
    ],
    "rp_noplace": [
        ("                    if (i == 0 || part[i] != part[i - 1]) at = atomicAdd(&cur[part[i]], len[i]);",
         "                    if (i == 0) at = t * 16u + len[i] * 0u;"),
    ],
    # the source as it is (an A/B baseline built before a product edit)
    "base": [],
    # k = 17's passes through k_repart<uint16_t, 8> (8 coarse slices a block: 512-B row spans, 64-B part segments)
    "rp17g8": [
        ("    hipLaunchKernelGGL(k_repart<uint16_t>, dim3(2048u / REPART_G), dim3(1024), 0, e->stream, pg, e->d_parts, alloc,\n                       meta, (uint64_t)e->parts_cap, alloc + 1, 15u, nullptr);",
         "    hipLaunchKernelGGL((k_repart<uint16_t, 8u>), dim3(2048u / 8u), dim3(1024), 0, e->stream, pg, e->d_parts, alloc,\n                       meta, (uint64_t)e->parts_cap, alloc + 1, 15u, nullptr);"),
    ],
    # k = 15 through k_repart<uint16_t, 4> (two blocks per CU) instead of 8 slices a block
    "k15g4": [
        ("        if (pg.split <= 4)\n", "        if (pg.split <= 3)\n"),
    ],
}


ENGINE_TUS = ("fk_engine", "fk_scan", "fk_part", "fk_part_pipe", "fk_part_res", "fk_sparse_pass", "fk_exchange")


def build_tree(name, files):
    """compile the engine's translation units from `files` ({file name:
    text}, every file of findkmer_amd/csrc) into build/exp/libfk_<name>.so,
    linked with the working tree's other objects (sparse, ingest, comm,
    writer: run `make` first)"""
    d = os.path.join(OUT, name)
    os.makedirs(d, exist_ok=True)
    for fn, text in files.items():
        open(os.path.join(d, fn), "w").write(text)
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + d]
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-value"]
    procs = [subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, *inc, "-c", "-x", "hip", os.path.join(d, t + ".hip"),
                               "-o", os.path.join(d, t + ".o")]) for t in ENGINE_TUS]
    assert all(p.wait() == 0 for p in procs), "compile failed"
    b = os.path.join(REPO, "build")
    lib = os.path.join(OUT, f"libfk_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] +
                   [os.path.join(d, t + ".o") for t in ENGINE_TUS] +
                   [os.path.join(b, f) for f in ("fk_sparse.o", "fk_ingest.o", "fk_comm.o", "fk_writer.o")] +
                   ["-lpthread", "-ldl"], check=True)
    print("built", lib)


def sources():
    return {fn: open(os.path.join(CSRC, fn)).read() for fn in os.listdir(CSRC)
            if fn.endswith((".hip", ".h"))}


def build(name):
    files = sources()
    for part in name.split("+"):
        for old, new in VARIANTS[part]:
            hits = [fn for fn, text in files.items() if old in text]
            assert len(hits) == 1 and files[hits[0]].count(old) == 1, (part, old[:80], hits)
            files[hits[0]] = files[hits[0]].replace(old, new)
    build_tree(name, files)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
