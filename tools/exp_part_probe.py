"""Experiment build (never the product): k_part with per-phase s_memtime
stamps, to see where a batch's time goes.

Writes build/exp/fk_engine_probe.hip (a copy of the engine with stamps
inserted), compiles it and links build/exp/libfk_probe.so against the
product's other objects (run `make` first).  tools/part_probe_run.py loads it
through FINDKMER_LIB and prints the phase shares.

Phases per batch (wave-level, lane 0 accumulates; one atomic per wave at
the end): tile = the fast-tile work of the batch's rounds (classification,
codes, loads issued), hist = issuing the (slice, lane bucket) count
atomics, bar1 = the barrier after them (includes draining the atomics),
scan_a = wave 0's slice scan (0 for the others), bar2, (scan_c, bar3 unused:
0), place = the placement atomics and code writes, bar4, out = the batch's
16-B pieces to HBM.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "findkmer_amd", "csrc", "fk_engine.hip")
OUT = os.path.join(REPO, "build", "exp")

STAMP = ('({ unsigned long long t_; __builtin_amdgcn_sched_barrier(0); '
         'asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); '
         '__builtin_amdgcn_sched_barrier(0); t_; })')


def patch(s):
    def rep(old, new, count=1):
        nonlocal s
        assert s.count(old) >= 1, old[:80]
        s = s.replace(old, new, count)

    # globals + reader
    rep('''template <bool PAIRS, bool MIX, uint32_t W>
__device__ __forceinline__ bool part_batch(''', '''__device__ unsigned long long g_pp[16];
#define PP_STAMP() ''' + STAMP + '''
extern "C" int fk_debug_part_phases(unsigned long long *out16) {
    if (out16 && hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_pp), sizeof(g_pp)) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pp), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
template <bool PAIRS, bool MIX, uint32_t W>
__device__ __forceinline__ bool part_batch(''')
    rep('''                                           uint32_t *cur, uint32_t *total, uint16_t *ent) {
    constexpr int NT = PART_TILES(PAIRS);''', '''                                           uint32_t *cur, uint32_t *total, uint16_t *ent,
                                           unsigned long long *pp) {
    constexpr int NT = PART_TILES(PAIRS);
    unsigned long long q0 = PP_STAMP();''')
    rep('''    /* (the barrier also tells whether any wave has tiles left) */
    const bool any_more = __syncthreads_or(more);''', '''    unsigned long long q1 = PP_STAMP();
    /* (the barrier also tells whether any wave has tiles left) */
    const bool any_more = __syncthreads_or(more);
    unsigned long long q2 = PP_STAMP();''')
    rep('''        if (lane == 63) *total = inc;
    }
    __syncthreads();''', '''        if (lane == 63) *total = inc;
    }
    unsigned long long q3 = PP_STAMP();
    __syncthreads();
    unsigned long long q4 = PP_STAMP();
    unsigned long long q5 = q4, q6 = q4;''')
    rep('''        if (haves[i]) part_entries<PAIRS, MIX>(f, mk, m1, sh, lowm, pg.npair, place);
    }
    __syncthreads();''', '''        if (haves[i]) part_entries<PAIRS, MIX>(f, mk, m1, sh, lowm, pg.npair, place);
    }
    unsigned long long q7 = PP_STAMP();
    __syncthreads();
    unsigned long long q8 = PP_STAMP();''')
    rep('''    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W)) dst[i] = src[i];
    return any_more;''', '''    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W)) dst[i] = src[i];
    unsigned long long q9 = PP_STAMP();
    pp[1] += q1 - q0; pp[2] += q2 - q1; pp[3] += q3 - q2; pp[4] += q4 - q3; pp[5] += q5 - q4;
    pp[6] += q6 - q5; pp[7] += q7 - q6; pp[8] += q8 - q7; pp[9] += q9 - q8; pp[10] += 1;
    return any_more;''')
    # k_part: accumulators, tile time, flush
    rep('''    Emit stash[NT];
    bool have_stash[NT];''', '''    Emit stash[NT];
    bool have_stash[NT];
    unsigned long long pp[16] = {};
    unsigned long long kt0 = PP_STAMP();''')
    rep('''#define FK_ROUND(X)                                                                  \\
    {                                                                                \\
        Emit em{0, 0, 0, 0, false, false, false};                                    \\''',
        '''#define FK_ROUND(X)                                                                  \\
    {                                                                                \\
        unsigned long long r0_ = PP_STAMP();                                         \\
        Emit em{0, 0, 0, 0, false, false, false};                                    \\''')
    rep('''        consume(X);                                                                  \\
        FK_LOADP(X, t + 2);                                                          \\
        {   /* static stash slots (no dynamic register indexing) */                 \\''',
        '''        consume(X);                                                                  \\
        FK_LOADP(X, t + 2);                                                          \\
        pp[0] += PP_STAMP() - r0_;                                                   \\
        {   /* static stash slots (no dynamic register indexing) */                 \\''')
    rep('''                                                          row0 + round / NT, hist, cur, &total, ent); \\''',
        '''                                                          row0 + round / NT, hist, cur, &total, ent, pp); \\''')
    rep('''#undef FK_ROUND
#undef FK_LOADP
    /* rows the block did not reach are empty */''', '''#undef FK_ROUND
#undef FK_LOADP
    pp[11] += PP_STAMP() - kt0;
    if (!RES && (threadIdx.x & 63) == 0)
        for (int i_ = 0; i_ < 12; i_++) atomicAdd(&g_pp[i_], pp[i_]);
    /* rows the block did not reach are empty */''')
    return s


def main():
    os.makedirs(OUT, exist_ok=True)
    src = patch(open(SRC).read())
    dst = os.path.join(OUT, "fk_engine_probe.hip")
    open(dst, "w").write(src)
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "findkmer_amd", "csrc")]
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-value",
             "-Wno-unused-variable"]
    obj = os.path.join(OUT, "probe.o")
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, *inc, "-c", "-x", "hip", dst, "-o", obj], check=True)
    b = os.path.join(REPO, "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(OUT, "libfk_probe.so"), obj] +
                   [os.path.join(b, f) for f in ("fk_sparse.o", "fk_ingest.o", "fk_comm.o", "fk_writer.o")] +
                   ["-lpthread", "-ldl"], check=True)
    print("built", os.path.join(OUT, "libfk_probe.so"))


if __name__ == "__main__":
    sys.exit(main())
