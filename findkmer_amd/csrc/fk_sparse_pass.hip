/*
 * fk_sparse_pass.hip -- 17 <= k <= 20 (findKmer.cpp:429-445, :663-690): the
 * sparse table built at finish by key-range passes over the retained input
 * (k_sp_emit or k_sp_wpart, then per pass k_kpart + k_repart + k_kp_cnt2 /
 * k_kp_sort), and
 * the sparse-table C-ABI (fk_engine_sparse*).
 */
#include "fk_engine_internal.h"

/*
 * 17 <= k <= 20: the table is built at finish by key-range passes over the
 * input the engine retained (1 byte per input byte, plus every range's exact
 * entering state from the feed's k_scan), never by materialising a slot per
 * byte.  k_sp_emit walks every range from its exact state, one 2 KiB tile at
 * a time, with tile_general -- the same per-byte rules as every other count
 * (findKmer.cpp:962-1069) -- writing each byte's window index (reference
 * order, :719-724) or short walk (:1059-1062) into the wave's LDS slots, and
 * then, per mode:
 *   SP_HIST  every window's bucket (key >> shift) into an LDS histogram
 *            (flushed with one atomic per bucket and block), every short
 *            walk to a global list;
 *   SP_KEYS  the windows with lo <= key < hi to a compact global list (one
 *            atomic per tile and wave for the space, ballot-ordered writes),
 *            and the short walks too when one pass takes every window (the
 *            feed counted them; no SP_HIST launch then);
 *   SP_DENSE the windows with lo <= key < hi counted in a dense u64 table
 *            (one bucket too large for a sorted pass: few distinct keys).
 */
/* SP_KEYS: one key range [lo, hi) of a walk and its list */
#define SP_MAXP 4u                  /* key ranges (passes) one SP_KEYS walk emits (round 5) */
struct SpPass {
    uint64_t lo, hi;
    uint64_t *out;                  /* the keys, or */
    uint32_t *out32;                /* ... (a range of <= 2^32 keys) key - lo as 32 bits */
    uint64_t cap;                   /* slots of the list */
    unsigned long long *ctr;        /* [0] slots claimed (whole SP_CHUNKs), [1] windows written (the rest: pads) */
};
struct SpEmit {
    int mode;
    uint32_t shift;                 /* bucket of a key: key >> shift */
    uint64_t lo, hi;                /* SP_DENSE: the key range [lo, hi) */
    unsigned long long *bhist;      /* SP_HIST: window count per bucket */
    uint32_t nbuckets;
    uint64_t *shorts;               /* SP_HIST: the short walks */
    unsigned long long *nshort;
    uint64_t short_cap;
    uint32_t np;                    /* SP_KEYS: the walk's key ranges, ascending (unused: lo = ~0) */
    uint64_t gend;                  /* ... the last range's hi */
    SpPass ps[SP_MAXP];
    unsigned long long *dense;      /* SP_DENSE: count of key lo + i */
};
enum { SP_HIST = 1, SP_KEYS = 2, SP_DENSE = 3 };
#define SP_WAVES 4u
#define SP_BUCKET_BITS 12u
/* SP_KEYS output: each wave claims SP_CHUNK slots at a time from the pass's
   counter and fills them in order; the unfilled end of its last chunk holds
   pads (4^k - 1, the largest key -- 0xFFFFFFFF in a 32-bit pass -- so the
   sort puts them last, and their number is taken off the last run).  Round 4: one claim per
   tile and wave -- 5 M same-address atomics per 10 GB pass -- made each keys
   pass take 60 ms against 10 ms for the histogram pass of the same walk. */
#define SP_CHUNK 8192u
struct SpOut {
    uint64_t base;    /* the wave's current chunk (wave-uniform) */
    uint32_t fill;    /* slots of it used (SP_CHUNK: none claimed yet) */
    uint64_t real;    /* windows written by the wave */
};
/* One window per lane (v, or SP_EMPTY / a short walk: none) into its key
   range's list, every lane of the wave calling together.  The ranges are
   told apart by a wave multisplit (3 ballots: range bits 0 and 1, and
   "in a range"), each range's entries placed at its chunk's fill point in
   lane order; a range claims a new SP_CHUNK (one atomic) when this step's
   entries run past its chunk.  One walk thus emits every range's keys:
   round 4 walked the input once per range, computing every window's key
   twice each time. */
static_assert(SP_MAXP == 4u, "sp_range compares three range starts");
/* the range of key v (SP_MAXP: none).  The host groups consecutive passes
   only: between two ranges lie empty buckets, which hold no key */
__device__ __forceinline__ uint32_t sp_range(const SpEmit &em, uint64_t v) {
    if (v < em.ps[0].lo || v >= em.gend) return SP_MAXP;
    return (uint32_t)(v >= em.ps[1].lo) + (uint32_t)(v >= em.ps[2].lo) + (uint32_t)(v >= em.ps[3].lo);
}
__device__ __forceinline__ void sp_place(const SpEmit &em, SpOut (&so)[SP_MAXP], uint64_t v, uint32_t lane) {
    const uint32_t q = sp_range(em, v);
    const unsigned long long bv = __ballot(q < SP_MAXP);
    if (!bv) return;
    const unsigned long long b0 = __ballot((q & 1u) != 0u), b1 = __ballot((q & 2u) != 0u);
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t i = 0; i < SP_MAXP; i++) {
        if (i >= em.np) break;
        const unsigned long long mi = bv & ((i & 1u) ? b0 : ~b0) & ((i & 2u) ? b1 : ~b1);
        if (!mi) continue;
        const uint32_t cnt = (uint32_t)__popcll(mi);
        const uint32_t rem = SP_CHUNK - so[i].fill;
        uint64_t nb = 0;
        if (cnt > rem) {
            unsigned long long c = 0;
            if (lane == 0) c = atomicAdd(em.ps[i].ctr, (unsigned long long)SP_CHUNK);
            nb = rdlane64(c, 0);
        }
        if (q == i) {
            const uint64_t p = (uint64_t)__popcll(mi & lt);
            const uint64_t at = p < rem ? so[i].base + so[i].fill + p : nb + (p - rem);
            if (at < em.ps[i].cap) {
                if (em.ps[i].out32) em.ps[i].out32[at] = (uint32_t)(v - em.ps[i].lo);
                else em.ps[i].out[at] = v;
            }
        }
        if (cnt > rem) { so[i].base = nb; so[i].fill = cnt - rem; }
        else so[i].fill += cnt;
        so[i].real += cnt;
    }
}
/* the end of the wave's walk: pad each range's chunk (4^k - 1, or
   0xFFFFFFFF in a 32-bit list), count its windows */
__device__ __forceinline__ void sp_close(const SpEmit &em, const SpOut (&so)[SP_MAXP], uint64_t pad) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t q = 0; q < SP_MAXP; q++) {
        if (q >= em.np) break;
        const SpPass &ps = em.ps[q];
        if (so[q].fill < SP_CHUNK)
            for (uint32_t i = so[q].fill + lane; i < SP_CHUNK; i += 64u) {
                if (so[q].base + i >= ps.cap) continue;
                if (ps.out32) ps.out32[so[q].base + i] = 0xFFFFFFFFu;
                else ps.out[so[q].base + i] = pad;
            }
        if (lane == 0 && so[q].real) atomicAdd(ps.ctr + 1, (unsigned long long)so[q].real);
    }
}

/* The windows of a fast tile (contiguous layout, tile_fast's Emit) as
 * reference-order keys, handed to the pass's mode.  Half h of a lane holds D
 * = 16 digits (15 with a '\n', right-aligned in its word R); the 32 digits
 * before the half are the previous half's {C, S2} (half 1: this lane's half
 * 0; half 0: the previous lane's half 1, lane 0: the tile's entering code),
 * so the window ending at digit j of the half is
 *   ((prev << 2(j+1)) | (R >> 2(D-1-j))) & (4^k - 1)
 * -- up to 20 bases from two words, which the 16-base {C, S2} of the dense
 * path cannot give. */
__device__ __forceinline__ void sp_fast_emit(const SpEmit &em, const Emit &fe, uint64_t c0, uint64_t maskk,
                                             uint32_t *bh, uint32_t lane, SpOut (&so)[SP_MAXP], uint64_t *stg) {
    const uint64_t pv0 = ((uint64_t)from_prev_lane(fe.BC, (uint32_t)(c0 >> 32)) << 32) |
                         from_prev_lane(fe.B2, (uint32_t)c0);
    const uint64_t pv1 = ((uint64_t)fe.AC << 32) | fe.A2;
    const uint32_t R0 = fe.h0 ? fe.A2 & 0x3FFFFFFFu : fe.A2, R1 = fe.h1 ? fe.B2 & 0x3FFFFFFFu : fe.B2;
    const uint32_t D0 = fe.h0 ? 15u : 16u, D1 = fe.h1 ? 15u : 16u;
    /* window jj (half jj / 16, digit jj % 16), or SP_EMPTY past the half's digits */
    auto key = [&](uint32_t jj) -> uint64_t {
        const bool h = jj >= 16u;
        const uint32_t j = jj & 15u, D = h ? D1 : D0, R = h ? R1 : R0;
        const uint64_t pv = h ? pv1 : pv0;
        if (j >= D) return SP_EMPTY;
        return fk_sigma(((pv << (2u * (j + 1u))) | (uint64_t)(R >> (2u * (D - 1u - j)))) & maskk);
    };
    if (em.mode == SP_KEYS) {
        /* the tile's <= 2048 windows staged in the wave's slots, grouped by
           range (a wave scan of each lane's per-range counts, packed two
           16-bit fields a word), then copied out range by range, 64
           consecutive entries a store */
        uint64_t kv[32];
        uint32_t c01 = 0, c23 = 0;
#pragma unroll
        for (uint32_t jj = 0; jj < 32u; jj++) {
            kv[jj] = key(jj);
            const uint32_t q = sp_range(em, kv[jj]), inc = 1u << (16u * (q & 1u));
            c01 += q < 2u ? inc : 0u;
            c23 += (q - 2u) < 2u ? inc : 0u;
        }
        const uint32_t i01 = wscan_incl32(c01), i23 = wscan_incl32(c23);
        const uint32_t t01 = rdlane(i01, 63), t23 = rdlane(i23, 63);
        const uint32_t T[4] = {t01 & 0xFFFFu, t01 >> 16, t23 & 0xFFFFu, t23 >> 16};
        const uint32_t S[4] = {0u, T[0], T[0] + T[1], T[0] + T[1] + T[2]};
        const uint32_t e01 = i01 - c01, e23 = i23 - c23;
        uint32_t p0 = e01 & 0xFFFFu, p1 = S[1] + (e01 >> 16), p2 = S[2] + (e23 & 0xFFFFu), p3 = S[3] + (e23 >> 16);
#pragma unroll
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint32_t q = sp_range(em, kv[jj]);
            if (q < SP_MAXP) {
                const uint32_t at = q == 0u ? p0 : q == 1u ? p1 : q == 2u ? p2 : p3;
                stg[at] = kv[jj];
                p0 += q == 0u; p1 += q == 1u; p2 += q == 2u; p3 += q == 3u;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (uint32_t q = 0; q < SP_MAXP; q++) {
            if (q >= em.np) break;
            const uint32_t t = T[q];
            if (!t) continue;
            const SpPass &ps = em.ps[q];
            const uint32_t rem = SP_CHUNK - so[q].fill;
            uint64_t nb = 0;
            if (t > rem) {   /* (t <= 2048 < SP_CHUNK: one new chunk at most) */
                unsigned long long c = 0;
                if (lane == 0) c = atomicAdd(ps.ctr, (unsigned long long)SP_CHUNK);
                nb = rdlane64(c, 0);
            }
            for (uint32_t j = lane; j < t; j += 64u) {
                const uint64_t v = stg[S[q] + j];
                const uint64_t at = j < rem ? so[q].base + so[q].fill + j : nb + (j - rem);
                if (at < ps.cap) {
                    if (ps.out32) ps.out32[at] = (uint32_t)(v - ps.lo);
                    else ps.out[at] = v;
                }
            }
            if (t > rem) { so[q].base = nb; so[q].fill = t - rem; }
            else so[q].fill += t;
            so[q].real += t;
        }
        __builtin_amdgcn_wave_barrier();
    } else if (em.mode == SP_DENSE) {
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint64_t v = key(jj);
            if (v >= em.lo && v < em.hi) atomicAdd(&em.dense[v - em.lo], 1ull);
        }
    } else {
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint64_t v = key(jj);
            if (v != SP_EMPTY) atomicAdd(&bh[v >> em.shift], 1u);
        }
    }
}

__global__ void __launch_bounds__(SP_WAVES * 64u)
k_sp_emit(const uint8_t *buf, uint64_t len, int k, uint64_t maskk, const XState *rst, uint64_t nranges,
          uint64_t cpw, uint64_t nchunks, SpEmit em) {
    extern __shared__ uint64_t sp_lds[];   /* SP_WAVES x 2048 slots, then (SP_HIST) the buckets */
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t *slots = sp_lds + (size_t)wv * FK_TILE_BYTES;
    uint32_t *bh = reinterpret_cast<uint32_t *>(sp_lds + (size_t)SP_WAVES * FK_TILE_BYTES);
    if (em.mode == SP_HIST) {
        for (uint32_t i = threadIdx.x; i < em.nbuckets; i += blockDim.x) bh[i] = 0;
        __syncthreads();
    }
    Ctx cx{buf, len, 0, nullptr, nullptr, nullptr, nullptr, nullptr, maskk, 0, k, nullptr, slots};
    const uint64_t nw = (uint64_t)gridDim.x * SP_WAVES;
    SpOut so[SP_MAXP];          /* SP_KEYS: the wave's output chunk in each range's list */
#pragma unroll
    for (uint32_t q = 0; q < SP_MAXP; q++) so[q] = SpOut{0, SP_CHUNK, 0};
    for (uint64_t r = (uint64_t)blockIdx.x * SP_WAVES + wv; r < nranges; r += nw) {
        const uint64_t c0 = r * cpw, c1 = min(c0 + cpw, nchunks);
        const uint64_t rb = c0 * FK_CHUNK_BYTES, re = min(c1 * FK_CHUNK_BYTES, len);
        const XState x = rst[r];
        DState st{x.code, (uint32_t)x.R, x.hdr};
        /* the next full tile's words load while this one is counted */
        uint32_t wn[8];
        auto load_full = [&](uint64_t at) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(buf + at + (uint64_t)lane * FK_LANE_BYTES);
            const u32x4 a = __builtin_nontemporal_load(p), c = __builtin_nontemporal_load(p + 1);
            wn[0] = a.x; wn[1] = a.y; wn[2] = a.z; wn[3] = a.w;
            wn[4] = c.x; wn[5] = c.y; wn[6] = c.z; wn[7] = c.w;
        };
        if (rb + FK_TILE_BYTES <= re) load_full(rb);
        for (uint64_t tb = rb; tb < re; tb += FK_TILE_BYTES) {
            uint32_t w[8];
            int nb = (int)FK_LANE_BYTES;
            if (tb + FK_TILE_BYTES <= re) {
#pragma unroll
                for (int d = 0; d < 8; d++) w[d] = wn[d];
            } else {
                nb = load_lane<FK_LANE_BYTES>(cx, (int64_t)(tb + (uint64_t)lane * FK_LANE_BYTES), w);
            }
            if (tb + 2 * FK_TILE_BYTES <= re) load_full(tb + FK_TILE_BYTES);
            Facts f{0, 0, 0, 0, 0, 0};
            Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF, 0};
            /* a fast tile (bases and at most one '\n' per half, deep in a run,
               outside a header: no short walks, every base ends a window)
               computes its 40-bit windows in registers: no byte walk, no
               slots */
            {
                const uint64_t c0 = st.code;
                Emit fe{0, 0, 0, 0, false, false, false};
                if (tb + FK_TILE_BYTES <= re && st.hdr == 0 &&
                    tile_fast<true, H_EMIT, false>(cx, w, st, f, cnt, 1u, &fe)) {
                    if (fe.deep) sp_fast_emit(em, fe, c0, maskk, bh, lane, so, slots);
                    continue;
                }
            }
            /* a lane reads back only the slots of its own 32 bytes */
#pragma unroll 8
            for (uint32_t j = 0; j < FK_LANE_BYTES; j++) slots[j * 64u + lane] = SP_EMPTY;
            tile_general<true, H_SPARSE>(cx, w, nb, 0u, st, f, cnt, 1u);
            if (em.mode == SP_KEYS) {
                if (em.shorts) {   /* (a single pass: no SP_HIST) */
#pragma unroll 8
                    for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                        const uint64_t v = slots[j * 64u + lane];
                        if (v >= SP_SHORT && v != SP_EMPTY) {
                            const unsigned long long i = atomicAdd(em.nshort, 1ull);
                            if (i < em.short_cap) em.shorts[i] = v;
                        }
                    }
                }
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) sp_place(em, so, slots[j * 64u + lane], lane);
            } else if (em.mode == SP_DENSE) {
#pragma unroll 8
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v >= em.lo && v < em.hi) atomicAdd(&em.dense[v - em.lo], 1ull);
                }
            } else {
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v < SP_SHORT) {
                        atomicAdd(&bh[v >> em.shift], 1u);
                    } else if (v != SP_EMPTY) {
                        const unsigned long long i = atomicAdd(em.nshort, 1ull);
                        if (i < em.short_cap) em.shorts[i] = v;
                    }
                }
            }
        }
    }
    if (em.mode == SP_KEYS) sp_close(em, so, (1ull << (2 * k)) - 1);
    if (em.mode == SP_HIST) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < em.nbuckets; i += blockDim.x)
            if (bh[i]) atomicAdd(&em.bhist[i], (unsigned long long)bh[i]);
    }
}

/* ---- finish ---- */

/* one k_sp_emit launch per retained segment */
int sp_emit_all(fk_engine *e, const SpEmit &em) {
    const size_t lds = (size_t)SP_WAVES * FK_TILE_BYTES * sizeof(uint64_t) +
                       (em.mode == SP_HIST ? (size_t)em.nbuckets * sizeof(uint32_t) : 0);
    for (const auto &sg : e->spsegs) {
        if (!sg.nranges) continue;
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((sg.nranges + SP_WAVES - 1) / SP_WAVES,
                                                                                 (uint64_t)e->cus * 8));
        hipLaunchKernelGGL(k_sp_emit, dim3(grid), dim3(SP_WAVES * 64u), lds, e->stream, sg.src ? sg.src : e->d_keep + sg.off, sg.len,
                           e->k, e->maskk, e->d_kst + sg.st, sg.nranges, sg.cpw, sg.nchunks, em);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

/*
 * A k = 17 key-range pass (keys lo + r, r < 2^32, emitted as 32-bit r) into
 * its runs without a sort (round 5; rocPRIM's radix sort and run-length
 * encode took 228 ms of a 10 G-base step's 390).  The pass is a 2^32-bin
 * count table, so it is counted the way k = 16's dense table is, and only
 * its nonzero bins are written:
 *   k_kpart       the key list in batches of 32 K keys, counting-sorted in LDS
 *                 by r's top 11 bits into 2048 coarse slices (k_part<C32>'s
 *                 row layout: each batch one row of runs of 21-bit codes and a
 *                 row of run words);
 *   k_repart      (as for k = 15, 16) each coarse slice into 64 contiguous
 *                 part streams of 15-bit codes;
 *   k_kp_cnt2     one block per part (2^15 bins, in key order): the part's
 *                 stream into LDS bins, the pads taken off the last bin, the
 *                 nonzero bins' offset from the parts before it (a chained
 *                 scan: each block publishes its distinct count, then looks
 *                 back for the earlier parts' total), then the bins written
 *                 as (key, u32 count) in ascending order with the statistics,
 *                 the rollover check and the adjacent keys' prefix histogram;
 *   k_kp_fold     the blocks' partial statistics into the pass accumulators,
 *                 the prefix histogram of each part's first key against the
 *                 last key of the nonempty part before it, and the pass's
 *                 distinct count.
 */
#define KP_BATCH 32768u      /* keys per k_kpart batch (16 waves x 2048) */
#define KP_SLOTS 64u         /* partial-statistics slots (block % KP_SLOTS) */
#define KP_SLOT_W 36u        /* per slot: 10 statistics, rollover, 24 prefix-histogram entries, spare */
#define KP_EMPTY (~0ull)

/* KT = uint32_t: 32-bit relative keys r (slice r >> 21, code r & (2^21 - 1));
   KT = uint64_t: keys lo + r with r < 2^(cs + 11) (slice r >> cs, code r &
   (2^cs - 1), cs <= 29); keys >= hi (pads past the pass's range) are left out */
/* The top key `tkey` (the pads' value: relative 0xFFFFFFFF, or 4^k - 1 when
   the pass holds it; ~0 for none) is left out of the partition and only
   counted into *tcount: the chunk pads of every emitting wave (tens of
   millions per pass) would otherwise crowd one part, whose k_repart block
   and LDS bin then serialise the whole pass. */
template <typename KT>
__global__ void __launch_bounds__(1024)
k_kpart(const KT *keys, uint64_t n, PartGeo pg, uint64_t lo, uint64_t hi, uint32_t cs, uint64_t tkey,
        unsigned long long *tcount) {
    constexpr bool WIDE = sizeof(KT) == 8;
    __shared__ uint32_t hist[2048], cur[2048], wtot[16];
    __shared__ uint32_t ntop;
    extern __shared__ uint32_t ent[];   /* KP_BATCH codes */
    const uint32_t t = threadIdx.x;
    const uint32_t sh = WIDE ? cs : 21u;
    const KT cmask = (KT)(((uint64_t)1 << sh) - 1);
    for (uint32_t i = t; i < 2048u; i += 1024u) hist[i] = 0;
    if (t == 0) ntop = 0;
    const uint64_t per = (uint64_t)pg.rounds * KP_BATCH;
    const uint64_t k0 = blockIdx.x * per, k1 = min(k0 + per, n);
    uint32_t *codes = reinterpret_cast<uint32_t *>(pg.codes);
    uint32_t mytop = 0;
    for (uint32_t r = 0; r < pg.rounds; r++) {
        const uint32_t row = blockIdx.x * pg.rounds + r;
        const uint64_t b0 = k0 + (uint64_t)r * KP_BATCH;
        const uint32_t nv = b0 < k1 ? (uint32_t)min<uint64_t>(KP_BATCH, k1 - b0) : 0u;
        __syncthreads();
        if (nv == 0) {   /* rows past the block's keys are empty */
            for (uint32_t b = t; b < 2048u; b += 1024u) pg.idx[(size_t)row * 2048u + b] = PART_NO_RUN;
            continue;
        }
        /* each key's slice (two 16-bit slices per word, 0xFFFF: left out --
           past hi, or the top key) and code: 48 registers where 32 64-bit
           keys took 64 and spilled */
        uint32_t cd[32], sp[16];
#pragma unroll
        for (uint32_t j = 0; j < 16u; j++) sp[j] = 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++) {
            cd[j] = 0;
            if (j * 1024u + t < nv) {
                const KT x = keys[b0 + j * 1024u + t];
                uint32_t sl = 0xFFFFu;
                if ((uint64_t)x == tkey) {
                    mytop++;
                } else if (!WIDE) {
                    sl = (uint32_t)x >> 21;
                    cd[j] = (uint32_t)x & 0x1FFFFFu;
                } else if ((uint64_t)x < hi) {
                    const uint64_t r = (uint64_t)x - lo;
                    sl = (uint32_t)(r >> sh);
                    cd[j] = (uint32_t)(r & (uint64_t)cmask);
                }
                sp[j >> 1] = (j & 1) ? (sp[j >> 1] & 0xFFFFu) | (sl << 16) : (sp[j >> 1] & 0xFFFF0000u) | sl;
            }
        }
#define KP_SL(j) ((sp[(j) >> 1] >> (((j) & 1) * 16)) & 0xFFFFu)
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++)
            if (KP_SL(j) != 0xFFFFu) atomicAdd(&hist[KP_SL(j)], 1u);
        __syncthreads();
        {   /* cursors and the row's run words: two slices per thread, a block
               scan (one wave walking 32 slices a lane kept 15 waiting) */
            const uint32_t b = 2u * t, c0 = hist[b], c1 = hist[b + 1u], sum = c0 + c1;
            const uint32_t inc = wscan_incl32(sum);
            if ((t & 63u) == 63u) wtot[t >> 6] = inc;
            __syncthreads();
            uint32_t run = inc - sum;
#pragma unroll
            for (uint32_t w = 0; w < 16u; w++) run += w < (t >> 6) ? wtot[w] : 0u;
            cur[b] = run;
            cur[b + 1u] = run + c0;
            reinterpret_cast<uint2 *>(pg.idx + (size_t)row * 2048u)[t] = make_uint2(run_word(run, c0), run_word(run + c0, c1));
            hist[b] = 0;
            hist[b + 1u] = 0;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++)
            if (KP_SL(j) != 0xFFFFu) ent[atomicAdd(&cur[KP_SL(j)], 1u)] = cd[j];
#undef KP_SL
        __syncthreads();
        /* the row: its runs end at cur[2047] (every entry placed) */
        const uint32_t tot = cur[2047];
        uint4 *dst = reinterpret_cast<uint4 *>(codes + (size_t)row * pg.batch);
        const uint4 *src = reinterpret_cast<const uint4 *>(ent);
        for (uint32_t i = t; i < (tot + 3u) / 4u; i += 1024u) dst[i] = src[i];
    }
    if (mytop) atomicAdd(&ntop, mytop);
    __syncthreads();
    if (t == 0 && ntop) atomicAdd(tcount, (unsigned long long)ntop);
}

/*
 * k = 17, round 6: a pass's partition fused into the walk (k_sp_wpart).  The
 * key-list route above walks the input once to emit every window's 32-bit
 * key into its pass's list (36 ms per 10 G-base step: 40 GB written), then
 * k_kpart reads each list back to partition it (4 x 9 ms), after a
 * histogram walk (10.6 ms) that sizes the passes.  Here pass q (the windows
 * whose first base is q: keys [q 2^32, (q + 1) 2^32)) walks the input
 * itself -- four walks, no key list, no histogram walk -- and writes k_kpart's
 * rows directly: each round every wave of a 16-wave block counts one tile;
 * after WP_NT rounds the block counting-sorts the in-pass windows of its
 * stashed fast tiles by coarse slice (the top 11 bits of the 32-bit key) in
 * LDS and writes the sorted batch as one row of 21-bit codes with its 2048
 * run words (the row claimed from a global counter).  A stashed fast tile is
 * five words a lane; its 17-mers are recomputed from them in each phase:
 * the 16-mer ending at slot i is one alignbit of the half's {context, word}
 * pair (as in k_part), and its first base the context's digit above it --
 * the context taken from the previous half's full 16-digit word, since a
 * '\n' half's context word (Emit::AC / BC) lost its top digit.  A batch with
 * more in-pass windows than a row holds (skewed input: at most WP_NT x 16 x
 * 2048) is written as several rows, each placing the entries whose sorted
 * position falls in its window.  A tile the fast path cannot take only
 * advances the wave's state (tile_general without counting: a few registers,
 * where the counting general path would crowd the fast tiles' loop out of
 * its 128 VGPRs); walk 0 records it with its entering state, and after walk
 * 0 k_sp_gtiles counts every recorded tile as k_sp_emit would (slots in
 * LDS), listing its windows by first base as 32-bit keys -- partitioned into
 * further rows of their pass by k_kpart -- and its short walks.  A row or
 * list past its capacity fails the walk, and the finish takes the key-list
 * route instead.
 */
#define SP_RETRY 1000      /* (host) the fused walks gave up: the key-list passes instead */
/* tiles per wave per batch, and the row: 16 x 4 x 2048 windows, a quarter
   of them (~32.8 K) in the pass on random input, in rows of 36 K codes
   (145 KiB of the 160 KiB of LDS).  Round 6: 3 tiles in 32 K rows filled
   them three quarters, and k_repart, reading runs of ~12 codes, took 14.4
   ms a pass against 12.7 for full rows */
#define WP_NT 4u
#define WP_BATCH 36352u
#define WP_FAULT 1ull
/* a tile the fast path did not take: where (its segment, offset) and its
   entering state */
struct SpDefer {
    uint64_t tb, code;
    uint32_t R, hdr, seg, pad;
};
struct SpWalk {
    uint32_t q;                    /* the pass's first base (reference order) */
    uint32_t ktop, cs;             /* k >= 18: the first base's bit 2k - 2, code bits */
    uint32_t *codes;               /* rows of WP_BATCH codes (k_kpart's layout) */
    uint32_t *idx;                 /* [row][2048] run words */
    unsigned long long *ctr;       /* [0] rows claimed, [1] tiles deferred, [3] windows placed in rows,
                                      [4] faults */
    uint64_t rows_cap;
    SpDefer *defer;                /* walk 0: the other tiles (else nullptr) */
    uint64_t defer_cap;
    uint32_t seg;                  /* the launch's segment */
    uint32_t dbg;                  /* FINDKMER_TUNE sp_walk_dbg: 1 = every tile deferred (tests) */
};
/* sigma32: fk_sigma of 16 digits (the internal A0 C1 T2 G3 to the
   reference's A0 C1 G2 T3, digit by digit: so a window of mapped words is
   the mapped window, and the stashed words are mapped once per tile) */
__device__ __forceinline__ uint32_t sigma32(uint32_t x) { return x ^ ((x >> 1) & 0x55555555u); }
struct WpTile {
    uint32_t c0, s0, c1, s1;       /* k = 17, per half: 16-digit context, 16-digit word (reference order) */
    uint32_t fl;                   /* bit 0: has windows, bits 1, 2: half 0 / 1 had a '\n' (slot 0 no window) */
};
/* 18 <= k <= 20 (windows up to 20 digits): as k_sp_emit's sp_fast_emit, the
   32 digits before half 0 (the previous lane's {BC, B2}) and the Emit words
   AC, A2, B2 (half 1's 32 digits before it are {AC, A2}), all mapped to the
   reference's digit order (fk_sigma maps digit by digit, so a window of the
   mapped words is the mapped window) */
struct WpTileW {
    uint32_t p0h, p0l, ac, a2, b2;
    uint32_t fl;
};
/* a stashed fast tile's in-pass windows: HIST into the slices' counts, else
   placed at their slices' cursors */
template <bool HIST>
__device__ __forceinline__ void wp_tile(const WpTile &x, uint32_t q, uint32_t *hist, uint32_t *cur, uint32_t *ent) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? x.c1 : x.c0, S = h ? x.s1 : x.s0;
        const bool skip0 = (x.fl >> (1 + h)) & 1u;
#pragma unroll
        for (int g = 0; g < 2; g++) {
            uint32_t b[8], cd[8], p[8];
            bool in[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int i = 8 * g + j;
                const uint32_t sh = 30u - 2u * (uint32_t)i;
                /* (the words are in reference digit order already: see WpTile) */
                const uint32_t r = i < 15 ? __builtin_amdgcn_alignbit(C, S, sh) : S;
                in[j] = __builtin_amdgcn_ubfe(C, sh, 2u) == q && (i > 0 || !skip0);
                b[j] = r >> 21;
                cd[j] = r & 0x1FFFFFu;
            }
            if (HIST) {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (in[j]) atomicAdd(&hist[b[j]], 1u);
            } else {
                /* the eight returning cursor atomics back to back, then the stores */
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (in[j]) p[j] = atomicAdd(&cur[b[j]], 1u);
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (in[j] && p[j] < WP_BATCH) ent[p[j]] = cd[j];
            }
        }
    }
}

/* the wide passes' windows: keys of 2k bits, the pass's first base q the
   top digit (bit ktop = 2k - 2 up), slice the top 11 bits of the relative
   key, code its low cs bits */
template <bool HIST>
__device__ __forceinline__ void wp_tile_w(const WpTileW &x, uint32_t q, uint32_t ktop, uint64_t maskk, uint32_t cs,
                                          uint32_t *hist, uint32_t *cur, uint32_t *ent) {
    (void)maskk;
    const uint32_t cm = (1u << cs) - 1u, tsh = ktop - 32u;   /* the first base: bits [ktop, ktop + 2) of the key */
#pragma unroll
    for (int h = 0; h < 2; h++) {
        /* the 96-bit stream {pvh, pvl, ra}: the 32 digits before the half,
           then its 16 (or, after a '\n', 15 left-aligned) digits; the window
           ending at the half's digit j is its bits [30 - 2j, 30 - 2j + 2k) */
        const uint32_t pvh = h ? x.ac : x.p0h, pvl = h ? x.a2 : x.p0l;
        const bool hf = (x.fl >> (1 + h)) & 1u;
        const uint32_t r = h ? x.b2 : x.a2;
        const uint32_t ra = hf ? r << 2 : r;
#pragma unroll
        for (int g = 0; g < 2; g++) {
            uint32_t b[8], cd[8], p[8];
            bool in[8];
#pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                const uint32_t j = 8u * (uint32_t)g + (uint32_t)jj, sh = 30u - 2u * j;
                const uint32_t lo = j < 15u ? __builtin_amdgcn_alignbit(pvl, ra, sh) : ra;
                const uint32_t hi = j < 15u ? __builtin_amdgcn_alignbit(pvh, pvl, sh) : pvl;
                in[jj] = (j < 15u || !hf) && __builtin_amdgcn_ubfe(hi, tsh, 2u) == q;
                b[jj] = __builtin_amdgcn_alignbit(hi, lo, cs) & 0x7FFu;
                cd[jj] = lo & cm;
            }
            if (HIST) {
#pragma unroll
                for (int jj = 0; jj < 8; jj++)
                    if (in[jj]) atomicAdd(&hist[b[jj]], 1u);
            } else {
#pragma unroll
                for (int jj = 0; jj < 8; jj++)
                    if (in[jj]) p[jj] = atomicAdd(&cur[b[jj]], 1u);
#pragma unroll
                for (int jj = 0; jj < 8; jj++)
                    if (in[jj] && p[jj] < WP_BATCH) ent[p[jj]] = cd[jj];
            }
        }
    }
}

template <bool WIDE>
__global__ void __launch_bounds__(1024, 1)
k_sp_wpart(const uint8_t *buf, uint64_t len, int k, uint64_t maskk, const XState *rst, uint64_t nranges, uint64_t cpw,
           uint64_t nchunks, SpWalk wk) {
    __shared__ uint32_t hist[2048], cur[2048], wtot[16];
    __shared__ uint32_t s_total;
    __shared__ unsigned long long s_row;
    extern __shared__ uint32_t ent[];   /* WP_BATCH codes */
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (uint32_t i = t; i < 2048u; i += 1024u) hist[i] = 0;
    __syncthreads();
    const uint64_t gw = (uint64_t)blockIdx.x * 16u + wv, nw = (uint64_t)gridDim.x * 16u;
    Ctx cx{buf, len, 0, nullptr, nullptr, nullptr, nullptr, nullptr, maskk, 0, k, nullptr, nullptr};
    /* the wave's tile cursor: range r, tile tb of [.., re), state st */
    uint64_t r = gw, tb = 0, re = 0;
    DState st{0, 0, 0};
    uint32_t wn[8] = {};
    auto load_full = [&](uint64_t at) {
        const u32x4 *p = reinterpret_cast<const u32x4 *>(buf + at + (uint64_t)lane * FK_LANE_BYTES);
        const u32x4 a = __builtin_nontemporal_load(p), c = __builtin_nontemporal_load(p + 1);
        wn[0] = a.x; wn[1] = a.y; wn[2] = a.z; wn[3] = a.w;
        wn[4] = c.x; wn[5] = c.y; wn[6] = c.z; wn[7] = c.w;
    };
    auto open = [&]() {   /* range r from its exact entering state */
        const uint64_t c0 = r * cpw, c1 = min(c0 + cpw, nchunks);
        tb = c0 * FK_CHUNK_BYTES;
        re = min(c1 * FK_CHUNK_BYTES, len);
        const XState x = rst[r];
        st = DState{x.code, (uint32_t)x.R, x.hdr};
        if (tb + FK_TILE_BYTES <= re) load_full(tb);
    };
    bool done = r >= nranges;
    if (!done) open();
    /* one tile of the wave's ranges: a fast tile stashed, any other only
       advancing the state (walk 0: recorded for k_sp_gtiles) */
    using Tile = typename std::conditional<WIDE, WpTileW, WpTile>::type;
    auto step = [&]() -> Tile {
        Tile x{};
        if (done) return x;
        uint32_t w[8];
        int nb = (int)FK_LANE_BYTES;
        const bool full = tb + FK_TILE_BYTES <= re;
        if (full) {
#pragma unroll
            for (int d = 0; d < 8; d++) w[d] = wn[d];
        } else {
            nb = load_lane<FK_LANE_BYTES>(cx, (int64_t)(tb + (uint64_t)lane * FK_LANE_BYTES), w);
        }
        if (tb + 2 * FK_TILE_BYTES <= re) load_full(tb + FK_TILE_BYTES);
        Facts f{0, 0, 0, 0, 0, 0};
        Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF, 0};
        const uint64_t c0 = st.code;
        Emit fe{0, 0, 0, 0, false, false, false};
        if (full && st.hdr == 0 && !(wk.dbg & 1u) && tile_fast<true, H_EMIT, false>(cx, w, st, f, cnt, 1u, &fe)) {
            if (fe.deep) {
                if constexpr (WIDE) {
                    x.p0h = sigma32(from_prev_lane(fe.BC, (uint32_t)(c0 >> 32)));
                    x.p0l = sigma32(from_prev_lane(fe.B2, (uint32_t)c0));
                    x.ac = sigma32(fe.AC);
                    /* (a '\n' half's word: its top digit is the digit before it, masked off) */
                    x.a2 = sigma32(fe.A2);
                    x.b2 = sigma32(fe.h1 ? fe.B2 & 0x3FFFFFFFu : fe.B2);
                } else {
                    const uint32_t xp = sigma32(from_prev_lane(fe.B2, (uint32_t)c0));   /* the 16 digits before half 0 */
                    const uint32_t a2 = sigma32(fe.A2);
                    x.c0 = fe.h0 ? xp >> 2 : xp;
                    x.s0 = a2;
                    x.c1 = fe.h1 ? a2 >> 2 : a2;
                    x.s1 = sigma32(fe.B2);
                }
                x.fl = 1u | (fe.h0 ? 2u : 0u) | (fe.h1 ? 4u : 0u);
            }
        } else {
            if (wk.defer && lane == 0) {
                const unsigned long long i = atomicAdd(&wk.ctr[1], 1ull);
                if (i < wk.defer_cap) wk.defer[i] = SpDefer{tb, st.code, st.R, st.hdr, wk.seg, 0u};
            }
            tile_general<false, H_NONE>(cx, w, nb, 0u, st, f, cnt, 1u);
        }
        tb += FK_TILE_BYTES;
        if (tb >= re) {
            r += nw;
            done = r >= nranges;
            if (!done) open();
        }
        return x;
    };
    Tile xs[WP_NT];
    auto apply = [&](const Tile &x, bool hst) {
        if constexpr (WIDE) {
            if (hst) wp_tile_w<true>(x, wk.q, wk.ktop, maskk, wk.cs, hist, cur, ent);
            else wp_tile_w<false>(x, wk.q, wk.ktop, maskk, wk.cs, hist, cur, ent);
        } else {
            if (hst) wp_tile<true>(x, wk.q, hist, cur, ent);
            else wp_tile<false>(x, wk.q, hist, cur, ent);
        }
    };
    /* the stashed tiles' in-pass windows into the slices' counts (sel: one
       stash slot, or ~0 all).  One stashed tile at a time: unrolled over the
       stash, the compiler interleaved all 96 windows and spilled */
    auto wp_hist = [&](uint32_t sel) {
#pragma unroll 1
        for (uint32_t i = 0; i < WP_NT; i++) {
            Tile x = xs[0];
#pragma unroll
            for (uint32_t ii = 1; ii < WP_NT; ii++)
                if (i == ii) x = xs[ii];
            if ((x.fl & 1u) && (sel == ~0u || sel == i)) apply(x, true);
        }
    };
    /* a new row, claimed by thread 0 (seen by all after the next barrier) */
    auto wp_claim = [&]() {
        if (t == 0) {
            const unsigned long long rw = atomicAdd(&wk.ctr[0], 1ull);
            s_row = rw;
            if (rw >= wk.rows_cap) atomicOr(&wk.ctr[4], WP_FAULT);
        }
    };
    /* sorted starts (two slices a thread, a block scan) as cursors and as
       the row's run words, the counts cleared for the next histogram;
       returns the total (past WP_BATCH the run words are rewritten) */
    auto wp_scan = [&]() -> uint32_t {
        const uint32_t b = 2u * t, n0 = hist[b], n1 = hist[b + 1u], sum = n0 + n1;
        const uint32_t inc = wscan_incl32(sum);
        if (lane == 63) wtot[wv] = inc;
        __syncthreads();
        uint32_t run = inc - sum;
#pragma unroll
        for (uint32_t w = 0; w < 16u; w++) run += w < wv ? wtot[w] : 0u;
        cur[b] = run;
        cur[b + 1u] = run + n0;
        hist[b] = 0;
        hist[b + 1u] = 0;
        const unsigned long long row = s_row;
        if (row < wk.rows_cap && run + sum <= 65536u)
            reinterpret_cast<uint2 *>(wk.idx + (size_t)row * 2048u)[t] = make_uint2(run_word(run, n0), run_word(run + n0, n1));
        if (t == 1023u) s_total = run + sum;
        __syncthreads();
        return s_total;
    };
    /* the stashed windows (sel: one slot, or ~0 all; T <= WP_BATCH of them)
       placed and written out as the claimed row */
    auto wp_row = [&](uint32_t sel, uint32_t T) {
#pragma unroll 1
        for (uint32_t i = 0; i < WP_NT; i++) {
            Tile x = xs[0];
#pragma unroll
            for (uint32_t ii = 1; ii < WP_NT; ii++)
                if (i == ii) x = xs[ii];
            if ((x.fl & 1u) && (sel == ~0u || sel == i)) apply(x, false);
        }
        __syncthreads();
        const unsigned long long row = s_row;
        if (row < wk.rows_cap) {
            if (t == 0) atomicAdd(&wk.ctr[3], (unsigned long long)T);
            uint4 *dst = reinterpret_cast<uint4 *>(wk.codes + (size_t)row * WP_BATCH);
            const uint4 *src = reinterpret_cast<const uint4 *>(ent);
            for (uint32_t i = t; i < (T + 3u) / 4u; i += 1024u) dst[i] = src[i];
        }
        __syncthreads();
    };
    for (;;) {
#pragma unroll 1
        for (uint32_t u = 0; u < WP_NT; u++) {
            const Tile x = step();
#pragma unroll
            for (uint32_t i = 0; i < WP_NT; i++)
                if (u == i) xs[i] = x;
        }
        wp_claim();   /* (a batch without windows leaves an empty row) */
        wp_hist(~0u);
        /* (the barrier also tells whether any wave has tiles left) */
        const bool more = __syncthreads_or(!done);
        const uint32_t T = wp_scan();
        if (T <= WP_BATCH) {
            if (T) wp_row(~0u, T);
        } else {
            /* more windows of the pass than a row holds (skewed input): one
               row per stash slot (16 x 2048 windows at most), each counted
               again on its own.  (Splitting the batch's sorted order at the
               row size instead let the atomics' order decide which of a
               straddling slice's entries fell before the split --
               differently in each row's placement: an entry twice, another
               lost.) */
#pragma unroll 1
            for (uint32_t i = 0; i < WP_NT; i++) {
                if (i) wp_claim();
                wp_hist(i);
                __syncthreads();
                wp_row(i, wp_scan());
            }
        }
        if (!more) break;
    }
}

/* the recorded tiles (walk 0), one wave at a time each from its entering
   state with k_sp_emit's general path: FILL = false counts each first
   base's windows (cnt[0..3]) and lists the short walks; FILL = true lists
   the windows, first base q at glist + goff[q], as key - q 4^(k - 1) (KT:
   32 bits at k = 17) */
struct SpSegDev {
    const uint8_t *src;
    uint64_t len;
};
template <bool FILL, typename KT>
__global__ void __launch_bounds__(SP_WAVES * 64u)
k_sp_gtiles(const SpDefer *df, uint64_t n, const SpSegDev *segs, int k, uint64_t maskk, KT *glist,
            const uint64_t *goff, unsigned long long *cnt, uint64_t *shorts, uint64_t short_cap) {
    const uint32_t ktop = 2u * (uint32_t)k - 2u;   /* a key's first base: its bits from 2k - 2 */
    const uint64_t relm = (1ull << ktop) - 1ull;
    extern __shared__ uint64_t gt_lds[];   /* SP_WAVES x 2048 slots */
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t *slots = gt_lds + (size_t)wv * FK_TILE_BYTES;
    const uint64_t nw = (uint64_t)gridDim.x * SP_WAVES;
    for (uint64_t i = (uint64_t)blockIdx.x * SP_WAVES + wv; i < n; i += nw) {
        const SpDefer d = df[i];
        const SpSegDev sg = segs[d.seg];
        Ctx cx{sg.src, sg.len, 0, nullptr, nullptr, nullptr, nullptr, nullptr, maskk, 0, k, nullptr, slots};
        uint32_t w[8];
        const int nb = load_lane<FK_LANE_BYTES>(cx, (int64_t)(d.tb + (uint64_t)lane * FK_LANE_BYTES), w);
        DState st{d.code, d.R, d.hdr};
        Facts f{0, 0, 0, 0, 0, 0};
        Counters c{0, 0, 0, 0, 0, FK_NO_EOF, 0};
#pragma unroll 8
        for (uint32_t j = 0; j < FK_LANE_BYTES; j++) slots[j * 64u + lane] = SP_EMPTY;
        tile_general<true, H_SPARSE>(cx, w, nb, 0u, st, f, c, 1u);
        /* per first base: this lane's windows (16-bit fields), then a wave scan */
        uint32_t c01 = 0, c23 = 0, nsh = 0;
        for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
            const uint64_t v = slots[j * 64u + lane];
            if (v < SP_SHORT) {
                const uint32_t q = (uint32_t)(v >> ktop), inc = 1u << (16u * (q & 1u));
                c01 += q < 2u ? inc : 0u;
                c23 += q >= 2u ? inc : 0u;
            } else if (v != SP_EMPTY) {
                nsh++;
            }
        }
        if (!FILL) {
            const uint32_t a01 = wsum32(c01), a23 = wsum32(c23), ash = shorts ? wscan_incl32(nsh) : 0u;
            const uint32_t tsh = rdlane(ash, 63);
            unsigned long long sb = 0;
            if (lane == 0) {
                if (a01 & 0xFFFFu) atomicAdd(&cnt[0], (unsigned long long)(a01 & 0xFFFFu));
                if (a01 >> 16) atomicAdd(&cnt[1], (unsigned long long)(a01 >> 16));
                if (a23 & 0xFFFFu) atomicAdd(&cnt[2], (unsigned long long)(a23 & 0xFFFFu));
                if (a23 >> 16) atomicAdd(&cnt[3], (unsigned long long)(a23 >> 16));
                if (tsh) sb = atomicAdd(&cnt[4], (unsigned long long)tsh);
            }
            sb = rdlane64(sb, 0) + (ash - nsh);
            if (shorts && nsh)
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v >= SP_SHORT && v != SP_EMPTY) {
                        if (sb < short_cap) shorts[sb] = v;
                        sb++;
                    }
                }
        } else {
            const uint32_t i01 = wscan_incl32(c01), i23 = wscan_incl32(c23);
            const uint32_t t01 = rdlane(i01, 63), t23 = rdlane(i23, 63);
            unsigned long long b4[4] = {0, 0, 0, 0};
            if (lane == 0) {
                if (t01 & 0xFFFFu) b4[0] = atomicAdd(&cnt[0], (unsigned long long)(t01 & 0xFFFFu));
                if (t01 >> 16) b4[1] = atomicAdd(&cnt[1], (unsigned long long)(t01 >> 16));
                if (t23 & 0xFFFFu) b4[2] = atomicAdd(&cnt[2], (unsigned long long)(t23 & 0xFFFFu));
                if (t23 >> 16) b4[3] = atomicAdd(&cnt[3], (unsigned long long)(t23 >> 16));
            }
            const uint32_t e01 = i01 - c01, e23 = i23 - c23;
            uint64_t at[4] = {rdlane64(b4[0], 0) + (e01 & 0xFFFFu), rdlane64(b4[1], 0) + (e01 >> 16),
                              rdlane64(b4[2], 0) + (e23 & 0xFFFFu), rdlane64(b4[3], 0) + (e23 >> 16)};
            if (c01 | c23)
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v < SP_SHORT) {
                        const uint32_t q = (uint32_t)(v >> ktop);
                        const uint64_t a = q == 0u ? at[0] : q == 1u ? at[1] : q == 2u ? at[2] : at[3];
                        glist[goff[q] + a] = (KT)(v & relm);
                        at[0] += q == 0u; at[1] += q == 1u; at[2] += q == 2u; at[3] += q == 3u;
                    }
                }
        }
        __builtin_amdgcn_wave_barrier();   /* (the slots are rewritten by the next tile) */
    }
}

/* A chained scan over the blocks in dispatch order (wave 0 of every block
   calls it): this block's `total` published (status A: aggregate), the
   earlier blocks' sum found by looking back 64 flags at a time -- up to the
   nearest one with status P (inclusive prefix) -- and this block's own
   inclusive prefix published.  Returns the exclusive prefix.  Parts are
   taken by start-order tickets, so every earlier part is already running
   and publishes unconditionally: a wait only lasts as long as a slow
   predecessor (a part holding one k-mer's billions of windows, counted
   twice over for its 16-bit wrap, takes seconds).  The bound is wall-clock
   (s_memrealtime, 100 MHz), CHAIN_WAIT_S seconds since this block started
   waiting -- far past any valid part -- and only guards a broken invariant
   (FK_FAULT_PARTS: the pass fails with FK_E_INTERNAL instead of hanging the
   GPU).  (Round 5 bounded it by 2^22 spin iterations, which a slow but
   valid predecessor could exceed.)  The flags are relaxed
   agent-scope atomics: a flag word carries all a reader needs (status and
   value in one 64-bit access), and a release store would write back this
   XCD's whole L2 -- the parts' output just written -- once per part. */
#define CHAIN_WAIT_S 60ull
__device__ unsigned long long chain_prefix(unsigned long long *flags, uint32_t blk, uint32_t total,
                                           unsigned long long *err) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long A = 1ull << 62, P = 2ull << 62, M = (1ull << 62) - 1;
    if (blk == 0) {
        if (lane == 0) __hip_atomic_store(&flags[0], P | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&flags[blk], A | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long pre = 0;
    int64_t j = (int64_t)blk - 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const int64_t idx = j - (int64_t)lane;
        unsigned long long f = idx >= 0 ? __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : P;
        /* wait only for the flags up to the nearest inclusive prefix (the
           blocks farther back may still be counting) */
        for (;;) {
            const unsigned long long pm0 = __ballot((f >> 62) == 2);
            const unsigned long long need = pm0 ? (pm0 & (~pm0 + 1)) * 2 - 1 : ~0ull;   /* lanes 0 .. first P */
            if (!(__ballot((f >> 62) == 0) & need)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > CHAIN_WAIT_S * 100000000ull) {
                if (lane == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
                return pre;
            }
            __builtin_amdgcn_s_sleep(1);
            if ((f >> 62) == 0) f = __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const unsigned long long pm = __ballot((f >> 62) == 2);
        const unsigned long long val = f & M;
        if (pm) {
            const uint32_t first = (uint32_t)__builtin_ctzll(pm);   /* the nearest prefix */
            pre += wsum64(lane <= first ? val : 0ull);
            break;
        }
        pre += wsum64(val);
        j -= 64;
    }
    if (lane == 0) __hip_atomic_store(&flags[blk], P | (pre + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

/* The part's 2^15 bins are 16-bit halves of 2^14 LDS words (64 KiB instead
   of 128: half the zeroing and reading, 16.9 -> 13.1 ms per k = 17 pass in
   round 5).  A half that wraps (a k-mer 65536 times in one part) makes the
   halves' sum fall short of the codes: the part is then counted again as two
   halves of 2^14 32-bit bins. */
#define KC_WORDS (1u << 14)
/*
 * k_kp_cnt2: one block per part, two blocks per CU (round 6), so that one
 * block's latency-bound phases -- the part's first loads, the barriers, the
 * chained scan's wait, the output -- overlap the other's.  Round 5's
 * k_kp_count held a thread's 32 bins in registers from the count to the
 * output (114 VGPRs, one block per CU: 12.7 ms per k = 17 pass against
 * 10.4 here); here the bins stay in LDS and are read twice, one 64-bin step of a wave's
 * 2048 at a time (consecutive 16-bit bins a lane each: no bank conflicts):
 * pass 1 takes the statistics, the wave's distinct count and its last
 * nonzero bin; after the chained scan, pass 2 writes each step's nonzero
 * bins compacted by a ballot (the wave's output one contiguous run) with
 * the first differing base of each adjacent pair (the nearest nonzero bin
 * below, in the step, the wave's earlier steps or the earlier waves).  A
 * lane's bins all end in base lane & 3.  A wrapped 16-bit bin: the part
 * counted again as two halves of 2^14 32-bit bins, each pass once per half
 * (32 virtual waves of 1024 bins).
 */
#define KC2_VW 32u
__global__ void __launch_bounds__(1024, 8)   /* 8 waves per SIMD: two blocks per CU */
k_kp_cnt2(const uint16_t *in, RepartSeg sg, uint32_t gp, uint64_t lo, uint64_t npads,
          const unsigned long long *tcount, uint32_t nparts, int k, unsigned long long *flags, uint64_t *out_k,
          uint32_t *out_c, unsigned long long *slots, uint64_t *fl, unsigned long long *err) {
    extern __shared__ uint32_t bins[];   /* KC_WORDS */
    __shared__ uint32_t wnz[KC2_VW], wlast[KC2_VW], hpre[8], s_hs, s_n;
    __shared__ unsigned long long wred[16][7];
    __shared__ unsigned long long bprefix;
    __shared__ uint32_t vblk;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) {
        /* the part: a ticket in the order blocks start, not blockIdx -- the
           chained scan may only wait on blocks that are already running,
           and across the 8 XCDs (and other processes' kernels) blockIdx
           order is not start order */
        vblk = (uint32_t)atomicAdd(&flags[nparts], 1ull);
        s_hs = 0;
        s_n = 0;
    }
    if (t < 8) hpre[t] = 0;
    __syncthreads();
    const uint32_t blk = vblk;
    /* the part's segments: row blk % gp of k_repart block blk / gp's table */
    const uint32_t sgb = blk / gp, spi = blk % gp;
    const unsigned long long dbase = sg.bmeta[2 * (size_t)sgb];
    const uint32_t R = (uint32_t)sg.bmeta[2 * (size_t)sgb + 1];
    /* bin b at half b & 1 of word b >> 1 (hsel: the 32-bit pass of half h,
       bins [h 2^14, (h + 1) 2^14) only) */
    auto count1 = [&](uint32_t b, int hsel) {
        b &= 0x7FFFu;
        if (hsel < 0) atomicAdd(&bins[b >> 1], 1u << ((b & 1u) << 4));
        else if ((b >> 14) == (uint32_t)hsel) atomicAdd(&bins[b & (KC_WORDS - 1u)], 1u);
    };
    auto zero = [&]() {
        for (uint32_t i = t; i < KC_WORDS / 4u; i += 1024u) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    };
    {
        const uint32_t mine = seg_codes(in, sg.desc, dbase, R, spi, [&](uint32_t c) { count1(c, -1); }, [&]() {
            zero();
            __syncthreads();
        });
        const uint32_t a = wsum32(mine);
        if (lane == 0 && a) atomicAdd(&s_n, a);
    }
    __syncthreads();
    /* the top key (relative 0xFFFFFFFF, the last bin of the last part) was
       only counted (k_kpart): its real windows, the pads taken off */
    const struct { uint32_t n; } m{s_n};
    const uint32_t extra = blk == nparts - 1u ? (uint32_t)(*tcount - npads) : 0u;
    const uint64_t kpart = lo + ((uint64_t)blk << 15);
    const uint32_t fd = (uint32_t)((kpart >> (2 * (k - 1))) & 3);
    const uint16_t *b16 = reinterpret_cast<const uint16_t *>(bins);
    /* bin i's count: 16-bit bins, or (wrap path, half h) 32-bit bins of [h 2^14, (h + 1) 2^14) */
    auto rd = [&](uint32_t i, int wrap) -> uint32_t {
        const uint32_t c = wrap ? bins[i & (KC_WORDS - 1u)] : (uint32_t)b16[i];
        return c + (i == 32767u ? extra : 0u);
    };
    uint32_t nz = 0, hs = 0;
    unsigned long long lsum = 0;
    /* pass 1 over virtual wave vw's bins [i0, i0 + 64 nsteps) */
    auto pass1 = [&](uint32_t vw, uint32_t i0, uint32_t nsteps, int wrap) {
        uint32_t cnt = 0, last = ~0u;
        for (uint32_t s = 0; s < nsteps; s++) {
            const uint32_t i = i0 + 64u * s + lane;
            const uint32_t c = rd(i, wrap);
            hs += c - (i == 32767u ? extra : 0u);
            nz += c != 0u;
            lsum += c;
            const unsigned long long bl = __ballot(c != 0u);
            cnt += (uint32_t)__popcll(bl);
            if (bl) last = i0 + 64u * s + 63u - (uint32_t)__clzll((long long)bl);
        }
        if (lane == 0) { wnz[vw] = cnt; wlast[vw] = last; }
    };
    pass1(wv, wv * 2048u, 32u, 0);
    {
        const uint32_t a = wsum32(hs);
        if (lane == 0) atomicAdd(&s_hs, a);
    }
    __syncthreads();
    const bool wrap = s_hs != m.n;   /* a 16-bit bin wrapped: the halves' sum falls short of the codes */
    if (wrap) {
        nz = 0;
        lsum = 0;
        for (int h = 0; h < 2; h++) {
            __syncthreads();
            zero();
            __syncthreads();
            seg_codes(in, sg.desc, dbase, R, spi, [&](uint32_t c) { count1(c, h); });
            __syncthreads();
            pass1(16u * h + wv, (uint32_t)h * 16384u + wv * 1024u, 16u, 1);
        }
    }
    const uint32_t nvw = wrap ? 32u : 16u;
    __syncthreads();
    uint32_t total = 0;
    for (uint32_t v = 0; v < nvw; v++) total += wnz[v];
    if (wv == 0) {
        const unsigned long long pre = chain_prefix(flags, blk, total, err);
        if (lane == 0) {
            bprefix = pre;
            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;
        }
    }
    __syncthreads();
    /* pass 2: the nonzero bins out, and the adjacent pairs' first differing base */
    uint32_t hc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto pass2 = [&](uint32_t vw, uint32_t i0, uint32_t nsteps, int wrap) {
        uint64_t o = bprefix;
        uint32_t prev = ~0u;   /* the nearest nonzero bin below (none: the part's first) */
        for (uint32_t v = 0; v < vw; v++) {
            o += wnz[v];
            if (wlast[v] != ~0u) prev = wlast[v];
        }
        for (uint32_t s = 0; s < nsteps; s++) {
            const uint32_t i = i0 + 64u * s + lane;
            const uint32_t c = rd(i, wrap);
            const unsigned long long bl = __ballot(c != 0u);
            if (c) {
                const unsigned long long below = bl & ((1ull << lane) - 1ull);
                const uint32_t at = (uint32_t)__popcll(below);
                __builtin_nontemporal_store((uint64_t)(kpart + i), out_k + o + at);
                __builtin_nontemporal_store(c, out_c + o + at);
                const uint32_t p = below ? i - lane + 63u - (uint32_t)__clzll((long long)below) : prev;
                if (p != ~0u) {
                    const uint32_t j = 7u - (hibit(i ^ p) >> 1);   /* depth k - 7 + j */
#pragma unroll
                    for (uint32_t q = 0; q < 8u; q++) hc[q] += j == q;
                } else {
                    fl[2 * (size_t)blk] = kpart + i;   /* the part's first key */
                }
            }
            o += (uint64_t)__popcll(bl);
            if (bl) prev = i0 + 64u * s + 63u - (uint32_t)__clzll((long long)bl);
        }
    };
    if (!wrap) {
        pass2(wv, wv * 2048u, 32u, 0);
    } else {
        for (int h = 0; h < 2; h++) {
            __syncthreads();
            zero();
            __syncthreads();
            seg_codes(in, sg.desc, dbase, R, spi, [&](uint32_t c) { count1(c, h); });
            __syncthreads();
            pass2(16u * h + wv, (uint32_t)h * 16384u + wv * 1024u, 16u, 1);
        }
    }
    /* the part's last key */
    if (t == 0 && total) {
        uint32_t last = 0;
        for (uint32_t v = 0; v < nvw; v++)
            if (wlast[v] != ~0u) last = wlast[v];
        fl[2 * (size_t)blk + 1] = kpart + last;
    }
#pragma unroll
    for (uint32_t q = 0; q < 8u; q++) {
        const uint32_t a = wsum32(hc[q]);
        if (lane == 0 && a) atomicAdd(&hpre[q], a);
    }
    /* statistics: distinct, sum, last-base marginals (lane & 3), first base fd */
    {
        unsigned long long v6[6];
        v6[0] = wsum32(nz);
#pragma unroll
        for (uint32_t d = 0; d < 4u; d++) {
            const unsigned long long x = (lane & 3u) == d ? lsum : 0ull;
            v6[2 + d] = wsum64(x);
        }
        v6[1] = v6[2] + v6[3] + v6[4] + v6[5];
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 6; q++) wred[wv][q] = v6[q];
    }
    __syncthreads();
    if (t < 10) {
        unsigned long long a = 0;
        const uint32_t q = t < 6u ? t : 1u;   /* 6..9: the sum under first base fd */
        for (uint32_t w = 0; w < 16u; w++) a += wred[w][q];
        if (t >= 6u && t - 6u != fd) a = 0;
        if (a) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + t], a);
        if (t == 1 && a != (uint64_t)m.n + extra) atomicOr(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 10], 1ull);
    }
    if (t < 8 && hpre[t]) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 11 + (k - 7 + (int)t)], (unsigned long long)hpre[t]);
}

/*
 * Wide passes (18 <= k <= 20, a key range of more than 2^32 keys): the same
 * two partition levels (64-bit keys in, the parts' codes 32-bit), then each
 * part -- up to KS_CAP keys of at most 23 bits, ~10 K at k = 20 over 10 G
 * bases -- sorted in LDS instead of counted: bucketed by its top 8 bits
 * (LDS histogram, scan, scatter), each bucket sorted by one wave in
 * registers (a bitonic network over 64 N keys, N = 1..16 per lane), then run-
 * length encoded.  A part or bucket above those sizes (a k-mer repeated
 * tens of thousands of times in one part) flags the pass, which then takes
 * the library sort (fks_sort_runs) instead.
 */
#define KS_CAP 24576u        /* k_kp_sort<KS_CAP>: one block per CU */
#define KS_CAP_S 12288u      /* k_kp_sort<KS_CAP_S>: two (every part of the pass fits) */
#define FK_FAULT_SORTCAP 8u

/* bitonic sort of the 64 N values x[i] (element i * 64 + lane), ascending */
template <int N>
__device__ __forceinline__ void wave_bitonic(uint32_t (&x)[N]) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t s2 = 2; s2 <= 64u * N; s2 <<= 1) {
#pragma unroll
        for (uint32_t d = s2 >> 1; d > 0; d >>= 1) {
            if (d >= 64) {
                const uint32_t dr = d / 64;
#pragma unroll
                for (int i = 0; i < N; i++) {
                    if ((uint32_t)i & dr) continue;
                    const int j = i | (int)dr;
                    const uint32_t e = (uint32_t)i * 64u + lane;
                    const bool up = (e & s2) == 0;
                    const uint32_t a = x[i], b = x[j];
                    x[i] = up ? min(a, b) : max(a, b);
                    x[j] = up ? max(a, b) : min(a, b);
                }
            } else {
#pragma unroll
                for (int i = 0; i < N; i++) {
                    const uint32_t e = (uint32_t)i * 64u + lane;
                    const uint32_t o = (uint32_t)__shfl_xor((int)x[i], (int)d, 64);
                    const bool up = (e & s2) == 0, low = (lane & d) == 0;
                    x[i] = (low == up) ? min(x[i], o) : max(x[i], o);
                }
            }
        }
    }
}

/* Batcher's odd-even merge sort of N (a power of two) registers, ascending
   (63 compare-exchanges at N = 16, every index a constant) */
template <int N>
__device__ __forceinline__ void reg_sort(uint32_t (&x)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; i++)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const uint32_t a = x[i + j], b = x[i + j + k];
                        x[i + j] = min(a, b);
                        x[i + j + k] = max(a, b);
                    }
}

template <int N>
__device__ __forceinline__ void wave_sort_bucket(uint32_t *k, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t e = (uint32_t)i * 64u + lane;
        x[i] = e < n ? k[e] : ~0u;
    }
    wave_bitonic<N>(x);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t e = (uint32_t)i * 64u + lane;
        if (e < n) k[e] = x[i];
    }
}

template <uint32_t CAP>
__global__ void __launch_bounds__(1024)
k_kp_sort(const uint32_t *in, const PartMeta *meta, uint64_t cap_in, uint64_t lo, uint32_t psh, uint64_t npads,
          const unsigned long long *tcount, uint32_t top_part, uint32_t nparts, int k, unsigned long long *flags,
          uint64_t *out_k, uint32_t *out_c, unsigned long long *slots, uint64_t *fl, unsigned long long *err) {
    constexpr uint32_t KSI = CAP / 1024u;
    extern __shared__ uint32_t keys[];   /* CAP keys, then CAP + 1 u16 run starts */
    uint16_t *const rs = reinterpret_cast<uint16_t *>(keys + CAP);
    /* the bucket cursors live where the run starts go later (two blocks of
       the small instance per CU: 80 KB of LDS each at most) */
    uint32_t *const bh = reinterpret_cast<uint32_t *>(rs);
    __shared__ uint32_t bo[1025];
    __shared__ unsigned long long wred[16][10];
    __shared__ uint32_t hpre[24];
    __shared__ uint32_t wnz[16];
    __shared__ unsigned long long bprefix;
    __shared__ uint32_t bad, vblk;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    bh[t] = 0;
    if (t < 24) hpre[t] = 0;
    if (t == 0) {
        bad = 0;
        vblk = (uint32_t)atomicAdd(&flags[nparts], 1ull);   /* (k_kp_cnt2: start order) */
    }
    __syncthreads();
    const uint32_t blk = vblk;
    PartMeta m = meta[blk];
    if (m.off + m.n > cap_in) {
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_META);
        m.n = 0;
        m.off = 0;
    }
    if (m.n > CAP) {   /* too many keys for one block's LDS: the library sort */
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_SORTCAP);
        m.n = 0;
    }
    const uint32_t n = m.n, bsh = psh - 10u;
    /* 1. bucket by the top 10 bits of the part's code (~10 keys a bucket) */
    uint32_t v[KSI];
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++) {
        v[j] = j * 1024u + t < n ? in[m.off + j * 1024u + t] : 0u;
        if (j * 1024u + t < n) atomicAdd(&bh[v[j] >> bsh], 1u);
    }
    __syncthreads();
    {   /* bucket t's start: a block scan */
        const uint32_t c = bh[t], inc = wscan_incl32(c);
        if (lane == 63) wnz[wv] = inc;
        __syncthreads();
        uint32_t before = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16u; w++) before += w < wv ? wnz[w] : 0u;
        bo[t] = bh[t] = before + inc - c;
        if (t == 1023) bo[1024] = before + inc;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++)
        if (j * 1024u + t < n) keys[atomicAdd(&bh[v[j] >> bsh], 1u)] = v[j];
    __syncthreads();
    /* 2. bucket t of up to 16 keys sorted by thread t in registers; the
       larger ones (~2 % at 10 a bucket on average) each by one wave */
    {
        const uint32_t b0 = bo[t], nb = bo[t + 1] - b0;
        if (nb > 1u && nb <= 16u) {
            uint32_t x[16];
#pragma unroll
            for (uint32_t i = 0; i < 16u; i++) x[i] = i < nb ? keys[b0 + i] : ~0u;
            reg_sort<16>(x);
#pragma unroll
            for (uint32_t i = 0; i < 16u; i++)
                if (i < nb) keys[b0 + i] = x[i];
        }
    }
    for (unsigned long long big = __ballot(bo[wv * 64u + lane + 1] - bo[wv * 64u + lane] > 16u); big; big &= big - 1) {
        const uint32_t b = wv * 64u + (uint32_t)__builtin_ctzll(big);
        const uint32_t b0 = bo[b], nb = bo[b + 1] - b0;
        if (nb <= 64) wave_sort_bucket<1>(keys + b0, nb);
        else if (nb <= 128) wave_sort_bucket<2>(keys + b0, nb);
        else if (nb <= 256) wave_sort_bucket<4>(keys + b0, nb);
        else if (nb <= 512) wave_sort_bucket<8>(keys + b0, nb);
        else if (nb <= 1024) wave_sort_bucket<16>(keys + b0, nb);
        else if (lane == 0) bad = 1;
    }
    __syncthreads();
    if (bad) {
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_SORTCAP);
    }
    const uint32_t nn = bad ? 0u : n;
    /* 3. runs: thread t takes positions [t * KSI, +KSI); a run
       starts where the key changes (the thread's keys read once, as 16-B
       pieces: its 48 or 96 bytes start 16-B aligned) */
    const uint32_t p0 = t * KSI;
    uint32_t kk[KSI];
    static_assert(KSI % 4u == 0u, "KSI keys as 16-B pieces");
#pragma unroll
    for (uint32_t j = 0; j < KSI; j += 4u) {
        const uint4 q = reinterpret_cast<const uint4 *>(keys + p0)[j / 4u];
        kk[j] = q.x; kk[j + 1] = q.y; kk[j + 2] = q.z; kk[j + 3] = q.w;
    }
    const uint32_t kprev = p0 ? keys[p0 - 1] : 0u;
    uint32_t starts = 0;   /* bit j: a run starts at p0 + j */
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++) {
        const uint32_t i = p0 + j;
        if (i < nn && (i == 0 || kk[j] != (j ? kk[j - 1] : kprev))) starts |= 1u << j;
    }
    const uint32_t nz = (uint32_t)__popc(starts);
    const uint32_t inc = wscan_incl32(nz);
    if (lane == 63) wnz[wv] = inc;
    __syncthreads();
    uint32_t before = 0, runs = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16u; w++) {
        const uint32_t x = wnz[w];
        before += w < wv ? x : 0u;
        runs += x;
    }
    /* the top key 4^k - 1 (when the pass holds it: the last key of the top
       part) was only counted (k_kpart): its real windows, the pads taken
       off, are one more run after this part's others */
    const unsigned long long extra = blk == top_part ? *tcount - npads : 0ull;
    const uint32_t total = runs + (extra ? 1u : 0u);
    const uint32_t off = before + inc - nz;
    /* every run's start in LDS (rs[runs] = the end), so that run r is
       written by thread r % 1024: contiguous stores */
    {
        uint32_t o = off;
#pragma unroll
        for (uint32_t j = 0; j < KSI; j++)
            if ((starts >> j) & 1u) rs[o++] = (uint16_t)(p0 + j);
        if (t == 0) rs[runs] = (uint16_t)nn;
    }
    if (wv == 0) {
        const unsigned long long pre = chain_prefix(flags, blk, total, err);
        if (lane == 0) {
            bprefix = pre;
            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;
        }
    }
    __syncthreads();
    const int fs = 2 * (k - 1);
    const uint64_t kb = lo + ((uint64_t)blk << psh);
    /* (named accumulators: a runtime index into a register array lives in
       scratch memory; the first base is the part's, psh < 2k - 2) */
    unsigned long long l0 = 0, l1 = 0, l2 = 0, l3 = 0, nd = 0;
    for (uint32_t r = t; r < runs; r += 1024u) {
        const uint32_t i = rs[r];
        const uint64_t key = kb + keys[i];
        const uint32_t c = (uint32_t)rs[r + 1] - i;
        __builtin_nontemporal_store(key, out_k + bprefix + r);
        __builtin_nontemporal_store(c, out_c + bprefix + r);
        const uint32_t ld = (uint32_t)(key & 3);
        nd += 1;
        l0 += ld == 0 ? c : 0u;
        l1 += ld == 1 ? c : 0u;
        l2 += ld == 2 ? c : 0u;
        l3 += ld == 3 ? c : 0u;
        if (r > 0) {   /* against the run before it, in this part */
            const int lz = __clzll((long long)(key ^ (kb + keys[i - 1]))) - (64 - 2 * k);
            atomicAdd(&hpre[lz / 2 + 1], 1u);
        }
        if (r == 0) fl[2 * (size_t)blk] = key;
        if (r + 1 == total) fl[2 * (size_t)blk + 1] = key;
    }
    if (t == 0 && extra) {   /* the top key's run, last in the part */
        const uint64_t key = (1ull << (2 * k)) - 1;
        const uint32_t c = (uint32_t)extra;
        out_k[bprefix + runs] = key;
        out_c[bprefix + runs] = c;
        nd += 1;
        l3 += c;   /* (the key 4^k - 1 ends in base T = 3) */
        if (runs) {
            const int lz = __clzll((long long)(key ^ (kb + keys[nn - 1]))) - (64 - 2 * k);
            atomicAdd(&hpre[lz / 2 + 1], 1u);
        } else {
            fl[2 * (size_t)blk] = key;
        }
        fl[2 * (size_t)blk + 1] = key;
        if (extra >> 32) atomicOr(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 10], 1ull);   /* a u32 count wrapped */
    }
    const unsigned long long sum = l0 + l1 + l2 + l3;
    const uint32_t fd = (uint32_t)((kb >> fs) & 3);
    const unsigned long long st[10] = {nd, sum, l0, l1, l2, l3, fd == 0 ? sum : 0ull, fd == 1 ? sum : 0ull,
                                       fd == 2 ? sum : 0ull, fd == 3 ? sum : 0ull};
    unsigned long long v10[10];
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(st[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wred[wv][q] = v10[q];
    __syncthreads();
    if (t < 10) {
        unsigned long long a = 0;
        for (uint32_t w = 0; w < 16u; w++) a += wred[w][t];
        if (a) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + t], a);
    }
    if (t < 24 && hpre[t]) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 11 + t], (unsigned long long)hpre[t]);
}

/* the partials into the pass accumulators (FKS_ACC layout), the prefix
   histogram of each nonempty part's first key against the last key of the
   nonempty part before it, and the pass's distinct count (res[0]) */
__global__ void __launch_bounds__(256)
k_kp_fold(const unsigned long long *slots, const uint64_t *fl, uint32_t nparts, int k,
          const unsigned long long *flags, unsigned long long *dacc, unsigned long long *res) {
    __shared__ uint32_t h[24];
    if (threadIdx.x < 24) h[threadIdx.x] = 0;
    __syncthreads();
    if (blockIdx.x == 0) {
        if (threadIdx.x < 10) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a += slots[sl * KP_SLOT_W + threadIdx.x];
            if (a) atomicAdd(&dacc[threadIdx.x], a);
        } else if (threadIdx.x == 10) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a |= slots[sl * KP_SLOT_W + 10];
            if (a) atomicAdd(&dacc[FKS_ACC_ROLL], 1ull);   /* (k_sp_stats adds wrapped counts' high words) */
        } else if (threadIdx.x >= 32 && threadIdx.x < 56) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a += slots[sl * KP_SLOT_W + 11 + (threadIdx.x - 32)];
            if (a) atomicAdd(&dacc[FKS_ACC_WPREFIX + (threadIdx.x - 32)], a);
        } else if (threadIdx.x == 64) {
            res[0] = flags[nparts - 1] & ((1ull << 62) - 1);
        }
    }
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += gridDim.x * blockDim.x) {
        const uint64_t first = fl[2 * (size_t)p];
        if (first == KP_EMPTY || p == 0) continue;
        uint32_t q = p - 1;
        while (q > 0 && fl[2 * (size_t)q] == KP_EMPTY) q--;
        if (fl[2 * (size_t)q] == KP_EMPTY) continue;
        const uint64_t pk = fl[2 * (size_t)q + 1];
        const int lz = __clzll((long long)(first ^ pk)) - (64 - 2 * k);
        atomicAdd(&h[lz / 2 + 1], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 24 && h[threadIdx.x]) atomicAdd(&dacc[FKS_ACC_WPREFIX + threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

/* The rows pg.rows of 21-bit codes under 2048 coarse slices of a 2^32-key
   pass [lo, lo + 2^32) -- k_kpart's over a key list, or the fused walk's
   (k_sp_wpart) -- into the pass's runs at out_k / out_c (*nw of them):
   k_repart, k_kp_cnt2, k_kp_fold.  n: the codes the rows hold; res: 16 B
   of zeroed device scratch, res[1] the top key counted apart by k_kpart
   (npads of them pads) */
static int sp_count_rows32(fk_engine *e, const PartGeo &pg, uint64_t n, uint64_t lo, uint64_t npads,
                           unsigned long long *res, unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c,
                           uint64_t *nw) {
    const int k = e->k;
    const uint32_t nparts = 2048u << 6, gp = REPART_G << 6;
    RepartSeg sgs{};
    int rc = repart_seg_alloc(e, pg, n, gp, &sgs);
    if (rc) return rc;
    if (!e->d_pmeta && hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
        return FK_E_OOM;
    PoolScratch flags(e, 0), slots(e, 1), fl(e, 2);
    if (!flags.alloc((size_t)(nparts + 1) * 8) || !slots.alloc((size_t)KP_SLOTS * KP_SLOT_W * 8) ||
        !fl.alloc((size_t)nparts * 16))
        return FK_E_OOM;
    PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
    unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
    HIPCHK(hipMemsetAsync(alloc, 0, 2 * sizeof(unsigned long long), e->stream));
    HIPCHK(hipMemsetAsync(flags.p, 0, (size_t)(nparts + 1) * 8, e->stream));   /* (+ the block tickets) */
    HIPCHK(hipMemsetAsync(slots.p, 0, (size_t)KP_SLOTS * KP_SLOT_W * 8, e->stream));
    hipLaunchKernelGGL((k_repart<uint16_t, REPART_G, true>), dim3(2048u / REPART_G), dim3(1024), 0, e->stream, pg,
                       e->d_parts, alloc, meta, (uint64_t)e->parts_cap, alloc + 1, 15u, nullptr, sgs);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_kp_cnt2, dim3(nparts), dim3(1024), (size_t)KC_WORDS * 4, e->stream, (const uint16_t *)e->d_parts,
                       sgs, gp, lo, npads, (const unsigned long long *)(res + 1), nparts,
                       k, flags.as<unsigned long long>(), out_k, out_c, slots.as<unsigned long long>(), fl.as<uint64_t>(),
                       alloc + 1);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_kp_fold, dim3(64), dim3(256), 0, e->stream, (const unsigned long long *)slots.p,
                       (const uint64_t *)fl.p, nparts, k, (const unsigned long long *)flags.p, dacc, res);
    HIPCHK(hipGetLastError());
    unsigned long long r[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&r[0], res, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&r[1], alloc + 1, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (r[1]) return FK_E_INTERNAL;
    *nw = r[0];
    return FK_OK;
}

/* The 2048-slice row geometry of a 32-bit pass (rows of `batch` codes);
   `rows0` rows already written (the fused walk's) before k_kpart's over n
   keys */
static PartGeo sp_geo32(fk_engine *e, uint64_t rows0, uint64_t n, uint32_t batch = KP_BATCH) {
    PartGeo pg{};
    pg.nslices = 2048u;
    pg.split = 6u;   /* 2^21-bin coarse slices, 64 parts of 2^15 */
    pg.batch = batch;
    const uint32_t grid = (uint32_t)std::max(1, e->cus);
    pg.rounds = (uint32_t)((n + (uint64_t)grid * KP_BATCH - 1) / ((uint64_t)grid * KP_BATCH));
    pg.rows = (uint32_t)rows0 + grid * pg.rounds;
    pg.flag = nullptr;
    return pg;
}

/* k_kpart over the n 32-bit keys into rows [rows0, pg.rows) of pg */
static int sp_kpart32(fk_engine *e, const PartGeo &pg, uint64_t rows0, const uint32_t *keys, uint64_t n,
                      unsigned long long *tcount) {
    if (!n) return FK_OK;
    PartGeo g = pg;
    g.codes = reinterpret_cast<uint16_t *>(reinterpret_cast<uint32_t *>(pg.codes) + rows0 * pg.batch);
    g.idx = pg.idx + rows0 * 2048u;
    const uint32_t grid = (uint32_t)std::max(1, e->cus);
    hipLaunchKernelGGL(k_kpart<uint32_t>, dim3(grid), dim3(1024), (size_t)KP_BATCH * 4, e->stream, keys, n, g, 0ull,
                       0ull, 21u, 0xFFFFFFFFull, tcount);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* The pass (keys lo + r for the n 32-bit r, npads of them the pad
   0xFFFFFFFF) into its runs at out_k / out_c: *nw of them */
int sp_count_runs32(fk_engine *e, const uint32_t *keys, uint64_t n, uint64_t lo, uint64_t npads,
                           unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw) {
    *nw = 0;
    if (n == 0) return FK_OK;
    PartGeo pg = sp_geo32(e, 0, n);
    const uint64_t ncodes = (uint64_t)pg.rows * KP_BATCH;   /* u32 codes */
    int rc = sp_ensure((void **)&e->d_codes, &e->codes_cap, 2 * ncodes, sizeof(uint16_t));
    if (!rc) rc = sp_ensure((void **)&e->d_pidx, &e->pidx_cap, (uint64_t)pg.rows * 2048u, sizeof(uint32_t));
    if (rc) return rc;
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    PoolScratch res(e, 3);
    if (!res.alloc(16)) return FK_E_OOM;
    HIPCHK(hipMemsetAsync(res.p, 0, 16, e->stream));
    unsigned long long *r = res.as<unsigned long long>();
    rc = sp_kpart32(e, pg, 0, keys, n, r + 1);
    if (!rc) rc = sp_count_rows32(e, pg, n, lo, npads, r, dacc, out_k, out_c, nw);
    return rc;
}

/* The rows pg.rows of cs-bit codes under 2048 coarse slices of a wide pass
   (keys lo + r, r < 2^(cs + 11)) -- k_kpart's over a key list, or the fused
   walk's -- into its runs at out_k / out_c (*nw): k_repart (128 parts a
   slice), k_kp_sort, k_kp_fold.  res: 16 B of zeroed device scratch, res[1]
   the top key counted apart (top_part: its part, ~0 none; npads of them
   pads).  `fallback`: a part or bucket too large for k_kp_sort -- nothing was
   folded into dacc. */
static int sp_sort_rows64(fk_engine *e, const PartGeo &pg, uint64_t n, uint64_t lo, uint32_t psh, uint64_t npads,
                          uint32_t top_part, unsigned long long *res, unsigned long long *dacc, uint64_t *out_k,
                          uint32_t *out_c, uint64_t *nw, bool *fallback) {
    const int k = e->k;
    const uint32_t nparts = 2048u << 7;
    /* (the part streams as 32-bit codes: twice the u16 capacity) */
    int rc = sp_ensure((void **)&e->d_parts, &e->parts_cap, 2 * (n + 8ull * nparts + 16), sizeof(uint16_t));
    if (rc) return rc;
    if (!e->d_pmeta && hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
        return FK_E_OOM;
    PoolScratch flags(e, 0), slots(e, 1), fl(e, 2);
    if (!flags.alloc((size_t)(nparts + 1) * 8) || !slots.alloc((size_t)KP_SLOTS * KP_SLOT_W * 8) ||
        !fl.alloc((size_t)nparts * 16))
        return FK_E_OOM;
    PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
    unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
    uint32_t *parts32 = reinterpret_cast<uint32_t *>(e->d_parts);
    const uint64_t cap32 = e->parts_cap / 2;
    HIPCHK(hipMemsetAsync(alloc, 0, 3 * sizeof(unsigned long long), e->stream));
    HIPCHK(hipMemsetAsync(flags.p, 0, (size_t)(nparts + 1) * 8, e->stream));   /* (+ the block tickets) */
    HIPCHK(hipMemsetAsync(slots.p, 0, (size_t)KP_SLOTS * KP_SLOT_W * 8, e->stream));
    const unsigned long long *tcount = res + 1;
    hipLaunchKernelGGL((k_repart<uint32_t, 4u>), dim3(2048u / 4u), dim3(1024), 0, e->stream, pg, parts32, alloc, meta,
                       cap32, alloc + 1, psh, alloc + 2);
    HIPCHK(hipGetLastError());
    unsigned long long pmax = 0;
    HIPCHK(hipMemcpyAsync(&pmax, alloc + 2, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (pmax > KS_CAP) {   /* a part past one block's LDS: the library sort */
        *fallback = true;
        return FK_OK;
    }
    const bool small = pmax <= KS_CAP_S;
    if (small)
        hipLaunchKernelGGL(k_kp_sort<KS_CAP_S>, dim3(nparts), dim3(1024), (size_t)KS_CAP_S * 6 + 16, e->stream,
                           (const uint32_t *)parts32, (const PartMeta *)meta, cap32, lo, psh, npads, tcount, top_part,
                           nparts, k, flags.as<unsigned long long>(), out_k, out_c, slots.as<unsigned long long>(),
                           fl.as<uint64_t>(), alloc + 1);
    else
        hipLaunchKernelGGL(k_kp_sort<KS_CAP>, dim3(nparts), dim3(1024), (size_t)KS_CAP * 6 + 16, e->stream,
                           (const uint32_t *)parts32, (const PartMeta *)meta, cap32, lo, psh, npads, tcount, top_part,
                           nparts, k, flags.as<unsigned long long>(), out_k, out_c, slots.as<unsigned long long>(),
                           fl.as<uint64_t>(), alloc + 1);
    HIPCHK(hipGetLastError());
    unsigned long long ferr = 0;
    HIPCHK(hipMemcpyAsync(&ferr, alloc + 1, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (ferr & FK_FAULT_SORTCAP) {
        *fallback = true;
        return FK_OK;
    }
    if (ferr) return FK_E_INTERNAL;
    hipLaunchKernelGGL(k_kp_fold, dim3(64), dim3(256), 0, e->stream, (const unsigned long long *)slots.p,
                       (const uint64_t *)fl.p, nparts, k, (const unsigned long long *)flags.p, dacc, res);
    HIPCHK(hipGetLastError());
    unsigned long long r0 = 0;
    HIPCHK(hipMemcpyAsync(&r0, res, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    *nw = r0;
    return FK_OK;
}

/* k_kpart over n 64-bit keys in [lo, hi) into rows [rows0, ..) of pg (cs-bit
   codes), the top key tkey counted apart into *tcount */
static int sp_kpart64(fk_engine *e, const PartGeo &pg, uint64_t rows0, const uint64_t *keys, uint64_t n, uint64_t lo,
                      uint64_t hi, uint32_t cs, uint64_t tkey, unsigned long long *tcount) {
    if (!n) return FK_OK;
    PartGeo g = pg;
    g.codes = reinterpret_cast<uint16_t *>(reinterpret_cast<uint32_t *>(pg.codes) + rows0 * pg.batch);
    g.idx = pg.idx + rows0 * 2048u;
    const uint32_t grid = (uint32_t)std::max(1, e->cus);
    hipLaunchKernelGGL(k_kpart<uint64_t>, dim3(grid), dim3(1024), (size_t)KP_BATCH * 4, e->stream, keys, n, g, lo, hi,
                       cs, tkey, tcount);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* A wide pass (keys[0, n) in [lo, hi), hi - lo > 2^32, npads of them the
   pad 4^k - 1) into its runs at out_k / out_c (*nw).  `fallback` is set
   when a part or bucket is too large for k_kp_sort: nothing was folded into
   dacc and the caller sorts the pass with the library instead. */
int sp_sort_runs64(fk_engine *e, const uint64_t *keys, uint64_t n, uint64_t lo, uint64_t hi, uint64_t npads,
                          unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw, bool *fallback) {
    *nw = 0;
    *fallback = false;
    if (n == 0) return FK_OK;
    const int k = e->k;
    uint32_t sbits = 33;
    while (sbits < 64 && ((hi - lo - 1) >> sbits)) sbits++;
    /* 2048 coarse slices of 128 parts (k_repart: 4 slices per block): at k
       = 20 a pass of up to 2^32 keys leaves ~16 K per part, within k_kp_sort's
       KS_CAP (64 parts per slice left ~33 K, and every pass took the library
       sort) */
    const uint32_t cs = sbits - 11, psh = cs - 7;
    PartGeo pg = sp_geo32(e, 0, n);
    pg.split = 7u;
    const uint64_t ncodes = (uint64_t)pg.rows * KP_BATCH;
    int rc = sp_ensure((void **)&e->d_codes, &e->codes_cap, 2 * ncodes, sizeof(uint16_t));
    if (!rc) rc = sp_ensure((void **)&e->d_pidx, &e->pidx_cap, (uint64_t)pg.rows * 2048u, sizeof(uint32_t));
    if (rc) return rc;
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    PoolScratch res(e, 3);
    if (!res.alloc(16)) return FK_E_OOM;
    HIPCHK(hipMemsetAsync(res.p, 0, 16, e->stream));
    unsigned long long *r = res.as<unsigned long long>();
    /* the top key 4^k - 1 (the pads' value; past hi they are left out as
       out of range) counted apart when the pass holds it */
    const uint64_t top = (1ull << (2 * k)) - 1;
    const bool top_in = top >= lo && top < hi;
    rc = sp_kpart64(e, pg, 0, keys, n, lo, hi, cs, top_in ? top : ~0ull, r + 1);
    if (rc) return rc;
    return sp_sort_rows64(e, pg, n, lo, psh, top_in ? npads : 0ull, top_in ? (uint32_t)((top - lo) >> psh) : ~0u, r,
                          dacc, out_k, out_c, nw, fallback);
}

/*
 * The sparse table (17 <= k <= 20) from the retained input, in key-range
 * passes (k_sp_emit):
 *   1. SP_HIST: window count per bucket (the top SP_BUCKET_BITS index bits)
 *      and every short walk;
 *   2. the passes: consecutive buckets merged while their windows fit one
 *      sorted pass (capped by free HBM, or FINDKMER_TUNE sp_pass); a single
 *      bucket above the cap is counted densely (2^(2k - SP_BUCKET_BITS) u64);
 *   3. per pass: emit, sort + run-length encode (or select the nonzero dense
 *      counts), statistics, prefix histogram, short-walk prefix marks, and
 *      the runs kept as one part of the table.
 * `seq`: the final run's length (its short walk if 1 <= seq < k).
 */
int sparse_finish(fk_engine *e, int32_t seq) {
    const int k = e->k;
    e->sp_distinct = 0;
    memset(e->sp_tstat, 0, sizeof e->sp_tstat);
    e->sp_roll = e->sp_nodes = 0;
    const uint32_t nbk = 1u << SP_BUCKET_BITS;
    const uint32_t shift = 2u * (uint32_t)k - SP_BUCKET_BITS;
    {   /* the HIST launch needs the larger LDS; set it once for every mode */
        const size_t lds = (size_t)SP_WAVES * FK_TILE_BYTES * sizeof(uint64_t) + (size_t)nbk * sizeof(uint32_t);
        HIPCHK(hipFuncSetAttribute((const void *)k_sp_emit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        for (const void *f : {(const void *)k_kpart<uint32_t>, (const void *)k_kpart<uint64_t>})
            HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(KP_BATCH * 4)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_sort<KS_CAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KS_CAP * 6 + 16)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_sort<KS_CAP_S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KS_CAP_S * 6 + 16)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_cnt2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KC_WORDS * 4)));
    }
    PoolScratch acc(e, 4), bh(e, 5), ctr(e, 6), pctr(e, 7);
    if (!acc.alloc(FKS_ACC_N * sizeof(unsigned long long)) || !bh.alloc((size_t)nbk * 8) || !ctr.alloc(24) ||
        !pctr.alloc(2 * SP_MAXP * sizeof(unsigned long long)))
        return FK_E_OOM;
    /* a keys pass claims its output in SP_CHUNKs per wave: at most one
       chunk's worth of pads per wave of every emit launch */
    uint64_t pad_max = 0;
    for (const auto &sg : e->spsegs)
        if (sg.nranges)
            pad_max += std::max<uint64_t>(1, std::min<uint64_t>((sg.nranges + SP_WAVES - 1) / SP_WAVES, (uint64_t)e->cus * 8)) *
                       SP_WAVES * SP_CHUNK;
    unsigned long long *dacc = acc.as<unsigned long long>();
    unsigned long long *nctr = ctr.as<unsigned long long>();
    HIPCHK(hipMemsetAsync(dacc, 0, FKS_ACC_N * sizeof(unsigned long long), e->stream));

    /* the pass cap: window keys one sorted pass may hold.  A pass needs
       ~56 B per key (emitted 8, sorted 8, runs 8, run lengths 8, rocPRIM's
       scratch ~8, the part's keys 8 + counts 4, handed over), and the parts
       of all passes together up to 12 B per window (distinct <= windows):
       reserve those first */
    const uint64_t wins = e->last.acc[ACC_WIN];
    uint64_t cap = e->sp_pass;
    uint64_t room = 0;   /* bytes for the passes' key lists and their processing */
    {
        size_t fr = 0, tot = 0;
        HIPCHK(hipMemGetInfo(&fr, &tot));
        /* plus what the engine's sparse buffers already hold (reused, or
           freed and reallocated larger) */
        const uint64_t held = e->spk_cap * 8 + e->spc_cap * 4 + e->emit_cap * 8 + e->spdense_cap * 8 +
                              e->fks.sorted_cap + e->fks.c64_cap + e->fks.tmp_cap + e->codes_cap * 2 +
                              e->parts_cap * 2 + e->pidx_cap * 4;
        const uint64_t avail = (uint64_t)fr + held;
        const uint64_t reserve = (1ull << 30) + 12 * wins;
        room = avail > reserve ? avail - reserve : 0;
    }
    /* a pass takes ~8 B per key for its list and ~9 for its processing
       (k_kpart's row codes 4 + run words, k_repart's part streams 2-4, the
       library sort's ~40 if a pass falls back to it: kept inside the cap) */
    if (!cap) cap = std::max<uint64_t>(1u << 20, std::min<uint64_t>(room / 56, 1ull << 32));
    /* the table's storage: room for every window (distinct <= windows) */
    {
        int rc = sp_ensure((void **)&e->d_spk, &e->spk_cap, wins + 1, 8);
        if (!rc) rc = sp_ensure((void **)&e->d_spc, &e->spc_cap, wins + 1, 4);
        if (rc) return rc;
    }
    /* all windows in one pass (the feed counted them): no histogram launch,
       the keys pass collects the short walks.  Not k = 17: its passes span
       2^32 keys, which sp_count_runs32 counts instead of sorting */
    const bool single = wins <= cap && k != 17;

    const bool tail = !e->state.hdr && seq >= 1 && seq < k;
    const bool nodes = e->opts.want_nodes != 0;
    uint64_t scap = std::max<uint64_t>(1024, e->keep_len / 64);
    PoolScratch shorts(e, 8), found(e, 9);
    uint64_t ns = 0;
    /* the collected short walks (+ the input's last run, shorter than k:
       :1059-1062 at EOF), distinct, with their found flags */
    auto prep_shorts = [&]() -> int {
        if (tail) {
            const uint64_t v = SP_SHORT | ((uint64_t)seq << 40) | fk_sigma(e->state.code & ((1ull << (2 * seq)) - 1));
            HIPCHK(hipMemcpyAsync(shorts.as<uint64_t>() + ns, &v, sizeof v, hipMemcpyHostToDevice, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            ns++;
        }
        if (!nodes) ns = 0;
        if (ns > 1) {   /* nodeCounter counts distinct prefixes: drop repeated walks */
            uint64_t nu = 0;
            if (fks_unique(&e->fks, shorts.as<uint64_t>(), ns, e->stream, &nu)) return FK_E_HIP;
            ns = nu;
        }
        if (ns) {
            if (!found.alloc(ns * 20)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(found.p, 0, ns * 20, e->stream));
        }
        return FK_OK;
    };

    struct Pass { uint32_t b0, b1; uint64_t n; bool dense; };
    std::vector<Pass> passes;
    /* the fused walks (k_sp_wpart) unless FINDKMER_TUNE sp_walk=0, or sp_pass
       (a test knob of the key-list passes) is set; k >= 18 while the four
       first-base passes leave k_kp_sort's parts (2048 x 128 a pass) within
       its two-blocks-per-CU size on uniform input */
    uint64_t kv = 1;
    const bool fused = wins > 0 && !e->sp_pass && (!tune_knob("sp_walk", &kv) || kv != 0) &&
                       (k == 17 || wins / 4 <= (2048ull << 7) * (KS_CAP_S - 1024));
    auto plan = [&]() -> int {
    if (single) {
        passes.push_back({0, nbk, wins, false});
    } else {
        /* 1. bucket histogram and short walks (a second run if the list overflowed) */
        for (int attempt = 0; attempt < 2; attempt++) {
            if (!shorts.alloc((scap + 1) * 8)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(bh.p, 0, (size_t)nbk * 8, e->stream));
            HIPCHK(hipMemsetAsync(nctr, 0, 16, e->stream));
            SpEmit em{};
            em.mode = SP_HIST;
            em.shift = shift;
            em.bhist = bh.as<unsigned long long>();
            em.nbuckets = nbk;
            em.shorts = shorts.as<uint64_t>();
            em.nshort = nctr + 1;
            em.short_cap = scap;
            int rc = sp_emit_all(e, em);
            if (rc) return rc;
            unsigned long long got = 0;
            HIPCHK(hipMemcpyAsync(&got, nctr + 1, sizeof got, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            ns = got;
            if (ns <= scap) break;
            if (attempt) return FK_E_HIP;
            scap = ns;
        }
        int rc = prep_shorts();
        if (rc) return rc;
        std::vector<unsigned long long> hb(nbk);
        HIPCHK(hipMemcpyAsync(hb.data(), bh.p, (size_t)nbk * 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        /* 2. passes: [b0, b1) buckets; dense when one bucket exceeds the
           cap.  A pass stays inside one aligned block of 2^P keys: k = 17
           (2^34 keys), P = 32, counts 32-bit keys (half the bytes; 4 such
           blocks, as many passes as a 10 G-base input needs anyway); k >= 18
           takes the largest P whose blocks hold at most `cap` windows on
           average, so that a sorted pass spans a power of two and
           sp_sort_runs64's 2^18 parts split it evenly (a pass of 0.28 x 2^40
           keys at k = 20 left half of them empty, and the rest twice as
           large as one block's LDS sorts at full occupancy) */
        uint32_t P = 2u * (uint32_t)k;
        if (k == 17) {
            P = 32;
        } else if (k > 17) {
            P = shift;
            while (P < 2u * (uint32_t)k && (wins >> (2u * (uint32_t)k - P - 1u)) <= cap) P++;
        }
        for (uint32_t b = 0; b < nbk;) {
            if (!hb[b]) { b++; continue; }
            if (hb[b] > cap) { passes.push_back({b, b + 1, hb[b], true}); b++; continue; }
            uint32_t b1 = b;
            uint64_t n = 0;
            while (b1 < nbk && hb[b1] <= cap && n + hb[b1] <= cap && (b1 >> (P - shift)) == (b >> (P - shift)))
                n += hb[b1++];
            passes.push_back({b, b1, n, false});
            b = b1;
        }
    }
    return FK_OK;
    };
    if (!fused) {
        int rc = plan();
        if (rc) return rc;
    }

    /* 3. the passes.  Consecutive sorted or counted passes share one walk
       (up to SP_MAXP key ranges, their lists side by side in d_emit) as
       far as their lists fit beside one pass's processing */
    uint64_t prev_last = 0;
    bool have_prev = false;
    std::vector<unsigned long long> edges(24, 0);   /* prefix histogram across pass boundaries */
    const uint64_t list_room = room > 9 * cap ? room - 9 * cap : 0;
    bool solo = false;   /* a pass fell back to the library sort: one pass per walk from there on */
    /* after a pass: its runs joined to the table (short-walk marks, the
       prefix pair across the pass boundary) */
    auto join = [&](uint64_t *out_k, uint64_t nw) -> int {
        if (!nw) return FK_OK;
        if (e->sp_distinct + nw > e->spk_cap) return FK_E_HIP;   /* cannot happen: distinct <= windows */
        if (ns && fks_short_mark(out_k, nw, shorts.as<uint64_t>(), ns, k, found.as<uint8_t>(), e->stream))
            return FK_E_HIP;
        uint64_t fl[2];
        HIPCHK(hipMemcpyAsync(&fl[0], out_k, 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipMemcpyAsync(&fl[1], out_k + (nw - 1), 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (have_prev) {   /* the adjacent pair across the boundary: first differing base */
            const uint64_t diff = fl[0] ^ prev_last;
            const int lz = __builtin_clzll(diff) - (64 - 2 * k);
            edges[lz / 2 + 1]++;
        }
        prev_last = fl[1];
        have_prev = true;
        e->sp_distinct += nw;
        return FK_OK;
    };
    /* the four first-base passes, each a walk that partitions its windows
       (k_sp_wpart) + the general tiles' list (k_kpart), then k_repart and
       k_kp_cnt2 (k = 17) or k_kp_sort (k >= 18); SP_RETRY: a row or list
       overflowed, a part past k_kp_sort's LDS, or it does not fit -- the
       key-list passes instead */
    auto walkq = [&]() -> int {
        const bool wide = k >= 18;
        const uint32_t ktop = 2u * (uint32_t)k - 2u, cs = ktop - 11u, psh = wide ? cs - 7u : 15u;
        const size_t gsz = wide ? 8 : 4;   /* a listed window: its key less the pass's base */
        const uint32_t grid = (uint32_t)std::max(1, e->cus);
        uint64_t nbatch = 0, ntiles = 0;   /* batches of all blocks: a row each (+ one per WP_BATCH windows) */
        std::vector<SpSegDev> hsegs;
        for (const auto &sg : e->spsegs) {
            hsegs.push_back({sg.src ? sg.src : e->d_keep + sg.off, sg.len});
            if (!sg.nranges) continue;
            const uint64_t rpw = (sg.nranges + (uint64_t)grid * 16 - 1) / ((uint64_t)grid * 16);
            const uint64_t tpr = (sg.cpw * FK_CHUNK_BYTES + FK_TILE_BYTES - 1) / FK_TILE_BYTES;
            nbatch += (uint64_t)grid * ((rpw * tpr + WP_NT - 1) / WP_NT + 1);
            ntiles += (sg.len + FK_TILE_BYTES - 1) / FK_TILE_BYTES + sg.nranges;
        }
        /* rows for a pass of up to half the windows, general-tile windows
           of up to an eighth, a quarter of the tiles recorded
           (FINDKMER_TUNE sp_walk_rows / sp_walk_glist: tests) */
        uint64_t rows_walk = nbatch + wins / 2 / WP_BATCH + 1, gcap = wins / 8 + (1u << 20), kv2 = 0;
        if (tune_knob("sp_walk_rows", &kv2)) rows_walk = kv2;
        if (tune_knob("sp_walk_glist", &kv2)) gcap = std::max<uint64_t>(1, kv2);
        const uint64_t dcap = ntiles / 4 + 1024;
        const uint64_t grows = (uint64_t)grid * ((gcap + (uint64_t)grid * KP_BATCH - 1) / ((uint64_t)grid * KP_BATCH));
        const uint64_t rows_all = rows_walk + grows;
        const uint64_t need = rows_all * (WP_BATCH * 4ull + 2048ull * 4) + 4 * gcap * gsz + dcap * sizeof(SpDefer) +
                              (wide ? 4 : 2) * wins + 32ull * (2048u << 7);
        if (need > room || rows_all > 0xFFFFFFFFull) return SP_RETRY;
        int rc = sp_ensure((void **)&e->d_codes, &e->codes_cap, 2 * rows_all * WP_BATCH, sizeof(uint16_t));
        if (!rc) rc = sp_ensure((void **)&e->d_pidx, &e->pidx_cap, rows_all * 2048u, sizeof(uint32_t));
        if (rc) return rc;
        PoolScratch wc(e, 10), gl(e, 11), dfr(e, 12), sgd(e, 13), res(e, 3);
        if (!wc.alloc(128) || !dfr.alloc(dcap * sizeof(SpDefer)) || !sgd.alloc(hsegs.size() * sizeof(SpSegDev) + 16) ||
            !res.alloc(16))
            return FK_E_OOM;
        if (nodes && !shorts.alloc((scap + 1) * 8)) return FK_E_OOM;
        unsigned long long *wctr = wc.as<unsigned long long>(), *r = res.as<unsigned long long>();
        unsigned long long *gctr = wctr + 8;   /* k_sp_gtiles: [0..3] windows per first base, [4] short walks */
        uint64_t *goff_d = reinterpret_cast<uint64_t *>(wctr + 12);
        HIPCHK(hipMemcpyAsync(sgd.p, hsegs.data(), hsegs.size() * sizeof(SpSegDev), hipMemcpyHostToDevice, e->stream));
        const void *wfn = wide ? (const void *)k_sp_wpart<true> : (const void *)k_sp_wpart<false>;
        HIPCHK(hipFuncSetAttribute(wfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(WP_BATCH * 4)));
        const uint32_t dbg = tune_knob("sp_walk_dbg", &kv2) ? (uint32_t)kv2 : 0u;
        uint64_t gn[4] = {0, 0, 0, 0}, goff[4] = {0, 0, 0, 0};
        for (uint32_t q = 0; q < 4; q++) {
            HIPCHK(hipMemsetAsync(wctr, 0, 64, e->stream));
            HIPCHK(hipMemsetAsync(r, 0, 16, e->stream));
            SpWalk wk{};
            wk.q = q;
            wk.ktop = ktop;
            wk.cs = cs;
            wk.codes = reinterpret_cast<uint32_t *>(e->d_codes);
            wk.idx = e->d_pidx;
            wk.ctr = wctr;
            wk.rows_cap = rows_walk;
            wk.defer = q == 0 ? dfr.as<SpDefer>() : nullptr;
            wk.defer_cap = dcap;
            wk.dbg = dbg;
            for (size_t si = 0; si < e->spsegs.size(); si++) {
                const auto &sg = e->spsegs[si];
                if (!sg.nranges) continue;
                wk.seg = (uint32_t)si;
                if (wide)
                    hipLaunchKernelGGL(k_sp_wpart<true>, dim3(grid), dim3(1024), (size_t)WP_BATCH * 4, e->stream,
                                       hsegs[si].src, sg.len, e->k, e->maskk, e->d_kst + sg.st, sg.nranges, sg.cpw,
                                       sg.nchunks, wk);
                else
                    hipLaunchKernelGGL(k_sp_wpart<false>, dim3(grid), dim3(1024), (size_t)WP_BATCH * 4, e->stream,
                                       hsegs[si].src, sg.len, e->k, e->maskk, e->d_kst + sg.st, sg.nranges, sg.cpw,
                                       sg.nchunks, wk);
                HIPCHK(hipGetLastError());
            }
            unsigned long long c[5];   /* rows, tiles deferred, -, windows in rows, faults */
            HIPCHK(hipMemcpyAsync(c, wctr, sizeof c, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            if (c[4] || c[0] > rows_walk) return SP_RETRY;
            if (q == 0) {   /* the deferred tiles: windows per first base and short walks, then listed */
                if (c[1] > dcap) return SP_RETRY;
                unsigned long long g[5] = {0, 0, 0, 0, 0};
                if (c[1]) {
                    const unsigned gg = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((c[1] + SP_WAVES - 1) / SP_WAVES,
                                                                                         (uint64_t)e->cus * 8));
                    const size_t lds = (size_t)SP_WAVES * FK_TILE_BYTES * sizeof(uint64_t);
                    for (const void *f : {(const void *)k_sp_gtiles<false, uint32_t>, (const void *)k_sp_gtiles<true, uint32_t>,
                                          (const void *)k_sp_gtiles<true, uint64_t>})
                        HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                    HIPCHK(hipMemsetAsync(gctr, 0, 40, e->stream));
                    hipLaunchKernelGGL((k_sp_gtiles<false, uint32_t>), dim3(gg), dim3(SP_WAVES * 64u), lds, e->stream,
                                       (const SpDefer *)dfr.p, (uint64_t)c[1], (const SpSegDev *)sgd.p, e->k, e->maskk,
                                       (uint32_t *)nullptr, (const uint64_t *)nullptr, gctr,
                                       nodes ? shorts.as<uint64_t>() : nullptr, scap);
                    HIPCHK(hipGetLastError());
                    HIPCHK(hipMemcpyAsync(g, gctr, sizeof g, hipMemcpyDeviceToHost, e->stream));
                    HIPCHK(hipStreamSynchronize(e->stream));
                    uint64_t tot = 0;
                    for (int j = 0; j < 4; j++) {
                        gn[j] = g[j];
                        goff[j] = tot;
                        tot += g[j];
                        if (g[j] > gcap) return SP_RETRY;
                    }
                    if (nodes && g[4] > scap) return SP_RETRY;
                    if (tot) {
                        if (!gl.alloc(tot * gsz)) return FK_E_OOM;
                        HIPCHK(hipMemcpyAsync(goff_d, goff, sizeof goff, hipMemcpyHostToDevice, e->stream));
                        HIPCHK(hipMemsetAsync(gctr, 0, 32, e->stream));
                        if (wide)
                            hipLaunchKernelGGL((k_sp_gtiles<true, uint64_t>), dim3(gg), dim3(SP_WAVES * 64u), lds, e->stream,
                                               (const SpDefer *)dfr.p, (uint64_t)c[1], (const SpSegDev *)sgd.p, e->k,
                                               e->maskk, gl.as<uint64_t>(), (const uint64_t *)goff_d, gctr,
                                               (uint64_t *)nullptr, scap);
                        else
                            hipLaunchKernelGGL((k_sp_gtiles<true, uint32_t>), dim3(gg), dim3(SP_WAVES * 64u), lds, e->stream,
                                               (const SpDefer *)dfr.p, (uint64_t)c[1], (const SpSegDev *)sgd.p, e->k,
                                               e->maskk, gl.as<uint32_t>(), (const uint64_t *)goff_d, gctr,
                                               (uint64_t *)nullptr, scap);
                        HIPCHK(hipGetLastError());
                    }
                }
                ns = nodes ? g[4] : 0;
                rc = prep_shorts();
                if (rc) return rc;
            }
            if (c[3] + gn[q] == 0) continue;
            PartGeo pg = sp_geo32(e, c[0], gn[q], WP_BATCH);
            pg.codes = e->d_codes;
            pg.idx = e->d_pidx;
            if (pg.rows > rows_all) return FK_E_INTERNAL;   /* (cannot happen: grows rows hold gcap keys) */
            uint64_t nw = 0;
            uint64_t *ok = e->d_spk + e->sp_distinct;
            uint32_t *oc = e->d_spc + e->sp_distinct;
            if (wide) {
                pg.split = 7u;
                bool fb = false;
                rc = sp_kpart64(e, pg, c[0], gl.as<uint64_t>() + goff[q], gn[q], 0, 1ull << ktop, cs, ~0ull, r + 1);
                if (!rc) rc = sp_sort_rows64(e, pg, c[3] + gn[q], (uint64_t)q << ktop, psh, 0, ~0u, r, dacc, ok, oc, &nw, &fb);
                if (!rc && fb) return SP_RETRY;   /* (the library sort needs the pass's key list) */
            } else {
                rc = sp_kpart32(e, pg, c[0], gl.as<uint32_t>() + goff[q], gn[q], r + 1);
                if (!rc) rc = sp_count_rows32(e, pg, c[3] + gn[q], (uint64_t)q << 32, 0, r, dacc, ok, oc, &nw);
            }
            if (!rc) rc = join(ok, nw);
            if (rc) return rc;
        }
        return FK_OK;
    };
    if (fused) {
        int rc = walkq();
        if (rc == SP_RETRY) {   /* from the start, by the key-list passes */
            e->sp_distinct = 0;
            HIPCHK(hipMemsetAsync(dacc, 0, FKS_ACC_N * sizeof(unsigned long long), e->stream));
            prev_last = 0;
            have_prev = false;
            std::fill(edges.begin(), edges.end(), 0ull);
            ns = 0;
            rc = plan();
        }
        if (rc) return rc;
    }
    for (size_t pi = 0; pi < passes.size();) {
        const Pass &p0 = passes[pi];
        uint64_t *out_k = e->d_spk + e->sp_distinct;   /* this pass's runs follow the earlier ones' */
        uint32_t *out_c = e->d_spc + e->sp_distinct;
        if (p0.dense) {
            SpEmit em{};
            em.shift = shift;
            em.lo = (uint64_t)p0.b0 << shift;
            em.hi = (uint64_t)p0.b1 << shift;
            uint64_t nw = 0;
            const uint64_t nd = 1ull << shift;
            int rc = sp_ensure((void **)&e->d_spdense, &e->spdense_cap, nd, 8);
            if (rc) return rc;
            HIPCHK(hipMemsetAsync(e->d_spdense, 0, nd * 8, e->stream));
            em.mode = SP_DENSE;
            em.dense = e->d_spdense;
            rc = sp_emit_all(e, em);
            if (rc) return rc;
            if (fks_dense_runs(&e->fks, em.dense, nd, em.lo, k, e->stream, dacc, out_k, out_c, &nw)) return FK_E_HIP;
            rc = join(out_k, nw);
            if (rc) return rc;
            pi++;
            continue;
        }
        /* the group: its lists' offsets (16-B aligned) in d_emit */
        size_t pj = pi;
        uint64_t bytes = 0, offs[SP_MAXP];
        while (pj < passes.size() && !passes[pj].dense && pj - pi < (solo ? 1u : SP_MAXP)) {
            const uint64_t span = (uint64_t)(passes[pj].b1 - passes[pj].b0) << shift;
            const uint64_t need = (((passes[pj].n + pad_max) * (span <= (1ull << 32) ? 4u : 8u)) + 15) & ~15ull;
            if (pj > pi && bytes + need > list_room) break;
            offs[pj - pi] = bytes;
            bytes += need;
            pj++;
        }
        {
            int rc = sp_ensure((void **)&e->d_emit, &e->emit_cap, bytes / 8 + 2, 8);
            if (rc) return rc;
        }
        SpEmit em{};
        em.shift = shift;
        em.mode = SP_KEYS;
        em.np = (uint32_t)(pj - pi);
        for (uint32_t q = 0; q < SP_MAXP; q++) em.ps[q].lo = ~0ull;
        em.gend = (uint64_t)passes[pj - 1].b1 << shift;
        unsigned long long *pc = pctr.as<unsigned long long>();
        for (uint32_t q = 0; q < em.np; q++) {
            const Pass &ps = passes[pi + q];
            SpPass &sp = em.ps[q];
            sp.lo = (uint64_t)ps.b0 << shift;
            sp.hi = (uint64_t)ps.b1 << shift;
            uint8_t *base = reinterpret_cast<uint8_t *>(e->d_emit) + offs[q];
            const bool rel32 = sp.hi - sp.lo <= (1ull << 32);
            sp.out = rel32 ? nullptr : reinterpret_cast<uint64_t *>(base);
            sp.out32 = rel32 ? reinterpret_cast<uint32_t *>(base) : nullptr;
            sp.cap = ps.n + pad_max;
            sp.ctr = pc + 2 * q;
        }
        unsigned long long got[2 * SP_MAXP] = {};
        for (int attempt = 0; attempt < 2; attempt++) {
            if (single && !shorts.alloc((scap + 1) * 8)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(nctr, 0, 24, e->stream));
            HIPCHK(hipMemsetAsync(pc, 0, 2 * SP_MAXP * sizeof(unsigned long long), e->stream));
            em.shorts = single ? shorts.as<uint64_t>() : nullptr;   /* the single pass collects them */
            em.nshort = nctr + 1;
            em.short_cap = scap;
            int rc = sp_emit_all(e, em);
            if (rc) return rc;
            unsigned long long nsh = 0;
            HIPCHK(hipMemcpyAsync(got, pc, 2 * SP_MAXP * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipMemcpyAsync(&nsh, nctr + 1, sizeof nsh, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            if (!single || nsh <= scap) {
                if (single) ns = nsh;
                break;
            }
            if (attempt) return FK_E_HIP;
            scap = nsh;
        }
        if (single) {
            int rc = prep_shorts();
            if (rc) return rc;
        }
        for (uint32_t q = 0; q < em.np; q++) {
            const Pass &ps = passes[pi + q];
            const SpPass &sp = em.ps[q];
            const uint64_t claimed = got[2 * q], real = got[2 * q + 1];
            /* the feed's (or the histogram's) count and the walk agree, and
               the claimed slots (windows + pads) fit */
            if (real != ps.n || claimed > sp.cap) return FK_E_HIP;
            uint64_t *ok = e->d_spk + e->sp_distinct;
            uint32_t *oc = e->d_spc + e->sp_distinct;
            uint64_t nw = 0;
            bool lib = false;
            if (sp.out32) {   /* counted, not sorted (sp_count_runs32) */
                int rc = sp_count_runs32(e, sp.out32, claimed, sp.lo, claimed - real, dacc, ok, oc, &nw);
                if (rc) return rc;
            } else {          /* partitioned and sorted in LDS (sp_sort_runs64) */
                int rc = sp_sort_runs64(e, sp.out, claimed, sp.lo, sp.hi, claimed - real, dacc, ok, oc, &nw, &lib);
                if (rc) return rc;
            }
            /* a part or bucket past k_kp_sort's sizes: the library sort,
               which needs the room the group's other lists hold: walk this
               pass again alone */
            if (lib && em.np > 1) {
                solo = true;
                pj = pi + q;
                break;
            }
            if (lib && fks_sort_runs(&e->fks, sp.out, claimed, k, e->stream, dacc, ok, oc, &nw, claimed - real))
                return FK_E_HIP;
            int rc = join(ok, nw);
            if (rc) return rc;
        }
        pi = pj;
    }

    /* 4. totals: statistics, rollover, nodeCounter */
    unsigned long long r[FKS_ACC_N];
    HIPCHK(hipMemcpyAsync(r, dacc, sizeof r, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int q = 0; q < 10; q++) e->sp_tstat[q] = r[q];
    e->sp_roll = r[FKS_ACC_ROLL];
    if (nodes) {
        unsigned long long left = 0;
        if (ns && fks_short_count(&e->fks, shorts.as<uint64_t>(), ns, found.as<uint8_t>(), e->stream, &left))
            return FK_E_HIP;
        if (e->sp_distinct || ns) {
            unsigned long long nd = 0;
            if (e->sp_distinct) {
                unsigned long long run = 1;
                for (int d = 1; d <= k; d++) {
                    run += r[FKS_ACC_WPREFIX + d] + edges[d];
                    nd += run;
                }
            }
            e->sp_nodes = 1 + nd + left;
        }
    }
    return FK_OK;
}


int sparse_copy(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n,
                       hipMemcpyKind kind) {
    if (!e || !n) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    *n = e->sp_distinct;
    if (!keys && !counts) return FK_OK;
    if (cap < e->sp_distinct) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    if (e->sp_distinct) {
        if (keys) HIPCHK(hipMemcpyAsync(keys, e->d_spk, e->sp_distinct * sizeof(uint64_t), kind, e->stream));
        if (counts) HIPCHK(hipMemcpyAsync(counts, e->d_spc, e->sp_distinct * sizeof(uint32_t), kind, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* The sparse table (17 <= k <= 20) after fk_engine_finish: the distinct
   k-mer indices (reference order, ascending = CSV row order) and their u32
   frequencies.  keys/counts may be NULL to ask for *n only. */
extern "C" int fk_engine_sparse(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n) {
    return sparse_copy(e, keys, counts, cap, n, hipMemcpyDeviceToHost);
}

/* The same into device buffers (the multi-GPU exchange's send buffers). */
extern "C" int fk_engine_sparse_device(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n) {
    return sparse_copy(e, keys, counts, cap, n, hipMemcpyDeviceToDevice);
}

/* first index of the ascending device keys[0, n) with key >= want (binary
   search, one key per probe) */
int sparse_lower_bound(fk_engine *e, uint64_t want, uint64_t *at) {
    uint64_t lo = 0, hi = e->sp_distinct;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        uint64_t v = 0;
        HIPCHK(hipMemcpyAsync(&v, e->d_spk + mid, 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (v < want) lo = mid + 1;
        else hi = mid;
    }
    *at = lo;
    return FK_OK;
}

/* The runs of the finished sparse table whose keys fall in [key_lo, key_hi)
   (a contiguous piece of it: CSV rows key_lo.. in order), to host memory:
   *n receives their number, min(cap, n) are copied (keys/counts may be
   NULL to ask for *n). */
extern "C" int fk_engine_sparse_range(fk_engine *e, uint64_t key_lo, uint64_t key_hi, uint64_t *keys,
                                      uint32_t *counts, uint64_t cap, uint64_t *n) {
    if (!e || !n || key_hi < key_lo) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    uint64_t a = 0, b = 0;
    if ((rc = sparse_lower_bound(e, key_lo, &a)) || (rc = sparse_lower_bound(e, key_hi, &b))) return rc;
    *n = b - a;
    const uint64_t m = std::min(cap, b - a);
    if (m && keys) HIPCHK(hipMemcpyAsync(keys, e->d_spk + a, m * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    if (m && counts)
        HIPCHK(hipMemcpyAsync(counts, e->d_spc + a, m * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* The finished sparse table's runs per owner rank: owner of index x is
   x / S, S = ceil(4^k / world) (fk_merge_layout's slices). */
extern "C" int fk_engine_sparse_split(fk_engine *e, int world, uint64_t *counts) {
    if (!e || !counts || world < 1) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    const uint64_t nb = 1ull << (2 * e->k), S = (nb + (uint64_t)world - 1) / (uint64_t)world;
    for (int r = 0; r < world; r++) counts[r] = 0;
    const uint64_t n = e->sp_distinct;
    if (!n) return FK_OK;
    /* the keys are ascending: owners' runs are contiguous; the boundaries by
       binary search over the device keys, one key per probe */
    const uint64_t *keys = e->d_spk;
    uint64_t first = 0, last = 0;
    HIPCHK(hipMemcpyAsync(&first, keys, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&last, keys + (n - 1), 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    const int r0 = (int)(first / S), r1 = (int)(last / S);
    uint64_t at = 0;
    for (int r = r0; r <= r1; r++) {
        uint64_t lo = at, hi = n;   /* first index with key >= (r + 1) * S */
        if (r == r1) {
            lo = n;
        } else {
            const uint64_t want = (uint64_t)(r + 1) * S;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                uint64_t v = 0;
                HIPCHK(hipMemcpyAsync(&v, keys + mid, 8, hipMemcpyDeviceToHost, e->stream));
                HIPCHK(hipStreamSynchronize(e->stream));
                if (v < want) lo = mid + 1;
                else hi = mid;
            }
        }
        counts[r] = lo - at;
        at = lo;
    }
    return FK_OK;
}

/* Replace the finished sparse table by the runs this rank owns after the
   exchange (keys/counts: device, any order, a key possibly from several
   ranks): counts of a key summed, stats[0] = distinct k-mers, stats[1] = the
   sum of their u32 counts (short of the windows when a sum wrapped: the
   rollover check). */
extern "C" int fk_engine_sparse_adopt(fk_engine *e, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                                      uint64_t *stats) {
    if (!e || !stats || (n && (!keys || !counts))) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    DevScratch acc;
    if (!acc.alloc(FKS_ACC_N * sizeof(unsigned long long))) return FK_E_OOM;
    HIPCHK(hipMemsetAsync(acc.p, 0, FKS_ACC_N * sizeof(unsigned long long), e->stream));
    rc = sp_ensure((void **)&e->d_spk, &e->spk_cap, n + 1, 8);
    if (!rc) rc = sp_ensure((void **)&e->d_spc, &e->spc_cap, n + 1, 4);
    if (rc) return rc;
    uint64_t nw = 0;
    e->sp_distinct = 0;
    if (fks_merge_runs(&e->fks, keys, counts, n, e->k, e->stream, acc.as<unsigned long long>(), e->d_spk, e->d_spc,
                       &nw))
        return FK_E_HIP;
    unsigned long long r[FKS_ACC_N];
    HIPCHK(hipMemcpyAsync(r, acc.p, sizeof r, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->sp_distinct = nw;
    memcpy(e->sp_tstat, r, sizeof e->sp_tstat);
    e->sp_roll = r[FKS_ACC_ROLL];
    stats[0] = r[0];
    stats[1] = r[1];
    return FK_OK;
}
