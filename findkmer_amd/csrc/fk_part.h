/*
 * fk_part.h -- the partition geometry shared by the k_part path and the sparse
 * passes (PartGeo, run index words), and k_repart (the second level).
 */
#pragma once
#include "fk_tiles.h"

/*
 * Partitioned counting for 8 <= k <= 12 (the 4^k table does not fit in LDS,
 * and global atomics top out near 27 G/s on this chip).  The state pass
 * (k_count / k_resume in H_NONE mode, then k_scan) gives every range its
 * exact entering state; then:
 *
 * k_part: one wave per range, three interleaved tiles in flight as in
 *   k_count.  Each round, every wave counts one tile: a fast tile hands its
 *   windows to the block's batch, any other tile is counted by the general
 *   path with global atomics.  The block counting-sorts the round's windows
 *   (up to 8 x 2048) by table slice (the top index bits) in LDS, writes the
 *   sorted batch contiguously to its code region (the low `sh` index bits,
 *   u16 each) and records each slice's run (start, count) in a slice-major
 *   index.
 * k_bucket_count: one block per slice (and group of rows) counts its runs in
 *   an LDS slice of 2^sh bins and adds the slice into the table.
 */
/* Waves per k_part block (template parameter W, 8 or 16; part_waves_of()).
   Larger blocks make k_part itself slower (more waves per barrier) but its
   batches larger, so k_bucket_count reads longer runs: one block per CU for
   the 512-slice tables (k = 11, 12: 16 waves, 132 KiB of LDS), two 8-wave
   blocks per CU for k <= 10 (<= 128 slices, long runs already).  Round 2:
   16-wave blocks took the k=11 FASTA step from 1.12 to 1.08 ms and k=12
   from 1.85 to 1.73 ms against 8-wave ones; 4-wave blocks made k=11 5 %
   slower and k=12 30 % slower. */
#define PART_BLOCK_W(W) ((W) * 64u)
/* tiles per wave per batch: 2 single-window tiles or 4 pair tiles fill the
   same LDS batch (a pair tile hands over half as many entries) */
#define PART_TILES(PAIRS) ((PAIRS) ? 4u : 2u)
#define PART_MAX_BATCH_W(W) (2u * (W) * FK_TILE_BYTES)   /* entries per batch */
/* k = 15, 16 (C32): 32-bit codes under 2048 coarse slices, one tile per wave
   per batch (W x 2048 entries, the same 128 KiB of LDS and row slot) */
#define PART_TILES3(PAIRS, C32) ((C32) ? 1u : PART_TILES(PAIRS))
#define PART_ROW_BYTES(W) (4u * (W) * FK_TILE_BYTES)   /* one batch's row slot in d_codes */
static_assert(PART_MAX_BATCH_W(16u) <= 65536u, "run index words hold 16-bit starts and counts - 1");
/* slices of a batch: k = 11 pairs 2^24 / 2^15 (the single k-mers fold into
   them, flagged), k = 12 2^24 / 2^15, k = 13 2^26 / 2^15; k <= 10 at most 128 */
#define PART_SM(W) ((W) >= 16u ? 2048u : 128u)   /* k = 13: 2^26 / 2^15 slices */
/* k = 14: 2^28 / 2^16 = 4096 slices of 16-bit codes (k_bucket_count counts a
   slice as two halves of 2^15 bins, PartGeo::split).  Their run cursors are
   packed two per word (16 KiB of counts + 8 KiB of cursors + the 128 KiB
   batch fit the 160 KiB of LDS): a cursor only reaches 2^16 at the batch's
   very end, where the carry lands on a slice with an empty run. */
#define PART_BIG 4096u
/* Measured and not kept (round 3): pairs mode keeping 8 batches' run words
   per slice in LDS and writing them as one 32-B piece (each scattered 4-B word
   costs a ~40-B write-back, 1.6 GB per 10 GB step): k_part 5.54 -> 5.67 ms,
   k=11 10 GB step 8.08 -> 8.21 ms (the flush and the extra LDS cost more). */
#define PART_SINGLE 0x8000u   /* a stored code with this bit: a single k-mer (pairs mode) */

/* A run index word: (start << 16) | (count - 1) for a run of count >= 1
   codes (a batch holds up to 2^16 of them, all possibly in one slice), and
   PART_NO_RUN for an empty one (start + count <= 2^16 never encodes to it) */
#define PART_NO_RUN 0xFFFFFFFFu
__device__ __forceinline__ uint32_t run_word(uint32_t start, uint32_t count) {
    return count ? (start << 16) | (count - 1u) : PART_NO_RUN;
}
__device__ __forceinline__ uint32_t run_count(uint32_t e) { return e == PART_NO_RUN ? 0u : (e & 0xFFFFu) + 1u; }

struct PartGeo {
    uint16_t *codes;       /* per row (batch): `batch` entries at row * batch */
    uint32_t batch;        /* entries per row slot: PART_MAX_BATCH_W of k_part's block size (+ 8 per slice
                              of pad pieces for PART_PAD) */
    uint32_t *idx;         /* [row][slice]: run_word(start, count) (row-major: one contiguous row of
                              words per batch; round 3: the slice-major layout's scattered 4-B writes
                              cost ~1.6 GB of write-backs per 10 GB step) */
    uint32_t rounds;       /* rows per block */
    uint32_t rows;         /* rows in all: grid * rounds */
    uint32_t nslices;      /* a multiple of 8 */
    uint32_t sh;           /* slice index = code >> sh; stored code = code & (2^sh - 1) */
    uint32_t npair;        /* pairs mode: slices [0, npair) hold (k+1)-mer pairs */
    /* pairs mode, a single k-mer x (a '\n' half's slot 1): slice sbase + ((x << slsh) >> sh), stored
       ((x << slsh) & lowm) | sflag.  2^15-bin slices: x filed under the pair code x << 2 with
       PART_SINGLE set (sbase 0, slsh 2); 2^16-bin slices (W16, k_bucket16): the singles' own slices
       [npair, npair + 4^k / 2^16) (sbase npair, slsh 0, sflag 0) */
    uint32_t sbase, slsh, sflag;
    uint32_t w16;          /* 2^16-bin slices counted in packed 16-bit LDS bins (k_bucket16): k = 11..14 */
    uint32_t nbk;          /* W16: slices k_bucket16 counts ([0, nbk): the index row may be wider) */
    uint32_t *pairs;       /* pairs mode: 4^(k+1) pair bins (k_bucket_count -> k_pair_fold) */
    uint32_t *singles;     /* pairs mode: 4^k single k-mer bins */
    uint32_t nomix;        /* no_mixed: tiles the fast path cannot take go to tile_general */
    uint32_t general;      /* general tiles (other than bases-only ones) k_part takes per range
                              before k_part<RES> takes the rest */
    uint32_t stride;       /* index row stride: rows of both regions (k_part, then k_part<RES>) */
    uint32_t *flag;        /* [0] != 0: some range went to k_part<RES>, region 2 holds rows */
    uint32_t split;        /* k = 15, 16: a coarse slice holds 2^split parts of 2^15 bins */
    uint32_t *glist;       /* k = 15, 16 over a fresh table: the general tiles' windows (hist_add), or nullptr */
    unsigned long long *fz;/* ... and the table statistics k_count_parts takes of it: FZ_SLOTS x 10 partials */
    uint32_t kk;           /* k */
};
#define FZ_SLOTS 1024u   /* (spread: 128 same-address atomics each at k = 16, not 2048) */

/* Every entry a fast tile's Emit hands to the partition, as f(slice, low).
 * Single windows: the 16 windows ending in each half (15 when slot 0 is not
 * a window).  PAIRS (as half_windows<H_PAIRS> does in LDS): the (k+1)-mers
 * ending at the odd slots 1, 3, .., 15 of each half, each standing for the
 * two k-mers ending at slots (2j, 2j+1); without a real slot 0 the first one
 * is the single k-mer x at slot 1, filed under the pair code x << 2 (its
 * slice) with PART_SINGLE set in the stored low bits. */
/* where a pairs-mode single k-mer goes (PartGeo::sbase, slsh, sflag) */
struct SingleEnc {
    uint32_t sbase, slsh, sflag;
};

#define W16_KS_DEFAULT ((1u << 12) | (1u << 13) | (1u << 14))

/*
 * k = 15, 16: the second partition level.  k_part leaves each of the 2048
 * coarse slices as runs of 32-bit codes (low 2k - 11 index bits) in every
 * batch row; a slice holds 2^(2k-26) parts of 2^15 bins (16 at k = 15, 64 at
 * k = 16).  k_repart (one block per REPART_G consecutive coarse slices)
 * reads the slices' runs -- counting their entries per part, then writing
 * each entry's low 15 bits as a 16-bit code into its part's contiguous
 * stream -- after taking the group's region of the output with one global
 * atomic.  k_count_parts (one block per part) then reads one contiguous
 * stream into 2^15 LDS bins and adds them to the table.
 *
 * Round 4 (k = 15 / 16, 1 G bases): one block per coarse slice, a lane per
 * row, and the entries stored one at a time at a per-part cursor moved 68-70
 * GB of HBM per step for ~14 GB of codes (10.3 / 11.8 ms): each lane's 64-B
 * run straddled lines no neighbour shared, and every 2-B store wrote back a
 * partial line.  Now the lanes of a row take the group's adjacent runs (one
 * contiguous span per row) and each round's entries are counting-sorted by
 * part in LDS and written out as contiguous segments.
 */
struct PartMeta {
    unsigned long long off;   /* first code of the part's stream (a multiple of 8) */
    uint32_t n, pad;
};
#define REPART_MAXP 64u       /* parts per coarse slice (k = 16) */
/* coarse slices per k_repart block, and (16-bit parts) two blocks per CU:
   <= 64 VGPRs (a few spill) beside 72 KiB of LDS each.  k = 16 1 G-base
   step 11.5 -> 10.5 ms, k = 17 10 G-base 204 -> 195 ms against G = 8 with
   one block per CU (G = 4 alone: 10.8 / 198) */
#define REPART_G 4u
#define REPART_MINW 8
/* parts per block: G x parts per slice (16-bit parts: up to REPART_MAXP a
   slice; the wide sparse passes' 32-bit parts: REPART_METAP) */
#define REPART_GP(OT, G) ((G) * (sizeof(OT) == 2 ? REPART_MAXP : REPART_METAP))
#define REPART_METAP 128u     /* meta entries per coarse slice (wide sparse passes: 128 parts, G = 4) */
#define REPART_CAP 32768u     /* entries per pass-B round: a batch (16 waves x 2048), the longest run */
static_assert(16u * FK_TILE_BYTES <= REPART_CAP, "a C32 row's run fits one k_repart round");

/* OT = uint16_t: a code's part is its bits [15, 15 + split), stored as its
   low 15 bits (k = 15, 16; k = 17 passes, psh = 15).  OT = uint32_t (wide
   sparse passes): part bits [psh, psh + 6), stored as the low psh bits. */
template <typename OT, uint32_t G = REPART_G>
__global__ void __launch_bounds__(1024, sizeof(OT) == 2 && G == REPART_G ? REPART_MINW : 1)
k_repart(PartGeo pg, OT *out, unsigned long long *alloc, PartMeta *meta, uint64_t cap,
         unsigned long long *err, uint32_t psh, unsigned long long *pmax) {
    /* (G coarse slices of 2^split parts: G << split <= GP, else nothing is
       done and the pass fails -- the arrays below are sized by GP) */
    constexpr uint32_t GP = REPART_GP(OT, G);
    /* per (slice in the group, part): entries, round count / offset /
       cursor, written so far, stream start */
    __shared__ uint32_t cnt[GP], hc[GP], ho[GP], cur[GP], wr[GP];
    __shared__ unsigned long long poff[GP];
    if ((G << pg.split) > GP) {
        if (threadIdx.x == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
        return;
    }
    __shared__ uint32_t scn[17];
    __shared__ __attribute__((aligned(16))) OT rbuf[REPART_CAP];
    const uint32_t pmask = (1u << psh) - 1u;
    const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const uint32_t np = 1u << pg.split, gp = G * np;   /* parts of the block */
    const uint32_t b0 = blockIdx.x * G;                /* its first coarse slice */
    for (uint32_t i = t; i < gp; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    const uint32_t nitems = nrows * G;   /* (row, slice) pairs, row-major: a row's runs side by side */
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    /* item i: row i / G, slice b0 + i % G; its codes as 16-B pieces (4 each)
       -- the G lanes of a row read one contiguous span */
    auto each_code = [&](uint32_t i, auto &&f) {
        const uint32_t r = i / G, sl = i % G;
        const uint32_t e = pg.idx[(size_t)r * pg.nslices + b0 + sl];
        if (e == PART_NO_RUN) return;
        const uint64_t s0 = (uint64_t)r * pg.batch + (e >> 16), s1 = s0 + run_count(e);
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
        auto piece = [&](const uint4 &v, uint64_t q) {
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int h = 0; h < 4; h++)
                if (q * 4 + h >= s0 && q * 4 + h < s1) f(sl * np + (w4[h] >> psh), w4[h]);
        };
        /* the pieces of a run of up to 17 codes in flight together (one
           load at a time left the kernel latency-bound) */
        uint4 v[5];
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++) v[u] = q0 + u < q1 ? g4[q0 + u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++)
            if (q0 + u < q1) piece(v[u], q0 + u);
        for (uint64_t q = q0 + 5u; q < q1; q++) piece(g4[q], q);
    };
    /* pass A: entries per part */
    for (uint32_t i = t; i < nitems; i += blockDim.x)
        each_code(i, [&](uint32_t p, uint32_t) { atomicAdd(&cnt[p], 1u); });
    __syncthreads();
    if (t < 64) {   /* the parts' 8-aligned stream starts in the group's region */
        uint32_t carry = 0;
        for (uint32_t p0 = 0; p0 < gp; p0 += 64u) {
            const uint32_t p = p0 + lane;
            const uint32_t sz = p < gp ? (cnt[p] + 7u) & ~7u : 0u;
            const uint32_t inc = wscan_incl32(sz);
            if (p < gp) ho[p] = carry + inc - sz;   /* (ho: scratch here) */
            carry += rdlane(inc, 63);
        }
        unsigned long long g0 = 0;
        if (lane == 0) g0 = atomicAdd(alloc, (unsigned long long)carry);
        g0 = rdlane64(g0, 0);
        /* bound check: the group's region inside the `cap` codes of `out`
           (the host sizes it for every entry a segment can hold); past it,
           nothing is written, the parts read as empty and the feed fails */
        const bool over = g0 + carry > cap;
        if (over && lane == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
        for (uint32_t p = lane; p < gp; p += 64u) {
            poff[p] = over ? ~0ull : g0 + ho[p];
            wr[p] = 0;
            /* slice-major: (b0 + p / np) * np + p % np */
            meta[(size_t)b0 * np + p] = over ? PartMeta{0, 0, 0} : PartMeta{g0 + ho[p], cnt[p], 0};
        }
        if (pmax) {   /* the largest part (k_kp_sort's LDS size) */
            uint32_t mx = 0;
            for (uint32_t p = lane; p < gp; p += 64u) mx = max(mx, cnt[p]);
            mx = wscan_max32(mx);
            if (lane == 63) atomicMax(pmax, (unsigned long long)mx);
        }
    }
    /* pass B: rounds of whole runs (a lane per item) holding up to
       REPART_CAP entries: counted by part, placed in LDS by part, and each
       part's segment written after the part's earlier rounds */
    uint32_t base = 0;
    __syncthreads();
    /* one item per lane and round, software-pipelined: the next round's
       items are known once this round's are taken, so their index words
       load during this round's count and their first pieces during its
       placement and write-out (each round was a chain of an index load, a
       code load and five barriers: k_repart latency-bound) */
    auto idx_word = [&](uint32_t i) -> uint32_t {
        return i < nitems ? pg.idx[(size_t)(i / G) * pg.nslices + b0 + i % G] : PART_NO_RUN;
    };
    auto span = [&](uint32_t i, uint32_t e, uint64_t &s0, uint64_t &s1) {
        /* (an empty run -- PART_NO_RUN, count 0 -- reads nothing) */
        s0 = (uint64_t)(i / G) * pg.batch + (e == PART_NO_RUN ? 0u : e >> 16);
        s1 = s0 + run_count(e);
    };
    auto load5 = [&](uint64_t s0, uint64_t s1, uint4 *v) {
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++) v[u] = q0 + u < q1 ? g4[q0 + u] : make_uint4(0, 0, 0, 0);
    };
    uint32_t ie = idx_word(base + t);
    uint4 pv[5];
    {
        uint64_t a0, a1;
        span(base + t, ie, a0, a1);
        load5(a0, a1, pv);
    }
    for (;;) {
        const uint32_t i = base + t;
        const uint32_t c = run_count(ie);
        const uint32_t wi = wscan_incl32(c);
        if (lane == 63) scn[wv] = wi;
        for (uint32_t p = t; p < gp; p += blockDim.x) hc[p] = 0;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += scn[w];
        /* the leading items whose runs fit (item `base`'s always does: a
           run holds at most one batch) */
        const bool take = i < nitems && before + wi <= REPART_CAP;
        const uint32_t ntake = (uint32_t)__syncthreads_count(take);
        const uint32_t nbase = base + ntake;
        const uint32_t ien = idx_word(nbase + t);   /* the next round's item */
        uint64_t s0, s1;
        span(i, take ? ie : PART_NO_RUN, s0, s1);
        const uint32_t sl = i % G;
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
        auto codes = [&](auto &&f) {
            auto piece = [&](const uint4 &v, uint64_t q) {
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int h = 0; h < 4; h++)
                    if (q * 4 + h >= s0 && q * 4 + h < s1) f(sl * np + (w4[h] >> psh), w4[h]);
            };
#pragma unroll
            for (uint32_t u = 0; u < 5u; u++)
                if (q0 + u < q1) piece(pv[u], q0 + u);
            for (uint64_t q = q0 + 5u; q < q1; q++) piece(g4[q], q);
        };
        codes([&](uint32_t p, uint32_t) { atomicAdd(&hc[p], 1u); });
        __syncthreads();
        if (t < 64) {
            uint32_t carry = 0;
            for (uint32_t p0 = 0; p0 < gp; p0 += 64u) {
                const uint32_t p = p0 + lane;
                const uint32_t n = p < gp ? hc[p] : 0u;
                const uint32_t inc = wscan_incl32(n);
                if (p < gp) { ho[p] = carry + inc - n; cur[p] = carry + inc - n; }
                carry += rdlane(inc, 63);
            }
        }
        __syncthreads();
        codes([&](uint32_t p, uint32_t v) {
            const uint32_t at = atomicAdd(&cur[p], 1u);
            rbuf[at] = (OT)(v & pmask);
        });
        /* the next round's first pieces (this round's are consumed) */
        {
            uint64_t a0, a1;
            span(nbase + t, ien, a0, a1);
            load5(a0, a1, pv);
        }
        ie = ien;
        __syncthreads();
        /* a wave per part: consecutive entries to consecutive 2-B slots */
        for (uint32_t p = wv; p < gp; p += 16u) {
            const uint32_t n = poff[p] == ~0ull ? 0u : hc[p], o = ho[p];
            OT *dst = out + poff[p] + wr[p];
            for (uint32_t j = lane; j < n; j += 64u) dst[j] = rbuf[o + j];
        }
        __syncthreads();
        for (uint32_t p = t; p < gp; p += blockDim.x) wr[p] += hc[p];
        base = nbase;
        if (base >= nitems || ntake == 0) break;
        __syncthreads();
    }
}

