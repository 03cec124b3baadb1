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
/*
 * Round 6: span-streamed.  The block's rows are taken RP_CHUNK at a time:
 * a lane per row reads the row's G run words (its span: the G slices' runs
 * lie side by side in slice order) into LDS -- the span's first code, the
 * cumulative run lengths, a block scan of the span's 16-B pieces -- and the
 * chunk's pieces are then streamed in rounds of 1024 x PPT pieces, PPT
 * consecutive pieces per thread (a piece's row by binary search over the
 * scan, its slice by the cumulative lengths).  Work per round is a fixed
 * number of codes whatever the runs' lengths: round 5's lane per run took a
 * round per pair of 16 K-code runs on skewed input (a 1 G-base poly-A
 * stretch: minutes in one block).  Codes of one thread that fall into the
 * same part consecutively are counted and placed with one atomic.
 * Pass A counts each part's entries (its stream is sized exactly, one global
 * atomic claims the group's region); pass B counts a round by part, places
 * it in LDS by part and writes each part's segment after its earlier rounds'.
 */
#define RP_CHUNK 1024u                  /* rows per chunk: a lane each */
#define RP_NOPART 0xFFFFu

/*
 * SEG (round 6, 16-bit parts): one pass over the codes instead of two.  A
 * round's codes, counting-sorted by part in LDS, are written as one
 * contiguous run at an offset claimed for the round (pass A sized every
 * part's stream exactly and pass B wrote each part's segment after its
 * earlier rounds', 30 % and 17 % of k = 16's k_repart); each part's
 * segment of the round -- (its codes' first position, count) -- goes to a
 * segment table, part-major per block, so that the consumer gathers a part
 * from its segments.  The block's rounds (counted from the run words alone
 * before the pass) size its table: desc[dbase + part * R + round], and
 * bmeta[2 blk] = dbase, [2 blk + 1] = R.  Table entries are staged in LDS
 * for RP_SEGS rounds and written as 64-B pieces per part.
 */
#define RP_SEGS 8u
struct RepartSeg {
    unsigned long long *desc;       /* (code position << 16) | count per (part, round) */
    uint64_t dcap;                  /* entries of desc */
    unsigned long long *dalloc;     /* entries claimed */
    unsigned long long *bmeta;      /* per block: dbase, rounds */
};

/* OT = uint16_t: a code's part is its bits [15, 15 + split), stored as its
   low 15 bits (k = 15, 16; k = 17 passes, psh = 15).  OT = uint32_t (wide
   sparse passes): part bits [psh, psh + 7), stored as the low psh bits.
   The rows' runs hold at most 65535 codes (C32 / k_kpart rows: 32 K). */
/* the codes of part i of a SEG k_repart block (its table row at desc +
   dbase + i R) as f(code); returns the codes of the segments this lane's
   entries named (their block sum is the part's size).  A wave takes 8
   segments at a time, 8 lanes each: a lane loads the segment's 16-B pieces
   sub, sub + 8, .. (a 64-code segment is ~9 pieces), two in flight, and
   hands on the codes inside the segment.  (Round 6: a lane per code, 2-B
   loads, took k = 16's k_count_parts from 3.5 to 4.8 ms.)  `pre` runs once
   per thread after the first batch's loads are issued (the consumers zero
   their bins there, as they did while a contiguous stream's first pieces
   loaded). */
template <typename F, typename P>
__device__ __forceinline__ uint32_t seg_codes(const uint16_t *in, const unsigned long long *desc,
                                              unsigned long long dbase, uint32_t R, uint32_t i, F &&f, P &&pre) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t sl = lane >> 3, sub = lane & 7u;
    const unsigned long long *d = desc + dbase + (unsigned long long)i * R;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(in);
    uint32_t mine = 0;
    uint64_t a = 0, q0 = 0;
    uint32_t n = 0, npc = 0;
    auto entry = [&](uint32_t r0) {
        const uint32_t r = r0 + sl;
        const unsigned long long e = r < R ? d[r] : 0ull;
        a = e >> 16;
        n = (uint32_t)(e & 0xFFFFu);
        q0 = a >> 3;
        npc = n ? (uint32_t)(((a + n + 7u) >> 3) - q0) : 0u;
    };
    uint4 v[2];
    auto load = [&](uint32_t x) {
#pragma unroll
        for (uint32_t u = 0; u < 2u; u++) v[u] = x + 8u * u < npc ? g4[q0 + x + 8u * u] : make_uint4(0, 0, 0, 0);
    };
    /* the first batch's entries and pieces in flight before `pre` (the
       caller's zeroing of its bins and barrier: every thread calls it once) */
    uint32_t r0 = wv * 8u;
    entry(r0);
    load(sub);
    pre();
    for (bool first = true; r0 < R; r0 += nw * 8u, first = false) {
        if (!first) entry(r0);
        if (sub == 0) mine += n;
        const uint32_t mxp = rdlane(wscan_max32(npc), 63);
        for (uint32_t x = sub; x < mxp; x += 16u) {
            if (!first || x != sub) load(x);
#pragma unroll
            for (uint32_t u = 0; u < 2u; u++) {
                if (x + 8u * u >= npc) continue;
                const uint64_t pb = (q0 + x + 8u * u) * 8u;   /* the piece's first code */
                const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (uint32_t h = 0; h < 8u; h++) {
                    const uint64_t pos = pb + h;
                    if (pos >= a && pos < a + n) f((w4[h >> 1] >> (16u * (h & 1u))) & 0xFFFFu);
                }
            }
        }
    }
    return mine;
}
template <typename F>
__device__ __forceinline__ uint32_t seg_codes(const uint16_t *in, const unsigned long long *desc,
                                              unsigned long long dbase, uint32_t R, uint32_t i, F &&f) {
    return seg_codes(in, desc, dbase, R, i, f, []() {});
}

template <typename OT, uint32_t G = REPART_G, bool SEG = false>
__global__ void __launch_bounds__(1024, sizeof(OT) == 2 && G == REPART_G ? REPART_MINW : 1)
k_repart(PartGeo pg, OT *out, unsigned long long *alloc, PartMeta *meta, uint64_t cap,
         unsigned long long *err, uint32_t psh, unsigned long long *pmax, RepartSeg sg = RepartSeg{}) {
    static_assert(!SEG || sizeof(OT) == 2, "SEG: 16-bit parts");
    /* (G coarse slices of 2^split parts: G << split <= GP, else nothing is
       done and the pass fails -- the arrays below are sized by GP) */
    constexpr uint32_t GP = REPART_GP(OT, G);
    /* 16-B pieces per thread and round: 4 (16 K codes, 64 a part at k =
       16) for 16-bit parts; 8 (32 K codes, 64 a part) for the wide passes'
       512 parts of 32-bit codes, one block per CU (with 4, or 2 and two
       blocks per CU, their 128 / 64-B segments took the k = 20 step from
       274 to 287 / 308 ms) */
    constexpr uint32_t PPT = sizeof(OT) == 2 ? 4u : 8u, ROUND = 1024u * PPT;
    /* per (slice in the group, part): entries, round count / offset /
       cursor, written so far, stream start */
    __shared__ uint32_t cnt[GP], hc[GP], ho[GP], cur[GP], wr[GP];
    __shared__ unsigned long long poff[GP];
    /* the chunk's rows: pieces before each, the span's first code in the
       row, its cumulative run lengths after slices 0 .. G-1 */
    __shared__ uint32_t pre[RP_CHUNK + 1], rs0[RP_CHUNK];
    __shared__ uint16_t rcum[RP_CHUNK][G];
    __shared__ uint32_t wsc[16];
    __shared__ __attribute__((aligned(16))) OT rbuf[ROUND * 4u];
    __shared__ unsigned long long stage[SEG ? RP_SEGS : 1u][SEG ? GP : 1u];
    __shared__ unsigned long long s_base, s_dbase;
    __shared__ uint32_t s_n;
    if ((G << pg.split) > GP) {
        if (threadIdx.x == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
        return;
    }
    const uint32_t pmask = (1u << psh) - 1u;
    const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const uint32_t np = 1u << pg.split, gp = G * np;   /* parts of the block */
    const uint32_t b0 = blockIdx.x * G;                /* its first coarse slice */
    for (uint32_t i = t; i < gp; i += blockDim.x) { cnt[i] = 0; hc[i] = 0; }
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);   /* u32 codes, 4 a piece */
    /* one chunk's rows into LDS; returns its pieces (block-uniform) */
    auto load_chunk = [&](uint32_t c0) -> uint32_t {
        const uint32_t r = c0 + t;
        uint32_t npc = 0, s0 = 0, cum = 0;
        if (r < nrows) {
            bool have = false;
            /* the row's G run words as 16-B pieces (b0 and the row stride
               are multiples of 4 words) */
            static_assert(G % 4u == 0u, "G run words as 16-B pieces");
            uint32_t ew[G];
#pragma unroll
            for (uint32_t j = 0; j < G; j += 4u) {
                const uint4 q = *reinterpret_cast<const uint4 *>(pg.idx + (size_t)r * pg.nslices + b0 + j);
                ew[j] = q.x; ew[j + 1] = q.y; ew[j + 2] = q.z; ew[j + 3] = q.w;
            }
#pragma unroll
            for (uint32_t j = 0; j < G; j++) {
                const uint32_t e = ew[j];
                const uint32_t c = run_count(e);
                if (c && !have) { s0 = e >> 16; have = true; }
                cum += c;
                rcum[t][j] = (uint16_t)cum;
            }
            if (cum) {
                const uint64_t a = (uint64_t)r * pg.batch + s0;
                npc = (uint32_t)(((a + cum + 3u) >> 2) - (a >> 2));
            }
        }
        rs0[t] = s0;
        const uint32_t inc = wscan_incl32(npc);
        if (lane == 63) wsc[wv] = inc;
        __syncthreads();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16u; w++) {
            const uint32_t x = wsc[w];
            before += w < wv ? x : 0u;
            all += x;
        }
        pre[t] = before + inc - npc;
        if (t == 0) pre[RP_CHUNK] = all;
        __syncthreads();
        return all;
    };
    /* this thread's pieces [q, q + PPT) of the chunk (q < tot): codes and
       their parts (RP_NOPART: outside the span).  (Round 6: pieces q0 +
       1024 u + t instead -- a wave's loads 1 KiB contiguous -- took k = 16's
       k_repart from 5.1 to 5.8 ms: four row searches a thread, and the
       spans' 256 B are what a load can use either way) */
    auto load_pieces = [&](uint32_t c0, uint32_t q, uint32_t tot, uint32_t (&code)[4 * PPT],
                           uint32_t (&part)[4 * PPT]) {
        /* the row holding piece q: the last row whose pieces start at or before it */
        uint32_t lo = 0, hi = RP_CHUNK;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= q) lo = mid;
            else hi = mid;
        }
        uint32_t rr = lo;
        uint4 v[PPT];
        uint64_t a[PPT];
        uint32_t rw[PPT];
#pragma unroll
        for (uint32_t u = 0; u < PPT; u++) {
            const uint32_t qq = q + u;
            if (qq < tot) {
                while (pre[rr + 1] <= qq) rr++;
                a[u] = (uint64_t)(c0 + rr) * pg.batch + rs0[rr];   /* the span's first code */
                v[u] = g4[(a[u] >> 2) + (qq - pre[rr])];
            } else {
                a[u] = 0;
                v[u] = make_uint4(0, 0, 0, 0);
            }
            rw[u] = rr;
        }
#pragma unroll
        for (uint32_t u = 0; u < PPT; u++) {
            const uint32_t qq = q + u;
            const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            const uint32_t rr2 = rw[u];
            const uint32_t span = rcum[rr2][G - 1];
            const uint64_t pb = ((a[u] >> 2) + (qq - pre[rr2])) * 4u;   /* the piece's first code */
#pragma unroll
            for (uint32_t h = 0; h < 4u; h++) {
                const int64_t off = (int64_t)(pb + h) - (int64_t)a[u];
                uint32_t pt = RP_NOPART;
                if (qq < tot && off >= 0 && off < (int64_t)span) {
                    uint32_t j = 0;
#pragma unroll
                    for (uint32_t g = 0; g + 1 < G; g++) j += (uint32_t)off >= rcum[rr2][g];
                    pt = j * np + (w4[h] >> psh);
                }
                code[4 * u + h] = w4[h];
                part[4 * u + h] = pt;
            }
        }
    };
    uint32_t R = 0;   /* SEG: the block's rounds */
    if constexpr (SEG) {
        for (uint32_t c0 = 0; c0 < nrows; c0 += RP_CHUNK) R += (load_chunk(c0) + ROUND - 1u) / ROUND;
        if (t == 0) {
            const unsigned long long d = atomicAdd(sg.dalloc, (unsigned long long)gp * R);
            const bool over = d + (unsigned long long)gp * R > sg.dcap;
            if (over) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
            s_dbase = over ? ~0ull : d;
            sg.bmeta[2 * (size_t)blockIdx.x] = over ? 0ull : d;
            sg.bmeta[2 * (size_t)blockIdx.x + 1] = over ? 0ull : R;
        }
        __syncthreads();
    }
    /* pass A: entries per part (runs of one part in a thread's codes: one atomic) */
    for (uint32_t c0 = 0; c0 < (SEG ? 0u : nrows); c0 += RP_CHUNK) {
        const uint32_t tot = load_chunk(c0);
        for (uint32_t q0 = 0; q0 < tot; q0 += ROUND) {
            const uint32_t q = q0 + t * PPT;
            if (q < tot) {
                uint32_t code[4 * PPT], part[4 * PPT];
                load_pieces(c0, q, tot, code, part);
                uint32_t rp = RP_NOPART, rn = 0;
#pragma unroll
                for (uint32_t i = 0; i < 4 * PPT; i++) {
                    if (part[i] != rp) {
                        if (rn) atomicAdd(&cnt[rp], rn);
                        rp = part[i];
                        rn = 0;
                    }
                    rn += part[i] != RP_NOPART;
                }
                if (rn) atomicAdd(&cnt[rp], rn);
            }
        }
        __syncthreads();   /* (the chunk's LDS rows are rewritten next) */
    }
    if (!SEG && t < 64) {   /* the parts' 8-aligned stream starts in the group's region */
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
    __syncthreads();
    /* pass B: each round counted by part, placed in LDS by part, and each
       part's segment written after its earlier rounds' (SEG: the round
       written as one run, its segments to the table) */
    uint32_t rr = 0;   /* SEG: the round's index in the block */
    for (uint32_t c0 = 0; c0 < nrows; c0 += RP_CHUNK) {
        const uint32_t tot = load_chunk(c0);
        for (uint32_t q0 = 0; q0 < tot; q0 += ROUND) {
            const uint32_t q = q0 + t * PPT;
            uint32_t code[4 * PPT], part[4 * PPT];
            if (q < tot) {
                load_pieces(c0, q, tot, code, part);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4 * PPT; i++) { code[i] = 0; part[i] = RP_NOPART; }
            }
            /* count (a run of one part: one atomic) */
            {
                uint32_t rp = RP_NOPART, rn = 0;
#pragma unroll
                for (uint32_t i = 0; i < 4 * PPT; i++) {
                    if (part[i] != rp) {
                        if (rn) atomicAdd(&hc[rp], rn);
                        rp = part[i];
                        rn = 0;
                    }
                    rn += part[i] != RP_NOPART;
                }
                if (rn) atomicAdd(&hc[rp], rn);
            }
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
                if constexpr (SEG) {
                    /* the round's run: claimed (8-aligned), its parts' segments staged */
                    unsigned long long g0 = 0;
                    if (lane == 0) g0 = atomicAdd(alloc, (unsigned long long)((carry + 7u) & ~7u));
                    g0 = rdlane64(g0, 0);
                    const bool over = g0 + carry > cap;
                    if (over && lane == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
                    if (lane == 0) { s_base = over ? ~0ull : g0; s_n = carry; }
                    for (uint32_t p = lane; p < gp; p += 64u) {
                        stage[rr % RP_SEGS][p] = over ? 0ull : ((g0 + ho[p]) << 16) | hc[p];
                        hc[p] = 0;
                    }
                }
            }
            __syncthreads();
            /* place: a run of one part takes its slots with one atomic (its
               length from a backward pass over the thread's codes) */
            {
                uint32_t len[4 * PPT];
                uint32_t follow = 0;
#pragma unroll
                for (int i = 4 * PPT - 1; i >= 0; i--) {
                    const bool same = i + 1 < (int)(4 * PPT) && part[i] == part[i + 1];
                    follow = same ? follow + 1u : 1u;
                    len[i] = follow;
                }
                uint32_t at = 0;
#pragma unroll
                for (uint32_t i = 0; i < 4 * PPT; i++) {
                    if (part[i] == RP_NOPART) continue;
                    if (i == 0 || part[i] != part[i - 1]) at = atomicAdd(&cur[part[i]], len[i]);
                    rbuf[at++] = (OT)(code[i] & pmask);
                }
            }
            __syncthreads();
            if constexpr (SEG) {
                /* the round as one run (16-B pieces: the claim and rbuf are
                   8-code aligned); every RP_SEGS rounds, and after the last,
                   the staged segments to the table, 64 B a part */
                const unsigned long long base = s_base;
                if (base != ~0ull) {
                    const uint32_t n8 = (s_n + 7u) >> 3;
                    uint4 *dst = reinterpret_cast<uint4 *>(out + base);
                    const uint4 *src = reinterpret_cast<const uint4 *>(rbuf);
                    for (uint32_t i = t; i < n8; i += blockDim.x) dst[i] = src[i];
                }
                const uint32_t s = rr % RP_SEGS;
                if ((s == RP_SEGS - 1u || rr + 1u == R) && s_dbase != ~0ull) {
                    const uint32_t r0 = rr - s;
                    for (uint32_t i = t; i < gp * (s + 1u); i += blockDim.x) {
                        const uint32_t p = i / (s + 1u), j = i % (s + 1u);
                        sg.desc[s_dbase + (unsigned long long)p * R + r0 + j] = stage[j][p];
                    }
                }
                rr++;
                __syncthreads();
                continue;
            }
            /* a wave per part: consecutive entries to consecutive slots; the
               part's round count cleared and its written count advanced by
               that wave alone.  (Round 6: whole aligned 16-B pieces with the
               unaligned rest carried to the next round measured slower.) */
            for (uint32_t p = wv; p < gp; p += 16u) {
                const uint32_t n = hc[p], o = ho[p];
                if (poff[p] != ~0ull) {
                    OT *dst = out + poff[p] + wr[p];
                    for (uint32_t j = lane; j < n; j += 64u) dst[j] = rbuf[o + j];
                }
                if (lane == 0) { wr[p] += n; hc[p] = 0; }
            }
            __syncthreads();
        }
    }
}

