/*
 * fk_part.hip -- the partitioned count for 8 <= k <= 16 (findKmer.cpp:1035-1042
 * into the trie of :663-690): k_part (fast tiles into LDS-sorted batches of
 * slice codes), k_bucket_count / k_bucket16 (a slice of the table per block
 * in LDS), k_repart + k_count_parts (k = 15, 16), k_pair_fold, and launch_part.
 */
#include "fk_part_kern.h"

/* (compiled in fk_part_pipe.hip / fk_part_res.hip) */
FK_PART_PIPE_INSTANCES(FK_PART_EXTERN)
FK_PART_OTHER_INSTANCES(FK_PART_EXTERN)

/* k_bucket_count's first loads per quad: BUCKET_ROWS rows at once, each
   with BUCKET_U 16-B pieces per lane (64 B per quad each).  2 x 4 (256 B
   of a ~200-B run, k=11 with 16-wave k_part blocks) beat 4 x 2 by ~1 %
   (k=11 step 1.082 -> 1.070 ms); 3 x 3, 3 x 4 and 1 x 8 fell in between.
   2 x 5 (95 VGPRs, still 4 waves per SIMD): a k=11 pair run is ~120 codes,
   so 4 pieces per lane (128 codes from the aligned-down start) sent a third
   of the runs -- and so nearly every wave of 16 runs -- through the
   long-run loop for a few codes; k_bucket_count 334 -> 325 us, k=11 step
   1.081 -> 1.074 ms, k=12 1.684 -> 1.669 ms, k=8 unchanged (2 x 6: the
   same within noise; 3 x 5 at 128 VGPRs 331 -> 351 us, 1 x 10 -> 341 us). */
#define BUCKET_U 5
#define BUCKET_ROWS 2
/* MODE (a template parameter, so that the hot loop of the common k carries
   no test of it: a runtime flag there cost ~0.9 ms of a k=11 10 GB step):
   BK_PLAIN 16-bit codes, one block per slice (and row group).  (Round 4's
            BK_SPLIT, k = 14 counted as two blocks per 2^16-bin slice that
            each read all of its codes, is k_bucket16's now.) */
/* BK_PAD: BK_PLAIN over padded runs (PART_PAD: a run starts on a 16-B
            piece, its index word holds that piece; only its last piece
            needs a mask) */
enum { BK_PLAIN = 0, BK_PAD = 2 };
template <int MODE>
__global__ void __launch_bounds__(1024)
k_bucket_count(PartGeo pg, uint32_t groups, uint32_t *table) {
    extern __shared__ uint32_t slice[];
    constexpr bool PADDED = MODE == BK_PAD;
    constexpr uint32_t CPP = 8u;   /* 16-bit codes per 16-B piece */
    constexpr uint32_t PSH = 3u;
    const uint32_t nb = 1u << pg.sh;
    /* pairs mode: the slice's 2^sh pair bins, then the 2^(sh-2) bins of the
       single k-mers filed under it (PART_SINGLE codes) */
    const uint32_t ns = pg.pairs ? nb >> 2 : 0u;
    /* consecutive slices on one XCD (blocks b, b + 8, .. share an XCD): the
       128-B line two neighbouring runs of a row share is fetched once into
       that XCD's L2 (k=11: 1 GB step 1.085 -> 1.065 ms, 10 GB 8.10 -> 8.04) */
    const uint32_t b = groups == 1 && (pg.nslices & 7u) == 0 ? (blockIdx.x & 7u) * (pg.nslices >> 3) + (blockIdx.x >> 3)
                                                             : blockIdx.x % pg.nslices;
    const uint32_t g = blockIdx.x / pg.nslices;
    for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) slice[i] = 0;
    __syncthreads();
    const uint32_t *ix = pg.idx + b;
    /* region 2 (k_part<RES>) holds rows only if some range went there */
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    /* four lanes share a run and read it as contiguous 64-byte pieces (one
       request per quad instead of one per lane).  (k = 14, round 4: a lane
       per run with 4 rows and 3 pieces each in flight fetched 19.4 GB per
       G-base instead of 5.3 -- 33 MB of lines in flight per XCD evict the
       lines the slice's other half and its neighbours would read from L2 --
       and took 3.46 ms instead of 2.86.)  A quad takes BUCKET_ROWS
       rows at once: their first 64 * BUCKET_U bytes of codes and the next
       rows' index words are all in flight together (a run is ~50-250 codes, so one
       dependent chain per run would leave the CU waiting on latency; rows
       sit at fixed offsets, so a run's position needs no further load) */
    constexpr uint32_t QL = 4u;   /* lanes per run */
    const uint32_t sub = threadIdx.x & (QL - 1u);
    const uint32_t quads = blockDim.x / QL, step = groups * quads;
    auto add16 = [&](const uint4 &v, uint64_t q, uint64_t s0, uint64_t s1) {
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const uint32_t nv = PADDED ? (uint32_t)min<uint64_t>(CPP, s1 - q * CPP) : 0u;   /* codes of the run in q */
#pragma unroll
        for (int h = 0; h < (int)CPP; h++) {
            const uint64_t at = q * CPP + h;
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            if (PADDED) {   /* the run starts on this lane's first piece: only its end bounds it */
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if ((uint32_t)h < nv) atomicAdd(&slice[a], 1u);
            } else {
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if (at >= s0 && at < s1) atomicAdd(&slice[a], 1u);
            }
        }
    };
    uint32_t en[BUCKET_ROWS];   /* the next iteration's index words, loaded with this one's codes */
    const uint32_t r00 = g * quads + threadIdx.x / QL;
#pragma unroll
    for (int j = 0; j < BUCKET_ROWS; j++) en[j] = r00 + j * step < nrows ? ix[(size_t)(r00 + j * step) * pg.nslices] : PART_NO_RUN;
    for (uint32_t r = r00; r < nrows; r += BUCKET_ROWS * step) {
        uint32_t e[BUCKET_ROWS];
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) e[j] = en[j];
        const uint32_t rn = r + BUCKET_ROWS * step;
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) en[j] = rn + j * step < nrows ? ix[(size_t)(rn + j * step) * pg.nslices] : PART_NO_RUN;
        uint64_t s0[BUCKET_ROWS], s1[BUCKET_ROWS];
        uint4 v[BUCKET_ROWS][BUCKET_U];
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) {
            s0[j] = (uint64_t)(r + j * step) * pg.batch + (e[j] == PART_NO_RUN ? 0u : (e[j] >> 16) * (PADDED ? CPP : 1u));
            s1[j] = s0[j] + run_count(e[j]);
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (int u = 0; u < BUCKET_U; u++) v[j][u] = q0 + QL * u < q1 ? g4[q0 + QL * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) {
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (int u = 0; u < BUCKET_U; u++)
                if (q0 + QL * u < q1) add16(v[j][u], q0 + QL * u, s0[j], s1[j]);
            /* the rest of a long run */
            for (uint64_t q = q0 + QL * BUCKET_U; q < q1; q += 4 * QL) {
                uint4 w[4];
#pragma unroll
                for (int u = 0; u < 4; u++) w[u] = q + QL * u < q1 ? g4[q + QL * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (q + QL * u < q1) add16(w[u], q + QL * u, s0[j], s1[j]);
            }
        }
    }
    __syncthreads();
    if (pg.pairs) {
        /* pairs mode: the slice's bins, in kernel index order, into the pair
           and single bins (k_pair_fold reduces them into the table) */
        uint32_t *dp = pg.pairs + ((size_t)b << pg.sh), *ds = pg.singles + ((size_t)b << (pg.sh - 2));
        for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) {
            const uint32_t v = slice[i];
            uint32_t *dst = i < nb ? dp + i : ds + (i - nb);
            if (groups == 1) *dst = v;   /* this block owns the slice: every bin written */
            else if (v) atomicAdd(dst, v);
        }
        return;
    }
    const uint64_t base = (uint64_t)b << pg.sh;
    if (groups != 1) {
        for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
            const uint32_t v = slice[i];
            if (v) atomicAdd(&table[fk_sigma(base | i)], v);
        }
        return;
    }
    /* this block owns the slice: eight loads in flight per lane before the
       adds and stores (one load-add-store chain at a time is latency-bound) */
    constexpr uint32_t U = 8u;
    for (uint32_t i0 = threadIdx.x; i0 < nb; i0 += U * blockDim.x) {
        uint32_t v[U], o[U];
#pragma unroll
        for (uint32_t j = 0; j < U; j++) {
            const uint32_t i = i0 + j * blockDim.x;
            v[j] = i < nb ? slice[i] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < U; j++) o[j] = v[j] ? table[fk_sigma(base | (i0 + j * blockDim.x))] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < U; j++)
            if (v[j]) table[fk_sigma(base | (i0 + j * blockDim.x))] = o[j] + v[j];
    }
}

/*
 * W16 (k = 11..14): slices of 2^16 bins counted in 16-bit LDS bins, two per
 * word (128 KiB for the whole slice).  Against 2^15-bin slices in 32-bit bins
 * that halves the slices, so every run a block reads is twice as long (k =
 * 11: ~240 codes, 480 B) and the reads of a run's partial first and last
 * lines are half as many; k = 14 counts a slice in one block instead of two
 * blocks that each read all of its codes.  A code c adds 1 << 16 (c & 1) to
 * word c >> 1 (non-returning, as the 32-bit bins).  A 16-bit bin that wraps
 * carries into its neighbour (low half) or out of the word (high half): both
 * make the sum of the halves fall short of the codes counted, and nothing
 * else does, so the block checks that sum against its exact count and, only
 * if it fell short (a bin past 65535 codes in one slice: poly-A stretches),
 * counts the slice again as two halves of 2^15 32-bit bins.  (Round 2 tried
 * 16-bit bins with returning atomics to catch wraps as they happen: 20 %
 * slower; the sum check costs one add per word.)
 *
 * Blocks: pairs mode puts the single k-mers (a '\n' half's slot 1) in their
 * own slices [npair, nbk), lightly loaded: they come first, so the pair
 * slices -- consecutive ones on one XCD, as k_bucket_count -- start at most
 * one light block late.
 */
/* Every code of slice b's runs (index column ix) as f(code): QL lanes per
   run reading 16-B pieces (QL x 16 B contiguous per request), ROWS rows per
   lane group in flight with U pieces each, the next rows' index words loaded
   with this iteration's codes (k_bucket_count's shape) */
template <uint32_t QL, uint32_t ROWS, uint32_t U, bool PADDED, typename F>
__device__ __forceinline__ void walk_runs(const PartGeo &pg, const uint32_t *ix, uint32_t nrows, F &&f) {
    constexpr uint32_t CPP = 8u, PSH = 3u;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    const uint32_t sub = threadIdx.x & (QL - 1u), groups = blockDim.x / QL;
    auto add16 = [&](const uint4 &v, uint64_t q, uint64_t s0, uint64_t s1) {
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const uint32_t nv = PADDED ? (uint32_t)min<uint64_t>(CPP, s1 - q * CPP) : 0u;
#pragma unroll
        for (int h = 0; h < (int)CPP; h++) {
            const uint64_t at = q * CPP + h;
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            if (PADDED ? (uint32_t)h < nv : (at >= s0 && at < s1)) f(c);
        }
    };
    uint32_t en[ROWS];
    const uint32_t r00 = threadIdx.x / QL;
#pragma unroll
    for (uint32_t j = 0; j < ROWS; j++)
        en[j] = r00 + j * groups < nrows ? ix[(size_t)(r00 + j * groups) * pg.nslices] : PART_NO_RUN;
    for (uint32_t r = r00; r < nrows; r += ROWS * groups) {
        uint32_t e[ROWS];
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) e[j] = en[j];
        const uint32_t rn = r + ROWS * groups;
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++)
            en[j] = rn + j * groups < nrows ? ix[(size_t)(rn + j * groups) * pg.nslices] : PART_NO_RUN;
        uint64_t s0[ROWS], s1[ROWS];
        uint4 v[ROWS][U];
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) {
            s0[j] = (uint64_t)(r + j * groups) * pg.batch + (e[j] == PART_NO_RUN ? 0u : (e[j] >> 16) * (PADDED ? CPP : 1u));
            s1[j] = s0[j] + run_count(e[j]);
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (uint32_t u = 0; u < U; u++) v[j][u] = q0 + QL * u < q1 ? g4[q0 + QL * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) {
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (uint32_t u = 0; u < U; u++)
                if (q0 + QL * u < q1) add16(v[j][u], q0 + QL * u, s0[j], s1[j]);
            for (uint64_t q = q0 + QL * U; q < q1; q += 4 * QL) {
                uint4 w[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) w[u] = q + QL * u < q1 ? g4[q + QL * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    if (q + QL * u < q1) add16(w[u], q + QL * u, s0[j], s1[j]);
            }
        }
    }
}

/* the heavy (pair or plain) slices' walk shape: 4 lanes per run, 2 rows x 3
   pieces in flight (QL 1, 2, 8 and U 4, 5 measured slower); the singles' slices hold a few codes
   per run, so a lane per run and 4 rows in flight (their walk is a chain of
   index and code loads: with the heavy shape the 64 single-slice blocks of
   k = 11 took ~0.3 ms, which the pair slices' last blocks waited out) */
/* W16 for k = 12, 13, 14 (1 G-base FASTA steps, round 5: k = 12 1.33 ->
   1.22 ms, k = 13 2.12 -> 1.84 ms, k = 14 4.4 -> 3.35 ms).  Not k = 11:
   its runs are long already (~120 codes), and with half the slices k_part's
   histogram and cursor atomics collide more often within a wave (k_part
   4.40 -> 4.51 ms per 10 G bases) while k_bucket16's 256 heavy blocks run
   as one round (k_bucket 2.31 -> 2.6-3.0 ms over the shapes tried): step
   6.79 -> 7.2-7.7 ms.  k = 14 has no other path (2^16-bin slices). */

#define B16_QL 4
#define B16_ROWS 2
#define B16_U 3   /* (5: k = 12 1.250, 13 1.837, 14 3.348 ms per G-base; 3: 1.228, 1.820, 3.294) */
#define B16L_QL 1
#define B16L_ROWS 4
#define B16L_U 1
template <bool PADDED>
__global__ void __launch_bounds__(1024)
k_bucket16(PartGeo pg, uint32_t *table) {
    extern __shared__ uint32_t bins[];
    constexpr uint32_t NW = 1u << 15;   /* words: 2^16 16-bit bins, or 2^15 32-bit ones */
    const uint32_t nsing = pg.pairs ? pg.nbk - pg.npair : 0u;
    uint32_t b;
    if (blockIdx.x < nsing) {
        b = pg.npair + blockIdx.x;
    } else {
        const uint32_t j = blockIdx.x - nsing, nh = pg.nbk - nsing;   /* (nh a multiple of 8) */
        b = (j & 7u) * (nh >> 3) + (j >> 3);
    }
    const bool light = b >= pg.npair && nsing;
    const uint32_t *ix = pg.idx + b;
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    auto walk = [&](auto &&f) {
        if (light) walk_runs<B16L_QL, B16L_ROWS, B16L_U, PADDED>(pg, ix, nrows, f);
        else walk_runs<B16_QL, B16_ROWS, B16_U, PADDED>(pg, ix, nrows, f);
    };
    /* where bin i of the slice goes: pairs mode -> the pair or single bins
       (k_pair_fold reduces them, this block owns them: stored), else the
       table (added, reference index order) */
    uint32_t *dst = nullptr;
    if (pg.pairs) dst = b < pg.npair ? pg.pairs + ((size_t)b << 16) : pg.singles + ((size_t)(b - pg.npair) << 16);
    const uint64_t base = (uint64_t)b << 16;
    /* fresh (round 5: the segment's k_zero left the table out, the general
       tiles' windows wait in pg.glist): every bin of the slice written, no
       read, and the table statistics taken here (pg.fz, as k_count_parts) */
    const bool fresh = pg.glist != nullptr && !pg.pairs;
    unsigned long long sd = 0, l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    auto out2 = [&](uint32_t i2, uint32_t lo, uint32_t hi) {   /* bins 2 i2, 2 i2 + 1 */
        if (!(lo | hi) && !pg.pairs && !fresh) return;
        if (pg.pairs) {
            reinterpret_cast<uint2 *>(dst)[i2] = make_uint2(lo, hi);
        } else {
            /* sigma maps the last digit 0 1 2 3 -> 0 1 3 2: the pair stays
               adjacent, swapped when the last digit of 2 i2 is 2 */
            uint2 *t2 = reinterpret_cast<uint2 *>(table + (fk_sigma(base | (2u * i2)) & ~1ull));
            if (fresh) {   /* (streaming stores, as the sparse outputs: not read back soon) */
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 ov = (i2 & 1u) ? u32x2{hi, lo} : u32x2{lo, hi};
                __builtin_nontemporal_store(ov, reinterpret_cast<u32x2 *>(t2));
                sd += (lo != 0u) + (hi != 0u);
                if (i2 & 1u) { l3 += lo; l2 += hi; } else { l0 += lo; l1 += hi; }
                return;
            }
            uint2 o = *t2;
            if (i2 & 1u) { o.x += hi; o.y += lo; } else { o.x += lo; o.y += hi; }
            *t2 = o;
        }
    };
    /* the block's statistics into one of the FZ_SLOTS partials: distinct,
       sum, last-base marginals, and the sum under the slice's first base
       (the slice's bins share their top 16 index bits) */
    __shared__ unsigned long long fzw[16][6];
    auto fz_flush = [&]() {
        if (!fresh) return;
        unsigned long long v6[6] = {sd, l0 + l1 + l2 + l3, l0, l1, l2, l3};
#pragma unroll
        for (int q = 0; q < 6; q++) v6[q] = wsum64(v6[q]);
        if ((threadIdx.x & 63) == 0)
#pragma unroll
            for (int q = 0; q < 6; q++) fzw[threadIdx.x >> 6][q] = v6[q];
        __syncthreads();
        if (threadIdx.x < 10) {
            const uint32_t q = threadIdx.x;
            unsigned long long t = 0;
            for (uint32_t w = 0; w < 16; w++) t += fzw[w][q < 6 ? q : 1u];
            if (q >= 6 && (uint32_t)((fk_sigma(base) >> (2 * pg.kk - 2)) & 3u) != q - 6u) t = 0;
            if (t) atomicAdd(&pg.fz[(blockIdx.x % FZ_SLOTS) * 10u + q], t);
        }
    };
    for (uint32_t i = threadIdx.x; i < NW / 4u; i += blockDim.x) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    uint32_t n = 0;
    walk([&](uint32_t c) {
        atomicAdd(&bins[c >> 1], 1u << ((c & 1u) << 4));
        n++;
    });
    __syncthreads();
    /* the wrap check: sum of the halves == codes counted */
    unsigned long long hs = 0;
    for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) hs += (bins[i] & 0xFFFFu) + (bins[i] >> 16);
    __shared__ unsigned long long red[2][16];
    {
        const unsigned long long a = wsum64(hs), c = wsum64((unsigned long long)n);
        if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = c; }
    }
    __syncthreads();
    unsigned long long sa = 0, sc = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) { sa += red[0][w]; sc += red[1][w]; }
    if (sa == sc) {
        for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) out2(i, bins[i] & 0xFFFFu, bins[i] >> 16);
        fz_flush();
        return;
    }
    /* a 16-bit bin wrapped: the slice again, as two halves of 2^15 32-bit bins */
    for (uint32_t h = 0; h < 2u; h++) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < NW / 4u; i += blockDim.x) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        walk([&](uint32_t c) {
            if ((c >> 15) == h) atomicAdd(&bins[c & 0x7FFFu], 1u);
        });
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < NW / 2u; i += blockDim.x) {
            const uint32_t i2 = (h << 14) + i;   /* bins (h << 15) + 2 i, + 1 */
            out2(i2, bins[2u * i], bins[2u * i + 1u]);
        }
    }
    fz_flush();
}


/* k_count_parts: one block per part, its stream into 2^15 LDS bins, then
   into the table.  The bins are 16-bit halves of 2^14 LDS words (64 KiB, two
   blocks per CU: one block's count overlaps the other's table writes; round
   5's 128 KiB of 32-bit bins left one block per CU alternating between them:
   k = 16 1 G-base step 10.1 -> 9.5 ms, k = 15 equal).  A wrapped bin (the
   halves' sum short of the part's codes) counts the part again as two
   halves of 2^14 32-bit bins.  The part's first pieces load while the bins
   are zeroed (round 6: the stream had been read one latency-bound piece at a
   time after the zeroing).  On a fresh table (the segment's k_zero left it
   out) every bin is written, no read (k = 16: 17 GB of zeroing and 17 GB of
   reads less per step), with streaming stores (the 16 GiB table is not read
   back soon: 10.74 -> 10.42 ms), and the statistics k_table_stats would
   read the table for (distinct, sum, last- and first-base marginals) taken
   here: they stand unless the general tiles' list or k_redo adds to the
   table afterwards. */
__global__ void __launch_bounds__(1024, 8)
k_count_parts(PartGeo pg, const uint16_t *in, RepartSeg sg, uint32_t *table) {
    extern __shared__ uint32_t bins[];   /* 2^14 words */
    __shared__ uint32_t s_hs, s_n;
    __shared__ unsigned long long wred[16][6];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t np = 1u << pg.split, gp = REPART_G * np;
    const uint32_t b = blockIdx.x / np, part = blockIdx.x % np;
    /* the part's segments: row blockIdx % gp of k_repart block blockIdx / gp's table */
    const uint32_t g = blockIdx.x / gp, pi = blockIdx.x % gp;
    const unsigned long long dbase = sg.bmeta[2 * (size_t)g];
    const uint32_t R = (uint32_t)sg.bmeta[2 * (size_t)g + 1];
    if (t == 0) { s_hs = 0; s_n = 0; }
    /* hsel < 0: bin c at half c & 1 of word c >> 1; else only bins [hsel 2^14, ..) as 32-bit words */
    auto add1 = [&](uint32_t c, int hsel) {
        c &= 0x7FFFu;
        if (hsel < 0) atomicAdd(&bins[c >> 1], 1u << ((c & 1u) << 4));
        else if ((c >> 14) == (uint32_t)hsel) atomicAdd(&bins[c & 0x3FFFu], 1u);
    };
    auto zero = [&]() {
        for (uint32_t i = t; i < (1u << 12); i += 1024u) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    };
    {
        const uint32_t mine = seg_codes(in, sg.desc, dbase, R, pi, [&](uint32_t c) { add1(c, -1); }, [&]() {
            zero();
            __syncthreads();
        });
        const uint32_t a = wsum32(mine);
        if (lane == 0 && a) atomicAdd(&s_n, a);
    }
    __syncthreads();
    const struct { uint32_t n; } m{s_n};
    {   /* the wrap check */
        uint32_t hs = 0;
        for (uint32_t i = t; i < (1u << 14); i += 1024u) hs += (bins[i] & 0xFFFFu) + (bins[i] >> 16);
        const uint32_t a = wsum32(hs);
        if (lane == 0) atomicAdd(&s_hs, a);
    }
    __syncthreads();
    const bool wrap = s_hs != m.n;
    const uint64_t base = ((uint64_t)b << pg.sh) | ((uint64_t)part << 15);
    const bool fresh = pg.glist != nullptr;
    uint32_t dist = 0;
    unsigned long long last[4] = {0, 0, 0, 0};
    /* bins 4 m4 .. 4 m4 + 3 of the part: kernel bins 4m + d land at reference
       index sigma(base | 4m) + sigma(d), i.e. the last digits 0 1 3 2: one
       16-B store on a fresh table (streaming: the table is not read back
       soon), else each nonzero bin added */
    auto out4 = [&](uint32_t m4, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
        const uint64_t r = fk_sigma(base | ((uint64_t)m4 << 2));
        if (fresh) {
            const u32x4 ov = {c0, c1, c3, c2};
            __builtin_nontemporal_store(ov, reinterpret_cast<u32x4 *>(table) + (r >> 2));
            dist += (c0 != 0) + (c1 != 0) + (c2 != 0) + (c3 != 0);
            last[0] += c0; last[1] += c1; last[2] += c3; last[3] += c2;
        } else {
            const uint32_t cc[4] = {c0, c1, c3, c2};
#pragma unroll
            for (int d = 0; d < 4; d++)
                if (cc[d]) table[r + (uint64_t)d] += cc[d];
        }
    };
    if (!wrap) {
        for (uint32_t m4 = t; m4 < (1u << 13); m4 += 1024u) {
            const uint2 w = reinterpret_cast<const uint2 *>(bins)[m4];
            out4(m4, w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16);
        }
    } else {
        for (int h = 0; h < 2; h++) {
            __syncthreads();
            zero();
            __syncthreads();
            seg_codes(in, sg.desc, dbase, R, pi, [&](uint32_t c) { add1(c, h); });
            __syncthreads();
            for (uint32_t i = t; i < (1u << 12); i += 1024u) {
                const uint4 w = reinterpret_cast<const uint4 *>(bins)[i];
                out4(((uint32_t)h << 12) + i, w.x, w.y, w.z, w.w);
            }
        }
    }
    if (!fresh) return;
    const int fs = 2 * pg.kk - 2;
    const unsigned long long sum = last[0] + last[1] + last[2] + last[3];
    unsigned long long v6[6] = {dist, sum, last[0], last[1], last[2], last[3]};
#pragma unroll
    for (int q = 0; q < 6; q++) v6[q] = wsum64(v6[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 6; q++) wred[wv][q] = v6[q];
    __syncthreads();
    if (t < 10) {
        unsigned long long a = 0;
        if (t < 6) {
            for (uint32_t w = 0; w < 16; w++) a += wred[w][t];
        } else {   /* the first base of every bin of the part: one digit */
            for (uint32_t w = 0; w < 16; w++) a += wred[w][1];
            if ((uint32_t)((fk_sigma(base) >> fs) & 3u) != t - 6u) a = 0;
        }
        if (a) atomicAdd(&pg.fz[(blockIdx.x % FZ_SLOTS) * 10u + t], a);
    }
}

/* the general tiles' windows of a fresh two-level table (hist_add's list) */
__global__ void k_list_init(uint32_t *list, uint32_t cap, unsigned long long *fz) {
    if (threadIdx.x == 0) { list[0] = 0; list[1] = cap; }
    for (uint32_t i = threadIdx.x; i < FZ_SLOTS * 10u; i += blockDim.x) fz[i] = 0;
}
__global__ void __launch_bounds__(256)
k_list_add(const uint32_t *list, uint32_t *table, int k, unsigned long long *fz) {
    const uint32_t n = min(list[0], list[1]);
    const int fs = 2 * k - 2;
    /* with what each window changes in the statistics k_count_parts took
       (the old value of its bin tells whether it was distinct before) */
    unsigned long long v10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t x = list[2 + i];
        const uint32_t old = atomicAdd(&table[x], 1u);
        v10[0] += old == 0;
        v10[1] += 1;
        v10[2 + (x & 3u)] += 1;
        v10[6 + ((x >> fs) & 3u)] += 1;
    }
#pragma unroll
    for (int q = 0; q < 10; q++) {
        const unsigned long long t = wsum64(v10[q]);
        if ((threadIdx.x & 63) == 0 && t) atomicAdd(&fz[((blockIdx.x * 4u + (threadIdx.x >> 6)) % FZ_SLOTS) * 10u + q], t);
    }
}

/* pairs mode: every k-mer x (kernel order) is the prefix of the pairs
 * 4x + b and the suffix of the pairs b*4^k + x (a pair stands for both of
 * its k-mers), plus the single windows counted at x */
__global__ void __launch_bounds__(256)
k_pair_fold(const uint32_t *pairs, const uint32_t *singles, uint64_t nbins, uint32_t *table, int fresh) {
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < nbins; x += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 pre = reinterpret_cast<const uint4 *>(pairs)[x];
        uint32_t v = pre.x + pre.y + pre.z + pre.w + singles[x];
#pragma unroll
        for (int b = 0; b < 4; b++) v += pairs[(uint64_t)b * nbins + x];
        if (fresh) table[fk_sigma(x)] = v;   /* (a fresh table: k_zero left it out) */
        else if (v) table[fk_sigma(x)] += v;
    }
}


/* k_part + k_bucket_count over a resolved segment (exact range states in
   d_rtrue): the counting of the partitioned path */
int launch_part(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int has_init,
                       const XState *exact) {
    PartGeo pg;
    const int k = e->k;
    /* k <= 12: (k+1)-mer pairs at every other base (half the entries), plus
       the single k-mers at the first slot of halves with a '\n' */
    const bool pairs = k <= e->part_pairs_kmax;
    const int kb = pairs ? k + 1 : k;                      /* bits of a pair (or window) code: 2 kb */
    /* >= 64 slices, <= 2^15 bins (128 KiB) each; k = 14: 2^16 codes per slice,
       counted as two halves (PART_BIG); k = 15, 16: 2048 coarse slices of
       2^19 / 2^21 32-bit codes, counted in 2^15-bin parts */
    const bool c32 = k >= 15;
    /* 2^16-bin slices counted in 16-bit LDS bins (k_bucket16) for the k in
       e->w16_ks (12 <= k <= 14) */
    const bool w16 = !c32 && k >= 12 && ((e->w16_ks >> k) & 1u);
    pg.w16 = w16 ? 1u : 0u;
    pg.sh = c32 ? 2 * k - 11 : w16 ? 16 : std::min(15, 2 * kb - 6);
    pg.split = c32 ? (uint32_t)(pg.sh - 15) : 0u;
    pg.npair = pairs ? 1u << (2 * kb - pg.sh) : 0u;
    if (pairs && w16) {
        /* the single k-mers in their own 2^16-bin slices after the pair slices */
        pg.sbase = pg.npair;
        pg.slsh = 0;
        pg.sflag = 0;
        pg.nbk = pg.npair + (1u << (2 * k - 16));
        /* (k = 12: 1280 slices in an index row of 2048, the width k_part's
           all-wave scan divides among its 16 waves) */
        pg.nslices = pg.nbk <= 512u ? pg.nbk : (pg.nbk + 1023u) & ~1023u;
    } else {
        /* singles filed under the pair code x << 2 (PART_SINGLE) */
        pg.sbase = 0;
        pg.slsh = 2;
        pg.sflag = PART_SINGLE;
        pg.nslices = pairs ? pg.npair : 1u << (2 * k - pg.sh);
        pg.nbk = pg.nslices;
    }
    pg.pairs = pg.singles = nullptr;
    pg.nomix = e->no_mixed ? 1u : 0u;
    pg.glist = nullptr;
    pg.fz = nullptr;
    pg.kk = (uint32_t)k;
    e->fz_ready = false;
    e->glist_live = false;
    if ((c32 || w16) && e->tab_fresh && !exact) {
        /* the general tiles' windows go to a list (hist_add): at most
           part_general + 3 general tiles per range (the comment lines or run
           breaks k_part takes and the bases-only tiles around them, the
           ragged last tile in k_part<RES>; tile_mixed takes every other tile
           outside the int32 zone, which tab_fresh excludes, and with
           no_mixed there is no fresh table).  Should a segment hold more,
           hist_add drops what does not fit and k_table_stats flags it
           (FK_FAULT_LIST): resolve_and_fetch counts the segment again */
        uint64_t cap = (uint64_t)g.nranges * (e->part_general + 3u) * FK_TILE_BYTES + 4096u;
        if (e->glist_force) cap = e->glist_force;
        if (cap + 2 > e->glist_cap) {
            hipFree(e->d_glist);
            e->d_glist = nullptr;
            e->glist_cap = 0;
            if (hipMalloc((void **)&e->d_glist, (cap + 2) * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
            e->glist_cap = cap + 2;
        }
        if (!e->d_fz && hipMalloc((void **)&e->d_fz, FZ_SLOTS * 10 * sizeof(unsigned long long)) != hipSuccess)
            return FK_E_OOM;
        hipLaunchKernelGGL(k_list_init, dim3(1), dim3(256), 0, e->stream, e->d_glist, (uint32_t)cap, e->d_fz);
        HIPCHK(hipGetLastError());
        pg.glist = e->d_glist;
        pg.fz = e->d_fz;
        /* the statistics: k_count_parts / k_bucket16 take them (pairs mode:
           k_table_stats reads the folded table) */
        e->fz_ready = !pairs;
        e->glist_live = true;
    }
    e->tab_fresh = false;
    if (pairs) {
        const uint64_t need = e->nbins * 5;                 /* 4^(k+1) pair bins + 4^k single bins */
        if (need > e->pair_cap) {
            hipFree(e->d_pairs);
            e->d_pairs = nullptr;
            if (hipMalloc((void **)&e->d_pairs, need * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
            e->pair_cap = need;
        }
        pg.pairs = e->d_pairs;
        pg.singles = e->d_pairs + e->nbins * 4;
    }
    pg.rounds = (uint32_t)((g.cpw * FK_CHUNK_TILES + 2) / PART_TILES3(pairs, c32) + 2);   /* rows (batches) per block */
    /* block size: 16 waves (larger batches, longer runs for k_bucket_count)
       for the tables of 512 slices or more, else 8 */
    const uint32_t W = part_waves_of(e);
    pg.batch = c32 ? W * FK_TILE_BYTES : PART_MAX_BATCH_W(W);   /* entries per row slot */
    const unsigned pgrid = (unsigned)((g.nranges + W - 1) / W);   /* the same ranges as k_count's waves */
    pg.rows = pgrid * pg.rounds;
    /* mixed tiles: ranges past their general tiles go to k_part<RES>, whose
       rows (region 2, as many as k_part's) follow k_part's */
    const bool mixed = !e->no_mixed;
    /* one comment line (or run break) per range stays here; a second one
       sends the range to k_part<RES>, whose block-wide rounds only pay off
       when many ranges go there */
    pg.general = e->part_general;
    pg.stride = mixed ? 2 * pg.rows : pg.rows;
    if (!e->d_pflag && hipMalloc((void **)&e->d_pflag, 64) != hipSuccess) return FK_E_OOM;
    pg.flag = e->d_pflag;
    HIPCHK(hipMemsetAsync(e->d_pflag, 0, sizeof(uint32_t), e->stream));
    /* runs padded to 16-B pieces (PART_PAD: the instances of at most 512
       slices, i.e. the 8-wave blocks of k <= 10 and k = 11's pairs): the row
       slot grows by one pad piece per slice */
    const bool padded = !c32 && k != 14 && (W == 8u || (k == 11 && pairs));
    if (padded) pg.batch += PART_ROW_PAD(W == 8u ? PART_SM(8u) : PART_PAD_MAX_SM) / 2u;
    const uint64_t ncodes = (uint64_t)pg.stride * pg.batch * (c32 ? 2u : 1u),
                   nidx = (uint64_t)pg.nslices * pg.stride;
    if (ncodes > e->codes_cap) {
        hipFree(e->d_codes);
        e->d_codes = nullptr;
        if (hipMalloc((void **)&e->d_codes, ncodes * sizeof(uint16_t)) != hipSuccess) return FK_E_OOM;
        e->codes_cap = ncodes;
    }
    if (nidx > e->pidx_cap) {
        hipFree(e->d_pidx);
        e->d_pidx = nullptr;
        if (hipMalloc((void **)&e->d_pidx, nidx * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
        e->pidx_cap = nidx;
    }
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    /* the main pass: pipelined batches (PIPE) for k = 8..13 (<= 512 slices,
       wave 0 scanning alone; k = 12 pairs and k = 13: 2048 slices, the scan
       over all waves), phase by phase for k = 14 (PART_BIG) and k = 15, 16
       (C32); the headline k = 11 with k a compile-time constant */
    auto kmain = c32 ? k_part<false, false, 16u, PART_SM(16u), true>
                 : k == 14 ? k_part<false, false, 16u, PART_BIG>
                 : W == 16u ? (pairs ? (k == 11 ? k_part<true, false, 16u, PART_PAD_MAX_SM, false, true, 11u>
                                                : k_part<true, false, 16u, PART_SM(16u), false, true>)
                                     : k_part<false, false, 16u, PART_SM(16u), false, true>)
                            : (pairs ? k_part<true, false, 8u, PART_SM(8u), false, true>
                                     : k_part<false, false, 8u, PART_SM(8u), false, true>);
    hipExtLaunchKernelGGL(kmain, dim3(pgrid), dim3(PART_BLOCK_W(W)), 0, e->stream, tev(e, 0), tev(e, 1), 0, buf, len,
                          lo, e->k, e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nchunks, g.cpw,
                          e->d_state, has_init, pg, e->d_resume, exact);
    HIPCHK(hipGetLastError());
    if (mixed) {
        auto kres = c32 ? k_part<false, true, 16u, PART_SM(16u), true>
                    : k == 14 ? k_part<false, true, 16u, PART_BIG>
                    : W == 16u ? (pairs ? (k == 11 ? k_part<true, true, 16u, PART_PAD_MAX_SM> : k_part<true, true, 16u>)
                                        : k_part<false, true, 16u>)
                               : (pairs ? k_part<true, true, 8u> : k_part<false, true, 8u>);
        hipLaunchKernelGGL(kres, dim3(pgrid), dim3(PART_BLOCK_W(W)), 0, e->stream, buf, len, lo, e->k, e->maskk,
                           e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nchunks, g.cpw, e->d_state,
                           has_init, pg, e->d_resume, exact);
        HIPCHK(hipGetLastError());
    } else {
        pg.flag = nullptr;
    }
    const uint32_t groups = w16 ? 1u : std::max<uint32_t>(1, (uint32_t)e->cus / pg.nslices);
    if (pairs && groups > 1) HIPCHK(hipMemsetAsync(e->d_pairs, 0, e->nbins * 5 * sizeof(uint32_t), e->stream));
    const size_t bc_lds = ((size_t)1 << (pg.sh - pg.split)) * sizeof(uint32_t) * (pairs ? 5 : 4) / 4;   /* + single bins */
    if (c32) {
        /* the second partition level: each coarse slice's runs into one
           contiguous 16-bit stream per part, then one block per part */
        const uint64_t nparts = (uint64_t)pg.nslices << pg.split;
        RepartSeg sgs{};
        {   /* (entries <= bytes) */
            int rc = repart_seg_alloc(e, pg, len, REPART_G << pg.split, &sgs);
            if (rc) return rc;
        }
        if (!e->d_pmeta &&
            hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
            return FK_E_OOM;
        PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
        /* [0]: the output claim, [1]: bound-check bits (DevRes::fault) */
        unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
        e->d_perr = alloc + 1;
        e->perr_live = true;
        HIPCHK(hipMemsetAsync(alloc, 0, 2 * sizeof(unsigned long long), e->stream));
        /* k = 15 (16 parts a slice) as k = 16: 4 coarse slices a block, two
           blocks per CU.  (Round 5's lane-per-run k_repart took 8 slices a
           block there: 4.27 ms per G-base against 4.68 with two blocks of 4;
           the span-streamed one 5.42 with 8, 4.50 with 4.) */
        hipLaunchKernelGGL((k_repart<uint16_t, REPART_G, true>), dim3(pg.nslices / REPART_G), dim3(1024), 0, e->stream,
                           pg, e->d_parts, alloc, meta, (uint64_t)e->parts_cap, e->d_perr, 15u, nullptr, sgs);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_count_parts, dim3((unsigned)nparts), dim3(1024), (size_t)1 << 16, e->stream, pg,
                           (const uint16_t *)e->d_parts, sgs, e->d_table);
        if (pg.glist) {
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
        }
    } else if (w16) {
        if (padded)
            hipLaunchKernelGGL(k_bucket16<true>, dim3(pg.nbk), dim3(1024), (size_t)1 << 17, e->stream, pg, e->d_table);
        else
            hipLaunchKernelGGL(k_bucket16<false>, dim3(pg.nbk), dim3(1024), (size_t)1 << 17, e->stream, pg, e->d_table);
        if (pg.glist && !pairs) {   /* (pairs mode: after k_pair_fold below) */
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
        }
    } else if (padded) {
        hipLaunchKernelGGL(k_bucket_count<BK_PAD>, dim3(pg.nslices * groups), dim3(1024), bc_lds, e->stream, pg,
                           groups, e->d_table);
    } else
        hipLaunchKernelGGL(k_bucket_count<BK_PLAIN>, dim3(pg.nslices * groups), dim3(1024), bc_lds, e->stream, pg,
                           groups, e->d_table);
    HIPCHK(hipGetLastError());
    if (pairs) {
        const unsigned fg = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 4, (e->nbins + 255) / 256);
        hipLaunchKernelGGL(k_pair_fold, dim3(fg), dim3(256), 0, e->stream, e->d_pairs, e->d_pairs + e->nbins * 4,
                           e->nbins, e->d_table, pg.glist ? 1 : 0);
        HIPCHK(hipGetLastError());
        if (pg.glist) {
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
            HIPCHK(hipGetLastError());
        }
    }
    return FK_OK;
}

int repart_seg_alloc(fk_engine *e, const PartGeo &pg, uint64_t ncodes, uint32_t gp, RepartSeg *sg) {
    /* rounds: a block's chunk of up to RP_CHUNK rows takes ceil(pieces /
       4096) rounds, a row's span adding at most two partial pieces */
    const uint64_t nrows = pg.flag ? (uint64_t)pg.stride : (uint64_t)pg.rows;   /* (both regions at most) */
    const uint64_t nblocks = pg.nslices / REPART_G, nchunks = (nrows + RP_CHUNK - 1) / RP_CHUNK;
    const uint64_t rounds = (ncodes / 4 + 2 * nrows * nblocks) / (1024u * 4u) + nblocks * nchunks + 1;
    int rc = sp_ensure((void **)&e->d_parts, &e->parts_cap, ncodes + 8 * rounds + 16, sizeof(uint16_t));
    if (!rc) rc = sp_ensure((void **)&e->d_rdesc, &e->rdesc_cap, (uint64_t)gp * rounds, sizeof(unsigned long long));
    if (!rc) rc = sp_ensure((void **)&e->d_rbm, &e->rbm_cap, 2 * nblocks + 2, sizeof(unsigned long long));
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(e->d_rbm + 2 * nblocks, 0, 2 * sizeof(unsigned long long), e->stream));
    sg->desc = e->d_rdesc;
    sg->dcap = e->rdesc_cap;
    sg->dalloc = e->d_rbm + 2 * nblocks;
    sg->bmeta = e->d_rbm;
    return FK_OK;
}

/* k_bucket_count: one 2^15-bin slice + its 2^13 single bins (160 KiB) in
   LDS; k_bucket16: 128 KiB of bins beside its static reduction words */
int part_kernels_init() {
    for (const void *f : {(const void *)k_bucket_count<BK_PLAIN>,
                          (const void *)k_bucket_count<BK_PAD>, (const void *)k_bucket16<true>,
                          (const void *)k_bucket16<false>})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (f == (const void *)k_bucket16<true> || f == (const void *)k_bucket16<false>)
                                    ? 1 << 17 : 5 << 15) != hipSuccess)
            return FK_E_HIP;
    if (hipFuncSetAttribute((const void *)k_count_parts, hipFuncAttributeMaxDynamicSharedMemorySize, 1 << 16) != hipSuccess)
        return FK_E_HIP;
    return FK_OK;
}
