/*
 * fk_part_kern.h -- k_part, the partition pass of 8 <= k <= 16 (fast tiles'
 * windows counting-sorted by table slice in LDS, written as u16 / u32 codes
 * with a run index).  Its instances are compiled in two translation units
 * (fk_part_pipe.hip: the pipelined main passes, fk_part_res.hip: the rest) and
 * launched from launch_part (fk_part.hip).
 */
#pragma once
#include "fk_engine_internal.h"

template <bool PAIRS, bool MIX, typename F>
__device__ __forceinline__ void part_entries(const Emit &em, uint32_t mk, uint32_t m1, uint32_t sh, uint32_t lowm,
                                             const SingleEnc &se, F &&f) {
    if (MIX && em.masked) {
        /* a mixed tile: only the slots in the mask end windows; a pair where
           both of its slots do, else the single k-mer of the one that does */
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
            const uint32_t cm = (em.cm >> (16 * h)) & 0xFFFFu;
            if (PAIRS) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t two = (cm >> (14 - 2 * j)) & 3u;
                    if (two == 3u) {
                        const uint32_t v = (j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2) & m1;
                        f(v >> sh, v & lowm);
                    } else if (two) {
                        const uint32_t s = 2u * (uint32_t)j + (two == 1u ? 1u : 0u);
                        const uint32_t v = ((s < 15u ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - s)) : S2) & mk) << se.slsh;
                        f(se.sbase + (v >> sh), (v & lowm) | se.sflag);
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    if ((cm >> (15 - i)) & 1u) {
                        const uint32_t v = (i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2) & mk;
                        f(v >> sh, v & lowm);
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
        if (PAIRS) {
            const uint32_t v0 = __builtin_amdgcn_alignbit(C, S2, 28u);
            const uint32_t c0 = skip0 ? (v0 & mk) << se.slsh : (v0 & m1);
            f((skip0 ? se.sbase : 0u) + (c0 >> sh), (c0 & lowm) | (skip0 ? se.sflag : 0u));
#pragma unroll
            for (int j = 1; j < 8; j++) {
                const uint32_t v = (j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2) & m1;
                f(v >> sh, v & lowm);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t v = (i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2) & mk;
                if (i > 0 || !skip0) f(v >> sh, v & lowm);
            }
        }
    }
}

/*
 * Padded runs (PART_PAD: the k_part instances of at most 512 slices, i.e.
 * 8 <= k <= 11 in pairs mode).  A batch's runs start on 16-B pieces in LDS
 * and in its row (the up to 7 codes after a run's last one are whatever the
 * LDS held: k_bucket_count<BK_PAD> masks them by the run's count), so that
 * k_bucket_count reads a run as whole aligned pieces with one mask for its
 * last piece instead of a bounds check per code.  The row slot grows by 16 B
 * per slice (<= 1 pad piece per run).  Measured and dropped (round 4):
 * appending each slice's runs to its own 4 KiB chunks (tools/chunk_probe.hip:
 * whole-chunk reads at 6.1 TB/s): k_bucket_count 2.46 -> 1.93 ms at k = 11
 * over 10 G bases, but k_part 4.40 -> 6.75 ms -- the runs' scattered,
 * line-unaligned stores cost 1.6 ms and the per-slice chunk bookkeeping 0.8.
 */
#define PART_PAD_MAX_SM 512u
#define PART_ROW_PAD(SM) (16u * (SM))   /* bytes of pad pieces a row slot adds */

/* The block-wide batch of one round: windows of the waves whose tile was
 * fast (have), counting-sorted by slice.  Every thread of the block calls
 * this the same number of times (it contains barriers).
 *
 * Round 3 measured (tools/exp_part_probe.py: s_memtime per phase, k=11,
 * 10 GB FASTA, cycles per wave and batch of 16 waves x 4 tiles): tiles 11.4 K,
 * histogram atomics 2.7 K + barrier 5.7 K, wave 0's scan 5.2 K (the others
 * wait 3.2 K), placement 14.3 K + barrier 3.0 K, write-out 2.4 K: the LDS
 * atomics bind.  Spreading each slice's counters over 8 lane buckets (2-way
 * instead of ~3.5-way bank conflicts) with a scan split over all waves did
 * not make the atomic phases cheaper (the atomic instructions' issue, not
 * the banks, sets their cost) and its extra barrier made the batch slower
 * (47.0 K vs 45.7 K cycles), so the scan stays on wave 0. */
template <bool PAIRS, bool MIX, uint32_t W, uint32_t SM, typename CT>
__device__ __forceinline__ bool part_batch(const Ctx &cx, const PartGeo &pg, const Emit *es, const bool *haves,
                                           bool more, uint32_t row, uint32_t *hist,
                                           uint32_t *cur, uint32_t *total, CT *ent, uint32_t *scr) {
    constexpr bool C32 = sizeof(CT) == 4;
    constexpr bool PAD = !C32 && SM <= PART_PAD_MAX_SM;   /* runs padded to 16-B pieces (PART_PAD) */
    constexpr int NT = PART_TILES3(PAIRS, C32);
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint32_t mk = (uint32_t)cx.maskk, sh = pg.sh, lowm = (1u << sh) - 1u;
    const uint32_t m1 = (mk << 2) | 3u;
    const SingleEnc se{pg.sbase, pg.slsh, pg.sflag};
    /* 1: slice histogram */
#pragma unroll
    for (int i = 0; i < NT; i++)
        if (haves[i]) part_entries<PAIRS, MIX>(es[i], mk, m1, sh, lowm, se, [&](uint32_t b, uint32_t) { atomicAdd(&hist[b], 1u); });
    /* (the barrier also tells whether any wave has tiles left) */
    const bool any_more = __syncthreads_or(more);
    /* 2: exclusive scan of the slice counts, index row: wave 0 alone for up
       to 512 slices; k = 13's 2048 slices split over all waves (each sums
       its contiguous share, one more barrier, then scans it from the sum of
       the shares before it) */
    if (!PAIRS && W >= 16u && pg.nslices > 512u) {
        const uint32_t per_w = pg.nslices / W, ppl = per_w / 64u;   /* multiples of 64 */
        const uint32_t wv = t >> 6, b0 = wv * per_w + lane * ppl;
        uint32_t mine = 0;
        for (uint32_t j = 0; j < ppl; j++) mine += hist[b0 + j];
        const uint32_t wt = wsum32(mine);
        if (lane == 0) scr[wv] = wt;
        __syncthreads();
        const uint32_t off = wsum32(lane < wv ? scr[lane] : 0u);
        const uint32_t inc = wscan_incl32(mine);
        uint32_t run = off + inc - mine;
        uint32_t lo16 = 0;
        for (uint32_t j = 0; j < ppl; j++) {
            const uint32_t b = b0 + j, c = hist[b];
            if (SM > 2048u) {   /* packed cursors (b0 and ppl are even) */
                if ((b & 1u) == 0) lo16 = run & 0xFFFFu;
                else cur[b >> 1] = lo16 | (run << 16);
            } else {
                cur[b] = run;
            }
            pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
            hist[b] = 0;
            run += c;
        }
        if (wv == W - 1u && lane == 63) *total = run;
    } else if (PAD && t < 64) {
        /* runs start on 16-B pieces; cursors and run index in entries / pieces */
        const uint32_t per = (pg.nslices + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) sum += (hist[b] + 7u) >> 3;
        }
        const uint32_t inc = wscan_incl32(sum);
        uint32_t run = inc - sum;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) {
                const uint32_t c = hist[b];
                cur[b] = 8u * run;
                pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
                hist[b] = 0;
                run += (c + 7u) >> 3;
            }
        }
        if (lane == 63) *total = 8u * inc;
    } else if (t < 64) {
        const uint32_t per = (pg.nslices + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) sum += hist[b];
        }
        const uint32_t inc = wscan_incl32(sum);
        uint32_t run = inc - sum;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) {
                const uint32_t c = hist[b];
                cur[b] = run;
                pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
                hist[b] = 0;
                run += c;
            }
        }
        if (lane == 63) *total = inc;
    }
    __syncthreads();
    /* 3: place each entry at its slot.  The codes are recomputed from the
       Emit words (laundered, so the compiler cannot keep phase 1's codes
       live across the barriers: that costs more VGPRs than it saves VALU) */
    auto place = [&](uint32_t b, uint32_t low) {
        uint32_t p;
        if (SM > 2048u) {
            const uint32_t h = (b & 1u) * 16u;
            p = (atomicAdd(&cur[b >> 1], 1u << h) >> h) & 0xFFFFu;
        } else {
            p = atomicAdd(&cur[b], 1u);
        }
        ent[p] = (CT)low;
    };
#pragma unroll
    for (int i = 0; i < NT; i++) {
        Emit f = es[i];
        asm volatile("" : "+v"(f.AC), "+v"(f.A2), "+v"(f.BC), "+v"(f.B2));
        if (haves[i]) part_entries<PAIRS, MIX>(f, mk, m1, sh, lowm, se, place);
    }
    __syncthreads();
    /* 4: the sorted batch into its row's fixed slot (pg.batch entries: a
       run's position needs no per-row base), as 16-B pieces; the up to 7
       codes past the batch's end are padding no run covers */
    const uint32_t n8 = (*total * (uint32_t)sizeof(CT) + 15u) >> 4;
    uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(pg.codes) + (size_t)row * pg.batch * sizeof(CT));
    const uint4 *src = reinterpret_cast<const uint4 *>(ent);
    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W)) dst[i] = src[i];
    return any_more;
}

/*
 * Pipelined batches (PIPE: the main pass of tables of at most 512 slices,
 * whose scan wave 0 runs alone, and of k = 13's 2048, whose scan all waves
 * share: part_scan_sum).  part_batch runs its phases one after
 * another on every wave -- tiles (VALU), histogram atomics, barrier, scan,
 * barrier, placement atomics (LDS), barrier, write-out -- so the CU's VALU
 * idles while its LDS works and the other way round.  Here batch j's
 * entries are placed while the waves count batch j+1's tiles: each round a
 * wave counts one tile, adds its entries to the histogram of batch j+1 and
 * places the entries of the tile it stashed in the same slot during batch j
 * (every tile of a batch sits in its own stash slot, so one stash serves
 * both batches).  At the end of a batch's tiles, one barrier (batch j's
 * placement and batch j+1's histogram done), then wave 0 scans batch j+1's
 * histogram (cursors, run index, total) while the other waves write batch j
 * out, then a second barrier: two barriers per batch instead of three, and
 * the tiles' VALU work overlaps the placement atomics across the waves.
 */
/* A fast tile's entries (as part_entries without mixed tiles) placed at
   their slices' cursors, eight at a time: the eight returning cursor
   atomics are issued back to back and only then the eight code stores.
   (One entry at a time -- atomic, wait, store -- the compiler cannot move
   the next atomic above the previous store into the same LDS, so every
   entry waited out a whole LDS round trip.) */
/* Entry j of group g of half h of a fast tile (as part_entries without
   mixed tiles): its slice (one bit-field extract: the code's bits [sh, sh +
   wsl), wsl = the slice bits) and its stored low bits (PAIRS: a single k-mer
   x at slot 1 of a '\n' half is the pair code x << 2 with PART_SINGLE) */
template <bool PAIRS>
__device__ __forceinline__ void part_entry(uint32_t C, uint32_t S2, bool skip0, int g, int j, uint32_t sh,
                                           uint32_t wsl, uint32_t lowm, const SingleEnc &se, uint32_t &b,
                                           uint32_t *low) {
    if (PAIRS) {
        const uint32_t v = j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2;
        if (j == 0 && skip0) {   /* x = v & mk, as (x << slsh): its slice is v's bits [sh - slsh, 2k) */
            b = se.sbase + __builtin_amdgcn_ubfe(v, sh - se.slsh, wsl - 2u + se.slsh);
            if (low) *low = ((v << se.slsh) & lowm) | se.sflag;
        } else {
            b = __builtin_amdgcn_ubfe(v, sh, wsl);
            if (low) *low = v & lowm;
        }
    } else {
        const int i = 8 * g + j;
        const uint32_t v = i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2;
        b = __builtin_amdgcn_ubfe(v, sh, wsl);
        if (low) *low = v & lowm;
    }
}

/* A fast tile's entries into the batch's slice histogram */
template <bool PAIRS>
__device__ __forceinline__ void part_hist8(const Emit &em, uint32_t sh, uint32_t wsl, const SingleEnc &se,
                                           uint32_t *hist) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
#pragma unroll
        for (int g = 0; g < (PAIRS ? 1 : 2); g++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;   /* slot 0 is not a window */
                uint32_t b;
                part_entry<PAIRS>(C, S2, skip0, g, j, sh, wsl, 0u, se, b, nullptr);
                atomicAdd(&hist[b], 1u);
            }
    }
}

/* A fast tile's entries placed at their slices' cursors (byte offsets into
   the batch), eight at a time: the eight returning cursor atomics are issued
   back to back and only then the eight code stores.  (One entry at a time --
   atomic, wait, store -- the compiler cannot move the next atomic above the
   previous store into the same LDS, so every entry waited out a whole LDS
   round trip.) */
typedef __attribute__((address_space(3))) uint16_t lds_u16;
template <bool PAIRS>
__device__ __forceinline__ void part_place8(const Emit &em, uint32_t sh, uint32_t wsl, uint32_t lowm,
                                            const SingleEnc &se, uint32_t *cur) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
#pragma unroll
        for (int g = 0; g < (PAIRS ? 1 : 2); g++) {
            uint32_t b[8], low[8], p[8];
#pragma unroll
            for (int j = 0; j < 8; j++) part_entry<PAIRS>(C, S2, skip0, g, j, sh, wsl, lowm, se, b[j], &low[j]);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;   /* slot 0 is not a window */
                p[j] = atomicAdd(&cur[b[j]], 2u);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;
                *(lds_u16 *)(uintptr_t)p[j] = (uint16_t)low[j];
            }
        }
    }
}

/* PAD: runs start on 16-B pieces (PART_PAD), the run index and the total in
   pieces / entries (8 per piece) */
template <bool PAD>
__device__ __forceinline__ void part_scan_w0(const PartGeo &pg, uint32_t row, uint32_t *hist, uint32_t *cur,
                                             uint32_t *tot, uint32_t ent_lds) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t per = (pg.nslices + 63) / 64;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; j++) {
        const uint32_t b = lane * per + j;
        if (b < pg.nslices) sum += PAD ? (hist[b] + 7u) >> 3 : hist[b];
    }
    const uint32_t inc = wscan_incl32(sum);
    uint32_t run = inc - sum;
    for (uint32_t j = 0; j < per; j++) {
        const uint32_t b = lane * per + j;
        if (b < pg.nslices) {
            const uint32_t c = hist[b];
            cur[b] = ent_lds + (PAD ? 16u : 2u) * run;   /* LDS byte addresses (part_place8) */
            pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
            hist[b] = 0;
            run += PAD ? (c + 7u) >> 3 : c;
        }
    }
    if (lane == 63) *tot = PAD ? 8u * inc : inc;
}

/* The same for 2048 slices (k = 13), over all W waves: each wave sums its
   contiguous share (part 1, beside the write-out), one more barrier, then
   scans its share from the sum of the shares before it (part 2) */
__device__ __forceinline__ uint32_t part_scan_sum(const PartGeo &pg, const uint32_t *hist, uint32_t nw, uint32_t *scr) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t per_w = pg.nslices / nw, ppl = per_w / 64u, b0 = wv * per_w + lane * ppl;
    uint32_t mine = 0;
    for (uint32_t j = 0; j < ppl; j++) mine += hist[b0 + j];
    const uint32_t wt = wsum32(mine);
    if (lane == 0) scr[wv] = wt;
    return mine;
}
__device__ __forceinline__ void part_scan_place(const PartGeo &pg, uint32_t row, uint32_t *hist, uint32_t *cur,
                                                uint32_t nw, const uint32_t *scr, uint32_t mine, uint32_t *tot,
                                                uint32_t ent_lds) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t per_w = pg.nslices / nw, ppl = per_w / 64u, b0 = wv * per_w + lane * ppl;
    const uint32_t off = wsum32(lane < wv ? scr[lane] : 0u);
    uint32_t run = off + wscan_incl32(mine) - mine;
    for (uint32_t j = 0; j < ppl; j++) {
        const uint32_t b = b0 + j, c = hist[b];
        cur[b] = ent_lds + 2u * run;
        pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
        hist[b] = 0;
        run += c;
    }
    if (wv == nw - 1u && lane == 63) *tot = run;
}

template <uint32_t W>
__device__ __forceinline__ void part_writeout(const PartGeo &pg, uint32_t row, uint32_t total, const uint16_t *ent,
                                              uint32_t t0, uint32_t nt) {
    const uint32_t n8 = (total * (uint32_t)sizeof(uint16_t) + 15u) >> 4;
    uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(pg.codes) + (size_t)row * pg.batch * 2u);
    const uint4 *src = reinterpret_cast<const uint4 *>(ent);
    for (uint32_t i = t0; i < n8; i += nt) dst[i] = src[i];
}

/* RES = false: the main pass.  With mixed tiles on, a range that needs more
 * than pg.general general tiles stops there (ResumeRec) and
 * RES = true -- the same blocks and ranges, their rows in region 2 -- counts
 * the rest of it, each tile fast, mixed (the masked entries of tile_mixed)
 * or general.  Two kernels: tile_mixed's registers stay out of the main
 * pass.  k_part<RES> returns at once unless some range stopped. */
template <bool PAIRS, bool RES, uint32_t W, uint32_t SM = PART_SM(W), bool C32 = false, bool PIPE = false,
          uint32_t KC = 0>
__global__ void __launch_bounds__(PART_BLOCK_W(W), 4) /* 4 waves per SIMD (<= 128 VGPRs): 16 waves per CU */
k_part(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
       uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr, uint64_t nchunks, uint64_t cpw,
       const XState *d_init, int has_init, PartGeo pg, ResumeRec *resume, const XState *exact) {
    static_assert(!PIPE || (!RES && !C32 && SM <= 2048u), "PIPE: the main pass, 16-bit codes, unpacked cursors");
    /* one LDS object: the histogram and the cursors first (below 64 KiB, so
       their base folds into the LDS instructions' offset field), then the
       batch */
    using CT = typename std::conditional<C32, uint32_t, uint16_t>::type;
    /* runs padded to 16-B pieces (PART_PAD) for the tables of at most 512 slices */
    constexpr bool PAD = !C32 && SM <= PART_PAD_MAX_SM;
    constexpr uint32_t CURW = SM > 2048u ? SM / 2u : SM;
    constexpr uint32_t ENT_OFF = (SM + CURW + 4u + W + 15u) & ~15u;   /* words, 64-B aligned */
    constexpr uint32_t ENT_BYTES = PART_ROW_BYTES(W) + (PAD ? PART_ROW_PAD(SM) : 0u);
    __shared__ __attribute__((aligned(64))) uint32_t lds_part[ENT_OFF + ENT_BYTES / 4u];
    uint32_t *const hist = lds_part, *const cur = lds_part + SM, &total = lds_part[SM + CURW],
                    *const tot = lds_part + SM + CURW + 1u, *const scr = lds_part + SM + CURW + 4u;
    CT *const ent = reinterpret_cast<CT *>(lds_part + ENT_OFF);
    if (RES && *(volatile uint32_t *)pg.flag == 0) return;   /* uniform: no range stopped */
    /* open the feed's result block (the kernels after this one accumulate
       into it) */
    if (!RES && blockIdx.x == 0) {
        if (threadIdx.x < 10) res->tstat[threadIdx.x] = 0;
        if (threadIdx.x == 10) res->eof_cand = ~0ull;
        if (threadIdx.x == 11) res->redo_n = 0;
    }
    for (uint32_t i = threadIdx.x; i < pg.nslices; i += PART_BLOCK_W(W)) hist[i] = 0;
    Ctx cx{buf, len, lo, table, nullptr, shortcnt, acc, res, maskk, 0, k, pg.glist};
    const int lane = threadIdx.x & 63;
    const uint64_t wave = blockIdx.x * W + wave_in_block();
    const uint64_t c0 = wave * cpw, c1 = min(c0 + cpw, nchunks);
    const bool has = c0 < c1 && (!RES || rr[wave].resume);
    RangeRec hdr_r;
    hdr_r.c0 = has ? c0 : 0;
    hdr_r.c1 = has ? c1 : 0;
    const Span sp = range_span(hdr_r, len);
    const uint64_t last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
    const bool ld = sp.nfull > 0;
    const ResumeRec *qr = resume + wave;   /* k_part<RES>: where k_part stopped (fields read where used) */
    uint64_t t = RES && has ? qr->tile : 0;
#define FK_LOADP(dst, t_)                                                            \
    if (ld) {                                                                        \
        const uint64_t tb_ = min(sp.rbase + (uint64_t)(t_) * FK_TILE_BYTES, last_tile); \
        const u32x4 *p_ = reinterpret_cast<const u32x4 *>(cx.buf + tb_) + lane;      \
        u32x4 v0_ = __builtin_nontemporal_load(p_);                                  \
        u32x4 v1_ = __builtin_nontemporal_load(p_ + 64);                             \
        dst[0] = v0_.x; dst[1] = v0_.y; dst[2] = v0_.z; dst[3] = v0_.w;               \
        dst[4] = v1_.x; dst[5] = v1_.y; dst[6] = v1_.z; dst[7] = v1_.w;               \
    }
    /* halo (lanes 0..7) and the first three tiles in flight before anything
       waits (as in k_count) */
    uint32_t hw[8] = {};
    const int64_t ho = (int64_t)sp.rbase - (int64_t)FK_HALO_BYTES + (int64_t)lane * FK_LANE_BYTES;
    const bool hv = has && lane < (int)(FK_HALO_BYTES / FK_LANE_BYTES) && ho >= lo;
    if (!RES) {
        const int64_t hc = max(min(ho, (int64_t)len - (int64_t)FK_LANE_BYTES), lo);
        const u32x4 *hp = reinterpret_cast<const u32x4 *>(buf + hc);
        u32x4 h0 = __builtin_nontemporal_load(hp), h1 = __builtin_nontemporal_load(hp + 1);
        hw[0] = h0.x; hw[1] = h0.y; hw[2] = h0.z; hw[3] = h0.w;
        hw[4] = h1.x; hw[5] = h1.y; hw[6] = h1.z; hw[7] = h1.w;
    }
    uint32_t A[8] = {}, B[8] = {}, C[8] = {};
    asm volatile("" ::: "memory");
    FK_LOADP(A, t);
    asm volatile("" ::: "memory");
    FK_LOADP(B, t + 1);
    asm volatile("" ::: "memory");
    FK_LOADP(C, t + 2);
    /* entering state: the known stream state for chunk 0, else a guess from
       the halo (k_scan checks it, k_redo recounts a range it got wrong);
       k_part<RES>: where k_part stopped */
    DState st{0, 0, 0}, first{0, 0, 0};
    Facts f{0, 0, 0, 0, 0, 0};
    if (RES) {
        if (has) {
            st = DState{qr->code, qr->R, qr->hdr};
            first = DState{qr->a_code, qr->a_R, qr->a_hdr};
            f = qr->f;
        }
    } else if (has) {
        if (exact) {
            /* a recount from the exact range states (resolve_and_fetch) */
            const XState x = exact[wave];
            st = DState{x.code, (uint32_t)x.R, x.hdr};
        } else if (c0 == 0 && has_init) {
            st = DState{d_init->code, (uint32_t)d_init->R, d_init->hdr};
        } else {
            st = halo_guess<H_EMIT>(cx, hw, hv);
        }
        first = st;
    }
    consume(hw);   /* waited on every path (see k_count) */
    Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
    bool done = !has || t >= sp.ntiles, stopped = false;
    uint32_t general_left = pg.nomix ? 0xFFFFFFFFu : pg.general;
    uint32_t round = 0;
    const uint32_t row0 = (RES ? pg.rows : 0u) + blockIdx.x * pg.rounds;
    constexpr uint32_t NT = PART_TILES3(PAIRS, C32);
    Emit stash[NT];
    bool have_stash[NT];
#pragma unroll
    for (uint32_t i = 0; i < NT; i++) {
        stash[i] = Emit{0, 0, 0, 0, false, false, false};
        have_stash[i] = false;
    }
    /* PIPE: the codes of an entry and its placement (unpacked cursors) */
    /* KC: k as a compile-time constant (the headline k = 11), so that the
       slice and low-bit extracts fold into single bit-field ops */
    constexpr uint32_t KBC = KC ? (PAIRS ? KC + 1u : KC) : 0u;
    /* (KC: 2^15-bin slices, singles filed under their pair code, PART_SINGLE) */
    const uint32_t shv = KC ? (2u * KBC - 6u < 15u ? 2u * KBC - 6u : 15u) : pg.sh;
    const uint32_t lowm = (1u << shv) - 1u;
    const SingleEnc se = KC ? SingleEnc{0u, 2u, PART_SINGLE} : SingleEnc{pg.sbase, pg.slsh, pg.sflag};
    /* the batch's LDS byte address (the PIPE cursors hold LDS addresses) */
    const uint32_t ent_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) CT *)ent;
    const uint32_t wsl = 2u * (KC ? KBC : (uint32_t)(PAIRS ? k + 1 : k)) - shv;   /* slice bits of a code */
    __syncthreads();
    /* PIPE: the stashed entry of this round's slot (batch j) to its place; odd
       waves place before their tile, even waves after it, so that the waves
       of a SIMD tend to be in different phases (VALU / LDS) */
    const bool early = PIPE && ((wave_in_block() >> 1) & 1u);
#define FK_PLACE_OLD()                                                               \
    {                                                                                \
        const uint32_t ph_ = round % NT;                                             \
        Emit old_ = stash[0];                                                        \
        bool hold_ = have_stash[0];                                                  \
        _Pragma("unroll") for (uint32_t i_ = 1; i_ < NT; i_++) if (ph_ == i_) {      \
            old_ = stash[i_];                                                        \
            hold_ = have_stash[i_];                                                  \
        }                                                                            \
        if (hold_) part_place8<PAIRS>(old_, shv, wsl, lowm, se, cur); \
    }
/* (a macro, not a lambda: the same body as an always-inline lambda called
   three times gave the compiler a different register allocation -- 107
   VGPRs and 256 SGPR spills instead of 123 and 207 -- and k_part at k = 11
   over 10 G bases 4.41 -> 4.85 ms, round 4) */
#define FK_ROUND(X)                                                                  \
    {                                                                                \
        Emit em{0, 0, 0, 0, false, false, false};                                    \
        if (PIPE && early) FK_PLACE_OLD();                                           \
        bool have = false, plain_ = false, kind_ = false;                            \
        if (!done) {                                                                 \
            if (t < sp.nfull && st.hdr == 0 && tile_fast<true, H_EMIT, true>(cx, X, st, f, cnt, 1u, &em, &kind_)) { \
                have = em.deep;                                                      \
                t++;                                                                 \
            } else if (RES && t < sp.nfull &&                                        \
                       tile_mixed<H_EMIT>(cx, X, (uint32_t)(t * FK_TILE_BYTES), st, f, cnt, 1u, plain_, &em)) { \
                have = true;                                                         \
                t++;                                                                 \
            } else if (!RES && !kind_ && general_left == 0) {                        \
                /* k_part<RES> counts this tile and the rest of the range (the  \
                   tile is skipped here: t advances on every path) */           \
                stopped = true;                                                      \
                t++;                                                                 \
            } else {                                                                 \
                general_left -= kind_ ? 0u : 1u;                                     \
                uint32_t v_[8];                                                      \
                const int64_t toff_ = (int64_t)(sp.rbase + t * FK_TILE_BYTES);       \
                const int nb_ = load_lane<FK_LANE_BYTES>(cx, toff_ + lane * (int64_t)FK_LANE_BYTES, v_); \
                tile_general<true, H_EMIT>(cx, v_, nb_, (uint32_t)(t * FK_TILE_BYTES), st, f, cnt, 1u); \
                consume(v_);                                                         \
                t++;                                                                 \
            }                                                                        \
            done = stopped || t >= sp.ntiles;                                        \
        }                                                                            \
        consume(X);                                                                  \
        FK_LOADP(X, t + 2);                                                          \
        if (PIPE) {   /* batch j+1's histogram, batch j's placement (see part_scan_w0) */ \
            const uint32_t ph_ = round % NT;                                         \
            if (have) part_hist8<PAIRS>(em, shv, wsl, se, hist);                   \
            if (!early) FK_PLACE_OLD();                                              \
            _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++) if (ph_ == i_) {  \
                stash[i_] = em;                                                      \
                have_stash[i_] = have;                                               \
            }                                                                        \
            if (ph_ == NT - 1) {                                                     \
                const uint32_t j_ = round / NT;                                      \
                const bool more_ = __syncthreads_or(!done);                          \
                if (KC == 0 && pg.nslices > 512u) {   /* 2048 slices: the scan over all waves */ \
                    const uint32_t mine_ = part_scan_sum(pg, hist, W, scr);          \
                    if (j_ > 0) part_writeout<W>(pg, row0 + j_ - 1, tot[(j_ - 1) & 1u], (const uint16_t *)ent, \
                                                 threadIdx.x, PART_BLOCK_W(W));       \
                    __syncthreads();                                                 \
                    part_scan_place(pg, row0 + j_, hist, cur, W, scr, mine_, &tot[j_ & 1u], ent_lds); \
                } else if (threadIdx.x < 64) {                                       \
                    part_scan_w0<PAD>(pg, row0 + j_, hist, cur, &tot[j_ & 1u], ent_lds); \
                } else if (j_ > 0) {                                                 \
                    part_writeout<W>(pg, row0 + j_ - 1, tot[(j_ - 1) & 1u], (const uint16_t *)ent, \
                                     threadIdx.x - 64u, PART_BLOCK_W(W) - 64u);       \
                }                                                                    \
                __syncthreads();                                                     \
                if (!more_ || j_ + 1 >= pg.rounds) {                                 \
                    /* the last batch: placed, then written out */                  \
                    _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++)           \
                        if (have_stash[i_]) part_place8<PAIRS>(stash[i_], shv, wsl, lowm, se, cur); \
                    __syncthreads();                                                 \
                    part_writeout<W>(pg, row0 + j_, tot[j_ & 1u], (const uint16_t *)ent, threadIdx.x, PART_BLOCK_W(W)); \
                    round++;                                                         \
                    break;                                                           \
                }                                                                    \
            }                                                                        \
        } else {   /* static stash slots (no dynamic register indexing) */          \
            const uint32_t ph_ = round % NT;                                         \
            _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++) if (ph_ == i_) {  \
                stash[i_] = em;                                                      \
                have_stash[i_] = have;                                               \
            }                                                                        \
            if (ph_ == NT - 1) {                                                     \
                const bool more_ = part_batch<PAIRS, RES, W, SM, CT>(cx, pg, stash, have_stash, !done, \
                                                          row0 + round / NT, hist, cur, &total, ent, scr); \
                if (!more_ || round / NT + 1 >= pg.rounds) { round++; break; }       \
            }                                                                        \
        }                                                                            \
        round++;                                                                     \
    }
    for (;;) {
        FK_ROUND(A);
        FK_ROUND(B);
        FK_ROUND(C);
    }
#undef FK_ROUND
#undef FK_PLACE_OLD
#undef FK_LOADP
    /* rows the block did not reach are empty */
    for (uint32_t r = (round + NT - 1) / NT; r < pg.rounds; r++) {
        const uint32_t row = row0 + r;
        for (uint32_t b = threadIdx.x; b < pg.nslices; b += PART_BLOCK_W(W)) pg.idx[(size_t)row * pg.nslices + b] = PART_NO_RUN;
    }
    if (!has) {
        flush_counters(cx, cnt, 1u);
        return;
    }
    if (!RES && stopped) {
        /* k_part<RES> counts the rest of the range */
        flush_counters(cx, cnt, 1u);
        const uint32_t unk = wsum32(cnt.unknown), eof = wmin32(cnt.eof);
        if (lane == 0) {
            ResumeRec w;
            w.tile = t - 1;   /* the tile it stopped at */
            w.code = st.code; w.R = st.R; w.hdr = st.hdr;
            w.a_code = first.code; w.a_R = first.R; w.a_hdr = first.hdr;
            w.range = (uint32_t)wave;
            w.unknown = unk;
            w.eof = eof;
            w.pad = 0;
            w.f = f;
            resume[wave] = w;
            RangeRec &r = rr[wave];
            r.c0 = c0; r.c1 = c1;
            r.resume = 1;
            atomicOr(pg.flag, 1u);
        }
        return;
    }
    /* the range's record: transfer function, guess, observations */
    RangeRec r;
    r.tf = fk_tf_span(first, st, f);
    r.a_code = first.code; r.a_R = first.R; r.a_hdr = first.hdr;
    r.c0 = c0; r.c1 = c1;
    r.resume = 0;
    range_obs(cx, cnt, 1u, sp, &r, true);
    if (lane == 0) {
        if (RES) {   /* plus what k_part observed before it stopped */
            r.unknown += qr->unknown;
            if (qr->eof != FK_NO_EOF) r.eof = min(r.eof, (uint64_t)qr->eof);
        }
        rr[wave] = r;
    }
}

/* the instances launch_part launches: (PAIRS, RES, W, SM, C32, PIPE, KC) */
#define FK_PART_PIPE_INSTANCES(X)                                               \
    X(true, false, 16u, PART_PAD_MAX_SM, false, true, 11u)                      \
    X(true, false, 16u, PART_SM(16u), false, true, 0u)                          \
    X(false, false, 16u, PART_SM(16u), false, true, 0u)                         \
    X(true, false, 8u, PART_SM(8u), false, true, 0u)                            \
    X(false, false, 8u, PART_SM(8u), false, true, 0u)
#define FK_PART_OTHER_INSTANCES(X)                                              \
    X(false, false, 16u, PART_SM(16u), true, false, 0u)                         \
    X(false, false, 16u, PART_BIG, false, false, 0u)                            \
    X(false, true, 16u, PART_SM(16u), true, false, 0u)                          \
    X(false, true, 16u, PART_BIG, false, false, 0u)                             \
    X(true, true, 16u, PART_PAD_MAX_SM, false, false, 0u)                       \
    X(true, true, 16u, PART_SM(16u), false, false, 0u)                          \
    X(false, true, 16u, PART_SM(16u), false, false, 0u)                         \
    X(true, true, 8u, PART_SM(8u), false, false, 0u)                            \
    X(false, true, 8u, PART_SM(8u), false, false, 0u)
#define FK_PART_ARGS const uint8_t *, uint64_t, int64_t, int, uint64_t, uint32_t *, uint32_t *, unsigned long long *, DevRes *, RangeRec *, uint64_t, uint64_t, const XState *, int, PartGeo, ResumeRec *, const XState *
#define FK_PART_EXTERN(P, R, W, SM, C32, PIPE, KC) \
    extern template __global__ void k_part<P, R, W, SM, C32, PIPE, KC>(FK_PART_ARGS);
#define FK_PART_INSTANTIATE(P, R, W, SM, C32, PIPE, KC) \
    template __global__ void k_part<P, R, W, SM, C32, PIPE, KC>(FK_PART_ARGS);
