/*
 * fk_scan.hip -- the state pass and the k <= 7 count (findKmer.cpp:962-1069):
 * k_count / k_resume / k_redo (one wave per range, LDS bins for k <= 7, the
 * scan state only for k >= 8), k_scan (exact range states), k_tail (the
 * one-pass k <= 7 feed), k_table_stats / k_table_final, and their launches.
 */
#include "fk_engine_internal.h"

template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 2)
k_count(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
        uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr,
        uint64_t nchunks, const XState *d_init, int has_init, uint64_t cpw, ResumeRec *resume,
        uint32_t general_tiles, uint32_t *subs, const OnePassCfg *opc, uint32_t op_flags,
        uint64_t nstatic, DynGeo dg, uint32_t *heads) {
    extern __shared__ uint32_t lds_bins[];
    /* open the feed's result block (the kernels after this one in the
       stream accumulate into it) */
    if (blockIdx.x == 0) {
        if (!(op_flags & OP_ON)) {
            if (threadIdx.x < 10) res->tstat[threadIdx.x] = 0;
            if (threadIdx.x == 10) res->eof_cand = ~0ull;
            if (threadIdx.x == 11) res->redo_n = 0;
        }
        /* one pass: k_tail writes the whole result block, and does a
           pending reset (table = 0 + the sub-tables) */
    }
    const uint32_t nw = lds_words(HM, k);
    /* the 509-odd blocks flush their bins into FK_SUBTABLES copies of the
       table (fewer same-address atomics at the end of the kernel);
       k_table_stats folds them into the table */
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k,
           subs ? subs + (size_t)(blockIdx.x % FK_SUBTABLES) * ((size_t)1 << (2 * k)) : nullptr};
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    /* the wave's static range; the static ranges end where the dynamic ones
       begin */
    const uint64_t send = dg.ndyn ? dg.base : nchunks;
    uint64_t rid = wave;
    uint64_t c0 = wave * cpw, c1 = min(c0 + cpw, send);
    if (dg.ndyn) static_span(dg, wave, c0, c1);
    bool has = wave < nstatic && c0 < c1;
    RangeRec hdr_r;
    hdr_r.c0 = has ? c0 : 0;
    hdr_r.c1 = has ? c1 : 0;
    Span sp = range_span(hdr_r, len);
    uint64_t last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
    /* prologue, all loads first; LDS is zeroed and the halo state computed
       while they fly */
    uint32_t hw[8], A[8], B[8], C[8];
    bool hv;
    range_prologue(cx, sp, last_tile, has, hw, hv, A, B, C);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    /* the wave's counters, flushed once per FK_FLUSH_BYTES of its ranges
       (packed 16-bit fields per lane) and at the end: one set of
       accumulator atomics per wave, not per range */
    Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
    uint32_t unk_seen = 0;
    uint64_t since = 0;
    for (;;) {
        if (has) {
            count_wave_range<HM>(cx, sp, last_tile, rid, c0, c1, hw, hv, A, B, C, d_init, has_init, op_flags,
                                 resume, rr, general_tiles, cnt, unk_seen);
            since += sp.rend - sp.rbase;
            if (since >= FK_FLUSH_BYTES) {
                flush_counters(cx, cnt, 1u, HM != H_NONE);
                cnt.unknown = 0;
                unk_seen = 0;
                since = 0;
            }
        }
        if (dg.ndyn == 0) break;
        const uint32_t d = claim_dyn(heads, dg);
        if (d >= dg.ndyn) break;
        rid = nstatic + d;
        dyn_span(dg, d, c0, c1);
        hdr_r.c0 = c0;
        hdr_r.c1 = c1;
        sp = range_span(hdr_r, len);
        last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
        has = true;
        range_prologue(cx, sp, last_tile, has, hw, hv, A, B, C);
    }
    flush_counters(cx, cnt, 1u, HM != H_NONE);
    if (LDS_MODE(HM)) {
        lds_flush<HM>(cx);
        if ((op_flags & OP_ON) && threadIdx.x < 64) block_summary(cx, opc, rr, nstatic);
    }
}
#undef FK_LOADI
#undef FK_LOADT

/*
 * k_resume: finish the ranges k_count stopped in (one wave per range, as in
 * k_count), with the general path wherever the fast path does not apply, and
 * write their RangeRecs.  Blocks without such a range exit at once.
 */
template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 4)   /* 4 waves per SIMD (<= 128 VGPRs): two blocks per CU */
k_resume(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
         uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr, uint64_t nranges,
         const ResumeRec *resume, uint32_t *heads, int mixed) {
    extern __shared__ uint32_t lds_bins[];
    /* k_scan lists the ranges to redo after this kernel (a one-pass k_count
       that gave up may have listed some already) */
    if (blockIdx.x == 0 && threadIdx.x == 0) res->redo_n = 0;
    /* k_count is done: reset its dynamic-range pools for the next launch */
    if (blockIdx.x == 0)
        for (uint32_t q = threadIdx.x; q < FK_MAX_POOLS; q += blockDim.x) heads[q * FK_HEAD_STRIDE] = 0;
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    const bool mine = wave < nranges && rr[wave].resume;
    /* uniform per block; in the LDS modes through the first bin (before the
       bins are zeroed): __syncthreads_or keeps its reduction in static LDS,
       which would move the bins off address 0 (lds_add) */
    bool any;
    if (LDS_MODE(HM)) {
        if (threadIdx.x == 0) lds_bins[0] = 0;
        __syncthreads();
        if (mine) lds_bins[0] = 1;
        __syncthreads();
        any = lds_bins[0] != 0;
        __syncthreads();
    } else {
        any = __syncthreads_or(mine);
    }
    if (!any) return;
    const uint32_t nw = lds_words(HM, k);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k};
    if (mine) {
        const ResumeRec q = resume[wave];
        RangeRec r = rr[wave];
        const Span sp = range_span(r, len);
        DState st{q.code, q.R, q.hdr};
        const DState a{q.a_code, q.a_R, q.a_hdr};
        Facts f = q.f;
        Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
        count_range<HM>(cx, sp, q.tile, st, f, cnt, 1u, mixed);
        r.tf = fk_tf_span(a, st, f);
        r.a_code = a.code; r.a_R = a.R; r.a_hdr = a.hdr;
        range_obs(cx, cnt, 1u, sp, &r, true, HM != H_NONE);
        if ((threadIdx.x & 63) == 0) {
            /* plus what k_count observed before the resume point */
            r.unknown += q.unknown;
            if (q.eof != FK_NO_EOF) r.eof = min(r.eof, (uint64_t)q.eof);
            rr[wave] = r;
        }
    }
    if (LDS_MODE(HM)) lds_flush<HM>(cx);
}

/*
 * k_redo, mode 0: each listed range (its guessed entering state would count
 * differently from the exact one) is counted again with weight -1 from the
 * guess, cancelling k_count + k_resume exactly, and with weight +1 from the
 * exact state, which also replaces its observations.  mode 1: cancel every
 * range from its exact state (a 0xFF byte truncates the input and the
 * segment is recounted).
 */
template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 4)
k_redo(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
       uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr,
       const XState *rtrue, const uint32_t *list, uint64_t nranges, int mode, int mixed) {
    extern __shared__ uint32_t lds_bins[];
    const uint64_t n = mode != 0 ? nranges : (uint64_t)res->redo_n;
    if ((uint64_t)blockIdx.x * FK_WAVES_PER_BLOCK >= n) return;   /* uniform per block */
    const uint32_t nw = lds_words(HM, k);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k};
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * FK_WAVES_PER_BLOCK;
    for (uint64_t i = wave; i < n; i += nwaves) {
        const uint64_t r = mode != 0 ? i : list[i];
        RangeRec q = rr[r];
        const Span sp = range_span(q, len);
        const XState t = rtrue[r];
        DState ts{t.code, (uint32_t)t.R, t.hdr};
        /* passes over the range (one inlined count_range: its register
           footprint decides this kernel's occupancy):
           mode 0: -1 from the guess, then +1 from the exact state -- except
                   when the whole range lies in the reference's negative
                   int32 zone (seqSize < 0 from its first base to its last,
                   no run break: a run longer than 2^31 bases, :977), where
                   the exact state counts nothing: one read instead of two;
           mode 1: -1 from the exact state;
           mode 2: +1 from the exact state (H_SPARSE: counters and
                   observations only; k_sp_emit emits the windows at finish). */
        const bool neg_zone = mode == 0 && !t.hdr && !q.tf.f0_const && (int32_t)(uint32_t)t.R < 0 &&
                              (uint64_t)(uint32_t)t.R + (sp.rend - sp.rbase) <= 0xFFFFFFFFull;
        const int npass = mode == 0 && !neg_zone ? 2 : 1;
#pragma unroll 1
        for (int pass = 0; pass < npass; pass++) {
            const bool cancel = mode == 1 || (mode == 0 && pass == 0);
            const uint32_t wt = cancel ? 0xFFFFFFFFu : 1u;
            DState st = (mode == 0 && pass == 0) ? DState{q.a_code, q.a_R, q.a_hdr} : ts;
            Facts f{0, 0, 0, 0, 0, 0};
            Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
            count_range<HM>(cx, sp, 0, st, f, cnt, wt, mixed);
            if (cancel) {
                flush_counters(cx, cnt, wt);
            } else {
                /* exact observations replace the guessed trajectory's */
                range_obs(cx, cnt, 1u, sp, &q, true);
                if ((threadIdx.x & 63) == 0) { rr[r].eof = q.eof; rr[r].unknown = q.unknown; }
            }
        }
    }
    if (LDS_MODE(HM)) lds_flush<HM>(cx);
}

/*
 * k_scan: exact entering state of every range, one thread per range.  Each
 * 256-thread block scans its ranges' transfer functions (wave shuffles, then
 * the four wave aggregates), publishes the block aggregate with an
 * epoch-tagged flag, waits for the flags of all blocks before it and
 * composes their aggregates with one wave scan (all predecessors publish at
 * about the same time, so this is one round trip, not a chain).
 * mode 0: resolve from *d_state, list the ranges whose guess is not
 * equivalent, write the exit state back to *d_state and res->exit.
 * mode 1: only the total transfer function (shard summary) into *tf_total.
 * Every block reads *d_state before publishing its flag; the last block
 * writes it only after seeing every flag.  All blocks are co-resident (a
 * handful), and a block only waits on blocks dispatched before it.
 */

__global__ void __launch_bounds__(SCAN_THREADS)
k_scan(const RangeRec *rr, uint64_t n, XState *d_state, XState *rtrue, uint32_t *redo_list,
       DevRes *res, int k, int mode, TF *tf_total, TF *aggs, uint32_t *flags, uint32_t epoch) {
    __shared__ TF wincl[SCAN_WAVES];   /* inclusive wave aggregates */
    __shared__ TF bprefix;
    __shared__ unsigned long long eof_min;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, b = blockIdx.x;
    const uint64_t r = (uint64_t)b * SCAN_THREADS + t;
    const XState init = *d_state;
    if (t == 0) eof_min = ~0ull;
    TF a = fk_identity();
    unsigned long long em = ~0ull;
    if (r < n) {
        a = rr[r].tf;
        const uint64_t e = rr[r].eof;
        if (e != FK_NO_EOF64) em = rr[r].c0 * FK_CHUNK_BYTES + e;
    }
    a = tf_wave_scan(a);
    if (lane == 63) wincl[w] = a;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        unsigned long long o = ((unsigned long long)__shfl_xor((unsigned)(em >> 32), d, 64) << 32) |
                               (unsigned)__shfl_xor((unsigned)em, d, 64);
        em = min(em, o);
    }
    __syncthreads();
    if (lane == 0 && em != ~0ull) atomicMin(&eof_min, em);
    if (t == 0) {
        for (int i = 1; i < SCAN_WAVES; i++) wincl[i] = fk_compose(wincl[i - 1], wincl[i]);
        aggs[b] = wincl[SCAN_WAVES - 1];
        __threadfence();
        __hip_atomic_store(&flags[b], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    /* prefix of all blocks before this one (wave 0) */
    if (w == 0) {
        TF carry = fk_identity();
        for (uint32_t base = 0; base < b; base += 64) {
            const uint32_t i = base + lane;
            TF x = fk_identity();
            if (i < b) {
                while (__hip_atomic_load(&flags[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch)
                    __builtin_amdgcn_s_sleep(1);
                x = aggs[i];
            }
            x = tf_wave_scan(x);
            /* lane 63 holds the chunk's aggregate (identity padding is neutral) */
            const TF chunk = tf_rdlane(x, 63);
            carry = fk_compose(carry, chunk);
        }
        if (lane == 0) bprefix = carry;
    }
    __syncthreads();
    if (mode == 1) {
        if (b == gridDim.x - 1 && t == 0) *tf_total = fk_compose(bprefix, wincl[SCAN_WAVES - 1]);
        return;
    }
    /* exclusive prefix of this thread's range */
    TF ex = tf_shup(a, 1);
    if (lane == 0) ex = fk_identity();
    if (w > 0) ex = fk_compose(wincl[w - 1], ex);
    ex = fk_compose(bprefix, ex);
    if (r < n) {
        const RangeRec &q = rr[r];
        const XState s = fk_apply(ex, init);
        rtrue[r] = s;
        DState as{q.a_code, q.a_R, q.a_hdr};
        if (!fk_equiv(as, s, k, (q.c1 - q.c0) * FK_CHUNK_BYTES)) {
            uint32_t slot = atomicAdd(&res->redo_n, 1u);
            redo_list[slot] = (uint32_t)r;
        }
        if (r == n - 1) {
            const XState fin = fk_apply(q.tf, s);
            *d_state = fin;
            res->exit = fin;
        }
    }
    if (t == 0 && eof_min != ~0ull) atomicMin(&res->eof_cand, eof_min);
}

/*
 * k_tail (one-pass feeds, after k_count; TAIL_BLOCKS x TAIL_THREADS).  Block
 * j takes 1/B of the table and 1/B of k_count's BlockSums:
 *  - table bins: table = (fresh ? 0 : table) + the FK_SUBTABLES sub-tables
 *    (zeroed), and their statistics;
 *  - BlockSums: each block's first guess against the previous block's last
 *    exit (the local check of block_summary, across blocks), flags, 0xFF
 *    candidates, and for the exit state's run length the last absorbing
 *    block (its exit R is exact) plus the bases of the blocks after it.
 * The last block to finish combines the B partial results (a segmented
 * reduction for the run length), merges the feed's accumulators and
 * publishes the result block.
 */
struct TailPart {
    unsigned long long st[10];   /* table statistics of the bin slice */
    uint64_t eof;                /* smallest 0xFF candidate */
    uint64_t Rj;                 /* exit R of the slice's last absorbing block */
    uint64_t nv_after;           /* bases of the slice's blocks after it (all, if none) */
    uint32_t need;               /* ONE_* bits */
    int32_t j;                   /* the slice's last absorbing block, or -1 */
};

__device__ __forceinline__ unsigned long long wmax64s(long long v) {
    return (unsigned long long)wred64((uint64_t)v, OpMaxS64{});
}

/* Item i of k_tail's chain: a k_count block's BlockSum (i < G), else the
 * dynamic range nstatic + (i - G), summarised here from its RangeRec as a
 * block of one range would be (block_summary). */
__device__ __forceinline__ BlockSum tail_item(const BlockSum *bsum, const RangeRec *rr, uint32_t G,
                                              uint64_t nstatic, uint32_t i) {
    if (i < G) return bsum[i];
    const RangeRec q = rr[nstatic + (i - G)];
    BlockSum b;
    if (q.resume) {
        b.e_R = 0; b.e_code = 0; b.e_hdr = 0;
        b.g_code = 0; b.g_R = 0; b.g_hdr = 0;
        b.nvb = 0; b.eof = ~0ull; b.nv = 0;
        b.flags = ONE_RESUME;
        return b;
    }
    const XState g{q.a_R, q.a_code, q.a_hdr, 0};
    const XState e = fk_apply(q.tf, g);
    b.e_R = e.R; b.e_code = e.code; b.e_hdr = e.hdr;
    b.g_code = q.a_code; b.g_R = q.a_R; b.g_hdr = q.a_hdr;
    b.nvb = (q.c1 - q.c0) * FK_CHUNK_BYTES;
    b.eof = q.eof != FK_NO_EOF64 ? q.c0 * FK_CHUNK_BYTES + q.eof : ~0ull;
    b.nv = q.tf.nv;
    b.flags = q.tf.f0_const ? BS_ABSORB : 0u;
    return b;
}

#define TAIL_KEEP 2
/* k_tail: bin i of the table, and zeros where the sub-tables held counts
   (streaming stores: no dirty L2 lines for a system fence to write back) */
__device__ __forceinline__ void tail_store(uint32_t *table, uint32_t *subs, uint32_t nbins, uint32_t i, uint32_t v,
                                           uint32_t m) {
#pragma unroll
    for (int j = 0; j < FK_SUBTABLES; j++)
        if (m & (1u << j)) __builtin_nontemporal_store(0u, &subs[(size_t)j * nbins + i]);
    __builtin_nontemporal_store(v, &table[i]);
}

__global__ void __launch_bounds__(TAIL_THREADS)
k_tail(const OnePassCfg *opc, uint32_t flags, uint32_t seq, uint32_t *table, int k, uint32_t *subs,
       unsigned long long *facc, DevRes *res, const XState *d_init, uint32_t G0, uint64_t seg_len,
       TailPart *part, uint32_t *done, const RangeRec *rr, uint64_t nstatic, uint32_t ndyn) {
    __shared__ unsigned long long sh[TAIL_THREADS / 64][16];
    __shared__ uint32_t bc[4];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, B = gridDim.x, jb = blockIdx.x;
    const uint32_t nbins = 1u << (2 * k);
    const bool fresh = (flags & OP_FRESH) != 0;
    const BlockSum *bsum = reinterpret_cast<const BlockSum *>(opc->bsum);
    /* the chain: G0 block summaries, then the dynamic ranges */
    const uint32_t G = G0 + ndyn;
    /* every load of the slice phase first (one round trip): this block's
       BlockSums [b0, b1) and their predecessors' exits, one per thread, and
       its table bins with the sub-tables (bins strided over the threads) */
    const uint32_t b0 = (uint32_t)((uint64_t)G * jb / B), b1 = (uint32_t)((uint64_t)G * (jb + 1) / B);
    const uint32_t lo = (uint32_t)((uint64_t)nbins * jb / B), hi = (uint32_t)((uint64_t)nbins * (jb + 1) / B);
    const uint32_t bi = b0 + t;
    const bool hb = bi < b1;   /* G <= B x TAIL_THREADS (host): one item per thread at most */
    BlockSum bs;
    uint64_t pe_R = 0, pe_code = 0;
    uint32_t pe_hdr = 0;
    if (hb) {
        bs = tail_item(bsum, rr, G0, nstatic, bi);
        if (bi > 0) {
            const BlockSum pb = tail_item(bsum, rr, G0, nstatic, bi - 1);
            pe_R = pb.e_R; pe_code = pb.e_code; pe_hdr = pb.e_hdr;
        }
        /* a dynamic range's guess is its exact entering state when the feed
           completes here (block_summary does this for the static ranges) */
        if (bi >= G0 && !(bs.flags & ONE_RESUME))
            opc->rtrue[nstatic + (bi - G0)] = XState{bs.g_R, bs.g_code, bs.g_hdr, 0};
    }
    const int fs = 2 * (k - 1);
    unsigned long long v10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    /* The stores (the table bins, zeros into the sub-tables) wait until this
       block has reported its partial record: a wave's returning atomics come
       back in order behind its earlier stores, so storing first made every
       block's report wait for its stores to complete (~5 us).  A thread
       keeps up to TAIL_KEEP bins (k <= 7: at most 2 with 16 blocks). */
    uint32_t keep_v[TAIL_KEEP], keep_m[TAIL_KEEP], nkeep = 0;
    for (uint32_t i = lo + t; i < hi; i += blockDim.x) {
        uint32_t a[FK_SUBTABLES];
#pragma unroll
        for (int j = 0; j < FK_SUBTABLES; j++) a[j] = subs[(size_t)j * nbins + i];
        uint32_t v = fresh ? 0u : table[i];
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < FK_SUBTABLES; j++) {
            v += a[j];
            m |= a[j] ? 1u << j : 0u;
        }
        if (nkeep < TAIL_KEEP) {
            keep_v[nkeep] = v;
            keep_m[nkeep] = m;
            nkeep++;
        } else {
            tail_store(table, subs, nbins, i, v, m);
        }
        v10[0] += v != 0;
        v10[1] += v;
        const uint32_t ld = i & 3u, fd = k == 1 ? ld : (i >> fs) & 3u;
        v10[2] += ld == 0 ? v : 0; v10[3] += ld == 1 ? v : 0; v10[4] += ld == 2 ? v : 0; v10[5] += ld == 3 ? v : 0;
        v10[6] += fd == 0 ? v : 0; v10[7] += fd == 1 ? v : 0; v10[8] += fd == 2 ? v : 0; v10[9] += fd == 3 ? v : 0;
    }
    /* BlockSum i: its first guess against block i-1's last exit (the local
       check of block_summary, across blocks), flags, 0xFF candidate */
    uint32_t need = 0;
    uint64_t eof = ~0ull;
    long long jmax = -1;
    if (hb) {
        need = bs.flags & (ONE_RESUME | ONE_SCAN);
        if (bi > 0 && !fk_equiv(DState{bs.g_code, bs.g_R, bs.g_hdr}, XState{pe_R, pe_code, pe_hdr, 0}, k, bs.nvb))
            need |= ONE_SCAN;
        eof = bs.eof;
        if (bs.flags & BS_ABSORB) jmax = bi;
    }
    /* the slice's last absorbing block, then the bases after it */
    const long long jw = (long long)wmax64s(jmax);
    if (lane == 0) sh[w][10] = (unsigned long long)jw;
    __syncthreads();
    long long js = -1;
    for (uint32_t q = 0; q < blockDim.x / 64; q++) js = max(js, (long long)sh[q][10]);
    uint64_t nv_after = hb && (long long)bi > js ? bs.nv : 0;
    if (hb && (long long)bi == js) sh[0][11] = bs.e_R;   /* the owner publishes its R */
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(v10[q]);
    nv_after = wsum64(nv_after);
    need = (uint32_t)wred64(need, OpOr64{});
    eof = wred64(eof, OpMin64{});
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 10; q++) sh[w][q] = v10[q];
        sh[w][12] = nv_after;
        sh[w][13] = need;
        sh[w][14] = eof;
    }
    __syncthreads();
    if (w == 0) {
        /* the partial record, with returning exchanges (waited for before
           the count below: no release fence) */
        uint32_t sink = 0;
        if (t < 16) {
            unsigned long long a = t == 14 ? ~0ull : 0ull;
            for (uint32_t q = 0; q < blockDim.x / 64; q++) {
                const unsigned long long v = sh[q][t];
                if (t < 10 || t == 12) a += v;
                else if (t == 13) a |= v;
                else if (t == 14) a = min(a, v);
            }
            TailPart &P = part[jb];
            if (t < 10) sink = xput(&P.st[t], a);
            if (t == 12) sink = xput(&P.nv_after, (uint64_t)a);
            if (t == 13) sink = xput(&P.need, (uint32_t)a);
            if (t == 14) sink = xput(&P.eof, (uint64_t)a);
            if (t == 15) sink = xput(&P.j, (int32_t)js) | xput(&P.Rj, (uint64_t)(js >= 0 ? sh[0][11] : 0));
        }
        keep(sink);
        /* 2. the last block to finish combines */
        if (t == 0) bc[0] = atomicAdd(done, 1u) == B - 1;
    }
    __syncthreads();
    /* k_count is done: block 0 resets its dynamic-range pools for the next
       launch (after its report, like the bin stores) */
    if (jb == 0)
        for (uint32_t q = t; q < FK_MAX_POOLS; q += blockDim.x) done[FK_HEADS_OFF + q * FK_HEAD_STRIDE] = 0;
    if (!bc[0]) {
        for (uint32_t q = 0; q < nkeep; q++) tail_store(table, subs, nbins, lo + t + q * blockDim.x, keep_v[q], keep_m[q]);
        return;
    }
    if (t < 64) {
        if (t == 0) *done = 0;
        /* every load of the combine first: partial `lane`, the last
           BlockSum, the entering state, the accumulators */
        const bool have = lane < B;
        uint32_t nd = 0;
        uint64_t ef = ~0ull, pR = 0, pn = 0;
        int32_t pj = -1;
        unsigned long long st[10];
        if (have) {
            const TailPart &P = part[lane];   /* device-coherent loads (other XCDs wrote them) */
            nd = xget(&P.need); ef = xget(&P.eof); pj = xget(&P.j); pR = xget(&P.Rj); pn = xget(&P.nv_after);
#pragma unroll
            for (int q = 0; q < 10; q++) st[q] = xget(&P.st[q]);
        } else {
#pragma unroll
            for (int q = 0; q < 10; q++) st[q] = 0;
        }
        const BlockSum lb = tail_item(bsum, rr, G0, nstatic, G - 1);
        /* a shard's entering state is unknown: count from its first guess
           (the host checks it against the stitched state at resolve) */
        const bool shard = (flags & OP_SHARD) != 0;
        const BlockSum b0s = bsum[0];
        const XState init = shard ? XState{b0s.g_R, b0s.g_code, b0s.g_hdr, 0}
                                  : fresh ? XState{0, 0, 0, 0} : *d_init;
        unsigned long long fa = 0;
        if (lane < ACC_N)
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) fa += facc[c * ACC_N + lane];
        const unsigned long long ta = lane < ACC_N && !fresh ? opc->acc_total[lane] : 0ull;
#pragma unroll
        for (int q = 0; q < 10; q++) st[q] = wsum64(st[q]);
        nd = (uint32_t)wred64(nd, OpOr64{});
        ef = wred64(ef, OpMin64{});
        /* exit run length: the last slice with an absorbing block, its R,
           plus the bases after it */
        const uint64_t hasj = __ballot(have && pj >= 0);
        const int sstar = hasj ? 63 - __builtin_clzll(hasj) : -1;
        const uint64_t add = wsum64((have && (int)lane > sstar) ? pn : 0);
        const uint64_t base = sstar >= 0 ? rdlane64(pR, sstar) + rdlane64(pn, sstar) : init.R;
        uint32_t need_all = nd;
        /* no run length in the segment reaches the int32 wrap (the local
           checks rely on it) */
        if (!shard && (uint64_t)(uint32_t)init.R + seg_len + FK_CHUNK_BYTES > 0x7FFFFFFFull) need_all |= ONE_SCAN;
        /* the exit state: header flag and last bases of the last block's
           exit (identical trajectories), exact when it absorbs or holds at
           least 32 bases; else the host path */
        if (!(lb.flags & BS_ABSORB) && lb.nv < 32) need_all |= ONE_SCAN;
#pragma unroll
        for (int q = 0; q < 10; q++)
            if (lane == (uint32_t)q) res->tstat[q] = st[q];
        if (need_all == 0 && lane < ACC_N) {
            const unsigned long long v = ta + fa;
            opc->acc_total[lane] = v;
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) facc[c * ACC_N + lane] = 0;
            res->acc[lane] = v;
        }
        if (lane == 0) {
            if (need_all == 0) {
                const uint64_t fR = base + add;
                XState *ps = opc->state;
                ps->R = fR; ps->code = lb.e_code; ps->hdr = lb.e_hdr; ps->pad = 0;
                res->exit.R = fR; res->exit.code = lb.e_code; res->exit.hdr = lb.e_hdr; res->exit.pad = 0;
            } else if (fresh) {
                XState *ps = opc->state;   /* k_scan starts from it */
                ps->R = 0; ps->code = 0; ps->hdr = 0; ps->pad = 0;
            }
            res->eof_cand = need_all ? ~0ull : ef;
            res->redo_n = 0;
            res->need = need_all;
            if (shard) {
                ShardSum &ss = res->shard;
                ss.g_code = b0s.g_code; ss.g_R = b0s.g_R; ss.g_hdr = b0s.g_hdr;
                ss.nvb0 = b0s.nvb;
                ss.absorb = sstar >= 0;
                ss.c_R = sstar >= 0 ? base + add : 0;
                ss.nv = add;
                ss.c_code = lb.e_code; ss.c_hdr = lb.e_hdr;
            }
        }
        publish_res_wave(res, opc->host_res, seq);
    }
    for (uint32_t q = 0; q < nkeep; q++) tail_store(table, subs, nbins, lo + t + q * blockDim.x, keep_v[q], keep_m[q]);
}

/* Sum the per-block partials of k_table_stats into res->tstat and publish
   the result block (one block of 256 threads). */
__device__ void stats_publish(DevRes *res, DevRes *host_res, const unsigned long long *part, uint32_t nparts,
                              uint32_t seq) {
    __shared__ unsigned long long wq[4][10];
    const uint32_t wv = threadIdx.x >> 6;
    unsigned long long acc10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nparts; b += blockDim.x)
#pragma unroll
        for (int q = 0; q < 10; q++) acc10[q] += part[(size_t)b * 10 + q];
#pragma unroll
    for (int q = 0; q < 10; q++) acc10[q] = wsum64(acc10[q]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wq[wv][q] = acc10[q];
    __syncthreads();
    if (threadIdx.x < 10) {
        unsigned long long s = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) s += wq[w][threadIdx.x];
        res->tstat[threadIdx.x] = s;
    }
    __syncthreads();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(res);
    uint32_t *dst = reinterpret_cast<uint32_t *>(host_res);
    for (uint32_t i = threadIdx.x; i < offsetof(DevRes, seq) / 4; i += blockDim.x) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&host_res->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* One pass over the final table: distinct k-mers, total, and the first- and
 * last-base marginals (-> depth-1 trie frequencies and base composition). */
__global__ void __launch_bounds__(256)
k_table_stats(uint32_t *table, uint64_t n, int k, DevRes *res,
              unsigned long long *acc, unsigned long long *facc, int fresh, DevRes *host_res, uint32_t *done,
              uint32_t seq, uint32_t *subs, int nsub, unsigned long long *part, int split,
              const unsigned long long *fz, const uint32_t *glist, const unsigned long long *perr) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            /* the segment's bound checks (k = 15, 16): the general tiles'
               list past its capacity, k_repart / k_count_parts past theirs */
            uint32_t f = perr ? (uint32_t)*perr : 0u;
            if (glist && glist[0] > glist[1]) f |= FK_FAULT_LIST;
            res->fault = f;
        }
        /* the feed's counters (facc, zero between feeds) join the engine's */
        if (threadIdx.x < ACC_N) {
            unsigned long long v = fresh ? 0ull : acc[threadIdx.x];
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) v += facc[c * ACC_N + threadIdx.x];
            acc[threadIdx.x] = v;
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) facc[c * ACC_N + threadIdx.x] = 0;
            res->acc[threadIdx.x] = v;
        }
        if (threadIdx.x == 0) res->need = 0;
    }
    unsigned long long dist = 0, sum = 0, last[4] = {0, 0, 0, 0}, first[4] = {0, 0, 0, 0};
    uint64_t n4 = n / 4;
    /* a fresh k = 15, 16 table whose statistics k_count_parts and
       k_list_add took: they stand unless k_redo changed it since */
    if (fz && res->redo_n == 0) {
        n4 = 0;
        if (threadIdx.x == 0) {
            for (uint32_t sl = blockIdx.x; sl < FZ_SLOTS; sl += gridDim.x) {
                const unsigned long long *z = fz + sl * 10u;
                dist += z[0]; sum += z[1];
                last[0] += z[2]; last[1] += z[3]; last[2] += z[4]; last[3] += z[5];
                first[0] += z[6]; first[1] += z[7]; first[2] += z[8]; first[3] += z[9];
            }
        }
    }
    uint4 *t4 = reinterpret_cast<uint4 *>(table);
    const int fs = 2 * (k - 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = t4[i];
        if (nsub) {
            /* fold k_count's sub-tables into the table (and clear them); all
               FK_SUBTABLES loads in flight at once */
            uint4 a[FK_SUBTABLES];
#pragma unroll
            for (int s = 0; s < FK_SUBTABLES; s++) a[s] = reinterpret_cast<uint4 *>(subs + (size_t)s * n)[i];
#pragma unroll
            for (int s = 0; s < FK_SUBTABLES; s++) {
                v.x += a[s].x; v.y += a[s].y; v.z += a[s].z; v.w += a[s].w;
                reinterpret_cast<uint4 *>(subs + (size_t)s * n)[i] = make_uint4(0, 0, 0, 0);
            }
            t4[i] = v;
        }
        dist += (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
        unsigned long long s4 = (unsigned long long)v.x + v.y + v.z + v.w;
        sum += s4;
        last[0] += v.x; last[1] += v.y; last[2] += v.z; last[3] += v.w;
        if (k == 1) {
            first[0] += v.x; first[1] += v.y; first[2] += v.z; first[3] += v.w;
        } else {
            uint32_t fd = (uint32_t)(((i * 4) >> fs) & 3);
            first[0] += fd == 0 ? s4 : 0; first[1] += fd == 1 ? s4 : 0;
            first[2] += fd == 2 ? s4 : 0; first[3] += fd == 3 ? s4 : 0;
        }
    }
    /* block partials (no same-address atomics across hundreds of blocks:
       the last block adds them up) */
    __shared__ unsigned long long wp[4][10];
    unsigned long long v10[10] = {dist, sum, last[0], last[1], last[2], last[3], first[0], first[1], first[2], first[3]};
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(v10[q]);
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wp[wv][q] = v10[q];
    __syncthreads();
    if (threadIdx.x < 10) {
        unsigned long long s = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) s += wp[w][threadIdx.x];
        part[(size_t)blockIdx.x * 10 + threadIdx.x] = s;
    }
    /* the last block to finish sums the partials, then publishes the whole
       result block to pinned host memory, sequence number last: the host
       spins on it instead of a copy plus a stream synchronisation.  With
       `split` (large tables: hundreds of blocks, whose release fences would
       each write back the L2 the table was just written into) the blocks
       stop here and k_table_final does that in a second launch. */
    if (split) return;
    __shared__ uint32_t is_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) is_last = atomicAdd(done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    stats_publish(res, host_res, part, gridDim.x, seq);
    if (threadIdx.x == 0) *done = 0;
}

__global__ void __launch_bounds__(256)
k_table_final(DevRes *res, DevRes *host_res, const unsigned long long *part, uint32_t nparts, uint32_t seq) {
    stats_publish(res, host_res, part, nparts, seq);
}

/* the LDS-counting kernels keep their bins at LDS address 0 (lds_add) */
bool lds_layout_ok() {
    static int ok = -1;
    if (ok < 0) {
        const void *fns[] = {(const void *)k_count<H_PAIRS>, (const void *)k_count<H_LDS>,
                             (const void *)k_resume<H_PAIRS>, (const void *)k_resume<H_LDS>,
                             (const void *)k_redo<H_PAIRS>, (const void *)k_redo<H_LDS>};
        int good = 1;
        for (const void *f : fns) {
            hipFuncAttributes a;
            if (hipFuncGetAttributes(&a, f) != hipSuccess || a.sharedSizeBytes != 0) good = 0;
        }
        ok = good;
    }
    return ok == 1;
}

int launch_count(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g,
                        int has_init, bool onepass, bool fresh, bool shard) {
    size_t sh = lds_bytes(e);
    const uint32_t flags = (onepass ? (OP_ON | (fresh ? OP_FRESH : 0u) | (shard ? OP_SHARD : 0u)) : 0u) |
                           (e->no_mixed ? (uint32_t)OP_NOMIX : 0u);
    FK_DISPATCH_COUNT(e,
                hipExtLaunchKernelGGL((k_count<HM>), dim3(g.grid), dim3(FK_BLOCK), sh, e->stream, tev(e, 0), tev(e, 1),
                                      0, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr,
                                   g.nchunks, e->d_state, has_init, g.cpw, e->d_resume, e->general_tiles,
                                   e->d_sub, e->d_opc, flags, g.nstatic, g.dg, e->d_ctl + FK_HEADS_OFF));
    HIPCHK(hipGetLastError());
    if (onepass) {
        if (++e->res_seq == 0) e->res_seq = 1;
        /* one chain item per thread: the block summaries, then the dynamic ranges */
        const uint64_t items = (uint64_t)g.grid + g.dg.ndyn;
        const unsigned tb = (unsigned)std::max<uint64_t>(TAIL_BLOCKS, (items + TAIL_THREADS - 1) / TAIL_THREADS);
        hipExtLaunchKernelGGL(k_tail, dim3(tb), dim3(TAIL_THREADS), 0, e->stream, nullptr, tev(e, 2), 0,
                              e->d_opc, flags, e->res_seq, e->d_table, e->k, e->d_sub, e->d_facc, e->d_res,
                              e->d_state, g.grid, len, reinterpret_cast<TailPart *>(e->d_tpart), e->d_ctl,
                              e->d_rr, g.nstatic, g.dg.ndyn);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

int launch_resume(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
    size_t sh = lds_bytes(e);
    FK_DISPATCH_COUNT(e,
                hipLaunchKernelGGL((k_resume<HM>), dim3(g.rgrid), dim3(FK_BLOCK), sh, e->stream, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nranges,
                                   e->d_resume, e->d_ctl + FK_HEADS_OFF, e->no_mixed ? 0 : 1));
    HIPCHK(hipGetLastError());
    return FK_OK;
}

int launch_redo(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int mode) {
    size_t sh = lds_bytes(e);
    FK_DISPATCH(hist_mode(e),
                hipLaunchKernelGGL((k_redo<HM>), dim3(g.rgrid), dim3(FK_BLOCK), sh, e->stream, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr,
                                   e->d_rtrue, e->d_redo, g.nranges, mode, e->no_mixed ? 0 : 1));
    HIPCHK(hipGetLastError());
    return FK_OK;
}


int launch_scan(fk_engine *e, const Geo &g, int mode) {
    {
        const int rc = flush_state(e);
        if (rc) return rc;
    }
    const unsigned blocks = (unsigned)((g.nranges + SCAN_THREADS - 1) / SCAN_THREADS);
    if (++e->scan_epoch == 0) {   /* flags hold epochs; never reuse 0 */
        HIPCHK(hipMemsetAsync(e->d_flags, 0, e->range_cap / SCAN_THREADS * sizeof(uint32_t) + 64, e->stream));
        e->scan_epoch = 1;
    }
    hipLaunchKernelGGL(k_scan, dim3(blocks), dim3(SCAN_THREADS), 0, e->stream, e->d_rr, g.nranges, e->d_state,
                       e->d_rtrue, e->d_redo, e->d_res, e->k, mode, e->d_tf, e->d_aggs, e->d_flags, e->scan_epoch);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* Table statistics and an accumulator snapshot into d_res, published to the
   pinned host copy (e->h_res) with a new sequence number.  The feed path's
   k_count has zeroed the sums already; other callers ask for a memset.
   `stop` (optional) is recorded when the kernel completes. */
int launch_table_stats(fk_engine *e, bool zero_first, hipEvent_t stop, bool subs,
                              bool fresh) {
    if (zero_first) HIPCHK(hipMemsetAsync(e->d_res->tstat, 0, sizeof(e->d_res->tstat), e->stream));
    unsigned gd = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 4, (e->nbins / 4 + 255) / 256 + 1);
    if (e->ts_blocks) gd = std::min<unsigned>(e->ts_blocks, (unsigned)e->cus * 4);
    const int split = gd > 16;   /* large tables: partials, then k_table_final */
    if (++e->res_seq == 0) e->res_seq = 1;
    const bool fz = e->fz_ready;   /* only for the statistics right after a fresh two-level count */
    e->fz_ready = false;
    const bool gl = fz || e->glist_live;
    e->glist_live = false;
    unsigned long long *perr = e->perr_live ? e->d_perr : nullptr;
    e->perr_live = false;
    hipExtLaunchKernelGGL(k_table_stats, dim3(gd), dim3(256), 0, e->stream, nullptr, split ? nullptr : stop, 0,
                          e->d_table, e->nbins, e->k, e->d_res, e->d_acc, e->d_facc, fresh ? 1 : 0, e->h_res_dev,
                          e->d_done, e->res_seq, e->d_sub, (subs && e->d_sub) ? FK_SUBTABLES : 0, e->d_tpart, split,
                          fz ? (const unsigned long long *)e->d_fz : nullptr, gl ? (const uint32_t *)e->d_glist : nullptr,
                          (const unsigned long long *)perr);
    HIPCHK(hipGetLastError());
    if (split) {
        hipExtLaunchKernelGGL(k_table_final, dim3(1), dim3(256), 0, e->stream, nullptr, stop, 0, e->d_res,
                              e->h_res_dev, e->d_tpart, gd, e->res_seq);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

/* Wait for the result block published by the last launch_table_stats() and
   copy it to e->last: spin on its sequence number in pinned memory, checking
   the stream for errors now and then. */
int wait_results(fk_engine *e) {
    const uint32_t want = e->res_seq;
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&e->h_res->seq, __ATOMIC_ACQUIRE) == want) break;
        if ((spin & 4095) == 0) {
            hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(&e->h_res->seq, __ATOMIC_ACQUIRE) == want) break;
                return FK_E_HIP;   /* stream drained without publishing */
            }
            if (q != hipErrorNotReady) return FK_E_HIP;
        }
        __builtin_ia32_pause();
    }
    memcpy(&e->last, e->h_res, sizeof(DevRes));
    return FK_OK;
}

/* the LDS bins of k_count / k_redo / k_resume (k <= 6: 5 x 4^k words) need
   more than the default dynamic-LDS limit */
int scan_kernels_init(size_t sh) {
    if (sh > 65536)
        for (const void *f : {(const void *)k_count<H_PAIRS>, (const void *)k_redo<H_PAIRS>,
                              (const void *)k_resume<H_PAIRS>})
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess)
                return FK_E_HIP;
    return FK_OK;
}
