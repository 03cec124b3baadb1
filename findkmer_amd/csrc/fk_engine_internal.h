/*
 * fk_engine_internal.h -- struct fk_engine and the host helpers the engine's
 * translation units share (fk_engine, fk_scan, fk_part, fk_sparse_pass,
 * fk_exchange).  Not part of the C-ABI (include/findkmer.h).
 */
#pragma once
#include "fk_tiles.h"
#include "fk_part.h"

/* ------------------------------------------------------------------------- */
/* host engine                                                                */
/* ------------------------------------------------------------------------- */

#define HIPCHK(x)                                                               \
    do {                                                                        \
        hipError_t _e = (x);                                                    \
        if (_e != hipSuccess) {                                                 \
            fprintf(stderr, "findkmer: %s failed: %s (%s:%d)\n", #x,             \
                    hipGetErrorString(_e), __FILE__, __LINE__);                 \
            return FK_E_HIP;                                                    \
        }                                                                       \
    } while (0)

/* A scratch device allocation, freed on every return path (hipFree waits for
   the work queued on it). */
struct DevScratch {
    void *p = nullptr;
    size_t bytes = 0;
    DevScratch() = default;
    DevScratch(const DevScratch &) = delete;
    DevScratch &operator=(const DevScratch &) = delete;
    ~DevScratch() { release(); }
    bool alloc(size_t n) {
        release();
        if (hipMalloc(&p, n) != hipSuccess) { p = nullptr; return false; }
        bytes = n;
        return true;
    }
    void release() { if (p) hipFree(p); p = nullptr; bytes = 0; }
    template <class T> T *as() const { return (T *)p; }
};

static const uint64_t SEG_MAX_BYTES = 1ull << 34;                 /* 16 GiB per segment */
static const uint64_t STAGE_BYTES = 256ull << 20;                 /* host feed staging */
static const unsigned long long NO_EOF64 = ~0ull;

struct fk_engine {
    int dev = 0, k = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    fk_opts opts{};
    uint64_t nbins = 0, nshort = 0, maskk = 0;
    int cus = 256;
    uint32_t ts_blocks = 0;                   /* k_table_stats grid override (0 = default) */
    bool part = false;                        /* 8 <= k <= 13: partitioned counting (k_part) */
    bool sparse = false;                      /* 17 <= k <= 20: key-range passes at finish (k_sp_emit) */
    uint8_t *d_keep = nullptr;                /* sparse: the input fed so far */
    XState *d_kst = nullptr;                  /* sparse: every retained range's exact entering state */
    uint64_t keep_len = 0, keep_cap = 0, kst_len = 0, kst_cap = 0;
    /* src: the caller's bytes (opts.borrow_input), else at d_keep + off */
    struct SpSeg { uint64_t off, len, st, nranges, cpw, nchunks; const uint8_t *src; };
    bool seg_borrow = false;                  /* the segment being fed lies in the caller's device buffer */
    std::vector<SpSeg> spsegs;                /* the retained segments */
    /* the finished table, contiguous (the passes append in key order): keys
       ascending + u32 counts; kept across steps (grown, never shrunk), as are
       a pass's emitted keys and the dense bucket table */
    uint64_t *d_spk = nullptr;
    uint32_t *d_spc = nullptr;
    uint64_t spk_cap = 0, spc_cap = 0;
    uint64_t *d_emit = nullptr;
    uint64_t emit_cap = 0;
    unsigned long long *d_spdense = nullptr;
    uint64_t spdense_cap = 0;
    uint64_t sp_distinct = 0;
    uint64_t sp_pass = 0;                     /* FINDKMER_TUNE sp_pass: window keys per pass (0: by free HBM) */
    FksState fks;
    bool sp_done = false;                     /* d_spk / d_spc hold the finished table */
    unsigned long long sp_nodes = 0, sp_roll = 0, sp_tstat[10] = {};
    uint16_t *d_codes = nullptr;              /* k_part: block code regions */
    uint32_t *d_pflag = nullptr;              /* k_part: a range went to k_part<RES> */
    uint32_t *d_pidx = nullptr;               /* k_part: slice-major run index */
    uint64_t codes_cap = 0, pidx_cap = 0;
    uint32_t *d_pairs = nullptr;              /* k_part pairs mode: 4^(k+1) pair bins + 4^k single bins */
    uint16_t *d_parts = nullptr;              /* k = 15, 16: the second level's part streams (k_repart) */
    uint64_t parts_cap = 0;
    void *d_pmeta = nullptr;                  /* k = 15, 16: PartMeta per part + the allocation counter */
    /* k_repart<SEG>'s segment table and per-block (base, rounds) + its claim counter */
    unsigned long long *d_rdesc = nullptr, *d_rbm = nullptr;
    uint64_t rdesc_cap = 0, rbm_cap = 0;
    int32_t *d_rsend = nullptr, *d_rrecv = nullptr;   /* routed sharded tables: blobs out / in (fk_engine_route_*) */
    uint64_t rsend_cap = 0, rrecv_cap = 0, rsend_words = 0;
    void *d_raux = nullptr;                   /* ... their per-destination geometry and slot offsets */
    uint64_t raux_cap = 0;
    int32_t *d_rsz = nullptr;                 /* ... the world x world blob-size matrix (16-bit limbs) */
    uint64_t rsz_cap = 0;
    int route_mode = 0;                       /* FINDKMER_TUNE route: 0 = reduce-scatter the table (default: the
                                                 routed send/recv has not run at world > 1 on hardware, ADVICE
                                                 r5), 1 = route it when world > 1 (at world 1 the reduce-scatter
                                                 is a local copy), 2 = route at any world (tests) */
    uint64_t pair_cap = 0;
    uint32_t w16_ks = W16_KS_DEFAULT;         /* k (bits) counted through k_bucket16 (FINDKMER_TUNE w16=mask) */
    int part_pairs_kmax = 12;                 /* pairs mode for k <= this (FINDKMER_TUNE pairs_kmax; k = 12 pairs:
                                                 2048 slices of 32-code runs, half the entries of
                                                 512 single-window slices: 1 G-base step 1.63 -> 1.36 ms) */
    uint32_t general_tiles = FK_COUNT_GENERAL_TILES;   /* per range in k_count */
    /* device state */
    uint32_t *d_table = nullptr, *d_short = nullptr;
    uint32_t *d_sub = nullptr;                /* FK_SUBTABLES table copies k_count flushes into (LDS modes) */
    unsigned long long *d_acc = nullptr;      /* ACC_N, engine lifetime (+ ACC_N: d_facc) */
    unsigned long long *d_facc = nullptr;     /* FK_ACC_COPIES x ACC_N the counting kernels of a feed add into;
                                                 merged into d_acc by the feed's publisher, zero between feeds */
    /* one-pass k_count (k <= 7, entering state known) */
    bool onepass = true;                      /* k <= 7: k_count + k_tail in one pass */
    BlockSum *d_bsum = nullptr;               /* per block of k_count */
    uint32_t *d_ctl = nullptr;                /* k_tail's finished-block count */
    uint32_t ranges_per_wave = 1;             /* k <= 7: ranges per k_count wave slot */
    bool no_mixed = false;                    /* FINDKMER_TUNE no_mixed=1: no mixed tiles (general byte walk) */
    uint32_t part_general = 1;                /* k_part: general tiles per range (FINDKMER_TUNE part_general) */
    uint32_t static_pct = 100;                /* k <= 7: % of a large segment in static ranges (FINDKMER_TUNE static_pct;
                                                 100 = no dynamic ranges: on a plain stream the waves that
                                                 finish early hand their bandwidth to the others, so
                                                 balancing gains nothing -- 1 GB k=6 0.174 ms either way --
                                                 while header-dense input gains 9 % at 75) */
    uint32_t cls_w[4] = {1000, 1000, 1000, 1000};   /* static share per wave class, per mille */
    uint64_t dyn_min_chunks = 0;              /* segments with dynamic ranges: >= this many chunks (0: 8 per
                                                 wave slot; FINDKMER_TUNE dyn_min_chunks, tests) */
    OnePassCfg *d_opc = nullptr;
    bool op_pending = false;                  /* the last count_segment launched a one-pass k_count */
    bool op_fresh = false;                    /* ... which did a pending reset itself */
    /* a shard counted in one pass: its k_tail result (compact summary) */
    bool shard_op = false, shard_waited = false, shard_full = false, shard_resumed = false;
    int dev_ev = 2;                           /* event that ends the last feed's device path */
    DevRes *d_res = nullptr;                  /* per feed */
    unsigned long long *d_tmp = nullptr;      /* scratch counters */
    XState *d_state = nullptr;                /* entering state of the next feed */
    RangeRec *d_rr = nullptr;
    XState *d_rtrue = nullptr;
    uint32_t *d_redo = nullptr;
    ResumeRec *d_resume = nullptr;            /* ranges k_count hands to k_resume */
    TF *d_aggs = nullptr;                     /* k_scan block aggregates */
    uint32_t *d_flags = nullptr;              /* ... and their epoch flags */
    uint32_t scan_epoch = 0;
    TF *d_tf = nullptr;
    uint64_t range_cap = 0;
    uint8_t *d_stage = nullptr, *h_stage = nullptr;
    hipEvent_t ev[3] = {};
    bool times_pending = false;               /* ev[] of the last feed not yet read */
    bool timing = true;                       /* record ev[] (FINDKMER_TUNE events=0: off) */
    bool zero_pending = false;                /* reset() not yet issued to the device */
    DevRes *h_res = nullptr, *h_res_dev = nullptr;   /* pinned, mapped result block */
    uint32_t *d_done = nullptr;               /* k_table_stats finished-block count */
    unsigned long long *d_tpart = nullptr;    /* k_table_stats per-block partial sums */
    uint32_t res_seq = 0;
    /* host bookkeeping */
    XState state{0, 0, 0, 0};
    DevRes last{};                            /* last feed's results */
    bool stats_valid = false;                 /* last.tstat describes the table */
    bool tail_added = false;                  /* end-of-input short run recorded */
    uint64_t fed = 0, scanned = 0, chunks = 0, redo = 0;
    int ended = 0;                            /* a 0xFF byte ended the input */
    int shard_pending = 0;
    const uint8_t *shard_buf = nullptr;
    uint64_t shard_len = 0;
    int64_t shard_lo = 0;
    double dev_ms = 0, main_ms = 0;
    uint64_t timed_n = 0;                     /* launches main_ms covers */
    uint64_t launch_no = 0;                   /* counting launches, for timing_every */
    uint32_t timing_every = 1;
    bool cur_timed = true;                    /* the current feed's launches record events */
    std::vector<uint8_t> unknown_bytes;
    std::vector<uint64_t> unknown_pos;        /* collect_unknown = 2: their stream offsets */
    /* partitioned path near the reference's int32 seqSize zone: a segment
       whose guessed range states are mostly wrong is recounted from the exact
       states instead of cancelled range by range (resolve_and_fetch) */
    XState dstate_val{0, 0, 0, 0};            /* d_state to write before the next kernel that reads it */
    bool dstate_pending = false;
    bool dirty = false;                       /* table / short walks changed since the last reset */
    bool seg_clean = true;                    /* ... not before the current segment */
    bool tab_fresh = false;                   /* k = 15, 16: this segment's k_zero left the table out
                                                 (k_count_parts writes every bin, k_list_add the rest) */
    uint32_t *d_glist = nullptr;              /* ... the general tiles' windows: [0] count, [1] cap, indices */
    uint64_t glist_cap = 0;
    unsigned long long *d_fz = nullptr;       /* ... and its statistics from k_count_parts (FZ_SLOTS x 10) */
    bool fz_ready = false;                    /* the next launch_table_stats may take them */
    bool glist_live = false;                  /* ... and must check the general tiles' list for overflow */
    unsigned long long *d_perr = nullptr;     /* k = 15, 16: k_repart / k_count_parts bound-check bits */
    bool perr_live = false;                   /* ... set by the last launch_part, for the next statistics */
    uint64_t glist_force = 0;                 /* FINDKMER_TUNE glist_cap=N: the list's capacity (tests) */
    uint64_t list_recounts = 0;               /* segments counted again after the list overflowed */
    bool seg_snap = false;                    /* d_snap holds them as before the current segment */
    uint32_t *d_snap = nullptr;
    uint64_t snap_cap = 0;
    /* fk_engine_shard_exchange: gathered pack rows, pinned and mapped (word
       0: sequence number, rows from word 32) */
    uint32_t *h_rows = nullptr, *h_rows_dev = nullptr;
    uint32_t *d_rows = nullptr;               /* the stitched exchange's rows (device) */
    uint32_t rows_cap = 0, rows_seq = 0;
    /* scratch buffers kept across calls (PoolScratch): the sparse finish
       and its passes took ~20 hipMalloc / hipFree pairs a step, and a
       hipFree waits for the device */
    static const int NPOOL = 14;
    void *pool_p[NPOOL] = {};
    size_t pool_cap[NPOOL] = {};
};

/* A scratch device buffer from the engine's pool slot `i` (grown on demand,
   freed with the engine): DevScratch's interface without a hipFree per use.
   Two buffers live at the same time must use different slots. */
struct PoolScratch {
    fk_engine *e;
    int i;
    void *p = nullptr;
    PoolScratch(fk_engine *eng, int slot) : e(eng), i(slot) {}
    bool alloc(size_t n) {
        if (n > e->pool_cap[i] || !e->pool_p[i]) {
            hipFree(e->pool_p[i]);
            e->pool_p[i] = nullptr;
            e->pool_cap[i] = 0;
            if (hipMalloc(&e->pool_p[i], n) != hipSuccess) return false;
            e->pool_cap[i] = n;
        }
        p = e->pool_p[i];
        return true;
    }
    template <class T> T *as() const { return (T *)p; }
};

static inline int hist_mode(const fk_engine *e) {
    return e->sparse ? H_SPARSE : e->k <= 6 ? H_PAIRS : e->k == 7 ? H_LDS : H_GLOBAL;
}

/* 128 VGPRs -> 4 waves/SIMD = two 512-thread blocks per CU */
static inline uint64_t blocks_per_cu(const fk_engine *) { return 2; }

static inline size_t lds_bytes(const fk_engine *e) {
    int m = hist_mode(e);
    if (m == H_PAIRS) return ((size_t)e->nbins * 4 + e->nbins) * sizeof(uint32_t);
    if (m == H_LDS) return (size_t)e->nbins * sizeof(uint32_t);
    return 0;
}

/* Zero table, counters and the stream state (asynchronous, stream-ordered). */
/* a sparse buffer of at least `n` elements of `sz` bytes (contents dropped) */
static inline int sp_ensure(void **p, uint64_t *cap, uint64_t n, size_t sz) {
    if (*p && *cap >= n) return FK_OK;
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t c = std::max<uint64_t>(n, 1024);
    if (hipMalloc(p, c * sz) != hipSuccess) return FK_E_OOM;
    *cap = c;
    return FK_OK;
}

/* A segment's decomposition into per-wave chunk ranges. */
struct Geo {
    uint64_t nchunks, cpw, nranges;
    uint64_t nstatic;     /* static ranges (one per k_count wave) */
    DynGeo dg;            /* the dynamic ranges after them (k <= 7) */
    unsigned grid;        /* k_count's blocks */
    unsigned rgrid;       /* blocks of the one-wave-per-range kernels (k_resume, k_redo) */
};
/* k_part's waves per block: 16 for the tables of 512 slices or more (one
   block per CU: only 16-wave blocks have the LDS for their cursors, PART_SM),
   else 8 (two per CU; 16 measured 1-5 % slower for k = 8..10, rounds 2, 3) */
static inline uint32_t part_waves_of(const fk_engine *e) { return e->k >= 11 ? 16u : 8u; }

static inline Geo geometry(const fk_engine *e, uint64_t len) {
    Geo g;
    g.nchunks = (len + FK_CHUNK_BYTES - 1) / FK_CHUNK_BYTES;
    uint64_t max_waves = (uint64_t)e->cus * blocks_per_cu(e) * FK_WAVES_PER_BLOCK;
    /* k_part: one range per wave of its blocks, the blocks one round over the CUs */
    if (e->part) max_waves = (uint64_t)e->cus * part_waves_of(e) * (part_waves_of(e) >= 16u ? 1u : 2u);
    /* k <= 7 (k_count counts in LDS): ranges_per_wave ranges per wave slot
       of the chip, i.e. that many rounds of blocks (experiment knob, default
       1).  Equal static ranges finish up to 35 % apart (tools/wave_times.py:
       per-XCD means differ by ~18 %), but more rounds of smaller blocks do
       not fix it -- the dispatcher deals blocks to the XCDs round-robin --
       and cost LDS zero/flush per block: 4 rounds 0.29 ms vs 0.18 ms. */
    if (!e->part && !e->sparse && LDS_MODE(hist_mode(e))) max_waves *= e->ranges_per_wave;
    memset(&g.dg, 0, sizeof g.dg);
    g.dg.nchunks = g.nchunks;
    const uint64_t min_chunks = e->dyn_min_chunks ? e->dyn_min_chunks : 8 * max_waves;
    const bool dyn = !e->part && !e->sparse && LDS_MODE(hist_mode(e)) && e->static_pct < 100 &&
                     g.nchunks >= std::max<uint64_t>(min_chunks, 4);
    if (dyn) {
        /* static ranges cover static_pct % of the segment (one per wave, or
           fewer for a short segment); the rest is cut into dynamic ranges of
           4u, 2u and u chunks (half, a quarter and a quarter of it), u chosen
           so that there are at most ~16 K of them */
        const uint64_t sc = std::max<uint64_t>(1, g.nchunks * e->static_pct / 100);
        g.cpw = std::max<uint64_t>(1, sc / max_waves);
        g.nstatic = std::min<uint64_t>(max_waves, sc / g.cpw);
        DynGeo &d = g.dg;
        const uint64_t grid = (g.nstatic + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK;
        /* one pool per pair of k_count blocks (the blocks one CU holds) */
        d.npools = (uint32_t)std::min<uint64_t>(FK_MAX_POOLS, std::max<uint64_t>(1, grid / blocks_per_cu(e)));
        for (int c = 0; c < 4; c++) d.cls[c] = (uint32_t)g.cpw;
        if (g.nstatic == max_waves && grid == 2ull * d.npools) {
            /* weighted static ranges per wave class (cls_w, per mille) */
            const uint64_t wsum = e->cls_w[0] + e->cls_w[1] + e->cls_w[2] + e->cls_w[3];
            const uint64_t avg = sc / max_waves;
            uint64_t tot = 0;
            for (int c = 0; c < 4; c++) {
                d.cls[c] = (uint32_t)std::max<uint64_t>(1, avg * e->cls_w[c] * 4 / wsum);
                tot += d.cls[c];
            }
            if (tot * (max_waves / 4) >= g.nchunks)
                for (int c = 0; c < 4; c++) d.cls[c] = (uint32_t)g.cpw;   /* keep a dynamic part */
        }
        const uint64_t stot = (uint64_t)d.npools * (4ull * d.cls[0] + 4ull * d.cls[1]) +
                              (grid - std::min<uint64_t>(grid, d.npools)) * (4ull * d.cls[2] + 4ull * d.cls[3]);
        const bool uniform = d.cls[0] == d.cls[1] && d.cls[1] == d.cls[2] && d.cls[2] == d.cls[3];
        d.base = uniform ? g.nstatic * g.cpw : stot;
        const uint64_t D = g.nchunks - d.base;
        const uint64_t u = std::max<uint64_t>(1, (D + 2 * FK_DYN_TARGET - 1) / (2 * FK_DYN_TARGET));
        d.sz[0] = (uint32_t)(4 * u); d.sz[1] = (uint32_t)(2 * u); d.sz[2] = (uint32_t)u;
        d.n[0] = (uint32_t)(D / 2 / d.sz[0]);
        d.n[1] = (uint32_t)(D / 4 / d.sz[1]);
        const uint64_t rem = D - (uint64_t)d.n[0] * d.sz[0] - (uint64_t)d.n[1] * d.sz[1];
        d.n[2] = (uint32_t)((rem + u - 1) / u);
        d.ndyn = d.n[0] + d.n[1] + d.n[2];
    } else {
        g.cpw = std::max<uint64_t>(1, (g.nchunks + max_waves - 1) / max_waves);
        g.nstatic = (g.nchunks + g.cpw - 1) / g.cpw;
    }
    g.nranges = g.nstatic + g.dg.ndyn;
    g.grid = (unsigned)std::max<uint64_t>(1, (g.nstatic + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK);
    g.rgrid = (unsigned)std::max<uint64_t>(1, (g.nranges + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK);
    return g;
}

#define FK_DISPATCH(HMV, ...)                                                   \
    switch (HMV) {                                                              \
    case H_PAIRS: { constexpr int HM = H_PAIRS; __VA_ARGS__; } break;          \
    case H_LDS: { constexpr int HM = H_LDS; __VA_ARGS__; } break;              \
    case H_SPARSE: { constexpr int HM = H_SPARSE; __VA_ARGS__; } break;        \
    default: { constexpr int HM = H_GLOBAL; __VA_ARGS__; } break;              \
    }
/* the counting passes of k_count / k_resume: state only (H_NONE) when the
   partitioned path (k_part) does the counting */
#define FK_DISPATCH_COUNT(e, ...)                                               \
    if ((e)->part || (e)->sparse) { constexpr int HM = H_NONE; __VA_ARGS__; }   \
    else FK_DISPATCH(hist_mode(e), __VA_ARGS__)

/* the timing events of a launch (none when timing is off) */
static inline hipEvent_t tev(const fk_engine *e, int i) { return e->timing && e->cur_timed ? e->ev[i] : nullptr; }

#define SCAN_THREADS 256                                    /* k_scan's blocks */
#define SCAN_WAVES (SCAN_THREADS / 64)
#define FK_SUMMARY_COMPACT 0x434F4D50414354ull   /* "COMPACT": tag in w[11] */

/* host functions defined in one translation unit, used by others */
int scan_kernels_init(size_t lds_bytes);
int part_kernels_init();
bool lds_layout_ok();
int launch_count(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g,
                        int has_init, bool onepass = false, bool fresh = false, bool shard = false);
int launch_resume(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g);
int launch_redo(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int mode);
int launch_scan(fk_engine *e, const Geo &g, int mode);
int launch_table_stats(fk_engine *e, bool zero_first, hipEvent_t stop = nullptr, bool subs = true,
                              bool fresh = false);
int wait_results(fk_engine *e);
int launch_part(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int has_init,
                       const XState *exact = nullptr);
int sp_count_runs32(fk_engine *e, const uint32_t *keys, uint64_t n, uint64_t lo, uint64_t npads,
                           unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw);
int sp_sort_runs64(fk_engine *e, const uint64_t *keys, uint64_t n, uint64_t lo, uint64_t hi, uint64_t npads,
                          unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw, bool *fallback);
int sparse_finish(fk_engine *e, int32_t seq);
int sparse_copy(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n,
                       hipMemcpyKind kind);
int sparse_lower_bound(fk_engine *e, uint64_t want, uint64_t *at);
int ensure_rows(fk_engine *e, uint32_t nrow);
int rows_fetch(fk_engine *e, const uint32_t *rows, uint32_t nrow);
uint64_t merge_table_words(uint64_t nbins, int world);
int route_pack(fk_engine *e, int world, bool counting, uint64_t *words);
int route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words, int32_t *slice,
                        unsigned long long *stats);
int route_exchange(fk_engine *e, fk_comm *comm, bool counting, int32_t *slice, unsigned long long *stats);
int stitched_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *first_end_out, bool scatter);
int flush_state(fk_engine *e);
hipError_t write_dstate(fk_engine *e, const XState &x);
int flush_zero(fk_engine *e, bool keep_table = false);
int set_dev(fk_engine *e, bool flush = true);
int zero_all(fk_engine *e);
bool tune_knob(const char *name, uint64_t *v);
/* k_repart<SEG> over pg's rows (ncodes codes at most): its segment table,
   block metadata and the parts buffer sized, the claim counters zeroed */
int repart_seg_alloc(fk_engine *e, const PartGeo &pg, uint64_t ncodes, uint32_t gp, RepartSeg *sg);
int grow_arrays(fk_engine *e, uint64_t nranges);
bool int32_zone_possible(const fk_engine *e, uint64_t len);
int check_fault(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g);
int resolve_and_fetch(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g);
int exact_eof(fk_engine *e, const Geo &g, unsigned long long &eof);
int collect_unknown(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g);
void add_times(fk_engine *e);
void settle_times(fk_engine *e, bool wait);
int count_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, int has_init, Geo &g,
                         bool shard = false);
int finish_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g,
                          const XState &entering);
int sp_grow(fk_engine *e, void **buf, uint64_t *cap, uint64_t used, uint64_t need);
int sp_retain(fk_engine *e, const uint8_t *dbuf, uint64_t len, const Geo &g);
int sparse_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, bool prefix = false);
int process_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len);
uint64_t segment_budget(fk_engine *e, uint64_t len);
int shard_wait(fk_engine *e);
int shard_full_tf(fk_engine *e);
bool compact_apply(const fk_summary *s, const XState &in, XState &out);
