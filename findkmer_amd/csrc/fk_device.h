/*
 * fk_device.h — device-side building blocks shared by the engine kernels.
 *
 * Scan semantics restated from findKmer/src/findKmer.cpp:962-1069 (see
 * DESIGN.md §2).  A stream position's scan state is (hdr, R, code):
 *   hdr  — inside a '>' comment line (:991-1008)
 *   R    — valid bases since the last run break, modulo 2^32: the reference's
 *          `int seqSize` (:977) is seq = (int32)R, so its wrap after 2^31-1 is
 *          reproduced exactly
 *   code — the last bases, 2 bits each, first base most significant
 *          (base2int :567-589; the window :947-958)
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FK_LANE_BYTES 32u              /* bytes per lane per tile */
#define FK_TILE_BYTES (64u * FK_LANE_BYTES)   /* one wave: 2 KiB */
#define FK_CHUNK_TILES 8u
#define FK_CHUNK_BYTES (FK_TILE_BYTES * FK_CHUNK_TILES)   /* 16 KiB per chunk */
#define FK_HALO_BYTES 256u             /* bytes before a chunk used to guess state */
#define FK_BLOCK 512u
#define FK_COUNT_GENERAL_TILES 8u      /* general-path tiles k_count takes per range */
#define FK_SUBTABLES 16                /* table copies k_count's blocks flush into (LDS modes) */
#define FK_WAVES_PER_BLOCK (FK_BLOCK / 64u)

/* accumulator slots (u64, device) */
enum {
    ACC_BASE = 0,        /* 4: bases a run's first window adds beyond its last
                            base (the rest of baseStatistics comes from the
                            table's last-base marginal) */
    ACC_VALID = 4,       /* baseCounter beyond one per window */
    ACC_WIN = 5,         /* TotalNumSequencesN */
    ACC_D1S = 10,        /* 4: depth-1 trie freq from short (<k) walks (the
                            window part is the table's first-base marginal) */
    ACC_UNK = 14,        /* "Unknown character" bytes */
    ACC_N = 16
};
/* The feed accumulators are FK_ACC_COPIES copies of ACC_N counters: a
 * wave flushes into copy (global wave index % FK_ACC_COPIES), so the
 * same-address atomics of thousands of waves finishing together spread over
 * 16 lines; k_tail / k_table_stats sum and clear the copies. */
#define FK_ACC_COPIES 16

#define FK_NO_EOF 0xFFFFFFFFu
#define FK_NO_EOF64 0xFFFFFFFFFFFFFFFFull

/* What a counted trajectory over a span of bytes (a wave's range) observed,
 * wave-uniform; with the entering and exit states it determines the span's
 * transfer function (fk_tf_span). */
struct Facts {
    uint32_t found_p1;        /* the span contains '\n' or '>' */
    uint32_t p1_gt;           /* ... and the first one is '>' */
    uint32_t any_reset;       /* the trajectory broke the run */
    uint32_t reset_after_p1;  /* ... after the first special byte */
    uint32_t R_at_p1;         /* R just before the first special byte */
    uint32_t nv_total;        /* bases processed (meaningful without a reset) */
};

struct DState {
    uint64_t code;
    uint32_t R;
    uint32_t hdr;
};

/* Exact (64-bit run) state and chunk transfer function for the state scan. */
struct XState {
    uint64_t R;
    uint64_t code;
    uint32_t hdr;
    uint32_t pad;
};
struct TF {
    XState c1;           /* result when entering inside a header (R = 0) */
    XState c0;           /* result when entering outside a header, if f0_const */
    uint64_t nv;         /* else: shift by nv bases ... */
    uint64_t cs;         /* ... whose last bases are cs */
    uint32_t f0_const;
    uint32_t pad;
};

/* Digit-wise map between the internal base encoding (A0 C1 T2 G3) and the
 * reference's (A0 C1 G2 T3): swaps digit values 2 and 3; an involution. */
__host__ __device__ inline uint64_t fk_sigma(uint64_t x) {
    return x ^ ((x >> 1) & 0x5555555555555555ull);
}

__host__ __device__ inline uint64_t fk_join(uint64_t x, uint64_t y, uint64_t n) {
    /* append n bases y (low 2n bits) after x; keep the last 32 bases */
    if (n >= 32) return y;
    uint64_t m = (1ull << (2 * n)) - 1;
    return (x << (2 * n)) | (y & m);
}

__host__ __device__ inline XState fk_apply(const TF &f, const XState &s) {
    if (s.hdr) return f.c1;
    if (f.f0_const) return f.c0;
    XState o;
    o.hdr = 0;
    o.pad = 0;
    o.R = s.R + f.nv;
    o.code = fk_join(s.code, f.cs, f.nv);
    return o;
}

/* h = f then g */
__host__ __device__ inline TF fk_compose(const TF &f, const TF &g) {
    TF h;
    h.c1 = fk_apply(g, f.c1);
    h.pad = 0;
    if (f.f0_const) {
        h.f0_const = 1;
        h.c0 = fk_apply(g, f.c0);
        h.nv = 0;
        h.cs = 0;
    } else if (g.f0_const) {
        h.f0_const = 1;
        h.c0 = g.c0;
        h.nv = 0;
        h.cs = 0;
    } else {
        h.f0_const = 0;
        h.c0 = XState{0, 0, 0, 0};
        h.nv = f.nv + g.nv;
        h.cs = fk_join(f.cs, g.cs, g.nv);
    }
    return h;
}

__host__ __device__ inline TF fk_identity() {
    TF t;
    t.c1 = XState{0, 0, 1, 0};
    t.c0 = XState{0, 0, 0, 0};
    t.nv = 0;
    t.cs = 0;
    t.f0_const = 0;
    t.pad = 0;
    return t;
}

/* Transfer function of a span counted from entering state a (exit x, facts f). */
__host__ __device__ inline TF fk_tf_span(const DState &a, const DState &x, const Facts &f) {
    TF t;
    t.pad = 0;
    XState xs{x.R, x.code, x.hdr, 0};
    if (a.hdr == 0) {
        if (f.any_reset) {
            t.f0_const = 1;
            t.c0 = xs;
            t.nv = 0;
            t.cs = 0;
        } else {
            t.f0_const = 0;
            t.c0 = XState{0, 0, 0, 0};
            t.nv = f.nv_total;
            t.cs = x.code;
        }
        if (!f.found_p1) {
            t.c1 = XState{0, 0, 1, 0};
        } else if (f.p1_gt) {
            t.c1 = xs;
        } else {
            uint32_t rr = f.reset_after_p1 ? x.R : (uint32_t)(x.R - f.R_at_p1);
            t.c1 = XState{rr, x.code, x.hdr, 0};
        }
    } else {
        /* entering inside a header was certain: f0 never applies */
        t.c1 = xs;
        t.f0_const = 1;
        t.c0 = xs;
        t.nv = 0;
        t.cs = 0;
    }
    return t;
}

/* A wave's contiguous run of chunks [c0, c1): its transfer function, the
 * state guessed for its start, and what its counted trajectory observed
 * (exact once the range is resolved). */
struct RangeRec {
    TF tf;
    uint64_t a_code;
    uint32_t a_R, a_hdr;
    uint64_t c0, c1;
    uint64_t eof;        /* first 0xFF outside a header, range-relative, or FK_NO_EOF64 */
    uint32_t unknown;    /* "Unknown character" bytes in the range */
    uint32_t resume;     /* k_count stopped early: resume[range] holds where */
};

/* A range k_count stopped in (first tile the fast path cannot take):
 * k_resume continues it from here.  Indexed by range. */
struct ResumeRec {
    uint64_t tile;       /* range-relative tile index */
    uint64_t code;       /* state entering that tile */
    uint32_t R, hdr;
    uint64_t a_code;     /* the range's guessed entering state */
    uint32_t a_R, a_hdr;
    uint32_t range;
    uint32_t unknown;    /* observations of the tiles before it */
    uint32_t eof;        /* range-relative, or FK_NO_EOF */
    uint32_t pad;
    Facts f;             /* facts of the range so far */
};

/* A shard counted in one pass (k_tail): its effect on the scan state, valid
 * for an entering state equivalent to its first range's guess (fk_equiv) and
 * far enough from the int32 wrap (the host checks both at resolve). */
struct ShardSum {
    uint64_t g_code;                /* the first range's guessed entering state */
    uint32_t g_R, g_hdr;
    uint64_t nvb0;                  /* bytes of the first range */
    uint64_t c_R, c_code;           /* absorb: the exit state; else a shift by nv bases ending in c_code */
    uint32_t c_hdr, absorb;
    uint64_t nv;
};

/* Per-feed results, fetched with one device-to-host copy. */
/* DevRes::fault: what a device-side bound check of the k = 15, 16 path saw.
   LIST: more general-tile windows than the fresh table's list holds (they
   were not written; the segment is counted again without the list).  PARTS /
   META: k_repart's output region or a part's stream past the parts buffer
   (nothing was written past it; the feed fails with FK_E_INTERNAL). */
#define FK_FAULT_LIST 1u
#define FK_FAULT_PARTS 2u
#define FK_FAULT_META 4u

struct DevRes {
    unsigned long long tstat[10];   /* k_table_stats: distinct, sum, last[4], first[4] */
    unsigned long long acc[16];     /* k_table_stats: snapshot of the accumulators */
    XState exit;                    /* stream state after the feed */
    unsigned long long eof_cand;    /* smallest 0xFF offset seen (a candidate) */
    uint32_t redo_n;                /* ranges re-counted */
    uint32_t need;                  /* one-pass k_count: 0 = complete, else ONE_* bits
                                       (the host runs the rest of the path) */
    uint32_t fault;                 /* k_table_stats: FK_FAULT_* bits of the counted segment */
    ShardSum shard;                 /* one-pass shard feeds */
    uint32_t pad2;
    uint32_t seq;                   /* host copy: written last (feed sequence number) */
};

/* k_count's dynamic ranges (k <= 7, LDS bins; large segments).  Static
 * ranges [0, nstatic) are one per wave, chunks [r*cpw, (r+1)*cpw); the rest
 * of the segment, from chunk `base` on, is cut into ndyn smaller ranges
 * (range ids nstatic + d, in stream order) in three tiers of shrinking size
 * (sz[0] > sz[1] > sz[2] chunks).  A wave that is done with its static
 * range claims dynamic ones from its block's pool (d % npools, in order of
 * d: largest first) until it is empty: the fast waves of a CU take the work
 * its slow ones would otherwise end with. */
struct DynGeo {
    uint64_t base;       /* first dynamic chunk */
    uint64_t nchunks;    /* chunks of the segment */
    uint32_t n[3];       /* ranges per tier */
    uint32_t sz[3];      /* chunks per range of each tier */
    uint32_t ndyn;       /* n[0] + n[1] + n[2] (0: static ranges only) */
    uint32_t npools;     /* claim pools (d % npools), one per CU's pair of blocks */
    /* static ranges by wave class: the first npools blocks (one per CU,
       dispatched first) and the rest, waves 0-3 and 4-7 of each block: a
       SIMD's four waves issue oldest first, so they stream at different
       speeds, and each class gets a share of the work to match */
    uint32_t cls[4];     /* chunks per static range: first-round waves 0-3, 4-7; second-round 0-3, 4-7 */
};
/* static range of wave w (dynamic-range mode) */
__host__ __device__ inline void static_span(const DynGeo &g, uint64_t w, uint64_t &c0, uint64_t &c1) {
    const uint64_t b = w / 8, wi = w % 8;
    const bool first = b < g.npools;
    const uint64_t a = first ? g.cls[0] : g.cls[2], bb = first ? g.cls[1] : g.cls[3];
    const uint64_t blk0 = 4ull * g.cls[0] + 4ull * g.cls[1], blk1 = 4ull * g.cls[2] + 4ull * g.cls[3];
    const uint64_t base = first ? b * blk0 : (uint64_t)g.npools * blk0 + (b - g.npools) * blk1;
    c0 = base + (wi < 4 ? wi * a : 4 * a + (wi - 4) * bb);
    c1 = c0 + (wi < 4 ? a : bb);
}
__host__ __device__ inline void dyn_span(const DynGeo &g, uint32_t d, uint64_t &c0, uint64_t &c1) {
    uint64_t off = g.base;
    uint32_t sz;
    if (d < g.n[0]) {
        off += (uint64_t)d * g.sz[0];
        sz = g.sz[0];
    } else if (d < g.n[0] + g.n[1]) {
        off += (uint64_t)g.n[0] * g.sz[0] + (uint64_t)(d - g.n[0]) * g.sz[1];
        sz = g.sz[1];
    } else {
        off += (uint64_t)g.n[0] * g.sz[0] + (uint64_t)g.n[1] * g.sz[1] + (uint64_t)(d - g.n[0] - g.n[1]) * g.sz[2];
        sz = g.sz[2];
    }
    c0 = off;
    c1 = off + sz < g.nchunks ? off + sz : g.nchunks;
}

/* what a one-pass k_count left for the host-launched kernels */
enum { ONE_SCAN = 1u,     /* a guess check failed (or could not be made): k_scan, k_redo, k_table_stats */
       ONE_RESUME = 2u }; /* some range ran out of general tiles: k_resume first */

/* Device state of one-pass feeds (k_count's block_summary, k_tail), in
 * device memory: k_count takes a pointer to it plus one flag word, so its
 * counting loop carries no extra kernel arguments. */
enum { OP_ON = 1u,        /* one pass: k_count summarises its blocks, k_tail finishes */
       OP_FRESH = 2u,     /* a reset is pending: zero table, state and accumulators */
       OP_SHARD = 4u,     /* a shard: the entering state is the first guess until resolved */
       OP_NOMIX = 8u };   /* no mixed tiles (FINDKMER_TUNE no_mixed=1: the general byte walk instead) */
struct OnePassCfg {
    void *bsum;                      /* per k_count block: a BlockSum (fk_engine.hip) */
    XState *rtrue;                   /* entering state per range */
    unsigned long long *acc_total;   /* the engine's accumulators (the feed counts into the feed accumulators) */
    DevRes *host_res;                /* pinned, mapped */
    XState *state;                   /* the engine's stream state (in: entering, out: exit) */
};

/* Would counting a span from state a and from state t give identical
 * contributions?  nvb bounds the bases in the span. */
__host__ __device__ inline bool fk_equiv(const DState &a, const XState &t, int k, uint64_t nvb) {
    if (a.hdr != t.hdr) return false;
    if (t.hdr) return true;
    uint32_t ra = a.R, rt = (uint32_t)t.R;
    bool deep_a = (int32_t)ra >= k && (uint64_t)ra + nvb <= 0x7FFFFFFFull;
    bool deep_t = (int32_t)rt >= k && (uint64_t)rt + nvb <= 0x7FFFFFFFull;
    if (!(ra == rt || (deep_a && deep_t))) return false;
    int32_t s = (int32_t)rt;
    int d = s <= 0 ? 0 : (s > k - 1 ? k - 1 : s);
    if (deep_a && deep_t) d = k - 1;
    uint64_t m = d ? ((d >= 32) ? ~0ull : ((1ull << (2 * d)) - 1)) : 0ull;
    return ((a.code ^ t.code) & m) == 0;
}
