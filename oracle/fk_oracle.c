/*
 * fk_oracle.c — TEST INFRASTRUCTURE ONLY (see fk_oracle.h).
 *
 * A sequential, byte-at-a-time restatement of the reference scan
 * (findKmer/src/findKmer.cpp:962-1069).  Every rule below cites the line it
 * restates.  It replaces the 4-ary trie (:107-111, :612-690) by the facts the
 * trie encodes: leaf frequency == window count, depth-1 frequency (for the
 * rollover check at :642), and the number of distinct trie nodes
 * (nodeCounter, :128) for the stats verdict (:544-558).
 *
 * Semantics (verified against the compiled reference):
 *  - '>' outside a header resets the run and starts a comment that runs to
 *    the next '\n' (:991-1008); an input that ends inside it makes the
 *    reference spin forever (:1005) -> unterminated_header.
 *  - '\n' is transparent (:1011).
 *  - A,C,G,T -> 0,1,2,3; 'N' and every other byte reset the run; bytes other
 *    than ACGTN print a warning (:567-589, :1019-1024).
 *  - A 0xFF byte outside a header equals EOF as a signed char and ends the
 *    scan (:988).
 *  - seqSize is a 32-bit int (:977) incremented per valid base (:1029): it
 *    wraps after 2^31-1, so in runs longer than that windows stop counting
 *    until the counter climbs back to k (verified: a 2^31+100 base run of 'A'
 *    at k=2 gives AA = 2147483646).
 *  - seqSize >  k : count window, baseCounter++, base[new]++    (:1035-1042)
 *    seqSize == k : count window, base[each of k]++, += k       (:1044-1057)
 *    0 < seqSize < k : a prefix-only trie walk of the last seqSize
 *                      bases (:1059-1062): touches nodes, counts nothing.
 */
#include "fk_oracle.h"
#include <stdlib.h>
#include <string.h>

/* base2int (:567-589) as a table: A0 C1 G2 T3, 'N' -2, any other byte -1 */
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Woverride-init"
static const signed char B2C[256] = {
    [0 ... 255] = -1, ['A'] = 0, ['C'] = 1, ['G'] = 2, ['T'] = 3, ['N'] = -2,
};
/* bytes that neither break a run nor start a comment: the bases and '\n' */
static const unsigned char BASE_OR_NL[256] = {
    [0 ... 255] = 0, ['A'] = 1, ['C'] = 1, ['G'] = 1, ['T'] = 1, ['\n'] = 1,
};
#pragma GCC diagnostic pop
static inline int base2code(uint8_t c) { return B2C[c]; }

/* Short trie walks that never reached depth k leave prefix nodes behind
 * (:1059-1062).  They matter only for nodeCounter; we record each maximal
 * segment of seqSize in [1, k-1] once (its longest walk covers the others). */
typedef struct { uint64_t code; int len; } fko_short;

typedef struct {
    fko_short *v;
    uint64_t n, cap;
} short_list;

static int short_push(short_list *s, uint64_t code, int len) {
    if (s->n == s->cap) {
        uint64_t nc = s->cap ? 2 * s->cap : 64;
        fko_short *nv = (fko_short *)realloc(s->v, nc * sizeof(*nv));
        if (!nv) return -1;
        s->v = nv; s->cap = nc;
    }
    s->v[s->n].code = code; s->v[s->n].len = len; s->n++;
    return 0;
}

/* Core scan.  emit(code) is called once per counted window. */
typedef void (*emit_fn)(void *ctx, uint64_t code);

/* The scan's state between bytes (the reference's locals of findKmer(),
 * :966-977): inside a comment line, seqSize, the window, and whether a walk
 * of 1..k-1 bases is open.  The stream starts from all zeros. */
typedef struct { int in_hdr; int32_t seq; uint64_t code; int short_open; } scan_state;

/* always inlined: each caller's emit() is inlined into its own copy */
static inline __attribute__((always_inline)) int scan(const uint8_t *buf, uint64_t len, int k, emit_fn emit,
                void *ctx, fko_result *res, short_list *shorts,
                uint8_t *unknown_out, uint64_t unknown_cap, const scan_state *init) {
    const uint64_t mask = (k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    int in_hdr = init ? init->in_hdr : 0;
    int32_t seq = init ? init->seq : 0;   /* seqSize, int at :977; wraps like the ref */
    uint64_t code = init ? init->code : 0; /* last k bases, first base most significant */
    int short_open = init ? init->short_open : 0;   /* a walk of length 1..k-1 is in progress */
    memset(res, 0, sizeof(*res));
    uint64_t i = 0;
    for (; i < len; i++) {
        uint8_t c = buf[i];
        if (in_hdr) {                       /* :999-1006 consume to '\n' */
            if (c == '\n') in_hdr = 0;
            continue;
        }
        if (c == 0xFF) {                    /* (char)c == EOF, :988 */
            res->hit_eof_byte = 1;
            break;
        }
        if (c == '>') {                     /* :991-994 */
            if (short_open && seq > 0 && seq < k) {
                if (short_push(shorts, code & ((1ull << (2 * seq)) - 1), seq)) return -1;
            }
            short_open = 0;
            seq = 0;
            in_hdr = 1;
            continue;
        }
        if (c == '\n') continue;            /* :1011 */
        int b = base2code(c);
        if (b < 0) {                        /* :1019-1024 */
            if (b == -1) {
                if (unknown_out && res->unknown_chars < unknown_cap)
                    unknown_out[res->unknown_chars] = c;
                res->unknown_chars++;
            }
            if (short_open && seq > 0 && seq < k) {
                if (short_push(shorts, code & ((1ull << (2 * seq)) - 1), seq)) return -1;
            }
            short_open = 0;
            seq = 0;
            continue;
        }
        code = ((code << 2) | (uint64_t)b) & mask;    /* :1028 */
        seq = (int32_t)((uint32_t)seq + 1u);          /* :1029, wraps */
        if (seq > k) {                                 /* :1035-1042 */
            emit(ctx, code);
            res->valid_bases++;
            res->base_count[b]++;
            res->windows++;
            res->depth1[(code >> (2 * (k - 1))) & 3]++;
        } else if (seq == k) {                         /* :1044-1057 */
            emit(ctx, code);
            for (int j = 0; j < k; j++) res->base_count[(code >> (2 * j)) & 3]++;
            res->valid_bases += (uint64_t)k;
            res->windows++;
            res->depth1[(code >> (2 * (k - 1))) & 3]++;
            short_open = 0;        /* this segment's prefixes are the window's */
        } else if (seq > 0) {                          /* :1059-1062 */
            res->depth1[(code >> (2 * (seq - 1))) & 3]++;
            short_open = 1;
        }
    }
    res->scanned_bytes = i;
    if (in_hdr) res->unterminated_header = 1;
    if (short_open && seq > 0 && seq < k) {
        if (short_push(shorts, code & ((1ull << (2 * seq)) - 1), seq)) return -1;
    }
    for (int b = 0; b < 4; b++)
        if (res->depth1[b] >= (1ull << 32)) res->rollover = 1;
    return 0;
}

/* ---------------- dense form ---------------- */

typedef struct { uint32_t *counts; } dense_ctx;

static inline void dense_emit(void *ctx, uint64_t code) {
    ((dense_ctx *)ctx)->counts[code]++;
}

/* nodeCounter = head + distinct prefixes (depth 1..k) of all walks. */
static uint64_t dense_nodes(const uint32_t *counts, int k, const short_list *s,
                            uint64_t any_walk) {
    if (!any_walk) return 0;           /* head is created by the first walk */
    uint64_t nodes = 1;
    uint64_t n = 1ull << (2 * k);
    /* presence at depth k, folded upward */
    uint8_t *cur = (uint8_t *)calloc(n, 1);
    if (!cur) return 0;
    for (uint64_t i = 0; i < n; i++) cur[i] = counts[i] != 0;
    for (int d = k; d >= 1; d--) {
        uint64_t nd = 1ull << (2 * d);
        for (uint64_t j = 0; j < s->n; j++)
            if (s->v[j].len >= d)
                cur[s->v[j].code >> (2 * (s->v[j].len - d))] = 1;
        uint64_t c = 0;
        for (uint64_t i = 0; i < nd; i++) c += cur[i];
        nodes += c;
        if (d > 1) {
            for (uint64_t i = 0; i < nd / 4; i++)
                cur[i] = cur[4 * i] | cur[4 * i + 1] | cur[4 * i + 2] | cur[4 * i + 3];
        }
    }
    free(cur);
    return nodes;
}

int fko_count_dense(const uint8_t *buf, uint64_t len, int k, uint32_t *counts,
                    fko_result *res, uint8_t *unknown_out, uint64_t unknown_cap) {
    if (k < 1 || k > 14) return -1;   /* (k = 14: a 1 GiB table; larger k: fko_count_sparse) */
    uint64_t n = 1ull << (2 * k);
    memset(counts, 0, n * sizeof(uint32_t));
    dense_ctx ctx = { counts };
    short_list s = { 0, 0, 0 };
    if (scan(buf, len, k, dense_emit, &ctx, res, &s, unknown_out, unknown_cap, NULL)) {
        free(s.v);
        return -1;
    }
    uint64_t distinct = 0;
    for (uint64_t i = 0; i < n; i++) distinct += counts[i] != 0;
    res->distinct = distinct;
    uint64_t any_walk = res->depth1[0] | res->depth1[1] | res->depth1[2] | res->depth1[3];
    res->nodes = dense_nodes(counts, k, &s, any_walk);
    free(s.v);
    return 0;
}

/* ---------------- dense form, split over threads ----------------
 *
 * The same scan cut into contiguous pieces, each scanned from its exact
 * entering state (scan_state), the results summed in stream order.  Exact
 * for any input: the entering state at a cut q is derived from the bytes
 * before q by the reference's own rules --
 *   j = the last byte before q that is not A/C/G/T/'\n' (:1011, :1019);
 *   j inside a comment line (a '>' earlier on its line, or j itself is '>',
 *   :991-1008): the comment ends at the next '\n' (state hdr=0, seqSize=0
 *   after it), or q is still inside it (hdr=1);
 *   else j broke the run (:1019-1024): seqSize=0 after j;
 *   no such j: the stream's initial state at byte 0;
 * then seqSize = the bases from there to q (mod 2^32, :977/:1029), the
 * window = the last of them, and a short walk is open iff 0 < seqSize < k
 * (:1059-1062).  A piece whose predecessor hit a 0xFF byte (:988) is
 * dropped.  Only the cost is parallel; the rules are scan()'s. */
#include <pthread.h>
#ifdef __SSE2__
#include <emmintrin.h>
#endif

/* j <= q with buf[j..q) all bases or '\n', j as small as possible */
static uint64_t back_over_bases(const uint8_t *buf, uint64_t q) {
    uint64_t j = q;
#ifdef __SSE2__
    const __m128i A = _mm_set1_epi8('A'), C = _mm_set1_epi8('C'), G = _mm_set1_epi8('G'),
                  T = _mm_set1_epi8('T'), NL = _mm_set1_epi8('\n');
    while (j >= 16) {
        __m128i v = _mm_loadu_si128((const __m128i *)(buf + j - 16));
        __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, A), _mm_cmpeq_epi8(v, C)),
                                 _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, G), _mm_cmpeq_epi8(v, T)),
                                              _mm_cmpeq_epi8(v, NL)));
        if (_mm_movemask_epi8(m) != 0xFFFF) break;
        j -= 16;
    }
#endif
    while (j > 0 && BASE_OR_NL[buf[j - 1]]) j--;
    return j;
}

/* the '\n' bytes in [p, q) */
static uint64_t count_nl(const uint8_t *buf, uint64_t p, uint64_t q) {
    uint64_t n = 0, x = p;
#ifdef __SSE2__
    const __m128i NL = _mm_set1_epi8('\n');
    for (; x + 16 <= q; x += 16)
        n += (uint64_t)__builtin_popcount((unsigned)_mm_movemask_epi8(
                 _mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(buf + x)), NL)));
#endif
    for (; x < q; x++) n += buf[x] == '\n';
    return n;
}


static void entry_state(const uint8_t *buf, uint64_t q, int k, scan_state *st) {
    memset(st, 0, sizeof(*st));
    uint64_t p = 0;                     /* state (hdr 0, seqSize 0) at p */
    uint64_t j = back_over_bases(buf, q);
    if (j > 0) {
        uint64_t b = j - 1;             /* the last breaker before q */
        int hdr = buf[b] == '>';
        for (uint64_t x = b; !hdr && x > 0 && buf[x - 1] != '\n'; x--)
            if (buf[x - 1] == '>') hdr = 1;
        if (hdr) {
            uint64_t e = b + 1;
            while (e < q && buf[e] != '\n') e++;
            if (e >= q) { st->in_hdr = 1; return; }
            p = e + 1;
        } else {
            p = b + 1;
        }
    }
    /* [p, q) holds only bases and '\n': seqSize = its bases, the window =
     * the last k of them */
    uint64_t R = q - p - count_nl(buf, p, q), code = 0;
    int got = 0;
    for (uint64_t x = q; x > p && got < k; x--) {
        if (buf[x - 1] == '\n') continue;
        code |= (uint64_t)base2code(buf[x - 1]) << (2 * got++);
    }
    st->seq = (int32_t)(uint32_t)R;
    st->code = code;
    st->short_open = st->seq > 0 && st->seq < k;
}

typedef struct {
    const uint8_t *buf;
    uint64_t lo, hi;
    int k;
    uint32_t *counts;
    fko_result res;
    short_list shorts;
    uint8_t *unknown;
    uint64_t unknown_cap;
    int rc;
} piece_t;

static void *piece_run(void *arg) {
    piece_t *p = (piece_t *)arg;
    scan_state st;
    entry_state(p->buf, p->lo, p->k, &st);
    dense_ctx ctx = { p->counts };
    /* counters on this thread's stack: the pieces' records share cache lines */
    fko_result res;
    short_list shorts = { 0, 0, 0 };
    int rc = scan(p->buf + p->lo, p->hi - p->lo, p->k, dense_emit, &ctx, &res, &shorts,
                  p->unknown, p->unknown_cap, p->lo ? &st : NULL);
    p->res = res;
    p->shorts = shorts;
    p->rc = rc;
    return NULL;
}

typedef struct { uint32_t *dst; uint32_t **src; int nsrc; uint64_t lo, hi; } sum_t;

static void *sum_run(void *arg) {
    sum_t *s = (sum_t *)arg;
    for (int t = 0; t < s->nsrc; t++)
        for (uint64_t i = s->lo; i < s->hi; i++) s->dst[i] += s->src[t][i];   /* u32, wraps like :110 */
    return NULL;
}

int fko_count_dense_par(const uint8_t *buf, uint64_t len, int k, uint32_t *counts,
                        fko_result *res, uint8_t *unknown_out, uint64_t unknown_cap, int threads) {
    if (k < 1 || k > 13) return -1;   /* (one table per thread) */
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > len / 4096 + 1) threads = (int)(len / 4096 + 1);
    if (threads == 1) return fko_count_dense(buf, len, k, counts, res, unknown_out, unknown_cap);
    const uint64_t n = 1ull << (2 * k);
    piece_t *pc = (piece_t *)calloc((size_t)threads, sizeof(piece_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    int rc = -1;
    if (!pc || !th) goto out;
    for (int t = 0; t < threads; t++) {
        pc[t].buf = buf;
        pc[t].lo = len * (uint64_t)t / (uint64_t)threads;
        pc[t].hi = len * (uint64_t)(t + 1) / (uint64_t)threads;
        pc[t].k = k;
        pc[t].counts = t ? (uint32_t *)calloc(n, sizeof(uint32_t)) : counts;
        if (!pc[t].counts) goto out;
        if (unknown_out && unknown_cap) {
            pc[t].unknown = (uint8_t *)malloc(unknown_cap);
            if (!pc[t].unknown) goto out;
            pc[t].unknown_cap = unknown_cap;
        }
    }
    memset(counts, 0, n * sizeof(uint32_t));
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, piece_run, &pc[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < threads; t++) if (pc[t].rc) goto out;
    /* pieces after the first that met a 0xFF byte outside a comment never
     * happen in the reference (:988): drop them */
    int used = threads;
    for (int t = 0; t < threads; t++)
        if (pc[t].res.hit_eof_byte) { used = t + 1; break; }
    {
        uint32_t **src = (uint32_t **)calloc((size_t)threads, sizeof(uint32_t *));
        if (!src) goto out;
        for (int t = 1; t < used; t++) src[t - 1] = pc[t].counts;
        sum_t *sm = (sum_t *)calloc((size_t)threads, sizeof(sum_t));
        if (!sm) { free(src); goto out; }
        for (int t = 0; t < threads; t++) {
            sm[t].dst = counts; sm[t].src = src; sm[t].nsrc = used - 1;
            sm[t].lo = n * (uint64_t)t / (uint64_t)threads;
            sm[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
            pthread_create(&th[t], NULL, sum_run, &sm[t]);
        }
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
        free(sm);
        free(src);
    }
    memset(res, 0, sizeof(*res));
    short_list all = { 0, 0, 0 };
    uint64_t nunk = 0;
    for (int t = 0; t < used; t++) {
        const fko_result *r = &pc[t].res;
        for (int b = 0; b < 4; b++) {
            res->base_count[b] += r->base_count[b];
            res->depth1[b] += r->depth1[b];
        }
        res->valid_bases += r->valid_bases;
        res->windows += r->windows;
        for (uint64_t u = 0; u < r->unknown_chars && unknown_out && nunk + u < unknown_cap && u < unknown_cap; u++)
            unknown_out[nunk + u] = pc[t].unknown[u];
        nunk += r->unknown_chars;
        for (uint64_t s = 0; s < pc[t].shorts.n; s++)
            if (short_push(&all, pc[t].shorts.v[s].code, pc[t].shorts.v[s].len)) { free(all.v); goto out; }
        if (t == used - 1) {
            res->scanned_bytes = pc[t].lo + r->scanned_bytes;
            res->hit_eof_byte = r->hit_eof_byte;
            res->unterminated_header = r->unterminated_header;
        }
    }
    res->unknown_chars = nunk;
    for (int b = 0; b < 4; b++)
        if (res->depth1[b] >= (1ull << 32)) res->rollover = 1;
    uint64_t distinct = 0;
    for (uint64_t i = 0; i < n; i++) distinct += counts[i] != 0;
    res->distinct = distinct;
    uint64_t any_walk = res->depth1[0] | res->depth1[1] | res->depth1[2] | res->depth1[3];
    res->nodes = dense_nodes(counts, k, &all, any_walk);
    free(all.v);
    rc = 0;
out:
    if (pc) {
        for (int t = 0; t < threads; t++) {
            if (t && pc[t].counts) free(pc[t].counts);
            free(pc[t].unknown);
            free(pc[t].shorts.v);
        }
    }
    free(pc);
    free(th);
    return rc;
}

/* ---------------- key ranges of a large-k table, split over threads ----
 *
 * The windows whose k-mer index falls in one of nr ascending, disjoint key
 * ranges [key_lo[r], key_hi[r]) -- slices of the reference's trie leaves in
 * DFS order (:719-724) -- counted in dense slice arrays, the stream cut into
 * pieces as in fko_count_dense_par (each from its exact entering state), so
 * that a 10 GB input's k >= 17 table can be checked slice by slice with
 * bounded host memory, several slices per scan. */
#define FKO_MAX_RANGES 8
typedef struct { uint32_t *counts; int nr; uint64_t lo[FKO_MAX_RANGES], span[FKO_MAX_RANGES], base[FKO_MAX_RANGES]; } range_ctx;

static inline void range_emit(void *ctx, uint64_t code) {
    range_ctx *c = (range_ctx *)ctx;
    for (int r = 0; r < c->nr; r++) {
        const uint64_t d = code - c->lo[r];   /* wraps above 2^64 for code < lo */
        if (d < c->span[r]) { c->counts[c->base[r] + d]++; return; }
    }
}

typedef struct {
    const uint8_t *buf;
    uint64_t lo, hi;
    int k;
    range_ctx ctx;
    fko_result res;
    int rc;
} rpiece_t;

static void *rpiece_run(void *arg) {
    rpiece_t *p = (rpiece_t *)arg;
    scan_state st;
    entry_state(p->buf, p->lo, p->k, &st);
    fko_result res;
    short_list shorts = { 0, 0, 0 };
    p->rc = scan(p->buf + p->lo, p->hi - p->lo, p->k, range_emit, &p->ctx, &res, &shorts, NULL, 0,
                 p->lo ? &st : NULL);
    free(shorts.v);
    p->res = res;
    return NULL;
}

int fko_count_sparse_range(const uint8_t *buf, uint64_t len, int k, const uint64_t *key_lo, const uint64_t *key_hi,
                           int nr, uint64_t *codes, uint32_t *counts, uint64_t cap, uint64_t *n_unique,
                           fko_result *res, int threads) {
    if (k < 1 || k > 20 || nr < 1 || nr > FKO_MAX_RANGES) return -1;
    range_ctx proto;
    memset(&proto, 0, sizeof proto);
    proto.nr = nr;
    uint64_t total = 0;
    for (int r = 0; r < nr; r++) {
        if (key_hi[r] <= key_lo[r] || (r && key_lo[r] < key_hi[r - 1])) return -1;
        proto.lo[r] = key_lo[r];
        proto.span[r] = key_hi[r] - key_lo[r];
        proto.base[r] = total;
        total += proto.span[r];
    }
    if (total > (1ull << 30)) return -1;
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > len / 4096 + 1) threads = (int)(len / 4096 + 1);
    rpiece_t *pc = (rpiece_t *)calloc((size_t)threads, sizeof(rpiece_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    int rc = -1;
    if (!pc || !th) goto out;
    for (int t = 0; t < threads; t++) {
        pc[t].buf = buf;
        pc[t].lo = len * (uint64_t)t / (uint64_t)threads;
        pc[t].hi = len * (uint64_t)(t + 1) / (uint64_t)threads;
        pc[t].k = k;
        pc[t].ctx = proto;
        pc[t].ctx.counts = (uint32_t *)calloc(total, sizeof(uint32_t));
        if (!pc[t].ctx.counts) goto out;
    }
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, rpiece_run, &pc[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < threads; t++) if (pc[t].rc) goto out;
    int used = threads;
    for (int t = 0; t < threads; t++)
        if (pc[t].res.hit_eof_byte) { used = t + 1; break; }
    for (int t = 1; t < used; t++)
        for (uint64_t i = 0; i < total; i++) pc[0].ctx.counts[i] += pc[t].ctx.counts[i];   /* u32, wraps like :110 */
    memset(res, 0, sizeof(*res));
    for (int t = 0; t < used; t++) {
        const fko_result *r = &pc[t].res;
        for (int b = 0; b < 4; b++) {
            res->base_count[b] += r->base_count[b];
            res->depth1[b] += r->depth1[b];
        }
        res->valid_bases += r->valid_bases;
        res->windows += r->windows;
        res->unknown_chars += r->unknown_chars;
        if (t == used - 1) {
            res->scanned_bytes = pc[t].lo + r->scanned_bytes;
            res->hit_eof_byte = r->hit_eof_byte;
            res->unterminated_header = r->unterminated_header;
        }
    }
    {
        uint64_t u = 0;
        for (int r = 0; r < nr; r++)
            for (uint64_t i = 0; i < proto.span[r]; i++) {
                const uint32_t c = pc[0].ctx.counts[proto.base[r] + i];
                if (c) {
                    if (u < cap) { codes[u] = proto.lo[r] + i; counts[u] = c; }
                    u++;
                }
            }
        *n_unique = u;
        res->distinct = u;   /* within the ranges */
        rc = u > cap ? -1 : 0;
    }
out:
    if (pc)
        for (int t = 0; t < threads; t++) free(pc[t].ctx.counts);
    free(pc);
    free(th);
    return rc;
}

/* ---------------- sparse form ---------------- */

typedef struct { uint64_t *v; uint64_t n, cap; int fail; } vec_ctx;

static void vec_emit(void *ctx, uint64_t code) {
    vec_ctx *c = (vec_ctx *)ctx;
    if (c->fail) return;
    if (c->n == c->cap) {
        uint64_t nc = c->cap ? 2 * c->cap : 1024;
        uint64_t *nv = (uint64_t *)realloc(c->v, nc * sizeof(uint64_t));
        if (!nv) { c->fail = 1; return; }
        c->v = nv; c->cap = nc;
    }
    c->v[c->n++] = code;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}

int fko_count_sparse(const uint8_t *buf, uint64_t len, int k, uint64_t *codes,
                     uint32_t *counts, uint64_t cap, uint64_t *n_unique,
                     fko_result *res) {
    if (k < 1 || k > 20) return -1;
    vec_ctx ctx = { 0, 0, 0, 0 };
    short_list s = { 0, 0, 0 };
    int rc = scan(buf, len, k, vec_emit, &ctx, res, &s, NULL, 0, NULL);
    if (rc || ctx.fail) { free(ctx.v); free(s.v); return -1; }
    qsort(ctx.v, ctx.n, sizeof(uint64_t), cmp_u64);
    uint64_t u = 0;
    for (uint64_t i = 0; i < ctx.n;) {
        uint64_t j = i;
        while (j < ctx.n && ctx.v[j] == ctx.v[i]) j++;
        if (u < cap) { codes[u] = ctx.v[i]; counts[u] = (uint32_t)(j - i); }
        u++;
        i = j;
    }
    *n_unique = u;
    res->distinct = u;
    /* nodes: distinct prefixes per depth over windows and short walks */
    uint64_t any_walk = res->depth1[0] | res->depth1[1] | res->depth1[2] | res->depth1[3];
    if (any_walk) {
        uint64_t m = u + s.n;
        uint64_t *pre = (uint64_t *)malloc((m ? m : 1) * sizeof(uint64_t));
        if (!pre) { free(ctx.v); free(s.v); return -1; }
        uint64_t nodes = 1;
        for (int d = 1; d <= k; d++) {
            uint64_t q = 0;
            /* distinct depth-d prefixes of the (sorted) windows ... */
            uint64_t prev = ~0ull; int have = 0;
            for (uint64_t i = 0; i < ctx.n; i++) {
                uint64_t p = ctx.v[i] >> (2 * (k - d));
                if (!have || p != prev) { pre[q++] = p; prev = p; have = 1; }
            }
            for (uint64_t j = 0; j < s.n; j++)
                if (s.v[j].len >= d) pre[q++] = s.v[j].code >> (2 * (s.v[j].len - d));
            qsort(pre, q, sizeof(uint64_t), cmp_u64);
            uint64_t c = 0;
            for (uint64_t i = 0; i < q; i++)
                if (i == 0 || pre[i] != pre[i - 1]) c++;
            nodes += c;
        }
        free(pre);
        res->nodes = nodes;
    }
    free(ctx.v);
    free(s.v);
    return (u > cap) ? -1 : 0;
}

/* ---------------- synthetic input ---------------- */

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint64_t fko_synth(uint8_t *out, uint64_t cap, uint64_t n_bases, uint64_t seed,
                   int fasta_line) {
    static const char acgt[4] = { 'A', 'C', 'G', 'T' };
    uint64_t o = 0;
    if (fasta_line > 0) {
        const char *h = ">synthetic\n";
        for (const char *p = h; *p && o < cap; p++) out[o++] = (uint8_t)*p;
    }
    uint64_t word = 0;
    for (uint64_t i = 0; i < n_bases && o < cap; i++) {
        if ((i & 31) == 0) word = splitmix64(seed + (i >> 5));
        out[o++] = (uint8_t)acgt[(word >> (2 * (i & 31))) & 3];
        if (fasta_line > 0 && ((i + 1) % (uint64_t)fasta_line) == 0 && o < cap)
            out[o++] = '\n';
    }
    return o;
}
