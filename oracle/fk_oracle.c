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

static inline int base2code(uint8_t c) {          /* :567-589 */
    switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'N': return -2;
    default:  return -1;
    }
}

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

static int scan(const uint8_t *buf, uint64_t len, int k, emit_fn emit,
                void *ctx, fko_result *res, short_list *shorts,
                uint8_t *unknown_out, uint64_t unknown_cap) {
    const uint64_t mask = (k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    int in_hdr = 0;
    int32_t seq = 0;          /* seqSize, int at :977; wraps like the ref */
    uint64_t code = 0;        /* last k bases, first base most significant */
    int short_open = 0;       /* a walk of length 1..k-1 is in progress */
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

static void dense_emit(void *ctx, uint64_t code) {
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
    if (k < 1 || k > 13) return -1;
    uint64_t n = 1ull << (2 * k);
    memset(counts, 0, n * sizeof(uint32_t));
    dense_ctx ctx = { counts };
    short_list s = { 0, 0, 0 };
    if (scan(buf, len, k, dense_emit, &ctx, res, &s, unknown_out, unknown_cap)) {
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
    int rc = scan(buf, len, k, vec_emit, &ctx, res, &s, NULL, 0);
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
