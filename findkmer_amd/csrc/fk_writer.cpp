/*
 * fk_writer.cpp — host side of the drop-in boundary: byte-identical output.
 *
 * Restates the reference's two output routines over the dense count table
 * produced by the GPU engine:
 *   statistics()      findKmer/src/findKmer.cpp:491-565
 *   histo_recursive() findKmer/src/findKmer.cpp:699-942
 *
 * Byte parity depends on evaluating every expression in the same types as
 * the reference (x86 80-bit long double, double log2/pow, long double sqrt),
 * so this translation unit is compiled by g++ WITHOUT -ffast-math and with
 * -ffp-contract=off (see Makefile).  Each row's h, H, p, mean and standard
 * deviation depend only on the k-mer's base composition, so they are
 * computed once per composition (C(k+3,3) of them) and rows are formatted in
 * parallel blocks that are written in index (= trie DFS, :719-724) order.
 */
#include "findkmer.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

/* estimate_RAM_usage()'s node bound (:1256-1260): 1 + sum_{n=1..k} 4^n,
 * accumulated exactly as the reference does (double pow into unsigned long). */
unsigned long max_nodes(int k) {
    unsigned long m = 1;
    double n = 1;
    while (n <= k) m += pow(4.0, n++);
    return m;
}

/* Per-composition constants of histo_recursive (:744-845). */
struct Comp {
    bool used = false;
    std::string hH;        /* ", %LE, %LE" of h and H */
    long double mean = 0;  /* n*p */
    long double sd = 0;    /* sqrt(n*p*q) */
    bool approx = false;   /* normal_approx_check (:189-198) */
};

inline int comp_key(int cA, int cC, int cG) { return (cA * 21 + cC) * 21 + cG; }

void build_comp(Comp &c, const int cnt[4], int k, const double prob[4],
                unsigned long long n) {
    /* :771-774 — long double field assigned from a double quotient */
    long double P[4];
    for (int i = 0; i < 4; i++) P[i] = (double)cnt[i] / (double)k;
    /* :793-801 */
    long double h = 0;
    for (int i = 0; i < 4; i++)
        if (P[i] != 0) h += (double)P[i] * log2(1 / (double)P[i]);
    /* :807 */
    long double H = h * k;
    /* :819-830 */
    double est = 1;
    for (int i = 0; i < 4; i++) est *= pow((double)prob[i], (double)cnt[i]);
    /* :833-839 */
    long double p = est;
    long double q = 1 - p;
    c.sd = sqrtl(n * p * q);
    c.mean = n * p;
    /* :875 normal_approx_check(n, p, 1 - p) */
    long double q2 = 1 - p;
    c.approx = (n * p >= 5) && (n * q2 >= 5);
    char buf[96];
    snprintf(buf, sizeof buf, ", %LE, %LE", h, H);
    c.hH = buf;
    c.used = true;
}

inline void digits_of(uint64_t idx, int k, int cnt[4], char *kmer) {
    static const char B[4] = { 'A', 'C', 'G', 'T' };   /* int2base :590-606 */
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
    for (int i = 0; i < k; i++) {
        int d = (int)((idx >> (2 * (k - 1 - i))) & 3);
        kmer[i] = B[d];
        cnt[d]++;
    }
}

struct RowCtx {
    int k;
    const uint32_t *counts;
    const uint64_t *keys;   /* sparse: row i is k-mer keys[i] with count counts[i] */
    unsigned long long n;   /* TotalNumSequencesN */
    int z_enable;
    long double z_thr;
    std::vector<Comp> *comps;
};

/* The tail of a row after h and H: the frequency and z (or nothing when
 * the z filter drops the row).  z depends only on the composition and the
 * count, so each (composition, count) pair is formatted once per thread:
 * ~70 K pairs instead of 4 M snprintf("%LE") calls at k = 11. */
struct Tail {
    bool keep;
    std::string s;
};
using TailCache = std::unordered_map<uint64_t, Tail>;

const Tail &row_tail(const RowCtx &c, const Comp &cp, int key, uint32_t f, TailCache &cache) {
    const uint64_t ck = ((uint64_t)key << 32) | f;
    auto it = cache.find(ck);
    if (it != cache.end()) return it->second;
    Tail t;
    unsigned long long x = f;
    long double z = (x - cp.mean) / cp.sd;                          /* :839 */
    t.keep = c.z_enable == 0 || (c.z_enable > 0 && fabsl(z) >= c.z_thr);   /* :852-854 */
    if (t.keep) {
        char num[64];
        int m = snprintf(num, sizeof num, ", %d", (int)f);          /* :872 */
        t.s.assign(num, (size_t)m);
        if (cp.approx) {                                            /* :876-886 */
            m = snprintf(num, sizeof num, ", %LE", z);
            t.s.append(num, (size_t)m);
        }
    }
    return cache.emplace(ck, std::move(t)).first->second;
}

/* format rows [lo, hi) into out */
void format_range(const RowCtx &c, uint64_t lo, uint64_t hi, std::string &out, TailCache &cache) {
    char kmer[32];
    int cnt[4];
    for (uint64_t i = lo; i < hi; i++) {
        const uint64_t idx = c.keys ? c.keys[i] : i;
        uint32_t f = c.counts[i];
        if (!f) continue;
        digits_of(idx, c.k, cnt, kmer);
        const int key = comp_key(cnt[0], cnt[1], cnt[2]);
        const Comp &cp = (*c.comps)[key];
        const Tail &t = row_tail(c, cp, key, f, cache);
        if (!t.keep) continue;
        out.push_back('\n');                                        /* :858 */
        out.append(kmer, (size_t)c.k);                              /* :861-863 */
        out.append(cp.hH);                                          /* :866-869 */
        out.append(t.s);                                            /* :872-886 */
    }
}

}  // namespace

extern "C" int fk_write_stats(const char *stats_path, int k, const fk_result *res,
                              void *log_v, double prob_out[4]) {
    FILE *log = (FILE *)log_v;
    FILE *sf = fopen(stats_path, "w");
    if (!sf) {
        fprintf(stderr, "Out file failed to open\nFile MUST be in current directory.\n");
        return FK_E_IO;
    }
    if (log)
        fprintf(log, "Statistics of occurrences and probability of A, C, G and T respectively: \n");
    unsigned long long baseCounter = res->valid_bases;
    for (int i = 0; i < 4; i++) {
        unsigned int count = (unsigned int)res->base_count[i];   /* u32, :94 */
        if (log) fprintf(log, "%u", count);
        long double P = (double)count / baseCounter;             /* :520-521 */
        if (prob_out) prob_out[i] = (double)P;
        if (P == 0.0) {                                          /* :522-525 */
            if (log) fprintf(log, "Division overflow detected in statistics.\n");
            fclose(sf);
            return 1;
        }
        if (log) fprintf(log, ", %Lf\n", P);
        fprintf(sf, "%Lf\n", P);
    }
    unsigned long maxN = max_nodes(k);
    if (log) {
        fprintf(log, "Found %llu valid bases total INSIDE sequences >= k.\n", baseCounter);
        fprintf(log, "%0.0f%% tree density.\n",
                ((double)(res->nodes) / (double)(maxN)) * 100);
    }
    /* nodeCounter == maxNodes  <=>  all 4^k leaves exist (:544) */
    uint64_t all = 1ull << (2 * k);
    if (res->distinct == all) {
        fprintf(sf, "All possible %dmers combinations were found.\n", k);
        if (log) fprintf(log, "All possible kmer combinations were found.\n");
    } else {
        if (log) fprintf(log, "FYI we did not find all possible combinations.\n");
        fprintf(sf, "did not find all possible %dmers combinations.\n", k);
    }
    fclose(sf);
    return FK_OK;
}

static int write_rows(FILE *out, int k, const uint64_t *keys, uint64_t n_rows, const uint32_t *counts,
                      const double prob[4], uint64_t windows, int z_enable, double z_threshold, int threads) {
    std::vector<Comp> comps(21 * 21 * 21);
    unsigned long long n = windows;
    /* memoise every composition that can occur */
    for (int a = 0; a <= k; a++)
        for (int c = 0; a + c <= k; c++)
            for (int g = 0; a + c + g <= k; g++) {
                int cnt[4] = { a, c, g, k - a - c - g };
                build_comp(comps[comp_key(a, c, g)], cnt, k, prob, n);
            }
    RowCtx ctx { k, counts, keys, n, z_enable, (long double)z_threshold, &comps };
    uint64_t total = keys ? n_rows : 1ull << (2 * k);
    if (threads <= 0) {
        unsigned hc = std::thread::hardware_concurrency();
        threads = hc ? (int)std::min(hc, 64u) : 1;
    }
    if (total < (1u << 16)) threads = 1;
    if (threads == 1) {
        std::string s;
        TailCache cache;
        format_range(ctx, 0, total, s, cache);
        if (fwrite(s.data(), 1, s.size(), out) != s.size()) return FK_E_IO;
        return FK_OK;
    }
    /* workers format slices in any order; this thread writes them in index
       order as they complete, so the writes overlap the formatting */
    const uint64_t slice = 1ull << 16;
    const uint64_t nsl = (total + slice - 1) / slice;
    std::vector<std::string> bufs((size_t)nsl);
    std::vector<uint8_t> done((size_t)nsl, 0);
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> next{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) {
        ts.emplace_back([&] {
            TailCache cache;
            for (uint64_t sl; (sl = next.fetch_add(1)) < nsl;) {
                std::string s;
                format_range(ctx, sl * slice, std::min((sl + 1) * slice, total), s, cache);
                std::lock_guard<std::mutex> g(mu);
                bufs[(size_t)sl] = std::move(s);
                done[(size_t)sl] = 1;
                cv.notify_all();
            }
        });
    }
    int rc = FK_OK;
    for (uint64_t sl = 0; sl < nsl; sl++) {
        std::string s;
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return done[(size_t)sl] != 0; });
            s = std::move(bufs[(size_t)sl]);
        }
        if (rc == FK_OK && !s.empty() && fwrite(s.data(), 1, s.size(), out) != s.size()) rc = FK_E_IO;
    }
    for (auto &th : ts) th.join();
    return rc;
}

extern "C" int fk_write_rows(void *out_v, int k, const uint32_t *counts,
                             const double prob[4], uint64_t windows, int z_enable,
                             double z_threshold, int threads) {
    FILE *out = (FILE *)out_v;
    if (!out || !counts || k < 1 || k > FK_K_MAX_DENSE) return FK_E_INVALID;
    return write_rows(out, k, nullptr, 0, counts, prob, windows, z_enable, z_threshold, threads);
}

/* The rows of a sparse table (17 <= k <= 20, fk_engine_sparse): the same
 * bytes fk_write_rows writes for the dense table with those counts. */
extern "C" int fk_write_rows_sparse(void *out_v, int k, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                                    const double prob[4], uint64_t windows, int z_enable, double z_threshold,
                                    int threads) {
    FILE *out = (FILE *)out_v;
    if (!out || (n && (!keys || !counts)) || k < 1 || k > FK_K_MAX_REF) return FK_E_INVALID;
    static const uint32_t zero = 0;
    return write_rows(out, k, keys ? keys : (const uint64_t *)&zero, n, counts ? counts : &zero, prob, windows,
                      z_enable, z_threshold, threads);
}

extern "C" int fk_write_csv_sparse(const char *csv_path, int k, const uint64_t *keys, const uint32_t *counts,
                                   uint64_t n, const double prob[4], uint64_t windows, int z_enable,
                                   double z_threshold, int threads) {
    FILE *f = fopen(csv_path, "w");
    if (!f) return FK_E_IO;
    fputs("Sequence, Shannon Entropy h, Shannon Entropy H, Frequency, Z score", f);
    int rc = fk_write_rows_sparse(f, k, keys, counts, n, prob, windows, z_enable, z_threshold, threads);
    if (fclose(f) != 0 && rc == FK_OK) rc = FK_E_IO;
    return rc;
}

extern "C" int fk_write_csv(const char *csv_path, int k, const uint32_t *counts,
                            const double prob[4], uint64_t windows, int z_enable,
                            double z_threshold, int threads) {
    FILE *f = fopen(csv_path, "w");
    if (!f) return FK_E_IO;
    /* OUT_FILE_COLUMN_HEADERS (:79), written without a newline (:354) */
    fputs("Sequence, Shannon Entropy h, Shannon Entropy H, Frequency, Z score", f);
    int rc = fk_write_rows(f, k, counts, prob, windows, z_enable, z_threshold, threads);
    if (fclose(f) != 0 && rc == FK_OK) rc = FK_E_IO;
    return rc;
}
