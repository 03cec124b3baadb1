/*
 * fk_sparse.h — the sparse count table for 17 <= k <= 20 (fk_sparse.hip).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

/* Device buffers of one engine's sparse table (grown on demand). */
struct FksState {
    uint64_t *sorted = nullptr;   /* a pass's keys, sorted */
    uint64_t *c64 = nullptr;      /* run lengths */
    void *tmp = nullptr;          /* rocPRIM temporary storage */
    unsigned long long *small = nullptr;
    uint64_t *cand = nullptr, *cand2 = nullptr;
    size_t sorted_cap = 0, c64_cap = 0, tmp_cap = 0, small_cap = 0,
           cand_cap = 0, cand2_cap = 0;
};

/* Device accumulators of a sparse finish (unsigned long long[FKS_ACC_N]):
 * the table statistics as k_table_stats's (distinct, u32 sum, last[4],
 * first[4]), the rollover flag (a count >= 2^32), and the prefix histogram
 * of adjacent sorted keys (first differing base at depth d, [d]). */
enum { FKS_ACC_ROLL = 10, FKS_ACC_WPREFIX = 11, FKS_ACC_N = 40 };

/* One key-range pass: sort and run-length encode the n window keys (bits
 * [0, 2k)) into out_keys (ascending distinct indices) and out_cnts (their u32
 * counts), *nw of them -- the caller's table storage, room for n; statistics,
 * rollover and prefix histogram accumulate into dacc.  `npads` of the keys
 * are the pad 4^k - 1 (the largest key: sorted last, with the real key
 * 4^k - 1 if any), taken off the last run's count (the run is dropped when
 * nothing else is in it).  Synchronises the stream.  0 or -1 (HIP error /
 * out of memory). */
int fks_sort_runs(FksState *st, uint64_t *keys, uint64_t n, int k, hipStream_t s, unsigned long long *dacc,
                  uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw, uint64_t npads = 0);
/* fks_sort_runs for a dense count table of keys [lo, lo + n) (room for its
 * nonzero entries). */
int fks_dense_runs(FksState *st, unsigned long long *dense, uint64_t n, uint64_t lo, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw);
/* Runs from several tables (any order, repeated keys): sorted, counts of a
 * key summed (u64, then the u32 frequency), into out_keys / out_cnts (room
 * for n), with statistics as fks_sort_runs.  The multi-GPU merge of the
 * ranks' sparse tables. */
int fks_merge_runs(FksState *st, const uint64_t *keys, const uint32_t *cnts, uint64_t n, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw);
/* Sort v[0, n) (all 64 bits) and keep the distinct values in place. */
int fks_unique(FksState *st, uint64_t *v, uint64_t n, hipStream_t s, uint64_t *n_out);
/* Mark which short-walk prefixes the sorted keys[0, nw) contain:
 * found[i * 20 + d - 1] for depth d of short walk i. */
int fks_short_mark(const uint64_t *keys, uint64_t nw, const uint64_t *shorts, uint64_t ns, int k, uint8_t *found,
                   hipStream_t s);
/* Distinct short-walk prefixes no window has (nodeCounter's short part). */
int fks_short_count(FksState *st, const uint64_t *shorts, uint64_t ns, const uint8_t *found, hipStream_t s,
                    unsigned long long *total);
void fks_free(FksState *st);
