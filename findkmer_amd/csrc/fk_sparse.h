/*
 * fk_sparse.h — the sparse count table for 17 <= k <= 20 (fk_sparse.hip).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

/* Device buffers of one engine's sparse table (grown on demand). */
struct FksState {
    uint64_t *sorted = nullptr;   /* the slots, sorted */
    uint64_t *keys = nullptr;     /* run values: window indices [0, nw), short walks [nw, nw+ns) */
    uint64_t *c64 = nullptr;      /* run lengths */
    uint32_t *lo = nullptr;       /* window counts as the reference's u32 frequency */
    uint32_t *hi = nullptr;
    void *tmp = nullptr;          /* rocPRIM temporary storage */
    unsigned long long *small = nullptr;
    uint64_t *cand = nullptr, *cand2 = nullptr;
    size_t sorted_cap = 0, keys_cap = 0, c64_cap = 0, lo_cap = 0, hi_cap = 0, tmp_cap = 0, small_cap = 0,
           cand_cap = 0, cand2_cap = 0;
    uint64_t nw = 0;              /* distinct k-mers */
    uint64_t ns = 0;              /* distinct short walks */
};

/* Sort and run-length encode the n slots; table statistics as
 * k_table_stats's (distinct, u32 sum, last[4], first[4]); *rollover != 0 if
 * some k-mer occurs 2^32 times or more; nodeCounter if want_nodes.
 * Synchronises the stream.  0 or -1 (HIP error / out of memory). */
int fks_finalize(FksState *st, uint64_t *slots, uint64_t n, int k, int want_nodes, hipStream_t s,
                 unsigned long long tstat[10], unsigned long long *rollover, unsigned long long *nodes);
void fks_free(FksState *st);
