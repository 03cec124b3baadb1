/*
 * fk_sparse.hip — the count table for 17 <= k <= 20 (the reference accepts
 * k <= 20, findKmer/src/findKmer.cpp:438; a dense 4^k table stops fitting at
 * k = 17..18 on one GPU).
 *
 * The engine's H_SPARSE pass writes one u64 slot per input byte (fk_engine.hip,
 * tile_general): the reference-order index of the window ending at that byte
 * (< 2^40), a short walk at a run break (SP_SHORT | depth << 40 | its code), or
 * SP_EMPTY.  At finish the slots are radix-sorted and run-length encoded
 * (rocPRIM): the windows' distinct indices in ascending order -- the trie's
 * DFS order, which is the CSV row order (histo_recursive :699-942) -- with
 * their counts, then the distinct short walks, then the empty slots.
 *
 * From those runs, on the GPU:
 *   - the table statistics k_table_stats computes for the dense table
 *     (distinct, u32 sum, last- and first-base marginals), so fk_result is
 *     filled the same way for every k;
 *   - nodeCounter (:128, :620): 1 + the distinct prefixes, at every depth,
 *     of the windows and of the short walks.  Window prefixes come from
 *     adjacent differences of the sorted indices; a short walk's prefixes
 *     count where no window has them (binary search), deduplicated by a
 *     second sort.
 */
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "fk_sparse.h"

#define SP_SHORT (1ull << 62)
#define SP_EMPTY (~0ull)

namespace {

__device__ __forceinline__ unsigned long long wsum(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

/* distinct, u32 sum, last[4], first[4] of the window runs; rollover flag */
__global__ void __launch_bounds__(256)
k_sp_stats(const uint64_t *keys, const uint32_t *cnt_lo, const uint32_t *cnt_hi, uint64_t nw, int k,
           unsigned long long *out10, unsigned long long *big) {
    unsigned long long v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long wrap = 0;
    const int fs = 2 * (k - 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = keys[i];
        const uint32_t c = cnt_lo[i];   /* the reference's u32 frequency (:110) */
        wrap |= cnt_hi[i];              /* a count >= 2^32: the rollover exit (:642) */
        v[0] += 1;
        v[1] += c;
        const uint32_t ld = (uint32_t)(key & 3), fd = (uint32_t)((key >> fs) & 3);
        v[2 + ld] += c;
        v[6 + fd] += c;
    }
    __shared__ unsigned long long sh[4][11];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 10; q++) v[q] = wsum(v[q]);
    wrap = wsum(wrap);
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 10; q++) sh[w][q] = v[q];
        sh[w][10] = wrap;
    }
    __syncthreads();
    if (threadIdx.x < 11) {
        unsigned long long s = 0;
        for (uint32_t j = 0; j < blockDim.x / 64; j++) s += sh[j][threadIdx.x];
        if (s) atomicAdd(threadIdx.x < 10 ? &out10[threadIdx.x] : big, s);
    }
}

/* the u64 run counts as (lo, hi) u32 halves */
__global__ void k_sp_split(const uint64_t *c64, uint64_t n, uint32_t *lo, uint32_t *hi) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        lo[i] = (uint32_t)c64[i];
        hi[i] = (uint32_t)(c64[i] >> 32);
    }
}

/* windows: hist[d] = adjacent pairs of sorted distinct indices whose first
   differing base is at depth d (1-based); distinct depth-d prefixes are
   1 + sum_{j <= d} hist[j] */
__global__ void __launch_bounds__(256)
k_sp_wprefix(const uint64_t *keys, uint64_t nw, int k, unsigned long long *hist) {
    __shared__ unsigned int h[24];
    if (threadIdx.x < 24) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = 1 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t diff = keys[i] ^ keys[i - 1];
        /* leading zero digits of the 2k-bit difference */
        const int lz = __clzll((long long)diff) - (64 - 2 * k);
        atomicAdd(&h[lz / 2 + 1], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 24 && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

/* a short walk's prefixes that no window has: candidates (depth << 40 | prefix) */
__global__ void k_sp_short_cand(const uint64_t *keys, uint64_t nw, const uint64_t *shorts, uint64_t ns, int k,
                                uint64_t *cand) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = shorts[i];
        const int seq = (int)((e >> 40) & 0x3F);
        const uint64_t code = e & ((1ull << 40) - 1);
        for (int d = 1; d <= 20; d++) {
            uint64_t out = SP_EMPTY;
            if (d <= seq) {
                const uint64_t p = code >> (2 * (seq - d));
                const int sh = 2 * (k - d);
                /* lower bound of p << sh among the window indices */
                uint64_t lo = 0, hi = nw;
                const uint64_t want = p << sh;
                while (lo < hi) {
                    const uint64_t mid = (lo + hi) / 2;
                    if (keys[mid] < want) lo = mid + 1;
                    else hi = mid;
                }
                const bool have = lo < nw && (keys[lo] >> sh) == p;
                if (!have) out = ((uint64_t)d << 40) | p;
            }
            cand[i * 20 + (uint64_t)(d - 1)] = out;
        }
    }
}

/* distinct candidates after the sort: adjacent differences per depth */
__global__ void __launch_bounds__(256)
k_sp_count_cand(const uint64_t *c, uint64_t n, unsigned long long *total) {
    unsigned long long v = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (c[i] != SP_EMPTY && (i == 0 || c[i] != c[i - 1])) v++;
    v = wsum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(total, v);
}

/* first index with value >= x among the *nruns sorted run keys */
__global__ void k_sp_bound(const uint64_t *keys, const unsigned long long *nruns, uint64_t x, unsigned long long *out) {
    uint64_t lo = 0, hi = *nruns;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (keys[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    *out = lo;
}

unsigned grid_for(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

#define CK(x)                                                                   \
    do {                                                                        \
        if ((x) != hipSuccess) return -1;                                       \
    } while (0)

int ensure(void **p, size_t *cap, size_t want) {
    if (*cap >= want && *p) return 0;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, want ? want : 16) != hipSuccess) return -1;
    *cap = want;
    return 0;
}

}  // namespace

void fks_free(FksState *st) {
    hipFree(st->sorted); hipFree(st->keys); hipFree(st->c64); hipFree(st->lo); hipFree(st->hi);
    hipFree(st->tmp); hipFree(st->small); hipFree(st->cand); hipFree(st->cand2);
    *st = FksState{};
}

int fks_finalize(FksState *st, uint64_t *slots, uint64_t n, int k, int want_nodes, hipStream_t s,
                 unsigned long long tstat[10], unsigned long long *rollover, unsigned long long *nodes) {
    st->nw = st->ns = 0;
    for (int q = 0; q < 10; q++) tstat[q] = 0;
    *rollover = 0;
    *nodes = 0;
    if (n == 0) return 0;
    /* 1. sort (all 64 bits: windows, then short walks, then empty slots) */
    if (ensure((void **)&st->sorted, &st->sorted_cap, n * 8) || ensure((void **)&st->keys, &st->keys_cap, n * 8) ||
        ensure((void **)&st->c64, &st->c64_cap, n * 8) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    size_t tb = 0, tb2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, slots, st->sorted, n, 0, 64, s));
    CK(rocprim::run_length_encode(nullptr, tb2, st->sorted, n, st->keys, st->c64, st->small, s));
    if (ensure(&st->tmp, &st->tmp_cap, tb > tb2 ? tb : tb2)) return -1;
    tb = st->tmp_cap;
    CK(rocprim::radix_sort_keys(st->tmp, tb, slots, st->sorted, n, 0, 64, s));
    tb2 = st->tmp_cap;
    /* 2. runs: keys[] distinct values, c64[] their counts, small[0] = runs */
    CK(rocprim::run_length_encode(st->tmp, tb2, st->sorted, n, st->keys, st->c64, st->small, s));
    unsigned long long *sm = st->small;
    /* sm[1] = first short walk, sm[2] = first empty slot */
    hipLaunchKernelGGL(k_sp_bound, dim3(1), dim3(1), 0, s, st->keys, sm, SP_SHORT, sm + 1);
    hipLaunchKernelGGL(k_sp_bound, dim3(1), dim3(1), 0, s, st->keys, sm, SP_EMPTY, sm + 2);
    unsigned long long h3[3];
    CK(hipMemcpyAsync(h3, sm, sizeof h3, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    const uint64_t runs = h3[0];
    const uint64_t nw = h3[1] < runs ? h3[1] : runs;
    const uint64_t se = h3[2] < runs ? h3[2] : runs;
    st->nw = nw;
    st->ns = se - nw;
    /* 3. u32 counts (and the high halves for the rollover check) */
    if (ensure((void **)&st->lo, &st->lo_cap, (nw + 1) * 4) || ensure((void **)&st->hi, &st->hi_cap, (nw + 1) * 4))
        return -1;
    CK(hipMemsetAsync(sm + 3, 0, 40 * sizeof(unsigned long long), s));
    if (nw) {
        hipLaunchKernelGGL(k_sp_split, dim3(grid_for(nw)), dim3(256), 0, s, st->c64, nw, st->lo, st->hi);
        hipLaunchKernelGGL(k_sp_stats, dim3(grid_for(nw)), dim3(256), 0, s, st->keys, st->lo, st->hi, nw, k,
                           sm + 3, sm + 13);
    }
    /* 4. nodeCounter */
    if (want_nodes) {
        if (nw > 1) hipLaunchKernelGGL(k_sp_wprefix, dim3(grid_for(nw)), dim3(256), 0, s, st->keys, nw, k, sm + 14);
        if (st->ns) {
            const uint64_t nc = st->ns * 20;
            if (ensure((void **)&st->cand, &st->cand_cap, nc * 8) || ensure((void **)&st->cand2, &st->cand2_cap, nc * 8))
                return -1;
            hipLaunchKernelGGL(k_sp_short_cand, dim3(grid_for(st->ns)), dim3(256), 0, s, st->keys, nw,
                               st->keys + nw, st->ns, k, st->cand);
            size_t tb3 = 0;
            CK(rocprim::radix_sort_keys(nullptr, tb3, st->cand, st->cand2, nc, 0, 64, s));
            if (ensure(&st->tmp, &st->tmp_cap, tb3)) return -1;
            tb3 = st->tmp_cap;
            CK(rocprim::radix_sort_keys(st->tmp, tb3, st->cand, st->cand2, nc, 0, 64, s));
            hipLaunchKernelGGL(k_sp_count_cand, dim3(grid_for(nc)), dim3(256), 0, s, st->cand2, nc, sm + 40);
        }
    }
    unsigned long long r[41];
    CK(hipMemcpyAsync(r, sm, sizeof r, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    for (int q = 0; q < 10; q++) tstat[q] = r[3 + q];
    *rollover = r[13];
    if (want_nodes && (nw || st->ns)) {
        /* windows: distinct depth-d prefixes for d = 1..k */
        unsigned long long nd = 0;
        if (nw) {
            unsigned long long run = 1;
            for (int d = 1; d <= k; d++) {
                run += r[14 + d];
                nd += run;
            }
        }
        *nodes = 1 + nd + r[40];
    }
    return 0;
}
