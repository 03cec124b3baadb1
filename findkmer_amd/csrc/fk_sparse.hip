/*
 * fk_sparse.hip — the count table for 17 <= k <= 20 (the reference accepts
 * k <= 20, findKmer/src/findKmer.cpp:438; a dense 4^k table stops fitting at
 * k = 17..18 on one GPU).
 *
 * The engine keeps the input it was fed and, at finish, builds the table in
 * key-range passes (fk_engine.hip, k_sp_emit): a histogram of the window
 * keys' top bits plans the passes; each pass emits the window indices of its
 * key range (reference order, < 2^40) compactly, and turns them into the
 * pass's distinct indices in ascending order -- the trie's DFS order, which
 * is the CSV row order (histo_recursive :699-942) -- with their counts.
 * Round 5: the engine does that itself for every pass (fk_engine.hip:
 * sp_count_runs32 counts a pass of at most 2^32 keys in LDS bins,
 * sp_sort_runs64 sorts a wider one in LDS); this file keeps the library
 * (rocPRIM) versions for what those do not take: fks_sort_runs for a pass
 * whose keys crowd one part past what a block's LDS sorts, fks_dense_runs
 * for a single bucket too large for any pass (a few k-mers repeated billions
 * of times), fks_merge_runs for the multi-GPU merge, fks_unique /
 * fks_short_count for the short walks' nodeCounter.  Device memory is
 * bounded by the input plus one pass, never one slot per input byte.
 *
 * From each pass's runs, on the GPU:
 *   - the table statistics k_table_stats computes for the dense table
 *     (distinct, u32 sum, last- and first-base marginals), so fk_result is
 *     filled the same way for every k;
 *   - nodeCounter (:128, :620): 1 + the distinct prefixes, at every depth,
 *     of the windows and of the short walks.  Window prefixes come from
 *     adjacent differences of the sorted indices (plus, on the host, the
 *     pair across each pass boundary); a short walk's prefixes count where
 *     no pass's windows have them (binary search per pass, fks_short_mark),
 *     deduplicated by a sort (fks_short_count).
 */
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "fk_sparse.h"

#define SP_EMPTY (~0ull)

namespace {

__device__ __forceinline__ unsigned long long wsum(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

/* distinct, u32 sum, last[4], first[4] of the window runs; rollover flag;
   the u32 counts (the reference's frequency) into cnt */
__global__ void __launch_bounds__(256)
k_sp_stats(const uint64_t *keys, const uint64_t *c64, uint32_t *cnt, uint64_t nw, int k,
           unsigned long long *out10, unsigned long long *big) {
    unsigned long long v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long wrap = 0;
    const int fs = 2 * (k - 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = keys[i];
        const uint64_t c6 = c64[i];
        const uint32_t c = (uint32_t)c6;   /* the reference's u32 frequency (:110) */
        cnt[i] = c;
        wrap |= c6 >> 32;                  /* a count >= 2^32: the rollover exit (:642) */
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

/* distinct candidates after the sort: adjacent differences per depth */
__global__ void __launch_bounds__(256)
k_sp_count_cand(const uint64_t *c, uint64_t n, unsigned long long *total) {
    unsigned long long v = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (c[i] != SP_EMPTY && (i == 0 || c[i] != c[i - 1])) v++;
    v = wsum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(total, v);
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

/* a dense bucket's nonzero counts as (key, count) runs */
struct NonZero {
    __device__ bool operator()(unsigned long long v) const { return v != 0; }
};
__global__ void k_sp_gather(const unsigned long long *dense, const uint64_t *keys, uint64_t n, uint64_t lo,
                            uint64_t *c64) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c64[i] = dense[keys[i] - lo];
}

/* a pass's short-walk prefixes found among its sorted window keys */
__global__ void k_sp_short_mark(const uint64_t *keys, uint64_t nw, const uint64_t *shorts, uint64_t ns, int k,
                                uint8_t *found) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = shorts[i];
        const int seq = (int)((e >> 40) & 0x3F);
        const uint64_t code = e & ((1ull << 40) - 1);
        for (int d = 1; d <= seq && d <= 20; d++) {
            if (found[i * 20 + (uint64_t)(d - 1)]) continue;
            const uint64_t p = code >> (2 * (seq - d));
            const int sh = 2 * (k - d);
            const uint64_t want = p << sh;
            uint64_t lo = 0, hi = nw;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (keys[mid] < want) lo = mid + 1;
                else hi = mid;
            }
            if (lo < nw && (keys[lo] >> sh) == p) found[i * 20 + (uint64_t)(d - 1)] = 1;
        }
    }
}

/* the prefixes of the short walks no window has, as candidates */
__global__ void k_sp_short_left(const uint64_t *shorts, uint64_t ns, const uint8_t *found, uint64_t *cand) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = shorts[i];
        const int seq = (int)((e >> 40) & 0x3F);
        const uint64_t code = e & ((1ull << 40) - 1);
        for (int d = 1; d <= 20; d++) {
            uint64_t out = SP_EMPTY;
            if (d <= seq && !found[i * 20 + (uint64_t)(d - 1)]) out = ((uint64_t)d << 40) | (code >> (2 * (seq - d)));
            cand[i * 20 + (uint64_t)(d - 1)] = out;
        }
    }
}

/* runs (out_keys, st->c64)[0, nw) -> u32 counts into out_cnts, statistics,
   prefix histogram */
static int runs_stats(FksState *st, uint64_t nw, int k, hipStream_t s, unsigned long long *dacc,
                      const uint64_t *out_keys, uint32_t *out_cnts) {
    if (!nw) return 0;
    hipLaunchKernelGGL(k_sp_stats, dim3(grid_for(nw)), dim3(256), 0, s, out_keys, st->c64, out_cnts, nw, k, dacc,
                       dacc + FKS_ACC_ROLL);
    if (nw > 1)
        hipLaunchKernelGGL(k_sp_wprefix, dim3(grid_for(nw)), dim3(256), 0, s, out_keys, nw, k, dacc + FKS_ACC_WPREFIX);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int fks_sort_runs(FksState *st, uint64_t *keys, uint64_t n, int k, hipStream_t s, unsigned long long *dacc,
                  uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw, uint64_t npads) {
    *nw = 0;
    if (n == 0) return 0;
    if (ensure((void **)&st->sorted, &st->sorted_cap, n * 8) || ensure((void **)&st->c64, &st->c64_cap, n * 8) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    const int bits = 2 * k;
    size_t tb = 0, tb2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, keys, st->sorted, n, 0, bits, s));
    CK(rocprim::run_length_encode(nullptr, tb2, st->sorted, n, out_keys, st->c64, st->small, s));
    if (ensure(&st->tmp, &st->tmp_cap, tb > tb2 ? tb : tb2)) return -1;
    tb = st->tmp_cap;
    CK(rocprim::radix_sort_keys(st->tmp, tb, keys, st->sorted, n, 0, bits, s));
    tb2 = st->tmp_cap;
    CK(rocprim::run_length_encode(st->tmp, tb2, st->sorted, n, out_keys, st->c64, st->small, s));
    unsigned long long runs = 0;
    CK(hipMemcpyAsync(&runs, st->small, sizeof runs, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (npads && runs) {
        /* the pads (4^k - 1, the largest key) are the last run, with the
           real key 4^k - 1 if the pass has it: take them off its count */
        uint64_t last = 0;
        CK(hipMemcpyAsync(&last, st->c64 + (runs - 1), sizeof last, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (last <= npads) {
            runs--;
        } else {
            last -= npads;
            CK(hipMemcpyAsync(st->c64 + (runs - 1), &last, sizeof last, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        }
    }
    *nw = runs;
    return runs_stats(st, runs, k, s, dacc, out_keys, out_cnts);
}

int fks_dense_runs(FksState *st, unsigned long long *dense, uint64_t n, uint64_t lo, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw) {
    *nw = 0;
    if (ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long))) return -1;
    rocprim::counting_iterator<uint64_t> idx(lo);
    auto flags = rocprim::make_transform_iterator(dense, NonZero());
    size_t tb = 0;
    CK(rocprim::select(nullptr, tb, idx, flags, out_keys, st->small, n, s));
    if (ensure(&st->tmp, &st->tmp_cap, tb)) return -1;
    tb = st->tmp_cap;
    CK(rocprim::select(st->tmp, tb, idx, flags, out_keys, st->small, n, s));
    unsigned long long runs = 0;
    CK(hipMemcpyAsync(&runs, st->small, sizeof runs, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *nw = runs;
    if (!runs) return 0;
    if (ensure((void **)&st->c64, &st->c64_cap, runs * 8)) return -1;
    hipLaunchKernelGGL(k_sp_gather, dim3(grid_for(runs)), dim3(256), 0, s, dense, out_keys, runs, lo, st->c64);
    return runs_stats(st, runs, k, s, dacc, out_keys, out_cnts);
}

struct WidenU32 {
    __device__ unsigned long long operator()(uint32_t v) const { return v; }
};

int fks_merge_runs(FksState *st, const uint64_t *keys, const uint32_t *cnts, uint64_t n, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw) {
    *nw = 0;
    if (n == 0) return 0;
    if (ensure((void **)&st->sorted, &st->sorted_cap, n * 8) || ensure((void **)&st->c64, &st->c64_cap, n * 8) ||
        ensure((void **)&st->cand2, &st->cand2_cap, n * 4) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    uint32_t *vs = reinterpret_cast<uint32_t *>(st->cand2);
    auto wide = rocprim::make_transform_iterator(vs, WidenU32());
    size_t tb = 0, tb2 = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, keys, st->sorted, cnts, vs, n, 0, 2 * k, s));
    CK(rocprim::reduce_by_key(nullptr, tb2, st->sorted, wide, n, out_keys, st->c64, st->small,
                              rocprim::plus<unsigned long long>(), rocprim::equal_to<uint64_t>(), s));
    if (ensure(&st->tmp, &st->tmp_cap, tb > tb2 ? tb : tb2)) return -1;
    tb = tb2 = st->tmp_cap;
    CK(rocprim::radix_sort_pairs(st->tmp, tb, keys, st->sorted, cnts, vs, n, 0, 2 * k, s));
    CK(rocprim::reduce_by_key(st->tmp, tb2, st->sorted, wide, n, out_keys, st->c64, st->small,
                              rocprim::plus<unsigned long long>(), rocprim::equal_to<uint64_t>(), s));
    unsigned long long runs = 0;
    CK(hipMemcpyAsync(&runs, st->small, sizeof runs, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *nw = runs;
    return runs_stats(st, runs, k, s, dacc, out_keys, out_cnts);
}

int fks_unique(FksState *st, uint64_t *v, uint64_t n, hipStream_t s, uint64_t *n_out) {
    *n_out = n;
    if (n < 2) return 0;
    if (ensure((void **)&st->cand2, &st->cand2_cap, n * 8) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    size_t tb = 0, tb2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, v, st->cand2, n, 0, 64, s));
    CK(rocprim::unique(nullptr, tb2, st->cand2, v, st->small + 41, n, rocprim::equal_to<uint64_t>(), s));
    if (ensure(&st->tmp, &st->tmp_cap, tb > tb2 ? tb : tb2)) return -1;
    tb = tb2 = st->tmp_cap;
    CK(rocprim::radix_sort_keys(st->tmp, tb, v, st->cand2, n, 0, 64, s));
    CK(rocprim::unique(st->tmp, tb2, st->cand2, v, st->small + 41, n, rocprim::equal_to<uint64_t>(), s));
    unsigned long long u = 0;
    CK(hipMemcpyAsync(&u, st->small + 41, sizeof u, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *n_out = u;
    return 0;
}

int fks_short_mark(const uint64_t *keys, uint64_t nw, const uint64_t *shorts, uint64_t ns, int k, uint8_t *found,
                   hipStream_t s) {
    if (!ns || !nw) return 0;
    hipLaunchKernelGGL(k_sp_short_mark, dim3(grid_for(ns)), dim3(256), 0, s, keys, nw, shorts, ns, k, found);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int fks_short_count(FksState *st, const uint64_t *shorts, uint64_t ns, const uint8_t *found, hipStream_t s,
                    unsigned long long *total) {
    *total = 0;
    if (!ns) return 0;
    const uint64_t nc = ns * 20;
    if (ensure((void **)&st->cand, &st->cand_cap, nc * 8) || ensure((void **)&st->cand2, &st->cand2_cap, nc * 8) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    hipLaunchKernelGGL(k_sp_short_left, dim3(grid_for(ns)), dim3(256), 0, s, shorts, ns, found, st->cand);
    size_t tb = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, st->cand, st->cand2, nc, 0, 64, s));
    if (ensure(&st->tmp, &st->tmp_cap, tb)) return -1;
    tb = st->tmp_cap;
    CK(rocprim::radix_sort_keys(st->tmp, tb, st->cand, st->cand2, nc, 0, 64, s));
    CK(hipMemsetAsync(st->small + 40, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_sp_count_cand, dim3(grid_for(nc)), dim3(256), 0, s, st->cand2, nc, st->small + 40);
    CK(hipMemcpyAsync(total, st->small + 40, sizeof *total, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    return 0;
}

void fks_free(FksState *st) {
    hipFree(st->sorted); hipFree(st->c64);
    hipFree(st->tmp); hipFree(st->small); hipFree(st->cand); hipFree(st->cand2);
    *st = FksState{};
}
