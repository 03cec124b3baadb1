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
 * Round 5: the engine does that itself for every pass (fk_sparse_pass.hip:
 * sp_count_runs32 counts a pass of at most 2^32 keys in LDS bins,
 * sp_sort_runs64 sorts a wider one in LDS).  This file keeps what those do
 * not take.  Round 6: all of it hand-written except one documented overflow
 * path -- fks_sort_runs, the library (rocPRIM) radix sort, for a pass whose
 * keys crowd one part past what a block's LDS sorts (a k-mer repeated tens
 * of thousands of times inside one 2^15-key part at k >= 18).  The rest:
 * fks_dense_runs (a single bucket too large for any pass: its nonzero bins
 * compacted by a block-count / scan / emit triple), fks_merge_runs (the
 * multi-GPU merge: the received tables' sorted runs merged pairwise by merge
 * path, then equal keys reduced), fks_unique / fks_short_count (the short
 * walks' nodeCounter: distinct values through an open-addressing hash set).
 * Device memory is bounded by the input plus one pass, never one slot per
 * input byte.
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
#include <vector>

#include <hip/hip_runtime.h>
/* the library radix sort: fks_sort_runs only (the documented overflow path) */
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

/* ---- compaction: a predicate over [0, n), its selected items written in
   order.  Three launches: per-tile counts, one block scanning them, then
   each tile again with a block-local scan.  A tile is FKS_T threads x
   FKS_I consecutive items each. */
#define FKS_T 256u
#define FKS_I 16u
#define FKS_TILE (FKS_T * FKS_I)

__device__ __forceinline__ uint32_t blk_excl_scan(uint32_t v, uint32_t *wsum4, uint32_t *total) {
    /* exclusive scan over the FKS_T threads (4 waves) */
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += o;
    }
    if (lane == 63) wsum4[w] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t j = 0; j < FKS_T / 64u; j++) {
        before += j < w ? wsum4[j] : 0u;
        all += wsum4[j];
    }
    *total = all;
    return before + inc - v;
}

template <class Pred>
__global__ void __launch_bounds__(FKS_T) k_sel_count(uint64_t n, Pred pred, uint32_t *tcount) {
    __shared__ uint32_t ws[FKS_T / 64u];
    const uint64_t i0 = (uint64_t)blockIdx.x * FKS_TILE + (uint64_t)threadIdx.x * FKS_I;
    uint32_t c = 0;
    for (uint32_t j = 0; j < FKS_I; j++)
        if (i0 + j < n && pred(i0 + j)) c++;
    uint32_t tot;
    blk_excl_scan(c, ws, &tot);
    if (threadIdx.x == 0) tcount[blockIdx.x] = tot;
}

/* tile offsets: toff[t] = sum of tcount[0, t), toff[nt] = the total (one
   block of 1024 threads, each a contiguous share) */
__global__ void __launch_bounds__(1024) k_sel_scan(const uint32_t *tcount, uint64_t nt, unsigned long long *toff) {
    __shared__ unsigned long long part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (nt + 1023) / 1024, b0 = min<uint64_t>(nt, per * t), b1 = min<uint64_t>(nt, b0 + per);
    unsigned long long v = 0;
    for (uint64_t i = b0; i < b1; i++) v += tcount[i];
    part[t] = v;
    __syncthreads();
    if (t == 0) {
        unsigned long long run = 0;
        for (uint32_t i = 0; i < 1024u; i++) {
            const unsigned long long x = part[i];
            part[i] = run;
            run += x;
        }
        toff[nt] = run;
    }
    __syncthreads();
    unsigned long long run = part[t];
    for (uint64_t i = b0; i < b1; i++) {
        toff[i] = run;
        run += tcount[i];
    }
}

template <class Pred, class Emit>
__global__ void __launch_bounds__(FKS_T) k_sel_emit(uint64_t n, Pred pred, Emit emit, const unsigned long long *toff) {
    __shared__ uint32_t ws[FKS_T / 64u];
    const uint64_t i0 = (uint64_t)blockIdx.x * FKS_TILE + (uint64_t)threadIdx.x * FKS_I;
    uint32_t m = 0;   /* selected items of this thread, as a bit mask */
    for (uint32_t j = 0; j < FKS_I; j++)
        if (i0 + j < n && pred(i0 + j)) m |= 1u << j;
    uint32_t tot;
    uint64_t at = toff[blockIdx.x] + blk_excl_scan(__popc(m), ws, &tot);
    for (uint32_t j = 0; j < FKS_I; j++)
        if (m & (1u << j)) emit(at++, i0 + j);
}

/* the selected items of pred over [0, n) to emit(position, index); the
   count to *nsel.  Synchronises the stream. */
template <class Pred, class Emit>
static int select_items(FksState *st, uint64_t n, Pred pred, Emit emit, hipStream_t s, uint64_t *nsel) {
    *nsel = 0;
    if (n == 0) return 0;
    const uint64_t nt = (n + FKS_TILE - 1) / FKS_TILE;
    if (nt > 0x7FFFFFFFull) return -1;
    if (ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)) ||
        ensure(&st->tmp, &st->tmp_cap, nt * 4 + (nt + 1) * 8 + 16))
        return -1;
    uint32_t *tc = static_cast<uint32_t *>(st->tmp);
    unsigned long long *toff = reinterpret_cast<unsigned long long *>(static_cast<char *>(st->tmp) + ((nt * 4 + 15) & ~15ull));
    hipLaunchKernelGGL(k_sel_count<Pred>, dim3((uint32_t)nt), dim3(FKS_T), 0, s, n, pred, tc);
    hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, s, (const uint32_t *)tc, nt, toff);
    hipLaunchKernelGGL((k_sel_emit<Pred, Emit>), dim3((uint32_t)nt), dim3(FKS_T), 0, s, n, pred, emit,
                       (const unsigned long long *)toff);
    CK(hipGetLastError());
    unsigned long long tot = 0;
    CK(hipMemcpyAsync(&tot, toff + nt, sizeof tot, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *nsel = tot;
    return 0;
}

struct DenseNZ {
    const unsigned long long *dense;
    __device__ bool operator()(uint64_t i) const { return dense[i] != 0; }
};
struct DenseOut {
    const unsigned long long *dense;
    uint64_t lo;
    uint64_t *keys, *c64;
    __device__ void operator()(uint64_t at, uint64_t i) const {
        keys[at] = lo + i;
        c64[at] = dense[i];
    }
};

int fks_dense_runs(FksState *st, unsigned long long *dense, uint64_t n, uint64_t lo, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw) {
    *nw = 0;
    /* (c64 room for every bin of the bucket: the count is known only after) */
    if (ensure((void **)&st->c64, &st->c64_cap, n * 8)) return -1;
    uint64_t runs = 0;
    if (select_items(st, n, DenseNZ{dense}, DenseOut{dense, lo, out_keys, st->c64}, s, &runs)) return -1;
    *nw = runs;
    return runs_stats(st, runs, k, s, dacc, out_keys, out_cnts);
}

/* ---- the multi-GPU merge: natural runs merged pairwise, equal keys reduced */

/* i starts an ascending run: i == 0 or keys[i] < keys[i - 1] */
struct RunStart {
    const uint64_t *keys;
    __device__ bool operator()(uint64_t i) const { return i == 0 || keys[i] < keys[i - 1]; }
};
struct IndexOut {
    uint64_t *out;
    __device__ void operator()(uint64_t at, uint64_t i) const { out[at] = i; }
};

/* One merge round: runs 2j and 2j + 1 (starts rs[], rs[nr] = n) merged into
 * the same span of the output; a lone last run is copied.  Thread t of the
 * grid writes outputs [8t, 8t + 8): for each pair it touches, the merge-path
 * split of its first output (A first on equal keys), then a sequential
 * merge. */
#define MP_PER 8u
__global__ void __launch_bounds__(256)
k_merge_pairs(const uint64_t *ka, const uint32_t *ca, uint64_t *kb, uint32_t *cb, uint64_t n, const uint64_t *rs,
              uint32_t nr) {
    const uint64_t o0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * MP_PER;
    if (o0 >= n) return;
    const uint64_t o1 = min<uint64_t>(o0 + MP_PER, n);
    const uint32_t np = (nr + 1) / 2;   /* pairs: pair j starts at rs[2j] */
    /* the pair holding o0: the last j with rs[2j] <= o0 */
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (rs[2 * mid] <= o0) lo = mid;
        else hi = mid;
    }
    for (uint32_t j = lo; j < np; j++) {
        /* A = [p0, pm), B = [pm, end) (empty for a lone last run: pm = n) */
        const uint64_t p0 = rs[2 * j], pm = rs[2 * j + 1], end = rs[min(2 * j + 2, nr)];
        const uint64_t a = max(o0, p0), z = min(o1, end);
        const uint64_t na = pm - p0, nb = end - pm, d = a - p0;
        /* merge-path split: the outputs before `a` take l items from A */
        uint64_t l = d > nb ? d - nb : 0, h = min(d, na);
        while (l < h) {
            const uint64_t m = (l + h) / 2;
            if (ka[p0 + m] <= ka[pm + (d - 1 - m)]) l = m + 1;
            else h = m;
        }
        uint64_t i = p0 + l, q = pm + (d - l);
        for (uint64_t o = a; o < z; o++) {
            const bool takeA = q >= end || (i < pm && ka[i] <= ka[q]);
            const uint64_t src = takeA ? i++ : q++;
            kb[o] = ka[src];
            cb[o] = ca[src];
        }
        if (end >= o1) break;
    }
}

/* the first of each run of equal keys, and the run's count summed (u64) */
struct KeyStart {
    const uint64_t *keys;
    __device__ bool operator()(uint64_t i) const { return i == 0 || keys[i] != keys[i - 1]; }
};
struct KeySum {
    const uint64_t *keys;
    const uint32_t *cnts;
    uint64_t n;
    uint64_t *out_keys, *c64;
    __device__ void operator()(uint64_t at, uint64_t i) const {
        const uint64_t key = keys[i];
        unsigned long long c = cnts[i];
        for (uint64_t j = i + 1; j < n && keys[j] == key; j++) c += cnts[j];
        out_keys[at] = key;
        c64[at] = c;
    }
};

int fks_merge_runs(FksState *st, const uint64_t *keys, const uint32_t *cnts, uint64_t n, int k, hipStream_t s,
                   unsigned long long *dacc, uint64_t *out_keys, uint32_t *out_cnts, uint64_t *nw) {
    *nw = 0;
    if (n == 0) return 0;
    /* the natural runs (each source's table is ascending: at most one per
       source; any order still merges, in more rounds) */
    if (ensure((void **)&st->cand, &st->cand_cap, n * 8)) return -1;
    uint64_t nr = 0;
    if (select_items(st, n, RunStart{keys}, IndexOut{st->cand}, s, &nr)) return -1;
    std::vector<uint64_t> rs(nr + 1);
    CK(hipMemcpyAsync(rs.data(), st->cand, nr * 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    rs[nr] = n;
    /* ping-pong buffers: keys in sorted / cand2 halves, counts u32 after */
    if (ensure((void **)&st->sorted, &st->sorted_cap, n * 12 + 16) ||
        ensure((void **)&st->cand2, &st->cand2_cap, n * 12 + 16) ||
        ensure((void **)&st->c64, &st->c64_cap, n * 8) ||
        ensure((void **)&st->cand, &st->cand_cap, (nr + 1) * 8))
        return -1;
    uint64_t *kbuf[2] = {st->sorted, st->cand2};
    uint32_t *cbuf[2] = {reinterpret_cast<uint32_t *>(st->sorted + n), reinterpret_cast<uint32_t *>(st->cand2 + n)};
    const uint64_t *kin = keys;
    const uint32_t *cin = cnts;
    int cur = 0;
    const unsigned grid = (unsigned)((n + MP_PER * 256 - 1) / (MP_PER * 256));
    do {
        CK(hipMemcpyAsync(st->cand, rs.data(), (nr + 1) * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_merge_pairs, dim3(grid), dim3(256), 0, s, kin, cin, kbuf[cur], cbuf[cur], n,
                           (const uint64_t *)st->cand, (uint32_t)nr);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));   /* (rs is rewritten below) */
        std::vector<uint64_t> nx;
        for (uint64_t j = 0; j < nr; j += 2) nx.push_back(rs[j]);
        nr = nx.size();
        nx.push_back(n);
        rs.swap(nx);
        kin = kbuf[cur];
        cin = cbuf[cur];
        cur ^= 1;
    } while (nr > 1);
    uint64_t runs = 0;
    if (select_items(st, n, KeyStart{kin}, KeySum{kin, cin, n, out_keys, st->c64}, s, &runs)) return -1;
    *nw = runs;
    return runs_stats(st, runs, k, s, dacc, out_keys, out_cnts);
}

/* ---- distinct values through an open-addressing hash set (~0: none) */
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}
__global__ void __launch_bounds__(256)
k_hash_insert(const uint64_t *v, uint64_t n, unsigned long long *table, uint64_t mask, unsigned long long *added) {
    unsigned long long mine = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long x = v[i];
        if (x == SP_EMPTY) continue;
        uint64_t h = mix64(x) & mask;
        for (uint64_t probe = 0; probe <= mask; probe++) {   /* (the table is at least twice the values) */
            const unsigned long long old = atomicCAS(&table[h], (unsigned long long)SP_EMPTY, x);
            if (old == SP_EMPTY) { mine++; break; }
            if (old == x) break;
            h = (h + 1) & mask;
        }
    }
    mine = wsum(mine);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(added, mine);
}
struct SlotUsed {
    const unsigned long long *table;
    __device__ bool operator()(uint64_t i) const { return table[i] != SP_EMPTY; }
};
struct SlotOut {
    const unsigned long long *table;
    uint64_t *out;
    __device__ void operator()(uint64_t at, uint64_t i) const { out[at] = table[i]; }
};

/* the distinct non-empty values of v[0, n) into a hash set of
   st->cand2 (its slot count to *slots); the count to *distinct */
static int hash_distinct(FksState *st, const uint64_t *v, uint64_t n, hipStream_t s, uint64_t *slots,
                         unsigned long long *distinct) {
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    if (ensure((void **)&st->cand2, &st->cand2_cap, cap * 8) ||
        ensure((void **)&st->small, &st->small_cap, 64 * sizeof(unsigned long long)))
        return -1;
    CK(hipMemsetAsync(st->cand2, 0xFF, cap * 8, s));
    CK(hipMemsetAsync(st->small + 40, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_hash_insert, dim3(grid_for(n)), dim3(256), 0, s, v, n,
                       reinterpret_cast<unsigned long long *>(st->cand2), cap - 1, st->small + 40);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(distinct, st->small + 40, sizeof *distinct, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *slots = cap;
    return 0;
}

int fks_unique(FksState *st, uint64_t *v, uint64_t n, hipStream_t s, uint64_t *n_out) {
    *n_out = n;
    if (n < 2) return 0;
    uint64_t slots = 0;
    unsigned long long u = 0;
    if (hash_distinct(st, v, n, s, &slots, &u)) return -1;
    uint64_t got = 0;   /* (in slot order: the callers need the set, not an order) */
    if (select_items(st, slots, SlotUsed{reinterpret_cast<const unsigned long long *>(st->cand2)},
                     SlotOut{reinterpret_cast<const unsigned long long *>(st->cand2), v}, s, &got))
        return -1;
    if (got != u) return -1;
    *n_out = got;
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
    if (ensure((void **)&st->cand, &st->cand_cap, nc * 8)) return -1;
    hipLaunchKernelGGL(k_sp_short_left, dim3(grid_for(ns)), dim3(256), 0, s, shorts, ns, found, st->cand);
    CK(hipGetLastError());
    uint64_t slots = 0;
    return hash_distinct(st, st->cand, nc, s, &slots, total);
}

void fks_free(FksState *st) {
    hipFree(st->sorted); hipFree(st->c64);
    hipFree(st->tmp); hipFree(st->small); hipFree(st->cand); hipFree(st->cand2);
    *st = FksState{};
}
