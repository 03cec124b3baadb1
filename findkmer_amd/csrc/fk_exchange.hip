/*
 * fk_exchange.hip -- multi-GPU: a shard's pack into the
 * merge buffer, the one-collective and stitched exchanges over the library's
 * RCCL communicator, and the routed k >= 15 sharded tables.
 */
#include "fk_engine_internal.h"

/* ---- one-collective shard exchange ---- */

/* The pending one-pass shard's result into a caller's merge buffer: the
 * table (every block, 16-B pieces), the counters as 16-bit limbs and the
 * pack rows (block 0).  `valid`: the host knows the shard went through
 * k_count + k_tail; the device adds k_tail's verdict (no ONE_* bits, no
 * 0xFF candidate).  The counter values are fk_engine_finish's formulas. */
__global__ void __launch_bounds__(1024)
k_shard_pack(const DevRes *res, const uint32_t *table, uint64_t nbins, uint32_t *dt, int32_t *dc, uint32_t *rows,
             int nrows, int slot, int is_last, int valid, uint64_t len, int k) {
    const bool ok = valid && res->need == 0 && res->eof_cand == ~0ull;
    if (valid) {
        /* nbins >= 4 (k >= 1); 16-B pieces while they fit, then words */
        const uint64_t n4 = nbins / 4;
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += stride)
            reinterpret_cast<uint4 *>(dt)[i] = reinterpret_cast<const uint4 *>(table)[i];
    }
    if (blockIdx.x != 0) return;
    const uint32_t t = threadIdx.x;
    if (t < FK_PACK_COUNTERS * 4) {
        const unsigned long long *acc = res->acc, *ts = res->tstat;
        const uint32_t c = t >> 2, limb = t & 3;
        unsigned long long v = 0;
        if (ok) {
            switch (c) {
            case 0: v = acc[ACC_WIN]; break;
            case 1: v = acc[ACC_WIN] + acc[ACC_VALID]; break;
            case 2: case 3: case 4: case 5: v = ts[2 + (c - 2)] + acc[ACC_BASE + (c - 2)]; break;
            case 6: case 7: case 8: case 9: v = ts[6 + (c - 6)] + acc[ACC_D1S + (c - 6)]; break;
            case 10: v = acc[ACC_UNK]; break;
            case 11: v = len; break;
            case 12: v = 0; break;                           /* ended: a 0xFF shard is never packed */
            default: v = is_last ? res->exit.hdr : 0u; break;   /* unterminated_header */
            }
        }
        dc[t] = (int32_t)((v >> (16 * limb)) & 0xFFFFu);
    }
    for (uint32_t i = t; i < (uint32_t)nrows * FK_PACK_ROW_WORDS; i += blockDim.x) {
        const uint32_t r = i / FK_PACK_ROW_WORDS, j = i % FK_PACK_ROW_WORDS;
        uint32_t v = 0;
        if ((int)r == slot && ok) {
            if (j < 24) {
                const ShardSum &ss = res->shard;
                uint64_t w = 0;
                switch (j >> 1) {
                case 0: w = ss.g_code; break;
                case 1: w = (uint64_t)ss.g_R | ((uint64_t)ss.g_hdr << 32); break;
                case 2: w = ss.nvb0; break;
                case 3: w = ss.c_R; break;
                case 4: w = ss.c_code; break;
                case 5: w = (uint64_t)ss.c_hdr | ((uint64_t)ss.absorb << 32); break;
                case 6: w = ss.nv; break;
                case 7: w = len; break;
                case 8: w = (uint64_t)k; break;
                case 11: w = FK_SUMMARY_COMPACT; break;
                default: w = 0; break;                        /* 9: no 0xFF byte; 10: unused */
                }
                v = (j & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
            } else if (j == 24) {
                v = 1u;
            }
        }
        rows[i] = v;
    }
}

extern "C" int fk_engine_shard_pack(fk_engine *e, uint32_t *table, int32_t *counters, uint32_t *rows, int nrows,
                                    int slot, int is_last) {
    if (!e || !table || !counters || !rows || nrows < 1 || slot < 0 || slot >= nrows) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: no dense table to merge */
    if (!e->shard_pending) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    /* packable: counted in one pass (k_count + k_tail, k <= 7), nothing of
       the multi-launch path run since */
    const int valid = e->shard_len && e->shard_op && !e->shard_full && !e->shard_resumed ? 1 : 0;
    const uint64_t n4 = e->nbins / 4;
    const unsigned grid = valid ? (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n4 + 1023) / 1024, 1024)) : 1u;
    hipLaunchKernelGGL(k_shard_pack, dim3(grid), dim3(1024), 0, e->stream, e->d_res, e->d_table, e->nbins, table,
                       counters, rows, nrows, slot, is_last ? 1 : 0, valid, e->shard_len, e->k);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* The gathered rows to pinned host memory, sequence number last (one block,
   one system fence per thread, then a block barrier before thread 0's
   release store: every thread's row stores are ordered before the sequence
   number the host spins on, whatever the block size). */
__global__ void __launch_bounds__(64) k_rows_publish(const uint32_t *rows, uint32_t n, uint32_t *host, uint32_t seq) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) host[32 + i] = rows[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&host[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* One row of a rows region (zeros elsewhere): words [0, nsrc) from src (a
   device transfer function), or w0 in word 0; word 24 = 1 (a valid row). */
__global__ void __launch_bounds__(64) k_fill_row(uint32_t *rows, int nrows, int slot, const uint32_t *src,
                                                 uint32_t nsrc, uint32_t w0) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)nrows * FK_PACK_ROW_WORDS; i += 64) {
        const uint32_t r = i / FK_PACK_ROW_WORDS, j = i % FK_PACK_ROW_WORDS;
        uint32_t v = 0;
        if ((int)r == slot) v = j == 24 ? 1u : (src ? (j < nsrc ? src[j] : 0u) : (j == 0 ? w0 : 0u));
        rows[i] = v;
    }
}

/* pinned, mapped scratch of the exchange: [0] sequence number, rows from
   word 32, counter and slice-statistics limbs (staging) after the rows */
int ensure_rows(fk_engine *e, uint32_t nrow) {
    if (e->rows_cap >= nrow) return FK_OK;
    if (e->h_rows) hipHostFree(e->h_rows);
    hipFree(e->d_rows);
    e->h_rows = e->h_rows_dev = nullptr;
    e->d_rows = nullptr;
    e->rows_cap = 0;
    const size_t words = 32 + nrow + 4 * FK_PACK_COUNTERS + FK_PACK_STATS;
    if (hipHostMalloc((void **)&e->h_rows, words * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&e->h_rows_dev, e->h_rows, 0) != hipSuccess ||
        hipMalloc((void **)&e->d_rows, nrow * sizeof(uint32_t)) != hipSuccess)
        return FK_E_OOM;
    memset(e->h_rows, 0, words * sizeof(uint32_t));
    e->rows_cap = nrow;
    return FK_OK;
}

/* The rows (device, already all-reduced on e->stream) into e->h_rows + 32;
   one host wait. */
int rows_fetch(fk_engine *e, const uint32_t *rows, uint32_t nrow) {
    if (++e->rows_seq == 0) e->rows_seq = 1;
    const uint32_t want = e->rows_seq;
    hipLaunchKernelGGL(k_rows_publish, dim3(1), dim3(64), 0, e->stream, rows, nrow, e->h_rows_dev, want);
    HIPCHK(hipGetLastError());
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&e->h_rows[0], __ATOMIC_ACQUIRE) == want) break;
        if ((spin & 4095) == 0) {
            hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(&e->h_rows[0], __ATOMIC_ACQUIRE) == want) break;
                return FK_E_HIP;   /* stream drained without publishing */
            }
            if (q != hipErrorNotReady) return FK_E_HIP;
        }
        __builtin_ia32_pause();
    }
    return FK_OK;
}

/* The stitched exchange with the library's communicator (the shard is
   pending): the shards' full transfer functions all-gathered (an
   all-reduce of rows), composed on the host, the shard resolved; the shards'
   end flags all-gathered the same way (a 0xFF byte, :988, exact only after
   the resolve); then the table and counter limbs, zero for ranks after the
   first ending shard, reduced onto rank 0. */
/* merge buffer layout (include/findkmer.h, fk_merge_layout): the table
   padded to a multiple of the world size, the counter limbs, the slice
   statistics, the rows */
uint64_t merge_table_words(uint64_t nbins, int world) {
    const uint64_t w = (uint64_t)std::max(1, world);
    return (nbins + w - 1) / w * w;
}

/* the u64 sum and the nonzero bins of one table slice (sharded table) */
__global__ void __launch_bounds__(256) k_slice_sum(const uint32_t *t, uint64_t n, unsigned long long *out2) {
    /* 16-B loads between a scalar head (to the first aligned word: a slice
       starts at rank * S) and tail; one 4-B load per lane left the k = 16
       slice at 2.2 TB/s */
    unsigned long long sum = 0, nz = 0;
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t head = std::min<uint64_t>(n, ((16u - ((uintptr_t)t & 15u)) & 15u) / 4u);
    const uint64_t n4 = (n - head) / 4;
    if (tid < head) { const uint32_t v = t[tid]; sum += v; nz += v != 0; }
    const u32x4 *t4 = reinterpret_cast<const u32x4 *>(t + head);
    for (uint64_t q = tid; q < n4; q += nth) {
        const u32x4 v = __builtin_nontemporal_load(t4 + q);
        sum += (unsigned long long)v.x + v.y + v.z + v.w;
        nz += (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
    }
    for (uint64_t i = head + n4 * 4 + tid; i < n; i += nth) { const uint32_t v = t[i]; sum += v; nz += v != 0; }
    sum = wsum64(sum);
    nz = wsum64(nz);
    if ((threadIdx.x & 63) == 0) {
        if (sum) atomicAdd(&out2[0], sum);
        if (nz) atomicAdd(&out2[1], nz);
    }
}

/* ... as 16-bit limbs in int32 words (sums over ranks stay exact) */
__global__ void k_slice_limbs(const unsigned long long *in2, int32_t *limbs8) {
    const uint32_t i = threadIdx.x;
    if (i < 8) limbs8[i] = (int32_t)((in2[i >> 2] >> (16 * (i & 3))) & 0xFFFFu);
}

/*
 * Routed sharded tables (k >= 15, FK_XCHG_SHARD_TABLE over RCCL or a gloo
 * rehearsal): instead of reduce-scattering the whole 4^k table (k = 16:
 * 16 GiB a rank, ~15 GiB of it over xGMI), each rank sends every owner only
 * the nonzero bins of the owner's range, as one blob of 4-B entries per
 * destination, and each owner counts the blobs it receives into its slice.
 * A shard of 1.25 G windows leaves ~1.1 G nonzero bins at k = 16: ~4.4 GB
 * sent instead of 15 GiB, and nothing sent for bins no rank saw.
 *
 * Parts: 2^15-bin blocks of the table (reference index order).  Owner d holds
 * bins [d S, min((d + 1) S, 4^k)), S = TW / world (fk_merge_layout), so a part
 * belongs to one owner or, at a range boundary, to two.  A (destination,
 * part) pair is a slot, slots destination-major.  Blob for destination d:
 *   [0, 4)           E_d (entries) and O_d (overflow pairs), u64 as 2 words
 *   [4, 4 + P_d)     entries per slot of d (P_d slots: its parts)
 *   [.., + E_d)      entries, slot by slot: (bin offset in the part << 17) | count
 *   [.., + 2 O_d)    overflow pairs (bin - d S, count): counts >= 2^17 - 1
 *   [.., + 2)        trailer: RT_MAGIC, the sum of the words before it
 */
#define RT_SH 15u
#define RT_ESC 0x1FFFFu
#define RT_HDR 4u
#define RT_STAT_SLOTS 512u
/* every blob ends in a trailer {RT_MAGIC, sum of the blob's other words mod
   2^32}: the owner checks it before trusting what it counted (a
   transfer that delivers only part of a blob would otherwise go unnoticed,
   and a receive buffer reused across steps would even hide it behind the
   previous step's identical blob).  The trailer words of the receive
   buffer are cleared before the transfer. */
#define RT_TRL 2u
#define RT_MAGIC 0x52544231u   /* "RTB1" */

/* per-destination arrays in one device buffer (u64 each, world W):
   p0 [0,W) first part, sb [W, 2W+1) first slot, np [2W+1, 3W+1) parts,
   bb [3W+1, 4W+1) blob start (words), ne [4W+1, 5W+1) entries,
   no [5W+1, 6W+1) overflow pairs, oc [6W+1, 7W+1) overflow cursor; then
   off[nslots + 1] (exclusive entry offset of each slot), then cnt[nslots] u32 */
struct RouteGeo {
    uint64_t nbins, S;
    uint32_t world, nparts;
    unsigned long long *aux;
    __device__ __forceinline__ unsigned long long *p0() const { return aux; }
    __device__ __forceinline__ unsigned long long *sb() const { return aux + world; }
    __device__ __forceinline__ unsigned long long *np() const { return aux + 2 * world + 1; }
    __device__ __forceinline__ unsigned long long *bb() const { return aux + 3 * world + 1; }
    __device__ __forceinline__ unsigned long long *ne() const { return aux + 4 * world + 1; }
    __device__ __forceinline__ unsigned long long *no() const { return aux + 5 * world + 1; }
    __device__ __forceinline__ unsigned long long *oc() const { return aux + 6 * world + 1; }
    __device__ __forceinline__ unsigned long long *off() const { return aux + 7 * world + 1; }
    uint32_t *ck;          /* per destination: the blob's word sum so far (k_route_write) */
};

/* a part's owner(s): d0 and, when the part crosses d0's end b, d0 + 1 */
__device__ __forceinline__ void rt_owners(const RouteGeo &g, uint64_t x0, uint32_t &d0, uint64_t &b, bool &two) {
    d0 = (uint32_t)min<uint64_t>(x0 / g.S, (uint64_t)g.world - 1);
    b = (uint64_t)(d0 + 1) * g.S;
    two = d0 + 1 < g.world && b < x0 + (1ull << RT_SH);
}

/* one block per part: its entries and overflow bins per owner, and per wave
   (a quarter of the part each: k_route_write's start positions, wc) */
__global__ void __launch_bounds__(256)
k_route_count(const uint32_t *table, RouteGeo g, int counting, uint32_t *cnt, uint32_t *wc) {
    __shared__ uint32_t ws[4][4];
    const uint32_t p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t x0 = (uint64_t)p << RT_SH;
    uint32_t d0;
    uint64_t b;
    bool two;
    rt_owners(g, x0, d0, b, two);
    uint32_t c[4] = {0, 0, 0, 0};   /* entries lo / hi, overflow lo / hi */
    if (counting) {
        const u32x4 *t4 = reinterpret_cast<const u32x4 *>(table + x0) + (size_t)wv * ((1u << RT_SH) / 16u);
        for (uint32_t q = lane; q < (1u << RT_SH) / 16u; q += 64u) {
            const u32x4 v4 = __builtin_nontemporal_load(t4 + q);
            const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const bool hi = x0 + wv * ((1u << RT_SH) / 4u) + q * 4u + (uint32_t)h >= b;
                const uint32_t v = w[h];
                c[hi ? 1 : 0] += v != 0u && v < RT_ESC;
                c[hi ? 3 : 2] += v >= RT_ESC;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) c[i] = wsum32(c[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 4; i++) ws[wv][i] = c[i];
        wc[(size_t)p * 8u + wv * 2u] = c[0];
        wc[(size_t)p * 8u + wv * 2u + 1u] = c[1];
    }
    __syncthreads();
    if (t == 0) {
        uint32_t s[4] = {0, 0, 0, 0};
        for (int w = 0; w < 4; w++)
            for (int i = 0; i < 4; i++) s[i] += ws[w][i];
        cnt[g.sb()[d0] + p - g.p0()[d0]] = s[0];
        if (s[2]) atomicAdd(&g.no()[d0], (unsigned long long)s[2]);
        if (two) {
            cnt[g.sb()[d0 + 1] + p - g.p0()[d0 + 1]] = s[1];
            if (s[3]) atomicAdd(&g.no()[d0 + 1], (unsigned long long)s[3]);
        }
    }
}

/* exclusive prefix of cnt[0, n) into off[0, n], off[n] = the total (one
   block: a few hundred K slots at most) */
__global__ void __launch_bounds__(1024)
k_route_scan(const uint32_t *cnt, uint64_t n, unsigned long long *off) {
    __shared__ unsigned long long part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (n + 1023) / 1024, b0 = min<uint64_t>(n, per * t), b1 = min<uint64_t>(n, b0 + per);
    unsigned long long s = 0;
    for (uint64_t i = b0; i < b1; i++) s += cnt[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        unsigned long long run = 0;
        for (uint32_t i = 0; i < 1024u; i++) {
            const unsigned long long v = part[i];
            part[i] = run;
            run += v;
        }
        off[n] = run;
    }
    __syncthreads();
    unsigned long long run = part[t];
    for (uint64_t i = b0; i < b1; i++) {
        off[i] = run;
        run += cnt[i];
    }
}

/* one block per part: its entries in bin order into each owner's blob (a
   wave per quarter of the part, its start from the waves before it),
   overflow bins appended to the owner's pairs, the slot counts, and (block
   0) every blob's header */
__global__ void __launch_bounds__(256)
k_route_write(const uint32_t *table, RouteGeo g, int counting, const uint32_t *cnt, const uint32_t *wc,
              uint32_t *send) {
    const uint32_t p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (p == 0 && t < g.world) {
        const unsigned long long e = g.ne()[t], o = g.no()[t];
        uint32_t *h = send + g.bb()[t];
        h[0] = (uint32_t)e; h[1] = (uint32_t)(e >> 32); h[2] = (uint32_t)o; h[3] = (uint32_t)(o >> 32);
        atomicAdd(&g.ck[t], h[0] + h[1] + h[2] + h[3]);
    }
    const uint64_t x0 = (uint64_t)p << RT_SH;
    uint32_t d0;
    uint64_t b;
    bool two;
    rt_owners(g, x0, d0, b, two);
    const uint32_t d1 = two ? d0 + 1 : d0;
    const uint64_t s0 = g.sb()[d0] + p - g.p0()[d0], s1 = g.sb()[d1] + p - g.p0()[d1];
    if (t == 0) {
        send[g.bb()[d0] + RT_HDR + (s0 - g.sb()[d0])] = cnt[s0];
        atomicAdd(&g.ck[d0], cnt[s0]);
        if (two) {
            send[g.bb()[d1] + RT_HDR + (s1 - g.sb()[d1])] = cnt[s1];
            atomicAdd(&g.ck[d1], cnt[s1]);
        }
    }
    if (!counting) return;
    constexpr uint32_t QW = (1u << RT_SH) / 4u;   /* bins per wave */
    const uint32_t *tw = table + x0 + (uint64_t)wv * QW;
    uint64_t pos0 = g.off()[s0] - g.off()[g.sb()[d0]], pos1 = g.off()[s1] - g.off()[g.sb()[d1]];
    for (uint32_t w = 0; w < wv; w++) { pos0 += wc[(size_t)p * 8u + w * 2u]; pos1 += wc[(size_t)p * 8u + w * 2u + 1u]; }
    uint32_t *e0 = send + g.bb()[d0] + RT_HDR + g.np()[d0], *e1 = send + g.bb()[d1] + RT_HDR + g.np()[d1];
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t ck0 = 0, ck1 = 0;   /* this lane's words into each blob */
    for (uint32_t i0 = 0; i0 < QW; i0 += 64u) {
        const uint32_t i = i0 + lane;
        const uint32_t v = tw[i];
        const uint64_t x = x0 + wv * QW + i;
        const bool hi = x >= b, nz = v != 0u && v < RT_ESC;
        const unsigned long long m0 = __ballot(nz && !hi), m1 = __ballot(nz && hi);
        const uint32_t ent = ((wv * QW + i) << 17) | v;
        if (nz) {
            if (hi) e1[pos1 + __popcll(m1 & lt)] = ent;
            else e0[pos0 + __popcll(m0 & lt)] = ent;
        }
        if (v >= RT_ESC) {
            const uint32_t d = hi ? d1 : d0;
            const unsigned long long at = atomicAdd(&g.oc()[d], 1ull);
            uint32_t *op = send + g.bb()[d] + RT_HDR + g.np()[d] + g.ne()[d] + 2 * at;
            op[0] = (uint32_t)(x - (uint64_t)d * g.S);
            op[1] = v;
        }
        const uint32_t w = (nz ? ent : 0u) + (v >= RT_ESC ? (uint32_t)(x - (uint64_t)(hi ? d1 : d0) * g.S) + v : 0u);
        if (hi) ck1 += w;
        else ck0 += w;
        pos0 += __popcll(m0);
        pos1 += __popcll(m1);
    }
    ck0 = wsum32(ck0);
    ck1 = wsum32(ck1);
    if (lane == 0) {
        if (ck0) atomicAdd(&g.ck[d0], ck0);
        if (ck1) atomicAdd(&g.ck[d1], ck1);
    }
}

/* each blob's trailer, once k_route_write has summed its words */
__global__ void __launch_bounds__(64) k_route_seal(RouteGeo g, uint32_t *send) {
    for (uint32_t d = threadIdx.x; d < g.world; d += 64u) {
        uint32_t *tr = send + g.bb()[d] + RT_HDR + g.np()[d] + g.ne()[d] + 2 * g.no()[d];
        tr[0] = RT_MAGIC;
        tr[1] = g.ck[d];
    }
}

/* the owner: one block per part of its range, every source's entries for
   the part into 2^15 LDS bins, then the part's owned bins into the slice
   (written, not added: the slice holds nothing before) */
__global__ void __launch_bounds__(1024)
k_route_absorb(const uint32_t *recv, const unsigned long long *rd, const unsigned long long *roff, uint32_t world,
               uint32_t np, uint64_t p0, uint64_t lo, uint64_t hi, uint32_t *out, unsigned long long *stats,
               uint32_t *vck) {
    extern __shared__ uint32_t bins[];
    const uint32_t j = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = t; i < (1u << RT_SH) / 4u; i += 1024u) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t s = 0; s < world; s++) {
        const uint32_t *blob = recv + rd[s];
        const uint32_t n = blob[RT_HDR + j];
        const uint32_t *ent = blob + RT_HDR + np + roff[(uint64_t)s * (np + 1) + j];
        uint32_t ck = t == 0 ? n : 0u;   /* (the slot's count word, read here) */
        for (uint32_t i = t; i < n; i += 1024u) {
            const uint32_t e = ent[i];
            ck += e;
            atomicAdd(&bins[e >> 17], e & RT_ESC);
        }
        ck = wsum32(ck);
        if ((t & 63) == 0 && ck) atomicAdd(&vck[s], ck);
    }
    __syncthreads();
    const uint64_t x0 = (p0 + j) << RT_SH;
    unsigned long long sum = 0, nz = 0;
    for (uint32_t i = t; i < (1u << RT_SH); i += 1024u) {
        const uint64_t x = x0 + i;
        if (x >= lo && x < hi) {
            const uint32_t v = bins[i];
            out[x - lo] = v;
            sum += v;
            nz += v != 0;
        }
    }
    /* the slice's total and nonzero bins (k_slice_sum's), before the
       overflow pairs add theirs (k_route_overflow): a block's sums into one
       of RT_STAT_SLOTS slot pairs (per-wave atomics on one address took
       50 ms at k = 16), k_route_stats folds them */
    if (stats) {
        __shared__ unsigned long long bs[16][2];
        sum = wsum64(sum);
        nz = wsum64(nz);
        if ((t & 63) == 0) { bs[t >> 6][0] = sum; bs[t >> 6][1] = nz; }
        __syncthreads();
        if (t < 2) {
            unsigned long long a = 0;
            for (int w = 0; w < 16; w++) a += bs[w][t];
            if (a) atomicAdd(&stats[(j % RT_STAT_SLOTS) * 2 + t], a);
        }
    }
}

/* every source's trailer against the sum of the words the owner read
   (k_route_absorb, k_route_overflow): bad[0] = 1 on any mismatch */
__global__ void __launch_bounds__(64)
k_route_verify(const uint32_t *recv, const unsigned long long *rd, uint32_t np, const uint32_t *vck, uint32_t world,
               uint32_t *bad) {
    for (uint32_t s = threadIdx.x; s < world; s += 64u) {
        const uint32_t *blob = recv + rd[s];
        const uint64_t ne = blob[0] | ((uint64_t)blob[1] << 32), no = blob[2] | ((uint64_t)blob[3] << 32);
        const uint32_t *tr = blob + RT_HDR + np + ne + 2 * no;
        if (tr[0] != RT_MAGIC || tr[1] != vck[s]) atomicOr(bad, 1u);
    }
}

__global__ void __launch_bounds__(256) k_route_stats(const unsigned long long *slots, unsigned long long *out2) {
    unsigned long long a = 0, b = 0;
    for (uint32_t i = threadIdx.x; i < RT_STAT_SLOTS; i += 256u) { a += slots[2 * i]; b += slots[2 * i + 1]; }
    a = wsum64(a);
    b = wsum64(b);
    if ((threadIdx.x & 63) == 0) {
        if (a) atomicAdd(&out2[0], a);
        if (b) atomicAdd(&out2[1], b);
    }
}

/* every source's overflow pairs added into the slice */
__global__ void __launch_bounds__(256)
k_route_overflow(const uint32_t *recv, const unsigned long long *rd, uint32_t np, uint32_t *out,
                 unsigned long long *stats, uint32_t *vck) {
    const uint32_t *blob = recv + rd[blockIdx.x];
    const uint64_t ne = blob[0] | ((uint64_t)blob[1] << 32), no = blob[2] | ((uint64_t)blob[3] << 32);
    const uint32_t *op = blob + RT_HDR + np + ne;
    uint32_t ck = threadIdx.x == 0 ? blob[0] + blob[1] + blob[2] + blob[3] : 0u;   /* (the header) */
    for (uint64_t i = threadIdx.x; i < no; i += 256u) ck += op[2 * i] + op[2 * i + 1];
    ck = wsum32(ck);
    if ((threadIdx.x & 63) == 0 && ck) atomicAdd(&vck[blockIdx.x], ck);
    for (uint64_t i = threadIdx.x; i < no; i += 256u) {
        const uint32_t old = atomicAdd(&out[op[2 * i]], op[2 * i + 1]);
        if (stats) {
            atomicAdd(&stats[0], (unsigned long long)op[2 * i + 1]);
            if (old == 0) atomicAdd(&stats[1], 1ull);
        }
    }
}

/* the owners' geometry for (nbins, world) on the host */
struct RouteHost {
    uint64_t S = 0, nslots = 0;
    uint32_t nparts = 0;
    std::vector<unsigned long long> p0, sb, np;
};
RouteHost route_geometry(uint64_t nbins, int world) {
    RouteHost h;
    h.S = merge_table_words(nbins, world) / (uint64_t)world;
    h.nparts = (uint32_t)(nbins >> RT_SH);
    h.p0.assign(world, 0);
    h.sb.assign(world + 1, 0);
    h.np.assign(world, 0);
    for (int d = 0; d < world; d++) {
        const uint64_t a = (uint64_t)d * h.S, z = std::min<uint64_t>((uint64_t)(d + 1) * h.S, nbins);
        if (a < z) {
            h.p0[d] = a >> RT_SH;
            h.np[d] = ((z - 1) >> RT_SH) - h.p0[d] + 1;
        } else {
            h.p0[d] = h.nparts;
        }
        h.sb[d + 1] = h.sb[d] + h.np[d];
    }
    h.nslots = h.sb[world];
    return h;
}

/* fk_engine_route_pack: the finished table's blobs, one per destination,
   side by side in e->d_rsend (words[d] each) */
int route_pack(fk_engine *e, int world, bool counting, uint64_t *words) {
    if (e->sparse || e->k < 8 || world < 1) return FK_E_INVALID;
    const RouteHost h = route_geometry(e->nbins, world);
    if (h.S < (1ull << RT_SH)) return FK_E_INVALID;   /* (a part spans at most two owners) */
    const uint64_t W = (uint64_t)world;
    const uint64_t naux = 7 * W + 1 + h.nslots + 1,
                   aux_bytes = naux * 8 + h.nslots * 4 + (uint64_t)h.nparts * 32 + W * 4 + 16;
    int rc = sp_ensure(&e->d_raux, &e->raux_cap, aux_bytes, 1);
    if (rc) return rc;
    unsigned long long *aux = static_cast<unsigned long long *>(e->d_raux);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(aux + naux), *wcnt = cnt + h.nslots,
             *ck = wcnt + (uint64_t)h.nparts * 8;
    std::vector<unsigned long long> ha(7 * W + 1, 0);
    for (int d = 0; d < world; d++) { ha[d] = h.p0[d]; ha[2 * W + 1 + d] = h.np[d]; }
    for (int d = 0; d <= world; d++) ha[W + d] = h.sb[d];
    HIPCHK(hipMemcpyAsync(aux, ha.data(), ha.size() * 8, hipMemcpyHostToDevice, e->stream));
    RouteGeo g{e->nbins, h.S, (uint32_t)world, h.nparts, aux, ck};
    hipLaunchKernelGGL(k_route_count, dim3(h.nparts), dim3(256), 0, e->stream, (const uint32_t *)e->d_table, g,
                       counting ? 1 : 0, cnt, wcnt);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, e->stream, (const uint32_t *)cnt, h.nslots,
                       aux + 7 * W + 1);
    HIPCHK(hipGetLastError());
    std::vector<unsigned long long> off(h.nslots + 1), no(W);
    HIPCHK(hipMemcpyAsync(off.data(), aux + 7 * W + 1, (h.nslots + 1) * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(no.data(), aux + 5 * W + 1, W * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t total = 0;
    for (int d = 0; d < world; d++) {
        const uint64_t ne = off[h.sb[d + 1]] - off[h.sb[d]];
        words[d] = RT_HDR + h.np[d] + ne + 2 * no[d] + RT_TRL;
        ha[3 * W + 1 + d] = total;   /* bb */
        ha[4 * W + 1 + d] = ne;      /* ne */
        total += words[d];
    }
    rc = sp_ensure((void **)&e->d_rsend, &e->rsend_cap, total, sizeof(uint32_t));
    if (rc) return rc;
    e->rsend_words = total;
    HIPCHK(hipMemcpyAsync(aux + 3 * W + 1, ha.data() + 3 * W + 1, 2 * W * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemsetAsync(aux + 6 * W + 1, 0, W * 8, e->stream));
    HIPCHK(hipMemsetAsync(ck, 0, W * 4, e->stream));
    hipLaunchKernelGGL(k_route_write, dim3(h.nparts), dim3(256), 0, e->stream, (const uint32_t *)e->d_table, g,
                       counting ? 1 : 0, (const uint32_t *)cnt, (const uint32_t *)wcnt,
                       reinterpret_cast<uint32_t *>(e->d_rsend));
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_seal, dim3(1), dim3(64), 0, e->stream, g, reinterpret_cast<uint32_t *>(e->d_rsend));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* fk_engine_route_absorb: the blobs received from every source (words[s]
   each, side by side at recv) into this rank's slice of the merged table */
int route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words, int32_t *slice,
                        unsigned long long *stats) {
    if (e->sparse || e->k < 8 || world < 1 || rank < 0 || rank >= world) return FK_E_INVALID;
    const RouteHost h = route_geometry(e->nbins, world);
    if (h.S < (1ull << RT_SH)) return FK_E_INVALID;
    const uint64_t np = h.np[rank];
    if (!np) return FK_OK;   /* (owns no bin) */
    const uint64_t W = (uint64_t)world;
    std::vector<unsigned long long> rd(W);
    uint64_t at = 0;
    for (int s = 0; s < world; s++) {
        rd[s] = at;
        if (words[s] < RT_HDR + np + RT_TRL) return FK_E_INVALID;
        at += words[s];
    }
    /* every blob's header against its size */
    std::vector<uint32_t> hdr(4 * W);
    for (int s = 0; s < world; s++)
        HIPCHK(hipMemcpyAsync(&hdr[4 * s], recv + rd[s], 16, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int s = 0; s < world; s++) {
        const uint64_t ne = hdr[4 * s] | ((uint64_t)hdr[4 * s + 1] << 32),
                       no = hdr[4 * s + 2] | ((uint64_t)hdr[4 * s + 3] << 32);
        if (RT_HDR + np + ne + 2 * no + RT_TRL != words[s]) return FK_E_RCCL;   /* (a header that does not fit) */
    }
    const uint64_t aux_bytes = (W + W * (np + 1) + 2 * RT_STAT_SLOTS) * 8 + W * 4 + 16;
    int rc = sp_ensure(&e->d_raux, &e->raux_cap, aux_bytes, 1);
    if (rc) return rc;
    unsigned long long *drd = static_cast<unsigned long long *>(e->d_raux), *roff = drd + W,
                       *sslots = roff + W * (np + 1);
    uint32_t *vck = reinterpret_cast<uint32_t *>(sslots + 2 * RT_STAT_SLOTS), *bad = vck + W;
    HIPCHK(hipMemsetAsync(vck, 0, W * 4 + 4, e->stream));
    if (stats) HIPCHK(hipMemsetAsync(sslots, 0, 2 * RT_STAT_SLOTS * 8, e->stream));
    HIPCHK(hipMemcpyAsync(drd, rd.data(), W * 8, hipMemcpyHostToDevice, e->stream));
    const uint32_t *r32 = reinterpret_cast<const uint32_t *>(recv);
    for (int s = 0; s < world; s++) {
        hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, e->stream, r32 + rd[s] + RT_HDR, np,
                           roff + (uint64_t)s * (np + 1));
        HIPCHK(hipGetLastError());
    }
    const uint64_t lo = (uint64_t)rank * h.S, hi = std::min<uint64_t>(lo + h.S, e->nbins);
    HIPCHK(hipFuncSetAttribute((const void *)k_route_absorb, hipFuncAttributeMaxDynamicSharedMemorySize, 1 << 17));
    uint32_t *out = reinterpret_cast<uint32_t *>(slice);
    hipLaunchKernelGGL(k_route_absorb, dim3((uint32_t)np), dim3(1024), (size_t)1 << 17, e->stream, r32,
                       (const unsigned long long *)drd, (const unsigned long long *)roff, (uint32_t)world, (uint32_t)np,
                       (uint64_t)h.p0[rank], lo, hi, out, stats ? sslots : nullptr, vck);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_overflow, dim3((uint32_t)world), dim3(256), 0, e->stream, r32,
                       (const unsigned long long *)drd, (uint32_t)np, out, stats, vck);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_verify, dim3(1), dim3(64), 0, e->stream, r32, (const unsigned long long *)drd,
                       (uint32_t)np, (const uint32_t *)vck, (uint32_t)world, bad);
    HIPCHK(hipGetLastError());
    if (stats) {
        hipLaunchKernelGGL(k_route_stats, dim3(1), dim3(256), 0, e->stream, (const unsigned long long *)sslots, stats);
        HIPCHK(hipGetLastError());
    }
    uint32_t hbad = 0;
    HIPCHK(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return hbad ? FK_E_RCCL : FK_OK;   /* a blob arrived short or corrupt */
}

extern "C" int fk_engine_route_pack(fk_engine *e, int world, int counting, uint64_t *words) {
    if (!e || !words) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    return route_pack(e, world, counting != 0, words);
}

extern "C" int fk_engine_route_copy(fk_engine *e, void *dst) {
    if (!e || !dst || !e->d_rsend) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(dst, e->d_rsend, e->rsend_words * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words,
                                      int32_t *slice) {
    if (!e || !recv || !words || !slice) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    return route_absorb(e, world, rank, recv, words, slice, nullptr);
}

/* the routed exchange over RCCL: blobs packed, their sizes all-reduced as a
   world x world matrix of 16-bit limbs, one grouped send/recv, the received
   blobs into this rank's slice */
int route_exchange(fk_engine *e, fk_comm *comm, bool counting, int32_t *slice, unsigned long long *stats) {
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    const uint64_t W = (uint64_t)world;
    std::vector<uint64_t> sw(W), rw(W), sd(W), rdsp(W);
    int rc = route_pack(e, world, counting, sw.data());
    if (rc) return rc;
    /* the size matrix in the engine's own buffer (a scratch allocation's
       hipFree synchronised the device inside the step) */
    const uint64_t nm = W * W * 3;
    rc = sp_ensure((void **)&e->d_rsz, &e->rsz_cap, nm, sizeof(int32_t));
    if (rc) return rc;
    std::vector<int32_t> hm(nm, 0);
    for (uint64_t d = 0; d < W; d++)
        for (int j = 0; j < 3; j++) hm[((uint64_t)rank * W + d) * 3 + j] = (int32_t)((sw[d] >> (16 * j)) & 0xFFFFu);
    HIPCHK(hipMemcpyAsync(e->d_rsz, hm.data(), nm * 4, hipMemcpyHostToDevice, e->stream));
    rc = fkc_allreduce_i32(comm, e->d_rsz, nm, e->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(hm.data(), e->d_rsz, nm * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t sat = 0, rat = 0;
    for (uint64_t s = 0; s < W; s++) {
        uint64_t v = 0;
        for (int j = 0; j < 3; j++) v |= (uint64_t)(uint32_t)hm[(s * W + (uint64_t)rank) * 3 + j] << (16 * j);
        rw[s] = v;
        rdsp[s] = rat;
        rat += v;
        sd[s] = sat;
        sat += sw[s];
    }
    rc = sp_ensure((void **)&e->d_rrecv, &e->rrecv_cap, rat, sizeof(int32_t));
    if (rc) return rc;
    /* the trailers cleared: each must arrive with its blob */
    for (uint64_t s = 0; s < W; s++)
        if (rw[s] >= RT_TRL)
            HIPCHK(hipMemsetAsync(e->d_rrecv + rdsp[s] + rw[s] - RT_TRL, 0, RT_TRL * sizeof(int32_t), e->stream));
    rc = fkc_alltoallv_i32(comm, e->d_rsend, sw.data(), sd.data(), e->d_rrecv, rw.data(), rdsp.data(), e->stream);
    if (rc) return rc;
    return route_absorb(e, world, rank, e->d_rrecv, rw.data(), slice, stats);
}

int stitched_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *first_end_out, bool scatter) {
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    const uint64_t tw = merge_table_words(e->nbins, world);
    const uint32_t nrow = (uint32_t)world * FK_PACK_ROW_WORDS;
    int rc = shard_full_tf(e);
    if (rc) return rc;
    if (e->shard_len == 0) {
        const TF id = fk_identity();
        HIPCHK(hipMemcpyAsync(e->d_tf, &id, sizeof id, hipMemcpyHostToDevice, e->stream));
    }
    hipLaunchKernelGGL(k_fill_row, dim3(1), dim3(64), 0, e->stream, e->d_rows, world, rank,
                       reinterpret_cast<const uint32_t *>(e->d_tf), (uint32_t)(sizeof(TF) / 4), 0u);
    HIPCHK(hipGetLastError());
    rc = fkc_allreduce_i32(comm, reinterpret_cast<int32_t *>(e->d_rows), nrow, e->stream);
    if (rc) return rc;
    rc = rows_fetch(e, e->d_rows, nrow);
    if (rc) return rc;
    XState s{0, 0, 0, 0}, in = s;   /* from the stream's initial state */
    for (int r = 0; r < world; r++) {
        TF t;
        memcpy(&t, e->h_rows + 32 + (size_t)r * FK_PACK_ROW_WORDS, sizeof t);
        if (r == rank) in = s;
        s = fk_apply(t, s);
    }
    fk_state ent{in.R, fk_sigma(in.code), in.hdr, 0};
    rc = fk_engine_resolve(e, &ent);
    if (rc) return rc;
    fk_result res;
    rc = fk_engine_finish(e, &res);
    if (rc != FK_OK && rc != FK_E_ROLLOVER && rc != FK_E_UNTERMINATED_HEADER && rc != FK_E_EMPTY) return rc;
    /* where the stream ends */
    hipLaunchKernelGGL(k_fill_row, dim3(1), dim3(64), 0, e->stream, e->d_rows, world, rank, (const uint32_t *)nullptr,
                       0u, res.hit_eof_byte ? 1u : 0u);
    HIPCHK(hipGetLastError());
    rc = fkc_allreduce_i32(comm, reinterpret_cast<int32_t *>(e->d_rows), nrow, e->stream);
    if (rc) return rc;
    rc = rows_fetch(e, e->d_rows, nrow);
    if (rc) return rc;
    int first_end = -1;
    for (int r = 0; r < world && first_end < 0; r++)
        if (e->h_rows[32 + (size_t)r * FK_PACK_ROW_WORDS]) first_end = r;
    const bool counting = first_end < 0 || rank <= first_end;
    const int last = first_end >= 0 ? first_end : world - 1;
    /* the table and the counters (fk_engine_finish's values, as 16-bit limbs) */
    uint64_t v[FK_PACK_COUNTERS] = {};
    if (counting) {
        v[0] = res.windows; v[1] = res.valid_bases;
        for (int b = 0; b < 4; b++) { v[2 + b] = res.base_count[b]; v[6 + b] = res.depth1[b]; }
        v[10] = res.unknown_chars; v[11] = res.scanned_bytes;
        v[12] = rank == first_end ? 1u : 0u;
        v[13] = rank == last ? (uint64_t)res.unterminated_header : 0u;
    }
    /* the reduce-scatter reads the engine's own table when its blocks divide
       it exactly (a power-of-two world): no copy of the whole table into
       the merge buffer first (k = 16: 16 GiB, ~5 ms per step); a rank whose
       shard the stream never reached sends zeros (its table, zeroed: the
       engine's count is discarded anyway) */
    const bool route = scatter && e->k >= FK_ROUTE_KMIN && fkc_has_alltoallv(comm) &&
                       (e->route_mode == 2 || (e->route_mode == 1 && world > 1));
    const bool direct = scatter && tw == e->nbins;
    if (route) {
        /* (the table stays where it is: route_pack reads it) */
    } else if (direct) {
        if (!counting) HIPCHK(hipMemsetAsync(e->d_table, 0, e->nbins * sizeof(uint32_t), e->stream));
    } else if (counting) {
        HIPCHK(hipMemcpyAsync(merge, e->d_table, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    } else {
        HIPCHK(hipMemsetAsync(merge, 0, e->nbins * sizeof(uint32_t), e->stream));
    }
    if (!route && !direct && tw > e->nbins)
        HIPCHK(hipMemsetAsync(merge + e->nbins, 0, (tw - e->nbins) * sizeof(uint32_t), e->stream));
    uint32_t *limbs = e->h_rows + 32 + e->rows_cap;   /* pinned staging */
    for (int i = 0; i < FK_PACK_COUNTERS; i++)
        for (int j = 0; j < 4; j++) limbs[4 * i + j] = (uint32_t)((v[i] >> (16 * j)) & 0xFFFFu);
    for (int j = 0; j < FK_PACK_STATS; j++) limbs[4 * FK_PACK_COUNTERS + j] = 0;
    HIPCHK(hipMemcpyAsync(merge + tw, limbs, (4 * FK_PACK_COUNTERS + FK_PACK_STATS) * sizeof(uint32_t),
                          hipMemcpyHostToDevice, e->stream));
    if (scatter) {
        /* the table sharded by its top index bits (the first bases): rank r
           keeps bins [r * S, (r + 1) * S) of the sum, S = tw / world; the
           counters and every slice's (sum, distinct) are all-reduced */
        const uint64_t S = tw / (uint64_t)world;
        HIPCHK(hipMemsetAsync(e->d_tmp, 0, 2 * sizeof(unsigned long long), e->stream));
        if (route) {   /* (the slice's total and nonzero bins as it is absorbed) */
            rc = route_exchange(e, comm, counting, merge + (uint64_t)rank * S, e->d_tmp);
        } else {
            rc = direct ? fkc_reduce_scatter_from_i32(comm, reinterpret_cast<const int32_t *>(e->d_table), merge, S,
                                                      e->stream)
                        : fkc_reduce_scatter_i32(comm, merge, S, e->stream);
        }
        if (rc) return rc;
        const uint64_t lo = (uint64_t)rank * S, n = lo < e->nbins ? std::min(S, e->nbins - lo) : 0;
        if (n && !route) {
            const unsigned gr = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 8, (n + 1023) / 1024);
            hipLaunchKernelGGL(k_slice_sum, dim3(gr), dim3(256), 0, e->stream,
                               reinterpret_cast<const uint32_t *>(merge) + lo, n, e->d_tmp);
        }
        hipLaunchKernelGGL(k_slice_limbs, dim3(1), dim3(64), 0, e->stream, e->d_tmp,
                           merge + tw + 4 * FK_PACK_COUNTERS);
        HIPCHK(hipGetLastError());
        rc = fkc_allreduce_i32(comm, merge + tw, 4 * FK_PACK_COUNTERS + FK_PACK_STATS, e->stream);
    } else {
        rc = fkc_reduce_i32(comm, merge, tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS, 0, e->stream);
    }
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (first_end_out) *first_end_out = first_end;
    return FK_OK;
}

extern "C" int fk_engine_shard_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *info) {
    if (!e || !comm || !merge) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;
    if (!e->shard_pending) return FK_E_STATE;
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    if (fkc_device(comm) != e->dev) return FK_E_INVALID;
    const int32_t flags = info ? info[0] : FK_XCHG_FAST;
    const bool try_fast = (flags & FK_XCHG_FAST) != 0;
    const bool scatter = (flags & FK_XCHG_SHARD_TABLE) != 0;
    int rc = set_dev(e);
    if (rc) return rc;
    const uint32_t nrow = (uint32_t)world * FK_PACK_ROW_WORDS;
    rc = ensure_rows(e, nrow);
    if (rc) return rc;
    const uint64_t tw = merge_table_words(e->nbins, world);
    if (try_fast) {
        /* one collective: pack, all-reduce table + counters + rows, compose */
        int32_t *stats = merge + tw + 4 * FK_PACK_COUNTERS;
        uint32_t *rows = reinterpret_cast<uint32_t *>(stats + FK_PACK_STATS);
        rc = fk_engine_shard_pack(e, reinterpret_cast<uint32_t *>(merge), merge + tw, rows, world, rank,
                                  rank == world - 1);
        if (rc) return rc;
        if (tw > e->nbins) HIPCHK(hipMemsetAsync(merge + e->nbins, 0, (tw - e->nbins) * sizeof(uint32_t), e->stream));
        HIPCHK(hipMemsetAsync(stats, 0, FK_PACK_STATS * sizeof(int32_t), e->stream));
        if (flags & FK_XCHG_TEST_INVALID)   /* tests: this rank's pack row reads as invalid */
            HIPCHK(hipMemsetAsync(rows + (size_t)rank * FK_PACK_ROW_WORDS + 24, 0, sizeof(uint32_t), e->stream));
        rc = fkc_allreduce_i32(comm, merge, tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS + nrow, e->stream);
        if (rc) return rc;
        rc = rows_fetch(e, rows, nrow);
        if (rc) return rc;
        fk_state st;
        rc = fk_shard_rows_compose(e->h_rows + 32, world, rank, &st);
        if (rc == FK_OK) {
            rc = fk_engine_resolve(e, &st);
            if (rc) return rc;
            if (info) { info[0] = 1; info[1] = -1; }
            return FK_OK;
        }
        if (rc != FK_E_SUMMARY) return rc;
        /* some guess did not hold (every rank sees it): stitched, below */
    }
    int32_t first_end = -1;
    rc = stitched_exchange(e, comm, merge, &first_end, scatter);
    if (rc) return rc;
    if (info) { info[0] = 0; info[1] = first_end; }
    return FK_OK;
}

extern "C" int fk_merge_layout(int k, int world, uint64_t *table_words, uint64_t *total_words) {
    if (k < FK_K_MIN || k > FK_K_MAX_DENSE || world < 1) return FK_E_INVALID;
    const uint64_t tw = merge_table_words(1ull << (2 * k), world);
    if (table_words) *table_words = tw;
    if (total_words)
        *total_words = tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS + (uint64_t)world * FK_PACK_ROW_WORDS;
    return FK_OK;
}

extern "C" int fk_engine_stream(fk_engine *e, void **stream) {
    if (!e || !stream) return FK_E_INVALID;
    *stream = (void *)e->stream;
    return FK_OK;
}

extern "C" int fk_shard_rows_compose(const uint32_t *rows, int world, int rank, fk_state *entering) {
    if (!rows || world < 1 || rank < 0 || rank >= world || !entering) return FK_E_INVALID;
    XState s{0, 0, 0, 0};   /* the stream's initial state */
    XState mine = s;
    for (int r = 0; r < world; r++) {
        const uint32_t *row = rows + (size_t)r * FK_PACK_ROW_WORDS;
        if (row[24] != 1u) return FK_E_SUMMARY;
        fk_summary sm;
        for (int j = 0; j < 12; j++) sm.w[j] = (uint64_t)row[2 * j] | ((uint64_t)row[2 * j + 1] << 32);
        if (sm.w[11] != FK_SUMMARY_COMPACT || sm.w[9] != 0) return FK_E_SUMMARY;
        if (r == rank) mine = s;
        XState y;
        if (!compact_apply(&sm, s, y)) return FK_E_SUMMARY;
        s = y;
    }
    entering->run = mine.R;
    entering->code = fk_sigma(mine.code);
    entering->hdr = mine.hdr;
    entering->ended = 0;
    return FK_OK;
}

/* 17 <= k <= 20 over the library's communicator (round 6; the all-to-all
 * had gone through torch.distributed, a stream gap per collective): this
 * rank's finished sparse table cut at the owners' bounds (each owner's runs
 * are contiguous: the keys ascend), the world x world run counts all-reduced
 * as 16-bit limbs, the keys (two words each) and the counts sent to their
 * owners by grouped ncclSend / ncclRecv (a rank's own runs by a device copy),
 * the received sorted runs merged (fk_engine_sparse_adopt: merge path,
 * equal keys summed), then the caller's counter limbs -- `limbs`, device,
 * FK_PACK_COUNTERS x 4 16-bit limbs already in place -- completed with the
 * slice's (total, distinct) and all-reduced, all on the engine's stream.
 * counting = 0: a rank the stream never reached (sends nothing). */
extern "C" int fk_engine_sparse_exchange(fk_engine *e, fk_comm *comm, int counting, int32_t *limbs,
                                         uint64_t *stats) {
    if (!e || !comm || !limbs || !stats) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    if (fkc_device(comm) != e->dev) return FK_E_INVALID;
    if (!fkc_has_alltoallv(comm)) return FK_E_RCCL;
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    const uint64_t W = (uint64_t)world;
    int rc = set_dev(e);
    if (rc) return rc;
    std::vector<uint64_t> cnt(W, 0), rw(W), sd(W), rdsp(W), w2(W), sd2(W), rw2(W), rdsp2(W);
    if (counting) {
        rc = fk_engine_sparse_split(e, world, cnt.data());
        if (rc) return rc;
    }
    const uint64_t nm = W * W * 4;
    rc = sp_ensure((void **)&e->d_rsz, &e->rsz_cap, nm, sizeof(int32_t));
    if (rc) return rc;
    std::vector<int32_t> hm(nm, 0);
    for (uint64_t d = 0; d < W; d++)
        for (int j = 0; j < 4; j++) hm[((uint64_t)rank * W + d) * 4 + j] = (int32_t)((cnt[d] >> (16 * j)) & 0xFFFFu);
    HIPCHK(hipMemcpyAsync(e->d_rsz, hm.data(), nm * 4, hipMemcpyHostToDevice, e->stream));
    rc = fkc_allreduce_i32(comm, e->d_rsz, nm, e->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(hm.data(), e->d_rsz, nm * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t m = 0, at = 0;
    for (uint64_t s = 0; s < W; s++) {
        uint64_t v = 0;
        for (int j = 0; j < 4; j++) v |= (uint64_t)(uint32_t)hm[(s * W + (uint64_t)rank) * 4 + j] << (16 * j);
        rw[s] = v;
        rdsp[s] = m;
        m += v;
        sd[s] = at;
        at += cnt[s];
        w2[s] = 2 * cnt[s]; sd2[s] = 2 * sd[s]; rw2[s] = 2 * rw[s]; rdsp2[s] = 2 * rdsp[s];
    }
    rc = sp_ensure((void **)&e->d_rrecv, &e->rrecv_cap, 3 * m + 2, sizeof(int32_t));
    if (rc) return rc;
    int32_t *rk = e->d_rrecv, *rcnt = e->d_rrecv + 2 * m;
    rc = fkc_alltoallv_i32(comm, reinterpret_cast<const int32_t *>(e->d_spk), w2.data(), sd2.data(), rk, rw2.data(),
                           rdsp2.data(), e->stream);
    if (!rc) rc = fkc_alltoallv_i32(comm, reinterpret_cast<const int32_t *>(e->d_spc), cnt.data(), sd.data(), rcnt,
                                    rw.data(), rdsp.data(), e->stream);
    if (rc) return rc;
    /* (the table the sends read is replaced next: let them finish first) */
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t st[2] = {0, 0};
    rc = fk_engine_sparse_adopt(e, reinterpret_cast<const uint64_t *>(rk), reinterpret_cast<const uint32_t *>(rcnt), m,
                                st);
    if (rc) return rc;
    /* the slice's (total, distinct) as limbs after the counters' */
    int32_t sl[FK_PACK_STATS];
    for (int j = 0; j < 4; j++) {
        sl[j] = (int32_t)((st[1] >> (16 * j)) & 0xFFFFu);
        sl[4 + j] = (int32_t)((st[0] >> (16 * j)) & 0xFFFFu);
    }
    HIPCHK(hipMemcpyAsync(limbs + 4 * FK_PACK_COUNTERS, sl, sizeof sl, hipMemcpyHostToDevice, e->stream));
    rc = fkc_allreduce_i32(comm, limbs, 4 * FK_PACK_COUNTERS + FK_PACK_STATS, e->stream);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    stats[0] = st[0];
    stats[1] = st[1];
    return FK_OK;
}
