/*
 * chunk_probe: the memory side of k = 11's partition round trip, measured in
 * isolation (no tile work): how fast the sorted codes can be written and read
 * back in two layouts.
 *
 *   rows   (today): each k_part batch is one contiguous 128 KiB row of 512
 *          runs of ~256 B; k_bucket_count's block for slice s reads run s of
 *          every row (one 256-B piece per 128 KiB).
 *   chunks (candidate): each (block, slice) appends its runs to 4 KiB chunks
 *          taken from a pool; k_bucket_count's block for slice s reads its
 *          chunks whole.
 *
 * Every kernel counts the codes it reads into LDS bins (one atomic per code)
 * as k_bucket_count does, so the read probes carry the same LDS load.
 * Build: hipcc --offload-arch=gfx950 -O3 tools/chunk_probe.hip -o /tmp/chunk_probe
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <random>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint4 rnd4(uint32_t a, uint32_t b) {
    const uint32_t h = mix(a * 0x9E3779B9u + b);
    return make_uint4(mix(h + 1), mix(h + 2), mix(h + 3), mix(h + 4));
}
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static const uint32_t NSLICE = 512, RUN = 128 /* codes */, ROWB = NSLICE * RUN * 2 /* 128 KiB */;
static const uint32_t CHUNK = 4096 /* bytes */, RUNS_PER_CHUNK = CHUNK / (RUN * 2);

/* rows layout write: block b writes its rows [b*R, (b+1)*R) contiguously */
__global__ void __launch_bounds__(1024) w_rows(uint4 *codes, uint32_t rows_per_block) {
    const uint64_t row0 = (uint64_t)blockIdx.x * rows_per_block;
    for (uint32_t r = 0; r < rows_per_block; r++) {
        uint4 *dst = codes + (row0 + r) * (ROWB / 16);
        for (uint32_t i = threadIdx.x; i < ROWB / 16; i += blockDim.x)
            dst[i] = rnd4((uint32_t)(row0 + r), i);
    }
}

/* chunk layout write: block b, batch r: slice s's run goes to chunk
   chunk_of[(b * NSLICE + s) * cpb + r / RUNS_PER_CHUNK] at piece r % RUNS_PER_CHUNK */
__global__ void __launch_bounds__(1024) w_chunks(uint4 *codes, uint32_t rows_per_block, const uint32_t *chunk_of,
                                                  uint32_t cpb) {
    const uint32_t lane16 = threadIdx.x & 15, grp = threadIdx.x >> 4;   /* 16 lanes per 256-B run */
    for (uint32_t r = 0; r < rows_per_block; r++) {
        for (uint32_t s = grp; s < NSLICE; s += blockDim.x / 16) {
            const uint32_t c = chunk_of[((uint64_t)blockIdx.x * NSLICE + s) * cpb + r / RUNS_PER_CHUNK];
            uint4 *dst = codes + (uint64_t)c * (CHUNK / 16) + (r % RUNS_PER_CHUNK) * (RUN * 2 / 16);
            dst[lane16] = rnd4(blockIdx.x * 4096u + r, s * 16u + lane16);
        }
    }
}

__device__ __forceinline__ void add8(uint32_t *bins, const uint4 &v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 8; h++) atomicAdd(&bins[(w[h >> 1] >> (16 * (h & 1))) & 0x7FFFu], 1u);
}

/* rows layout read: block per slice (XCD-consecutive), a quad per run,
   2 rows per quad at once, 4 pieces of 16 B per lane (a 256-B run) */
__global__ void __launch_bounds__(1024) r_rows(const uint4 *codes, uint64_t nrows, uint32_t *out) {
    extern __shared__ uint32_t bins[];
    const uint32_t s = (blockIdx.x & 7u) * (NSLICE / 8) + (blockIdx.x >> 3);
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    const uint32_t sub = threadIdx.x & 3, quads = blockDim.x / 4;
    for (uint64_t r = threadIdx.x / 4; r < nrows; r += 2 * quads) {
        uint4 v[2][4];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint64_t rr = r + j * quads;
            const uint4 *p = codes + rr * (ROWB / 16) + s * (RUN * 2 / 16) + sub;
#pragma unroll
            for (int u = 0; u < 4; u++) v[j][u] = rr < nrows ? p[4 * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int u = 0; u < 4; u++) add8(bins, v[j][u]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) out[(uint64_t)blockIdx.x * 40960 + i] = bins[i];
}

/* chunk layout read: block per slice, a wave per chunk (4 x 1 KiB), two
   chunks in flight per wave */
__global__ void __launch_bounds__(1024) r_chunks(const uint4 *codes, const uint32_t *list, uint32_t per_slice,
                                                  uint32_t *out) {
    extern __shared__ uint32_t bins[];
    const uint32_t s = (blockIdx.x & 7u) * (NSLICE / 8) + (blockIdx.x >> 3);
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x / 64;
    const uint32_t *mine = list + (uint64_t)s * per_slice;
    for (uint32_t c = wv; c < per_slice; c += 2 * nw) {
        uint4 v[2][4];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint32_t cc = c + j * nw;
            const uint4 *p = codes + (uint64_t)(cc < per_slice ? mine[cc] : 0) * (CHUNK / 16) + lane;
#pragma unroll
            for (int u = 0; u < 4; u++) v[j][u] = cc < per_slice ? p[64 * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int u = 0; u < 4; u++) add8(bins, v[j][u]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) out[(uint64_t)blockIdx.x * 40960 + i] = bins[i];
}


/* rows layout, as k_bucket_count<BK_PAD> reads it: run (row, slice) at the
   16-B piece idx >> 16 of its row, idx & 0xFFFF + 1 codes (variable), rows of
   ROWB + 16 * NSLICE bytes; QL lanes per run, RR rows per quad at once, U
   pieces per lane, index words one iteration ahead */
template <int QL, int RR, int U>
__global__ void __launch_bounds__(1024) r_rows_idx(const uint4 *codes, const uint32_t *idx, uint64_t nrows,
                                                    uint32_t rowp, uint32_t *out) {
    extern __shared__ uint32_t bins[];
    const uint32_t s = (blockIdx.x & 7u) * (NSLICE / 8) + (blockIdx.x >> 3);
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    const uint32_t sub = threadIdx.x & (QL - 1), runs = blockDim.x / QL;
    uint32_t en[RR];
    const uint64_t r00 = threadIdx.x / QL;
#pragma unroll
    for (int j = 0; j < RR; j++) en[j] = r00 + j * runs < nrows ? idx[(r00 + j * runs) * NSLICE + s] : 0xFFFFFFFFu;
    for (uint64_t r = r00; r < nrows; r += RR * runs) {
        uint32_t e[RR];
#pragma unroll
        for (int j = 0; j < RR; j++) e[j] = en[j];
        const uint64_t rn = r + RR * runs;
#pragma unroll
        for (int j = 0; j < RR; j++) en[j] = rn + j * runs < nrows ? idx[(rn + j * runs) * NSLICE + s] : 0xFFFFFFFFu;
        uint4 v[RR][U];
        uint32_t np[RR], last[RR];
#pragma unroll
        for (int j = 0; j < RR; j++) {
            const uint32_t c = e[j] == 0xFFFFFFFFu ? 0u : (e[j] & 0xFFFFu) + 1u;
            np[j] = (c + 7u) >> 3;
            last[j] = c & 7u;
            const uint4 *p = codes + (r + j * runs) * rowp + (e[j] >> 16) + sub;
#pragma unroll
            for (int u = 0; u < U; u++) v[j][u] = sub + QL * u < np[j] ? p[QL * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < RR; j++)
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t q = sub + QL * u;
                if (q < np[j]) {
                    const uint32_t nv = q + 1 == np[j] && last[j] ? last[j] : 8u;
                    const uint32_t w[4] = {v[j][u].x, v[j][u].y, v[j][u].z, v[j][u].w};
#pragma unroll
                    for (int h = 0; h < 8; h++)
                        if ((uint32_t)h < nv) atomicAdd(&bins[(w[h >> 1] >> (16 * (h & 1))) & 0x7FFFu], 1u);
                }
            }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 40960; i += blockDim.x) out[(uint64_t)blockIdx.x * 40960 + i] = bins[i];
}

int main(int argc, char **argv) {
    const uint64_t GB = argc > 1 ? strtoull(argv[1], 0, 10) : 10;   /* codes bytes, GB */
    const uint32_t blocks = 256;
    const uint64_t total = GB * 1000000000ull;
    const uint32_t rows_per_block = (uint32_t)(total / ROWB / blocks) / RUNS_PER_CHUNK * RUNS_PER_CHUNK;
    const uint64_t nrows = (uint64_t)rows_per_block * blocks;
    const uint64_t bytes = nrows * ROWB;
    const uint32_t cpb = rows_per_block / RUNS_PER_CHUNK;           /* chunks per (block, slice) */
    const uint64_t nchunks = bytes / CHUNK;
    printf("codes %.3f GB, rows %llu, chunks %llu (%u per block-slice)\n", bytes / 1e9, (unsigned long long)nrows,
           (unsigned long long)nchunks, cpb);
    uint4 *codes;
    uint32_t *out, *chunk_of, *list;
    CHK(hipMalloc(&codes, bytes));
    CHK(hipMalloc(&out, (size_t)NSLICE * 40960 * 4));
    std::vector<uint32_t> perm(nchunks);
    for (uint64_t i = 0; i < nchunks; i++) perm[i] = (uint32_t)i;
    std::mt19937_64 rng(1);
    std::shuffle(perm.begin(), perm.end(), rng);
    /* chunk_of[(b, s, j)] = perm[...]; list[s][b * cpb + j] the same ids */
    std::vector<uint32_t> lst((size_t)NSLICE * blocks * cpb);
    for (uint32_t b = 0; b < blocks; b++)
        for (uint32_t s = 0; s < NSLICE; s++)
            for (uint32_t j = 0; j < cpb; j++)
                lst[((size_t)s * blocks + b) * cpb + j] = perm[((size_t)b * NSLICE + s) * cpb + j];
    CHK(hipMalloc(&chunk_of, perm.size() * 4));
    CHK(hipMalloc(&list, lst.size() * 4));
    CHK(hipMemcpy(chunk_of, perm.data(), perm.size() * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(list, lst.data(), lst.size() * 4, hipMemcpyHostToDevice));
    CHK(hipFuncSetAttribute((const void *)r_rows, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
    CHK(hipFuncSetAttribute((const void *)r_chunks, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto timeit = [&](const char *name, auto &&launch) {
        float best = 1e9, sum = 0;
        for (int it = 0; it < 6; it++) {
            CHK(hipEventRecord(a));
            launch();
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (it) { best = std::min(best, ms); sum += ms; }
        }
        printf("%-10s best %.3f ms avg %.3f ms  %.2f TB/s\n", name, best, sum / 5, bytes / (best * 1e-3) / 1e12);
        fflush(stdout);
    };
    timeit("w_rows", [&] { hipLaunchKernelGGL(w_rows, dim3(blocks), dim3(1024), 0, 0, codes, rows_per_block); });
    timeit("r_rows", [&] { hipLaunchKernelGGL(r_rows, dim3(NSLICE), dim3(1024), 163840, 0, codes, nrows, out); });
    timeit("w_chunks", [&] {
        hipLaunchKernelGGL(w_chunks, dim3(blocks), dim3(1024), 0, 0, codes, rows_per_block, chunk_of, cpb);
    });
    timeit("r_chunks", [&] {
        hipLaunchKernelGGL(r_chunks, dim3(NSLICE), dim3(1024), 163840, 0, codes, list, blocks * cpb, out);
    });
    /* realistic rows: ROWB + 16 * NSLICE bytes per row; run lengths around 128 codes (a 64K-entry batch
       over 512 slices, multinomial), padded to 16-B pieces */
    {
        const uint32_t rowp = (ROWB + 16 * NSLICE) / 16;       /* pieces per row */
        const uint64_t nr = bytes / ((uint64_t)rowp * 16);
        std::vector<uint32_t> ix(nr * NSLICE);
        std::mt19937_64 g(7);
        std::vector<uint32_t> cnt(NSLICE);
        for (uint64_t r = 0; r < nr; r++) {
            for (uint32_t b = 0; b < NSLICE; b++) cnt[b] = RUN - 11 + (uint32_t)(g() % 23);   /* ~ binomial spread */
            uint32_t at = 0;
            for (uint32_t b = 0; b < NSLICE; b++) {
                ix[r * NSLICE + b] = cnt[b] ? (at << 16) | (cnt[b] - 1) : 0xFFFFFFFFu;
                at += (cnt[b] + 7) / 8;
            }
        }
        uint32_t *didx;
        CHK(hipMalloc(&didx, ix.size() * 4));
        CHK(hipMemcpy(didx, ix.data(), ix.size() * 4, hipMemcpyHostToDevice));
        CHK(hipFuncSetAttribute((const void *)r_rows_idx<4, 2, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        CHK(hipFuncSetAttribute((const void *)r_rows_idx<8, 2, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        CHK(hipFuncSetAttribute((const void *)r_rows_idx<4, 3, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        CHK(hipFuncSetAttribute((const void *)r_rows_idx<16, 2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        CHK(hipFuncSetAttribute((const void *)r_rows_idx<4, 4, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        timeit("idx q4r2u5", [&] { hipLaunchKernelGGL((r_rows_idx<4, 2, 5>), dim3(NSLICE), dim3(1024), 163840, 0, codes, didx, nr, rowp, out); });
        timeit("idx q8r2u3", [&] { hipLaunchKernelGGL((r_rows_idx<8, 2, 3>), dim3(NSLICE), dim3(1024), 163840, 0, codes, didx, nr, rowp, out); });
        timeit("idx q4r3u5", [&] { hipLaunchKernelGGL((r_rows_idx<4, 3, 5>), dim3(NSLICE), dim3(1024), 163840, 0, codes, didx, nr, rowp, out); });
        timeit("idx q16r2u2", [&] { hipLaunchKernelGGL((r_rows_idx<16, 2, 2>), dim3(NSLICE), dim3(1024), 163840, 0, codes, didx, nr, rowp, out); });
        timeit("idx q4r4u5", [&] { hipLaunchKernelGGL((r_rows_idx<4, 4, 5>), dim3(NSLICE), dim3(1024), 163840, 0, codes, didx, nr, rowp, out); });
    }
    CHK(hipDeviceSynchronize());
    return 0;
}
