// scatter_probe.hip — can k >= 8 windows be partitioned by their top 8 index
// bits at HBM speed?  1e9 pseudo-random 22-bit codes (k=11), 509 blocks:
//   A  LDS histogram of 256 buckets per block (pass A of the partition)
//   B  LDS cursor per bucket (ds_add with return) + scattered 2-byte store
//      of the low 14 bits into the bucket's contiguous region (pass B)
//   C  per-bucket count of 2-byte codes into a 16 Ki-bin LDS slice (pass C)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ unsigned code_of(unsigned long long i) {
    unsigned long long x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    return (unsigned)x & ((1u << 22) - 1);
}

__global__ void k_hist(unsigned long long n, unsigned long long per, unsigned *hist) {
    __shared__ unsigned h[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
    __syncthreads();
    unsigned long long b0 = blockIdx.x * per, b1 = min(b0 + per, n);
    for (unsigned long long i = b0 + threadIdx.x; i < b1; i += blockDim.x) atomicAdd(&h[code_of(i) >> 14], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[blockIdx.x * 256 + i] = h[i];
}

__global__ void k_scatter(unsigned long long n, unsigned long long per, const unsigned *offs, unsigned short *out) {
    __shared__ unsigned cur[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) cur[i] = offs[blockIdx.x * 256 + i];
    __syncthreads();
    unsigned long long b0 = blockIdx.x * per, b1 = min(b0 + per, n);
    for (unsigned long long i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        unsigned c = code_of(i);
        unsigned p = atomicAdd(&cur[c >> 14], 1u);
        out[p] = (unsigned short)(c & 0x3FFF);
    }
}

/* B2: block-batched scatter: 16 Ki windows per batch counting-sorted by
   bucket in LDS, then written out bucket run by bucket run (coalesced) */
#define BT 512
#define PER 32
__global__ void __launch_bounds__(BT) k_scatter2(unsigned long long n, unsigned long long per, const unsigned *offs,
                                                 unsigned short *out) {
    __shared__ unsigned hist[256], start[256], cur[256], gcur[256];
    __shared__ unsigned short ent[BT * PER];
    __shared__ unsigned char bid[BT * PER];
    const unsigned t = threadIdx.x;
    if (t < 256) gcur[t] = offs[blockIdx.x * 256 + t];
    unsigned long long b0 = blockIdx.x * per, b1 = min(b0 + per, n);
    for (unsigned long long base = b0; base < b1; base += BT * PER) {
        if (t < 256) hist[t] = 0;
        __syncthreads();
        unsigned c[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) {
            unsigned long long i = base + (unsigned long long)j * BT + t;
            c[j] = i < b1 ? code_of(i) : 0xFFFFFFFFu;
            if (c[j] != 0xFFFFFFFFu) atomicAdd(&hist[c[j] >> 14], 1u);
        }
        __syncthreads();
        if (t < 64) {   /* exclusive scan of 256 counts by one wave */
            unsigned a0 = hist[4 * t], a1 = hist[4 * t + 1], a2 = hist[4 * t + 2], a3 = hist[4 * t + 3];
            unsigned s = a0 + a1 + a2 + a3, inc = s;
            for (int d = 1; d < 64; d <<= 1) { unsigned v = __shfl_up(inc, d, 64); if (t >= (unsigned)d) inc += v; }
            unsigned ex = inc - s;
            start[4 * t] = ex; start[4 * t + 1] = ex + a0; start[4 * t + 2] = ex + a0 + a1; start[4 * t + 3] = ex + a0 + a1 + a2;
            cur[4 * t] = ex; cur[4 * t + 1] = ex + a0; cur[4 * t + 2] = ex + a0 + a1; cur[4 * t + 3] = ex + a0 + a1 + a2;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; j++) {
            if (c[j] != 0xFFFFFFFFu) {
                unsigned b = c[j] >> 14;
                unsigned p = atomicAdd(&cur[b], 1u);
                ent[p] = (unsigned short)(c[j] & 0x3FFF);
                bid[p] = (unsigned char)b;
            }
        }
        __syncthreads();
        const unsigned tot = start[255] + hist[255];
        for (unsigned e = t; e < tot; e += BT) {
            unsigned b = bid[e];
            out[gcur[b] + (e - start[b])] = ent[e];
        }
        __syncthreads();
        if (t < 256) gcur[t] += hist[t];
    }
}

/* C2: bucket count with 16-byte loads */
__global__ void __launch_bounds__(1024) k_count2(const unsigned short *codes, const unsigned *bstart, unsigned *table) {
    __shared__ unsigned slice[1 << 14];
    for (int i = threadIdx.x; i < (1 << 14); i += blockDim.x) slice[i] = 0;
    __syncthreads();
    const unsigned b = blockIdx.x;
    unsigned long long s0 = bstart[b], s1 = bstart[b + 1];
    unsigned long long a0 = (s0 + 7) & ~7ull;   /* 16-B aligned body */
    for (unsigned long long i = s0 + threadIdx.x; i < min(a0, s1); i += blockDim.x) atomicAdd(&slice[codes[i]], 1u);
    unsigned long long a1 = a0 + ((s1 > a0 ? s1 - a0 : 0) & ~7ull);
    const uint4 *v = reinterpret_cast<const uint4 *>(codes + a0);
    for (unsigned long long q = threadIdx.x; q < (a1 - a0) / 8; q += blockDim.x) {
        uint4 w = v[q];
        unsigned x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int h = 0; h < 4; h++) { atomicAdd(&slice[x[h] & 0xFFFF], 1u); atomicAdd(&slice[x[h] >> 16], 1u); }
    }
    for (unsigned long long i = a1 + threadIdx.x; i < s1; i += blockDim.x) atomicAdd(&slice[codes[i]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < (1 << 14); i += blockDim.x) table[(b << 14) + i] = slice[i];
}

__global__ void k_count(const unsigned short *codes, const unsigned *bstart, unsigned *table) {
    __shared__ unsigned slice[1 << 14];
    for (int i = threadIdx.x; i < (1 << 14); i += blockDim.x) slice[i] = 0;
    __syncthreads();
    const unsigned b = blockIdx.x;
    for (unsigned long long i = bstart[b] + threadIdx.x; i < bstart[b + 1]; i += blockDim.x) atomicAdd(&slice[codes[i]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < (1 << 14); i += blockDim.x) table[(b << 14) + i] = slice[i];
}

int main() {
    const unsigned long long n = 1000000000ull;
    const int blocks = 509;
    const unsigned long long per = (n + blocks - 1) / blocks;
    unsigned *hist, *offs, *bstart, *table;
    unsigned short *codes;
    CHECK(hipMalloc(&hist, blocks * 256 * 4)); CHECK(hipMalloc(&offs, blocks * 256 * 4));
    CHECK(hipMalloc(&bstart, 257 * 4)); CHECK(hipMalloc(&table, (1u << 22) * 4));
    CHECK(hipMalloc(&codes, n * 2));
    hipEvent_t e[4];
    for (int i = 0; i < 4; i++) CHECK(hipEventCreate(&e[i]));
    for (int rep = 0; rep < 3; rep++) {
        CHECK(hipEventRecord(e[0]));
        hipLaunchKernelGGL(k_hist, dim3(blocks), dim3(512), 0, 0, n, per, hist);
        CHECK(hipEventRecord(e[1]));
        /* host scan (bucket-major, block-minor) */
        unsigned *h = (unsigned *)malloc(blocks * 256 * 4), *o = (unsigned *)malloc(blocks * 256 * 4), bs[257];
        CHECK(hipMemcpy(h, hist, blocks * 256 * 4, hipMemcpyDeviceToHost));
        unsigned long long acc = 0;
        for (int b = 0; b < 256; b++) { bs[b] = (unsigned)acc; for (int k = 0; k < blocks; k++) { o[k * 256 + b] = (unsigned)acc; acc += h[k * 256 + b]; } }
        bs[256] = (unsigned)acc;
        CHECK(hipMemcpy(offs, o, blocks * 256 * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(bstart, bs, 257 * 4, hipMemcpyHostToDevice));
        free(h); free(o);
        CHECK(hipEventRecord(e[2]));
        if (rep == 0) hipLaunchKernelGGL(k_scatter, dim3(blocks), dim3(512), 0, 0, n, per, offs, codes);
        else hipLaunchKernelGGL(k_scatter2, dim3(blocks), dim3(BT), 0, 0, n, per, offs, codes);
        CHECK(hipEventRecord(e[3]));
        CHECK(hipEventSynchronize(e[3]));
        float ta, tb;
        CHECK(hipEventElapsedTime(&ta, e[0], e[1])); CHECK(hipEventElapsedTime(&tb, e[2], e[3]));
        CHECK(hipEventRecord(e[0]));
        if (rep == 0) hipLaunchKernelGGL(k_count, dim3(256), dim3(1024), 0, 0, codes, bstart, table);
        else hipLaunchKernelGGL(k_count2, dim3(256), dim3(1024), 0, 0, codes, bstart, table);
        CHECK(hipEventRecord(e[1]));
        CHECK(hipEventSynchronize(e[1]));
        float tc;
        CHECK(hipEventElapsedTime(&tc, e[0], e[1]));
        unsigned *t = (unsigned *)malloc((1u << 22) * 4);
        CHECK(hipMemcpy(t, table, (1u << 22) * 4, hipMemcpyDeviceToHost));
        unsigned long long tot = 0;
        for (unsigned i = 0; i < (1u << 22); i++) tot += t[i];
        free(t);
        printf("%s: hist %.3f ms  scatter %.3f ms  count %.3f ms  total %llu (want %llu)\n",
               rep == 0 ? "naive  " : "batched", ta, tb, tc, tot, n);
    }
    return 0;
}
