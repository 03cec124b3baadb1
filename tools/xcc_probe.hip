// xcc_probe.hip — which XCD runs each block (s_getreg HW_REG_XCC_ID) and
// the same-XCD L2 atomic throughput versus device-scope atomics on a 16 MiB
// table (the k=11 count table), 1e9 random increments.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ unsigned xcc_id() {
    /* s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0] */
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 0xF;
}

__global__ void k_probe(unsigned *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <int MODE>   /* 0 device-scope atomics on one table, 1 per-XCD copies + workgroup scope,
                         2 per-XCD L2-resident slice (nbins/8 bins) + workgroup scope */
__global__ void k_atomics(unsigned *table, unsigned long long n, unsigned nbins) {
    unsigned *t = MODE ? table + (size_t)xcc_id() * nbins : table;
    if (MODE == 2) nbins /= 8;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned b = (unsigned)mix(i) & (nbins - 1);
        if (MODE) __hip_atomic_fetch_add(&t[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else atomicAdd(&t[b], 1u);
    }
}

int main() {
    unsigned *d;
    CHECK(hipMalloc(&d, 4096 * sizeof(unsigned)));
    hipLaunchKernelGGL(k_probe, dim3(4096), dim3(64), 0, 0, d);
    unsigned h[4096];
    CHECK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
    int same = 0, hist[16] = {0};
    for (int b = 0; b < 4096; b++) { same += h[b] == (unsigned)(b % 8); hist[h[b] & 15]++; }
    printf("blocks with xcc == block%%8: %d / 4096; per-xcc:", same);
    for (int i = 0; i < 16; i++) if (hist[i]) printf(" %d:%d", i, hist[i]);
    printf("\n");
    const unsigned nbins = 1u << 22;
    const unsigned long long n = 1000000000ull;
    unsigned *tab;
    CHECK(hipMalloc(&tab, 8ull * nbins * sizeof(unsigned)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (int mode = 0; mode < 3; mode++) {
        CHECK(hipMemset(tab, 0, 8ull * nbins * sizeof(unsigned)));
        CHECK(hipEventRecord(a));
        if (mode == 0) hipLaunchKernelGGL((k_atomics<0>), dim3(8192), dim3(256), 0, 0, tab, n, nbins);
        else if (mode == 1) hipLaunchKernelGGL((k_atomics<1>), dim3(8192), dim3(256), 0, 0, tab, n, nbins);
        else hipLaunchKernelGGL((k_atomics<2>), dim3(8192), dim3(256), 0, 0, tab, n, nbins);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        unsigned *hv = (unsigned *)malloc(8ull * nbins * sizeof(unsigned));
        CHECK(hipMemcpy(hv, tab, 8ull * nbins * sizeof(unsigned), hipMemcpyDeviceToHost));
        unsigned long long tot = 0;
        for (size_t i = 0; i < 8ull * nbins; i++) tot += hv[i];
        free(hv);
        printf("mode %d (%s): %.2f ms, %.1f G atomics/s, total %llu (want %llu)\n", mode,
               mode == 2 ? "per-XCD 2 MiB slice, workgroup scope" : mode ? "per-XCD copy, workgroup scope" : "one table, device scope",
               ms, n / ms / 1e6, tot, n);
    }
    return 0;
}
