// atomic_scope_probe.hip — random u32 increments into a 4^11-bin table:
//   D  device-scope atomicAdd into one table (what k_part's general tiles do)
//   X  workgroup-scope atomics into one table copy per XCD (s_getreg XCC_ID):
//      performed in that XCD's L2, coherent there; copies folded afterwards
// Prints G atomics/s for each and checks that both sum to the same table.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ unsigned code_of(unsigned long long i) {
    unsigned long long x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    return (unsigned)x & ((1u << 22) - 1);
}
__device__ __forceinline__ unsigned xcc_id() {
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 0xF;
}
__global__ void k_dev(unsigned long long n, unsigned *t) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        atomicAdd(&t[code_of(i)], 1u);
}
__global__ void k_xcd(unsigned long long n, unsigned *t) {
    unsigned *mine = t + ((size_t)xcc_id() << 22);
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        __hip_atomic_fetch_add(&mine[code_of(i)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__global__ void k_fold(unsigned *t) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (1u << 22); i += gridDim.x * blockDim.x) {
        unsigned s = 0;
        for (int x = 0; x < 8; x++) s += t[((size_t)x << 22) + i];
        t[i] = s;
    }
}
int main() {
    const unsigned long long n = 1ull << 30;
    unsigned *d, *x;
    CHECK(hipMalloc(&d, 4u << 22));
    CHECK(hipMalloc(&x, 8 * (4u << 22)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipMemset(d, 0, 4u << 22));
        CHECK(hipMemset(x, 0, 8 * (4u << 22)));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_dev, dim3(2048), dim3(256), 0, 0, n, d);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        float ms_d; CHECK(hipEventElapsedTime(&ms_d, a, b));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_xcd, dim3(2048), dim3(256), 0, 0, n, x);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        float ms_x; CHECK(hipEventElapsedTime(&ms_x, a, b));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_fold, dim3(1024), dim3(256), 0, 0, x);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        float ms_f; CHECK(hipEventElapsedTime(&ms_f, a, b));
        std::vector<unsigned> hd(1u << 22), hx(1u << 22);
        CHECK(hipMemcpy(hd.data(), d, 4u << 22, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hx.data(), x, 4u << 22, hipMemcpyDeviceToHost));
        bool same = hd == hx;
        printf("device-scope %.3f ms (%.1f G/s)  per-XCD workgroup-scope %.3f ms (%.1f G/s) + fold %.3f ms  tables equal: %d\n",
               ms_d, n / ms_d / 1e6, ms_x, n / ms_x / 1e6, ms_f, (int)same);
    }
    return 0;
}
