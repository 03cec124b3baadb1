// Experiment (never the product): global u32 atomic throughput into a table
// region per XCD (blocks are dispatched round-robin over the 8 XCDs, so block
// b runs on XCD b % 8) of R bytes, versus one shared region.  Decides whether
// 14 <= k <= 16 could count a coarse partition's slices in L2 with global
// atomics instead of LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_atomics(uint32_t *t, uint64_t region_words, int per_xcd, uint32_t iters, uint32_t seed) {
    const uint32_t xcd = blockIdx.x & 7u;
    uint32_t *base = per_xcd ? t + (uint64_t)xcd * region_words : t;
    uint32_t x = seed ^ (blockIdx.x * 1024u + threadIdx.x) * 2654435761u;
    const uint64_t mask = region_words - 1;
    for (uint32_t i = 0; i < iters; i++) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        atomicAdd(base + (x & mask), 1u);
    }
}

int main(int argc, char **argv) {
    const uint32_t iters = 256;
    const unsigned grid = 256 * 8, block = 256;
    uint32_t *t = nullptr;
    const uint64_t total = 1ull << 30;   // 4 GiB of u32
    if (hipMalloc(&t, total * 4) != hipSuccess) return 1;
    hipMemset(t, 0, total * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    struct Case { uint64_t words; int per_xcd; const char *name; } cases[] = {
        {1u << 17, 1, "512 KiB per XCD"}, {1u << 19, 1, "2 MiB per XCD"}, {1u << 20, 1, "4 MiB per XCD"},
        {1u << 21, 1, "8 MiB per XCD"}, {1u << 22, 0, "16 MiB shared"}, {1ull << 28, 0, "1 GiB shared"},
        {1ull << 30, 0, "4 GiB shared"}};
    for (auto &c : cases) {
        hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(block), 0, 0, t, c.words, c.per_xcd, iters, 1u);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; r++)
            hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(block), 0, 0, t, c.words, c.per_xcd, iters, 7u + r);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double n = 5.0 * grid * block * iters;
        printf("%-18s %8.3f ms  %7.1f G atomics/s\n", c.name, ms / 5, n / (ms * 1e-3) / 1e9);
    }
    hipFree(t);
    return 0;
}
