// stream_ceiling.hip — measured HBM read ceiling on this MI355X for the access
// patterns the k-mer scan can use (SURVEY.md §8(d) "measured stream-read
// ceiling").  Each variant reads the same 1 GiB buffer once, 16 B per lane,
// and folds the bytes into a checksum so nothing is dead-code eliminated.
//   A  grid-stride: consecutive waves read consecutive 1 KiB tiles
//   B  per-wave contiguous ranges (the engine's layout), 4 tiles in flight
//   C  as B, 8 tiles in flight
//   D  as B without the non-temporal hint
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_ceiling.hip -o build/stream_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_grid(const u32x4 *p, size_t n16, unsigned *out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int DEPTH, bool NT>
__global__ void k_range(const u32x4 *p, size_t n16, size_t tiles_per_wave, unsigned *out) {
    const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const size_t t0 = wave * tiles_per_wave;
    unsigned acc = 0;
    u32x4 buf[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
        size_t i = (t0 + d) * 64 + lane;
        buf[d] = i < n16 ? (NT ? __builtin_nontemporal_load(p + i) : p[i]) : u32x4{0, 0, 0, 0};
    }
    for (size_t t = 0; t < tiles_per_wave; t += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            u32x4 v = buf[d];
            size_t i = (t0 + t + DEPTH + d) * 64 + lane;
            if (t + DEPTH + d < tiles_per_wave && i < n16) buf[d] = NT ? __builtin_nontemporal_load(p + i) : p[i];
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

/* 2 KiB tiles, two 16-B loads per lane; INTER: +1024 (contiguous per
   instruction) instead of +16 (lane stride 32) */
template <int DEPTH, bool INTER>
__global__ void k_tile2(const u32x4 *p, size_t n16, size_t tiles_per_wave, unsigned *out) {
    const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const size_t t0 = wave * tiles_per_wave;
    unsigned acc = 0;
    u32x4 a[DEPTH], b[DEPTH];
    auto idx = [&](size_t t, int h) -> size_t {
        return INTER ? t * 128 + h * 64 + lane : t * 128 + lane * 2 + h;
    };
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
        size_t i0 = idx(t0 + d, 0), i1 = idx(t0 + d, 1);
        a[d] = i0 < n16 ? __builtin_nontemporal_load(p + i0) : u32x4{0, 0, 0, 0};
        b[d] = i1 < n16 ? __builtin_nontemporal_load(p + i1) : u32x4{0, 0, 0, 0};
    }
    for (size_t t = 0; t < tiles_per_wave; t += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            u32x4 va = a[d], vb = b[d];
            size_t tn = t0 + t + DEPTH + d;
            size_t i0 = idx(tn, 0), i1 = idx(tn, 1);
            if (t + DEPTH + d < tiles_per_wave && i1 < n16) {
                a[d] = __builtin_nontemporal_load(p + i0);
                b[d] = __builtin_nontemporal_load(p + i1);
            }
            acc ^= va.x + va.y + va.z + va.w + vb.x + vb.y + vb.z + vb.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 1ull << 30);
    size_t n16 = bytes / 16;
    u32x4 *p; unsigned *out;
    CHECK(hipMalloc(&p, bytes)); CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(p, 0x41, bytes));
    hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    size_t tiles = n16 / 64;
    for (int wpc : {16, 32}) {
        size_t waves = (size_t)cus * wpc;
        size_t tpw = (tiles + waves - 1) / waves;
        unsigned blocks = (unsigned)((waves + 7) / 8);
        double a = time_ms([&] { hipLaunchKernelGGL(k_grid, dim3(blocks), dim3(512), 0, 0, p, n16, out); }, 20);
        double b4 = time_ms([&] { hipLaunchKernelGGL((k_range<4, true>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw, out); }, 20);
        double b8 = time_ms([&] { hipLaunchKernelGGL((k_range<8, true>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw, out); }, 20);
        double d4 = time_ms([&] { hipLaunchKernelGGL((k_range<4, false>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw, out); }, 20);
        size_t tpw2 = (tiles / 2 + waves - 1) / waves;
        double e3 = time_ms([&] { hipLaunchKernelGGL((k_tile2<3, false>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw2, out); }, 20);
        double f3 = time_ms([&] { hipLaunchKernelGGL((k_tile2<3, true>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw2, out); }, 20);
        double f4 = time_ms([&] { hipLaunchKernelGGL((k_tile2<4, true>), dim3(blocks), dim3(512), 0, 0, p, n16, tpw2, out); }, 20);
        printf("{\"waves_per_cu\": %d, \"bytes\": %zu, \"grid_stride_GBps\": %.1f, \"range_depth4_nt_GBps\": %.1f, "
               "\"range_depth8_nt_GBps\": %.1f, \"range_depth4_GBps\": %.1f, \"tile2k_stride32_d3_GBps\": %.1f, "
               "\"tile2k_inter_d3_GBps\": %.1f, \"tile2k_inter_d4_GBps\": %.1f}\n",
               wpc, bytes, bytes / a / 1e6, bytes / b4 / 1e6, bytes / b8 / 1e6, bytes / d4 / 1e6, bytes / e3 / 1e6,
               bytes / f3 / 1e6, bytes / f4 / 1e6);
    }
    return 0;
}
