/*
 * fk_ingest.hip — file -> HBM ingest for the drop-in ./findKmer.
 *
 * The reference reads its sequence file one fgetc() at a time inside the
 * scan loop (findKmer/src/findKmer.cpp:988).  Here the whole file is made
 * device-resident before the scan: T host threads pread() disjoint chunks
 * straight into their own small pinned buffers (two per thread, so a
 * thread's next read overlaps its previous chunk's H2D copy) and copy them with
 * hipMemcpyAsync on their own streams into one device buffer.  Page-cache
 * reads, which one thread does at a few GB/s, run in parallel, and PCIe
 * copies overlap the reads.  The engine then scans the buffer in one feed
 * (fk_engine_feed(..., on_device=1)), and a k sweep (./findKmer --sweep)
 * scans the same buffer once per k without reading the file again.
 */
#include "findkmer.h"

#include <hip/hip_runtime.h>

#include <ctype.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

struct fk_input {
    int device = 0;
    uint8_t *d = nullptr;
    uint64_t len = 0;
    double seconds = 0;
};

/* Bytes per pread + H2D, and threads.  Pinning host memory costs about
   0.5 ms per MiB on the MI355X boxes, so the pinned buffers are kept small:
   a 2 GB page-cache-resident file took 250-280 ms with 8 threads x 2 x 32 MiB
   (7-8 GB/s) and ~105 ms with 4 threads x 2 x 2 MiB (19 GB/s); more threads
   were slower at every chunk size (scripts/gpu_ingest_chunks.sh). */
static const uint64_t INGEST_CHUNK_DEFAULT = 2ull << 20;
static const unsigned INGEST_THREADS_DEFAULT = 4;
static const uint64_t INGEST_PAD = 64;              /* device bytes past the end (zeroed) */

extern "C" int fk_input_load(const char *path, int device, int threads, fk_input **out) {
    if (!path || !out) return FK_E_INVALID;
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return FK_E_IO;
    struct stat sb;
    if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
        close(fd);
        return FK_E_IO;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        close(fd);
        return FK_E_NO_DEVICE;
    }
    if (device < 0 && hipGetDevice(&device) != hipSuccess) device = 0;
    if (device >= ndev || hipSetDevice(device) != hipSuccess) {
        close(fd);
        return FK_E_INVALID;
    }
    fk_input *in = new fk_input;
    in->device = device;
    in->len = (uint64_t)sb.st_size;
    if (hipMalloc((void **)&in->d, in->len + INGEST_PAD) != hipSuccess) {
        close(fd);
        delete in;
        return FK_E_OOM;
    }
    if (hipMemset(in->d + in->len, 0, INGEST_PAD) != hipSuccess) {
        close(fd);
        fk_input_destroy(in);
        return FK_E_HIP;
    }
    uint64_t INGEST_CHUNK = INGEST_CHUNK_DEFAULT;
    if (const char *cm = getenv("FINDKMER_INGEST_CHUNK_MB")) INGEST_CHUNK = std::max<uint64_t>(1, strtoull(cm, nullptr, 10)) << 20;
    const uint64_t nchunks = (in->len + INGEST_CHUNK - 1) / INGEST_CHUNK;
    if (threads <= 0)
        threads = (int)std::min<unsigned>(INGEST_THREADS_DEFAULT, std::max(1u, std::thread::hardware_concurrency()));
    threads = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, nchunks));
    std::atomic<uint64_t> next{0};
    std::atomic<int> status{FK_OK};
    auto worker = [&]() {
        if (hipSetDevice(device) != hipSuccess) { status = FK_E_HIP; return; }
        hipStream_t s = nullptr;
        uint8_t *pin[2] = {nullptr, nullptr};
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool used[2] = {false, false};
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc((void **)&pin[0], INGEST_CHUNK, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&pin[1], INGEST_CHUNK, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
            status = FK_E_OOM;
        }
        for (int slot = 0; status == FK_OK; slot ^= 1) {
            const uint64_t c = next.fetch_add(1);
            if (c >= nchunks) break;
            const uint64_t off = c * INGEST_CHUNK, n = std::min(INGEST_CHUNK, in->len - off);
            if (used[slot] && hipEventSynchronize(ev[slot]) != hipSuccess) { status = FK_E_HIP; break; }
            uint64_t got = 0;
            while (got < n) {
                const ssize_t r = pread(fd, pin[slot] + got, n - got, (off_t)(off + got));
                if (r <= 0) break;
                got += (uint64_t)r;
            }
            if (got != n) { status = FK_E_IO; break; }
            if (hipMemcpyAsync(in->d + off, pin[slot], n, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipEventRecord(ev[slot], s) != hipSuccess) {
                status = FK_E_HIP;
                break;
            }
            used[slot] = true;
        }
        if (s && hipStreamSynchronize(s) != hipSuccess) status = FK_E_HIP;
        for (int i = 0; i < 2; i++) {
            if (ev[i]) hipEventDestroy(ev[i]);
            if (pin[i]) hipHostFree(pin[i]);
        }
        if (s) hipStreamDestroy(s);
    };
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
    close(fd);
    if (const char *tm = getenv("FINDKMER_TIMES")) {
        if (tm[0] == '1')
            fprintf(stderr, "[fk_input_load] %d threads: device buffer %.3f ms, read + copy %.3f ms (%.2f GB/s)\n",
                    threads, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count(),
                    in->len / 1e6 / std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    }
    if (status != FK_OK) {
        const int rc = status;
        fk_input_destroy(in);
        return rc;
    }
    in->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = in;
    return FK_OK;
}

extern "C" int fk_input_info(const fk_input *in, const uint8_t **dev_ptr, uint64_t *len, int *device,
                             double *seconds) {
    if (!in) return FK_E_INVALID;
    if (dev_ptr) *dev_ptr = in->d;
    if (len) *len = in->len;
    if (device) *device = in->device;
    if (seconds) *seconds = in->seconds;
    return FK_OK;
}

extern "C" void fk_input_destroy(fk_input *in) {
    if (!in) return;
    if (in->d) {
        hipSetDevice(in->device);
        hipFree(in->d);
    }
    delete in;
}

/*
 * Device choice for one process among many on a node.  The reference's sweep
 * driver starts 24 ./findKmer processes at once (k6thru11fullANDupstream.sh:
 * 16-24); with "the current device" every one of them would land on GPU 0.
 * FINDKMER_DEVICE=<ordinal> pins a process; otherwise the candidates are the
 * devices whose free HBM covers the run's estimated need, and the process
 * takes candidate (salt mod count) -- salt = its pid, so processes started
 * together spread round-robin instead of all picking the same emptiest GPU;
 * with no candidate, the device with the most free HBM.  Free HBM comes from
 * the amdgpu sysfs counters (no HIP context on the other GPUs), else from
 * hipMemGetInfo.
 */
extern "C" int fk_device_policy(int ndev, const uint64_t *free_bytes, uint64_t need, uint32_t salt) {
    if (ndev < 1 || !free_bytes) return FK_E_INVALID;
    std::vector<int> fits;
    int best = 0;
    for (int d = 0; d < ndev; d++) {
        if (free_bytes[d] >= need) fits.push_back(d);
        if (free_bytes[d] > free_bytes[best]) best = d;
    }
    return fits.empty() ? best : fits[salt % fits.size()];
}

static bool read_u64(const char *path, uint64_t *v) {
    FILE *f = fopen(path, "r");
    if (!f) return false;
    unsigned long long x = 0;
    const bool ok = fscanf(f, "%llu", &x) == 1;
    fclose(f);
    *v = (uint64_t)x;
    return ok;
}

static bool sysfs_free_vram(int dev, uint64_t *free_b) {
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, dev) != hipSuccess) return false;
    for (char *c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
    char path[256];
    uint64_t total = 0, used = 0;
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/mem_info_vram_total", bus);
    if (!read_u64(path, &total) || total == 0) return false;
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/mem_info_vram_used", bus);
    if (!read_u64(path, &used)) return false;
    *free_b = total > used ? total - used : 0;
    return true;
}

extern "C" int fk_device_select(uint64_t need, int *device) {
    if (!device) return FK_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return FK_E_NO_DEVICE;
    int dev = 0;
    if (const char *pin = getenv("FINDKMER_DEVICE")) {
        char *end = nullptr;
        const long v = strtol(pin, &end, 10);
        if (!*pin || *end || v < 0 || v >= ndev) return FK_E_INVALID;
        dev = (int)v;
    } else if (ndev > 1) {
        std::vector<uint64_t> fr((size_t)ndev, 0);
        bool sysfs = true;
        for (int d = 0; d < ndev && sysfs; d++) sysfs = sysfs_free_vram(d, &fr[(size_t)d]);
        /* without the sysfs counters, no probing: a hipMemGetInfo per device
           would create a HIP context (and its HBM) on every GPU in every one
           of the sweep's processes; spread them by pid alone */
        dev = sysfs ? fk_device_policy(ndev, fr.data(), need, (uint32_t)getpid()) : (int)((uint32_t)getpid() % (uint32_t)ndev);
    }
    if (hipSetDevice(dev) != hipSuccess) return FK_E_HIP;
    *device = dev;
    return FK_OK;
}

/*
 * Record progress for `-q 0` runs.  The reference prints, at every '>' that
 * starts a comment line, "Read %llu bases\n>" + the line (findKmer.cpp:
 * 996-1002), with baseCounter as of that byte.  baseCounter grows by k when a
 * run reaches k bases and by 1 per base after that (:1040-1057), so at a
 * header start it is the sum of g(L) = (L >= k ? L : 0) over the runs closed
 * so far (a header start closes the current run) -- exact while every run is
 * shorter than 2^31 bases (the reference's int32 seqSize, :977) and no 0xFF
 * byte ends the scan early (:988); otherwise the caller uses the engine's
 * streamed path.
 *
 * k_hdr_traj: one thread per 4 KiB chunk computes the chunk's two possible
 * trajectories of the (in_header, run) state: entering outside a header
 * (mode 0, with an unknown run length carried in) or inside one (mode 1: the
 * chunk is skipped up to its first '\n').  The host composes the chunks in
 * order (a few ns each), then k_hdr_list writes each chunk's header starts
 * from the trajectory it actually takes.
 */
#define HDR_CHUNK 4096u

struct HdrTraj {
    uint64_t inner;      /* sum of g(L) over runs closed after the first break */
    uint32_t head;       /* bases before the first break (joins the run carried in) */
    uint32_t tail;       /* bases after the last break */
    uint32_t nhdr;       /* header starts */
    uint8_t broke, exit_hdr, ff, pad;
};

template <bool WRITE>
__device__ void hdr_walk(const uint8_t *buf, uint64_t beg, uint64_t end, int mode, int k, HdrTraj &t,
                         uint64_t *pos_out, uint64_t *inner_out) {
    t = HdrTraj{0, 0, 0, 0, 0, 0, 0, 0};
    int in_hdr = mode;
    uint32_t L = 0;
    uint32_t n = 0;
    for (uint64_t p = beg; p < end; p++) {
        const uint8_t c = buf[p];
        if (in_hdr) {
            if (c == '\n') in_hdr = 0;
            continue;
        }
        if (c == 'A' || c == 'C' || c == 'G' || c == 'T') {
            L++;
        } else if (c == '\n') {
        } else if (c == 0xFF) {
            t.ff = 1;
            break;
        } else {
            if (!t.broke) {
                t.head = L;
                t.broke = 1;
            } else if (L >= (uint32_t)k) {
                t.inner += L;
            }
            L = 0;
            if (c == '>') {
                if (WRITE) {
                    pos_out[n] = p;
                    inner_out[n] = t.inner;
                }
                n++;
                in_hdr = 1;
            }
        }
    }
    if (!t.broke) t.head = L;
    t.tail = L;
    t.nhdr = n;
    t.exit_hdr = (uint8_t)in_hdr;
}

__global__ void k_hdr_traj(const uint8_t *buf, uint64_t len, uint64_t nchunks, int k, HdrTraj *traj) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t beg = c * HDR_CHUNK, end = std::min(len, beg + HDR_CHUNK);
    hdr_walk<false>(buf, beg, end, 0, k, traj[2 * c], nullptr, nullptr);
    hdr_walk<false>(buf, beg, end, 1, k, traj[2 * c + 1], nullptr, nullptr);
}

__global__ void k_hdr_list(const uint8_t *buf, uint64_t len, uint64_t nchunks, int k, const uint8_t *mode,
                           const uint64_t *off, uint64_t *pos, uint64_t *inner) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t beg = c * HDR_CHUNK, end = std::min(len, beg + HDR_CHUNK);
    HdrTraj t;
    hdr_walk<true>(buf, beg, end, mode[c], k, t, pos + off[c], inner + off[c]);
}

extern "C" int fk_input_headers(fk_input *in, int k, uint64_t *pos, uint64_t *bases, uint64_t cap, uint64_t *n) {
    if (!in || !n || k < 1 || k > 20 || (cap && (!pos || !bases))) return FK_E_INVALID;
    if (hipSetDevice(in->device) != hipSuccess) return FK_E_HIP;
    const uint64_t nchunks = (in->len + HDR_CHUNK - 1) / HDR_CHUNK;
    *n = 0;
    if (!nchunks) return FK_OK;
    HdrTraj *d_traj = nullptr;
    uint8_t *d_mode = nullptr;
    uint64_t *d_off = nullptr, *d_pos = nullptr, *d_inner = nullptr;
    int rc = FK_OK;
    std::vector<HdrTraj> traj(2 * nchunks);
    std::vector<uint8_t> mode(nchunks);
    std::vector<uint64_t> off(nchunks), cbase(nchunks);
    uint64_t total = 0;
    const unsigned grid = (unsigned)((nchunks + 255) / 256);
    do {
        if (hipMalloc((void **)&d_traj, 2 * nchunks * sizeof(HdrTraj)) != hipSuccess) { rc = FK_E_OOM; break; }
        hipLaunchKernelGGL(k_hdr_traj, dim3(grid), dim3(256), 0, nullptr, in->d, in->len, nchunks, k, d_traj);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpy(traj.data(), d_traj, 2 * nchunks * sizeof(HdrTraj), hipMemcpyDeviceToHost) != hipSuccess) {
            rc = FK_E_HIP;
            break;
        }
        /* compose the chunks in stream order */
        int in_hdr = 0;
        uint64_t L = 0, base = 0;
        auto g = [k](uint64_t x) { return x >= (uint64_t)k ? x : 0ull; };
        for (uint64_t c = 0; c < nchunks && rc == FK_OK; c++) {
            const int m = in_hdr;
            const HdrTraj &t = traj[2 * c + (size_t)m];
            mode[c] = (uint8_t)m;
            off[c] = total;
            if (t.ff) { rc = FK_E_STATE; break; }   /* 0xFF ends the scan: streamed path */
            const uint64_t L0 = m == 1 ? 0 : L;
            if (t.broke) {
                /* a run that crosses 2^31-1 bases and closes in this chunk:
                   the int32 seqSize zone as well */
                if (L0 + t.head >= 0x7FFFFFFFull) { rc = FK_E_STATE; break; }
                cbase[c] = base + g(L0 + t.head);
                base = cbase[c] + t.inner;   /* every run closed in the chunk; the tail run stays open */
                L = t.tail;
            } else {
                cbase[c] = base;
                L = L0 + t.head;
            }
            total += t.nhdr;
            in_hdr = t.exit_hdr;
            if (L >= 0x7FFFFFFFull) { rc = FK_E_STATE; break; }   /* int32 seqSize zone: streamed path */
        }
        if (rc) break;
        if (total > 0) {
            if (hipMalloc((void **)&d_mode, nchunks) != hipSuccess ||
                hipMalloc((void **)&d_off, nchunks * sizeof(uint64_t)) != hipSuccess ||
                hipMalloc((void **)&d_pos, total * sizeof(uint64_t)) != hipSuccess ||
                hipMalloc((void **)&d_inner, total * sizeof(uint64_t)) != hipSuccess) {
                rc = FK_E_OOM;
                break;
            }
            if (hipMemcpy(d_mode, mode.data(), nchunks, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(d_off, off.data(), nchunks * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess) {
                rc = FK_E_HIP;
                break;
            }
            hipLaunchKernelGGL(k_hdr_list, dim3(grid), dim3(256), 0, nullptr, in->d, in->len, nchunks, k, d_mode,
                               d_off, d_pos, d_inner);
            if (hipGetLastError() != hipSuccess) { rc = FK_E_HIP; break; }
        }
        *n = total;
        if (cap) {
            std::vector<uint64_t> inner((size_t)std::min(cap, total));
            const uint64_t m = std::min(cap, total);
            if (m && (hipMemcpy(pos, d_pos, m * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess ||
                      hipMemcpy(inner.data(), d_inner, m * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)) {
                rc = FK_E_HIP;
                break;
            }
            /* chunk of each header start -> its baseCounter */
            for (uint64_t i = 0; i < m; i++) bases[i] = cbase[pos[i] / HDR_CHUNK] + inner[i];
        }
    } while (0);
    hipFree(d_traj);
    hipFree(d_mode);
    hipFree(d_off);
    hipFree(d_pos);
    hipFree(d_inner);
    return rc;
}
