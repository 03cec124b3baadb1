/*
 * fk_ingest.hip — file -> HBM ingest for the drop-in ./findKmer.
 *
 * The reference reads its sequence file one fgetc() at a time inside the
 * scan loop (findKmer/src/findKmer.cpp:988).  Here the whole file is made
 * device-resident before the scan: T host threads pread() disjoint chunks
 * straight into their own pinned buffers (two per thread, so a thread's
 * next read overlaps its previous chunk's H2D copy) and copy them with
 * hipMemcpyAsync on their own streams into one device buffer.  Page-cache
 * reads, which one thread does at a few GB/s, run in parallel, and PCIe
 * copies overlap the reads.  The engine then scans the buffer in one feed
 * (fk_engine_feed(..., on_device=1)), and a k sweep (./findKmer --sweep)
 * scans the same buffer once per k without reading the file again.
 */
#include "findkmer.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
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

static const uint64_t INGEST_CHUNK = 32ull << 20;   /* bytes per pread + H2D */
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
    const uint64_t nchunks = (in->len + INGEST_CHUNK - 1) / INGEST_CHUNK;
    if (threads <= 0) threads = (int)std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
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
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
    close(fd);
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
