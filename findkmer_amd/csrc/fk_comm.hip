/*
 * fk_comm: an RCCL communicator owned by the library (one rank per GPU, over
 * xGMI), so that a sharded pass's exchange runs on the engine's own HIP
 * stream with no framework in between: pack kernel -> ncclAllReduce ->
 * rows publish kernel, one host wait (fk_engine_shard_exchange).
 *
 * RCCL is resolved at run time (dlopen) rather than linked: the drop-in
 * ./findKmer never needs it, and inside a PyTorch process the copy torch has
 * already loaded (same SONAME librccl.so.1) is the one used.  The unique id
 * is created by one rank (fk_comm_id) and handed to the others by the
 * caller (findkmer_amd/dist.py broadcasts it over torch.distributed).
 *
 * The reference has no counterpart: it is single-threaded
 * (findKmer/src/findKmer.cpp:962-1069); SURVEY.md §8(e).
 */
#include <dlfcn.h>
#include <string.h>

#include <algorithm>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "findkmer.h"
#include "fk_comm.h"

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    /* optional (fk_comm_info only; a missing one does not turn the
       communicator off) */
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;
    decltype(&ncclCommCuDevice) cu_device = nullptr;
    /* optional (the routed table exchange, fkc_alltoallv_i32; without them
       the sharded table is reduce-scattered) */
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    bool ok = false;
};

/* the process's RCCL: an already loaded copy first (torch's), else the
   system one */
const Rccl &rccl() {
    static Rccl r = [] {
        Rccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) return x;
        x.get_id = (decltype(x.get_id))dlsym(h, "ncclGetUniqueId");
        x.init_rank = (decltype(x.init_rank))dlsym(h, "ncclCommInitRank");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
        x.reduce = (decltype(x.reduce))dlsym(h, "ncclReduce");
        x.reduce_scatter = (decltype(x.reduce_scatter))dlsym(h, "ncclReduceScatter");
        x.count = (decltype(x.count))dlsym(h, "ncclCommCount");
        x.user_rank = (decltype(x.user_rank))dlsym(h, "ncclCommUserRank");
        x.cu_device = (decltype(x.cu_device))dlsym(h, "ncclCommCuDevice");
        x.send = (decltype(x.send))dlsym(h, "ncclSend");
        x.recv = (decltype(x.recv))dlsym(h, "ncclRecv");
        x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
        /* exactly the entry points the exchange calls */
        x.ok = x.get_id && x.init_rank && x.destroy && x.all_reduce && x.reduce && x.reduce_scatter;
        return x;
    }();
    return r;
}

}  // namespace

struct fk_comm {
    ncclComm_t nc = nullptr;
    int world = 0, rank = 0, device = 0;
};

static_assert(FK_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "fk_comm ids are RCCL unique ids");

extern "C" int fk_comm_id(uint8_t *id) {
    if (!id) return FK_E_INVALID;
    const Rccl &r = rccl();
    if (!r.ok) return FK_E_RCCL;
    ncclUniqueId u;
    if (r.get_id(&u) != ncclSuccess) return FK_E_RCCL;
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return FK_OK;
}

/* Everything fk_comm_create checks before its collective ncclCommInitRank,
   without joining anything: callers agree on it first (one all-reduce), so
   that no rank is left alone inside the collective init. */
extern "C" int fk_comm_available(int device) {
    if (!rccl().ok) return FK_E_RCCL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return FK_E_NO_DEVICE;
    if (device < 0 || device >= n) return FK_E_INVALID;
    return hipSetDevice(device) == hipSuccess ? FK_OK : FK_E_HIP;
}

extern "C" int fk_comm_create(const uint8_t *id, int world, int rank, int device, fk_comm **out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return FK_E_INVALID;
    *out = nullptr;
    const Rccl &r = rccl();
    if (!r.ok) return FK_E_RCCL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return FK_E_NO_DEVICE;
    if (device < 0 || device >= n) return FK_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return FK_E_HIP;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    fk_comm *c = new fk_comm;
    c->world = world;
    c->rank = rank;
    c->device = device;
    /* collective: returns when every rank has joined */
    if (r.init_rank(&c->nc, world, u, rank) != ncclSuccess) {
        delete c;
        return FK_E_RCCL;
    }
    *out = c;
    return FK_OK;
}

extern "C" void fk_comm_destroy(fk_comm *c) {
    if (!c) return;
    if (c->nc && rccl().ok) rccl().destroy(c->nc);
    delete c;
}

int fkc_world(const fk_comm *c) { return c->world; }
int fkc_rank(const fk_comm *c) { return c->rank; }
int fkc_device(const fk_comm *c) { return c->device; }

int fkc_allreduce_i32(fk_comm *c, int32_t *buf, size_t n, hipStream_t s) {
    if (!c || !c->nc || !rccl().ok) return FK_E_RCCL;
    return rccl().all_reduce(buf, buf, n, ncclInt32, ncclSum, c->nc, s) == ncclSuccess ? FK_OK : FK_E_RCCL;
}

int fkc_reduce_i32(fk_comm *c, int32_t *buf, size_t n, int root, hipStream_t s) {
    if (!c || !c->nc || !rccl().ok) return FK_E_RCCL;
    return rccl().reduce(buf, buf, n, ncclInt32, ncclSum, root, c->nc, s) == ncclSuccess ? FK_OK : FK_E_RCCL;
}

int fkc_reduce_scatter_i32(fk_comm *c, int32_t *buf, size_t per_rank, hipStream_t s) {
    if (!c || !c->nc || !rccl().ok) return FK_E_RCCL;
    /* in place: rank r's block of the sum lands at buf + r * per_rank */
    return rccl().reduce_scatter(buf, buf + (size_t)c->rank * per_rank, per_rank, ncclInt32, ncclSum, c->nc, s) ==
                   ncclSuccess
               ? FK_OK
               : FK_E_RCCL;
}

int fkc_reduce_scatter_from_i32(fk_comm *c, const int32_t *send, int32_t *buf, size_t per_rank, hipStream_t s) {
    if (!c || !c->nc || !rccl().ok) return FK_E_RCCL;
    return rccl().reduce_scatter(send, buf + (size_t)c->rank * per_rank, per_rank, ncclInt32, ncclSum, c->nc, s) ==
                   ncclSuccess
               ? FK_OK
               : FK_E_RCCL;
}

bool fkc_has_alltoallv(const fk_comm *c) {
    const Rccl &r = rccl();
    return c && c->nc && r.ok && r.send && r.recv && r.group_start && r.group_end;
}

/* every rank sends scount[p] words at send + sdispl[p] to rank p and
   receives rcount[p] words from rank p at recv + rdispl[p] (point-to-point
   pairs in one group: over xGMI each pair takes its own link) */
int fkc_alltoallv_i32(fk_comm *c, const int32_t *send, const uint64_t *scount, const uint64_t *sdispl,
                      int32_t *recv, const uint64_t *rcount, const uint64_t *rdispl, hipStream_t s) {
    if (!fkc_has_alltoallv(c)) return FK_E_RCCL;
    const Rccl &r = rccl();
    /* this rank's own blob: a device copy (a 1.5 GB ncclSend to self
       delivered about half of it at k = 16) */
    const int me = c->rank;
    if (scount[me] != rcount[me]) return FK_E_INVALID;
    if (scount[me] && hipMemcpyAsync(recv + rdispl[me], send + sdispl[me], scount[me] * sizeof(int32_t),
                                     hipMemcpyDeviceToDevice, s) != hipSuccess)
        return FK_E_HIP;
    if (c->world == 1) return FK_OK;
    /* the others in pieces of at most 2^28 words, matched in order */
    const uint64_t CH = 1ull << 28;
    if (r.group_start() != ncclSuccess) return FK_E_RCCL;
    int rc = FK_OK;
    for (int p = 0; p < c->world && rc == FK_OK; p++) {
        if (p == me) continue;
        for (uint64_t o = 0; o < scount[p] && rc == FK_OK; o += CH)
            if (r.send(send + sdispl[p] + o, std::min(CH, scount[p] - o), ncclInt32, p, c->nc, s) != ncclSuccess)
                rc = FK_E_RCCL;
        for (uint64_t o = 0; o < rcount[p] && rc == FK_OK; o += CH)
            if (r.recv(recv + rdispl[p] + o, std::min(CH, rcount[p] - o), ncclInt32, p, c->nc, s) != ncclSuccess)
                rc = FK_E_RCCL;
    }
    if (r.group_end() != ncclSuccess) rc = FK_E_RCCL;
    return rc;
}

/* What RCCL itself reports for the communicator: its rank count, this
   rank and the device it drives (-1 where this RCCL lacks the query). */
extern "C" int fk_comm_info(fk_comm *c, int *nranks, int *rank, int *device) {
    if (!c || !c->nc || !rccl().ok) return FK_E_RCCL;
    const Rccl &r = rccl();
    int n = -1, me = -1, dev = -1;
    if (r.count && r.count(c->nc, &n) != ncclSuccess) return FK_E_RCCL;
    if (r.user_rank && r.user_rank(c->nc, &me) != ncclSuccess) return FK_E_RCCL;
    if (r.cu_device && r.cu_device(c->nc, &dev) != ncclSuccess) return FK_E_RCCL;
    if (nranks) *nranks = n;
    if (rank) *rank = me;
    if (device) *device = dev;
    return FK_OK;
}
