/*
 * fk_engine.hip — MI355X (gfx950) k-mer counting engine behind include/findkmer.h.
 *
 * Replaces the reference hot path findKmer() (findKmer/src/findKmer.cpp:962-1069)
 * and its trie (:107-111, :612-690) with three HIP kernels per input segment:
 *
 *   k_count  each wave owns a contiguous range of 64 KiB chunks (8 waves per
 *            512-thread block, ~one range per wave slot of the chip).  16 B
 *            per lane per 1 KiB tile, coalesced, 4 tiles prefetched.  The
 *            range's entering scan state is guessed from the 256 bytes before
 *            it.  Fast tiles (only A/C/G/T and at most one '\n' per lane, deep
 *            in a run) pack each lane's bases into one 32-bit word with
 *            v_dot4_u32_u8 and cut windows out of {previous lane, own} with
 *            v_alignbit; other tiles take a general path (64-lane scan of
 *            per-lane run summaries, then a byte walk).  Windows go to LDS
 *            bins for k <= 7 ((k+1)-mers at every other base for k <= 6,
 *            marginalised at the flush) and to global u32 atomics otherwise.
 *            Each chunk records its transfer function; each range the
 *            composition.
 *   k_scan   one workgroup scans the range transfer functions into the exact
 *            entering state of every range (64-bit run length, so the
 *            reference's int32 seqSize wrap is exact) and lists the ranges
 *            whose guess would count differently.
 *   k_redo   walks only the listed ranges chunk by chunk: a chunk whose guess
 *            is not equivalent is counted again with weight -1 from the guess
 *            (cancelling k_count's contribution exactly) and +1 from the true
 *            state.  Normally the list is empty.
 *
 * Counting rules per valid base (seq = (int32)R after the increment):
 *   seq >  k : window, baseCounter++, base[new]++            (:1035-1042)
 *   seq == k : window, base[all k]++, baseCounter += k        (:1044-1057)
 *   0<seq<k  : depth-1 trie touch only (prefix walk)          (:1059-1062)
 * Runs break at '>' (then skip to '\n'), 'N' and any other non-ACGT byte;
 * '\n' is transparent; 0xFF outside a header ends the input (:988).
 */
#include "fk_engine_internal.h"

/* trie prefix presence, level d from level d+1 (or from the table at d = k-1) */
__global__ void k_fold_from_table(const uint32_t *table, const uint32_t *shortd, uint8_t *pres,
                                  uint64_t nd, unsigned long long *count) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = reinterpret_cast<const uint4 *>(table)[i];
        uint8_t p = (v.x | v.y | v.z | v.w) != 0 || shortd[i] != 0;
        pres[i] = p;
        c += p;
    }
    c = wsum32((uint32_t)c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}
__global__ void k_fold_level(const uint8_t *child, const uint32_t *shortd, uint8_t *pres,
                             uint64_t nd, unsigned long long *count) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t ch = reinterpret_cast<const uint32_t *>(child)[i];
        uint8_t p = ch != 0 || shortd[i] != 0;
        pres[i] = p;
        c += p;
    }
    c = wsum32((uint32_t)c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}


/* Header flag at each lane's start (last '>' vs last '\n' before it). */
__device__ __forceinline__ uint32_t lane_hdr_entry(const uint32_t w[4], int nb, uint32_t hdr_in) {
    const int lane = threadIdx.x & 63;
    uint32_t g = 0, n = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t c = fk_byte(w, j);
        uint32_t pos = (uint32_t)lane * 16u + (uint32_t)j + 1u;
        if (j < nb && c == '>') g = pos;
        if (j < nb && c == '\n') n = pos;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t tg = shup(g, d), tn = shup(n, d);
        if (lane >= d) { g = max(g, tg); n = max(n, tn); }
    }
    uint32_t gx = shup(g, 1), nx = shup(n, 1);
    if (lane == 0) { gx = 0; nx = 0; }
    return (gx | nx) ? (gx > nx ? 1u : 0u) : hdr_in;
}

/*
 * k_extract: copy the bytes that make the reference print "Unknown character
 * %c processed!" (:581-584) to out[], in stream order.  One wave per listed
 * range, entering header flag from the exact state scan.
 */
__global__ void __launch_bounds__(FK_BLOCK)
k_extract(const uint8_t *buf, uint64_t len, int64_t lo, const RangeRec *rr, const XState *rtrue,
          const uint32_t *list, const uint64_t *offs, uint32_t nlist, uint8_t *out, uint64_t *opos) {
    const int lane = threadIdx.x & 63;
    Ctx cx{buf, len, lo, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * FK_WAVES_PER_BLOCK;
    for (uint64_t i = wave; i < nlist; i += nwaves) {
        const uint32_t r = list[i];
        const Span sp = range_span(rr[r], len);
        uint32_t hdr = rtrue[r].hdr;
        uint64_t base = offs[i];
        const uint64_t ntiles = (sp.rend - sp.rbase + 1023) / 1024;
        for (uint64_t t = 0; t < ntiles; t++) {
            uint32_t w[4];
            const int64_t toff = (int64_t)(sp.rbase + t * 1024);
            int nb = load_lane<16>(cx, toff + lane * 16, w);
            nb = (int)min((int64_t)nb, max((int64_t)0, (int64_t)sp.rend - (toff + lane * 16)));
            uint32_t h = lane_hdr_entry(w, nb, hdr);
            uint32_t cntu = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if (j < nb) {
                    uint32_t ch = fk_byte(w, j);
                    if (h) { if (ch == '\n') h = 0; }
                    else if (ch == '>') h = 1;
                    else if (ch != '\n' && ch != 'N' && ch != 0xFFu && fk_sym(ch) < 0) cntu++;
                }
            }
            uint32_t incl = cntu;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                uint32_t tv = shup(incl, d);
                if (lane >= d) incl += tv;
            }
            uint64_t o = base + incl - cntu;
            h = lane_hdr_entry(w, nb, hdr);
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if (j < nb) {
                    uint32_t ch = fk_byte(w, j);
                    if (h) { if (ch == '\n') h = 0; }
                    else if (ch == '>') h = 1;
                    else if (ch != '\n' && ch != 'N' && ch != 0xFFu && fk_sym(ch) < 0) {
                        if (opos) opos[o] = (uint64_t)(toff + lane * 16 + j);   /* (collect_unknown = 2) */
                        out[o++] = (uint8_t)ch;
                    }
                }
            }
            base += rdlane(incl, 63);
            hdr = rdlane(h, 63);
        }
    }
}

__global__ void k_add_short(uint32_t *shortcnt, uint64_t idx) { atomicAdd(&shortcnt[idx], 1u); }

/* engine reset: table, short-walk counts, accumulators and stream state in
   one launch */
__global__ void k_zero(uint32_t *table, uint64_t nbins, uint32_t *shortcnt, uint64_t nshort,
                       unsigned long long *acc, XState *state, uint32_t *subs, int nsub) {
    const uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    uint4 *t4 = reinterpret_cast<uint4 *>(table);
    for (uint64_t i = i0; i < nbins / 4; i += step) t4[i] = make_uint4(0, 0, 0, 0);
    uint4 *s4 = reinterpret_cast<uint4 *>(subs);
    for (uint64_t i = i0; i < (uint64_t)nsub * nbins / 4; i += step) s4[i] = make_uint4(0, 0, 0, 0);
    for (uint64_t i = (nbins / 4) * 4 + i0; i < nbins; i += step) table[i] = 0;
    for (uint64_t i = i0; i < nshort; i += step) shortcnt[i] = 0;
    if (i0 < (1 + FK_ACC_COPIES) * ACC_N) acc[i0] = 0;   /* engine + feed accumulators */
    if (i0 == 0) *state = XState{0, 0, 0, 0};
}

/* synthetic input: byte[i] = "ACGT"[(splitmix64(seed + (i>>5)) >> 2(i&31)) & 3] */
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__global__ void k_synth(uint8_t *out, uint64_t total, uint64_t seed, int fasta_line, uint64_t hlen) {
    const uint64_t i16 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 16;
    if (i16 >= total) return;
    uint8_t b[16];
    const char *hdr = ">synthetic\n";
    for (int j = 0; j < 16; j++) {
        uint64_t o = i16 + j;
        uint8_t v = 0;
        if (o < total) {
            if (o < hlen) {
                v = (uint8_t)hdr[o];
            } else {
                uint64_t q = o - hlen, i;
                if (fasta_line > 0) {
                    uint64_t L = (uint64_t)fasta_line;
                    uint64_t line = q / (L + 1), r = q % (L + 1);
                    if (r == L) { b[j] = '\n'; continue; }
                    i = line * L + r;
                } else {
                    i = q;
                }
                uint64_t wv = splitmix64(seed + (i >> 5));
                v = (uint8_t)"ACGT"[(wv >> (2 * (i & 31))) & 3];
            }
        }
        b[j] = v;
    }
    if (i16 + 16 <= total) {
        uint4 v;
        memcpy(&v, b, 16);
        *reinterpret_cast<uint4 *>(out + i16) = v;
    } else {
        for (int j = 0; j < 16 && i16 + j < total; j++) out[i16 + j] = b[j];
    }
}

/* upstream-regions-like FASTA (fk_synth_upstream_device): record r =
   ">ENST%011u\n" + 1001 bases + "\n"; rs = splitmix64((seed << 40) ^ r)
   draws the record's N block (rs % 100 == 0: 50 'N' from base (rs >> 32) %
   951) and seeds its bases (word j of the record: splitmix64(rs + 1 + j)) */
#define UP_HDR 17u
#define UP_BASES 1001u
__device__ __forceinline__ uint8_t upstream_byte(uint64_t seed, uint64_t rec, uint32_t p) {
    if (p == 0) return '>';
    if (p < 5) return (uint8_t)"ENST"[p - 1];
    if (p < UP_HDR - 1) {   /* 11 decimal digits, most significant first */
        uint64_t v = rec;
        for (uint32_t d = p; d < UP_HDR - 2; d++) v /= 10;
        return (uint8_t)('0' + v % 10);
    }
    if (p == UP_HDR - 1 || p == FK_UPSTREAM_REC - 1) return '\n';
    const uint32_t j = p - UP_HDR;
    const uint64_t rs = splitmix64((seed << 40) ^ rec);
    if (rs % 100 == 0) {
        const uint32_t n0 = (uint32_t)((rs >> 32) % (UP_BASES - 50));
        if (j >= n0 && j < n0 + 50) return 'N';
    }
    const uint64_t w = splitmix64(rs + 1 + (j >> 5));
    return (uint8_t)"ACGT"[(w >> (2 * (j & 31))) & 3];
}
__global__ void k_synth_upstream(uint8_t *out, uint64_t total, uint64_t first_rec, uint64_t seed) {
    const uint64_t i16 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 16;
    if (i16 >= total) return;
    uint8_t b[16];
    for (int j = 0; j < 16; j++) {
        const uint64_t o = i16 + j;
        b[j] = o < total ? upstream_byte(seed, first_rec + o / FK_UPSTREAM_REC, (uint32_t)(o % FK_UPSTREAM_REC)) : 0;
    }
    if (i16 + 16 <= total) {
        uint4 v;
        memcpy(&v, b, 16);
        *reinterpret_cast<uint4 *>(out + i16) = v;
    } else {
        for (int j = 0; j < 16 && i16 + j < total; j++) out[i16 + j] = b[j];
    }
}


__global__ void k_zero(uint32_t *table, uint64_t nbins, uint32_t *shortcnt, uint64_t nshort,
                       unsigned long long *acc, XState *state, uint32_t *subs, int nsub);

/* A reset is issued lazily, with the next device work (every API entry that
   touches the device goes through set_dev), so that it reaches the GPU
   back to back with that work. */
/* d_state written lazily, as a kernel argument (no pageable host copy on
   the host's critical path after a compact resolve), before the next kernel
   that reads it (count_segment's launches, k_scan); a direct write replaces
   a pending one */
__global__ void k_set_state(XState *d, XState v) { *d = v; }
int flush_state(fk_engine *e) {
    if (!e->dstate_pending) return FK_OK;
    e->dstate_pending = false;
    hipLaunchKernelGGL(k_set_state, dim3(1), dim3(1), 0, e->stream, e->d_state, e->dstate_val);
    HIPCHK(hipGetLastError());
    return FK_OK;
}
hipError_t write_dstate(fk_engine *e, const XState &x) {
    e->dstate_pending = false;
    return hipMemcpyAsync(e->d_state, &x, sizeof x, hipMemcpyHostToDevice, e->stream);
}

int flush_zero(fk_engine *e, bool keep_table) {
    if (!e->zero_pending) return FK_OK;
    e->zero_pending = false;
    const uint64_t nb = keep_table ? 0 : e->nbins;   /* (a fresh two-level count writes every bin itself) */
    const uint64_t work = std::max<uint64_t>(nb / 4, std::max<uint64_t>(e->nshort, (1 + FK_ACC_COPIES) * ACC_N));
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 8, (work + 255) / 256);
    hipLaunchKernelGGL(k_zero, dim3(grid), dim3(256), 0, e->stream, e->d_table, nb, e->d_short, e->nshort,
                       e->d_acc, e->d_state, e->d_sub, e->d_sub ? FK_SUBTABLES : 0);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* make e's device current; flush a pending reset unless the caller launches
   it itself right before its first kernel (count_segment: no host work
   between the two launches, so the GPU does not idle after k_zero) */
int set_dev(fk_engine *e, bool flush) {
    HIPCHK(hipSetDevice(e->dev));
    return flush ? flush_zero(e) : FK_OK;
}

extern "C" int fk_abi_version(void) { return FK_ABI_VERSION; }



extern "C" const char *fk_strerror(int s) {
    switch (s) {
    case FK_OK: return "ok";
    case FK_E_INVALID: return "invalid argument";
    case FK_E_K_UNSUPPORTED: return "k outside the dense-table range of this engine (1..16)";
    case FK_E_NO_DEVICE: return "no HIP device available";
    case FK_E_HIP: return "HIP runtime error";
    case FK_E_OOM: return "out of memory";
    case FK_E_EMPTY: return "Sequence File Is Empty, Ending Program";
    case FK_E_UNTERMINATED_HEADER: return "input ends inside a '>' header line";
    case FK_E_ROLLOVER: return "COUNTER ROLLOVER DETECTED";
    case FK_E_STATE: return "engine API called out of order";
    case FK_E_IO: return "I/O error";
    case FK_E_RCCL: return "collective failed";
    case FK_E_SUMMARY: return "shard summary does not apply to this state (exchange the full summaries)";
    case FK_E_INTERNAL: return "device-side bound check failed (counts not valid)";
    default: return "unknown error";
    }
}

extern "C" int fk_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}





int zero_all(fk_engine *e) {
    e->zero_pending = true;
    e->dirty = false;
    e->dstate_pending = false;   /* the reset zeroes d_state */
    e->state = XState{0, 0, 0, 0};
    memset(&e->last, 0, sizeof e->last);
    e->stats_valid = false;
    e->tail_added = false;
    e->fed = e->scanned = e->chunks = e->redo = 0;
    e->ended = 0;
    e->shard_pending = 0;
    e->dev_ms = e->main_ms = 0;
    e->timed_n = 0;
    e->keep_len = e->kst_len = 0;
    e->spsegs.clear();
    e->sp_distinct = 0;
    e->sp_done = false;
    e->unknown_bytes.clear();
    e->unknown_pos.clear();
    /* statistics a fresh two-level count left for the next launch_table_stats
       belong to the count this reset discards */
    e->fz_ready = false;
    e->glist_live = false;
    e->perr_live = false;
    return FK_OK;
}

extern "C" void fk_engine_destroy(fk_engine *e) {
    if (!e) return;
    hipSetDevice(e->dev);
    if (e->stream) hipStreamSynchronize(e->stream);
    hipFree(e->d_table); hipFree(e->d_short); hipFree(e->d_sub); hipFree(e->d_snap);
    hipFree(e->d_pairs);
    hipFree(e->d_parts); hipFree(e->d_pmeta); hipFree(e->d_rdesc); hipFree(e->d_rbm); hipFree(e->d_glist); hipFree(e->d_fz);
    hipFree(e->d_rsend); hipFree(e->d_rrecv); hipFree(e->d_raux); hipFree(e->d_rsz);
    for (int i = 0; i < fk_engine::NPOOL; i++) hipFree(e->pool_p[i]);
    hipFree(e->d_codes); hipFree(e->d_pidx); hipFree(e->d_pflag); hipFree(e->d_acc); hipFree(e->d_res); hipFree(e->d_tmp);
    hipFree(e->d_state); hipFree(e->d_rr); hipFree(e->d_rtrue);
    hipFree(e->d_redo); hipFree(e->d_tf); hipFree(e->d_stage); hipFree(e->d_resume);
    hipFree(e->d_aggs); hipFree(e->d_flags);
    hipFree(e->d_bsum); hipFree(e->d_ctl); hipFree(e->d_opc);
    hipFree(e->d_keep);
    hipFree(e->d_kst);
    hipFree(e->d_spk); hipFree(e->d_spc); hipFree(e->d_emit); hipFree(e->d_spdense);
    fks_free(&e->fks);
    if (e->h_stage) hipHostFree(e->h_stage);
    for (int i = 0; i < 3; i++) if (e->ev[i]) hipEventDestroy(e->ev[i]);
    if (e->h_res) hipHostFree(e->h_res);
    if (e->h_rows) hipHostFree(e->h_rows);
    hipFree(e->d_rows);
    hipFree(e->d_done);
    hipFree(e->d_tpart);
    if (e->own_stream && e->stream) hipStreamDestroy(e->stream);
    delete e;
}


/* One knob of FINDKMER_TUNE ("name=value,name=value"): true and *v = value
   when `name` is set. */
bool tune_knob(const char *name, uint64_t *v) {
    const char *t = getenv("FINDKMER_TUNE");
    if (!t) return false;
    const size_t n = strlen(name);
    for (const char *p = t; *p;) {
        if (strncmp(p, name, n) == 0 && p[n] == '=') {
            *v = strtoull(p + n + 1, nullptr, 10);
            return true;
        }
        const char *c = strchr(p, ',');
        if (!c) break;
        p = c + 1;
    }
    return false;
}

extern "C" int fk_engine_create(int k, const fk_opts *opts, fk_engine **out) {
    if (!out) return FK_E_INVALID;
    *out = nullptr;
    if (k < FK_K_MIN || k > FK_K_MAX_REF) return FK_E_INVALID;
    int ndev = fk_device_count();
    if (ndev <= 0) return FK_E_NO_DEVICE;
    fk_engine *e = new fk_engine();
    if (opts) e->opts = *opts;
    e->k = k;
    if (e->opts.device >= 0) e->dev = e->opts.device;
    else if (hipGetDevice(&e->dev) != hipSuccess) e->dev = 0;
    if (e->dev >= ndev) { delete e; return FK_E_NO_DEVICE; }
    int rc = set_dev(e);
    if (rc) { delete e; return rc; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, e->dev) == hipSuccess && prop.multiProcessorCount > 0)
        e->cus = prop.multiProcessorCount;
    /* test and tuning knobs, all in one variable FINDKMER_TUNE="name=value,..."
       (tune_knob): no_mixed=1 (tile_general instead of mixed tiles),
       part_general=N (general tiles k_part takes per range before
       k_part<RES>), static_pct=P / dyn_min_chunks=N (k_count's dynamic
       ranges), events=0 (no HIP events),
       seg_kb=N (device feeds cut into N-KiB segments), sp_pass=N (17 <= k:
       at most N window keys per sorted pass; smaller buckets merge, larger
       ones take the dense path; the key-list route), route=0/1/2 (k = 15,
       16 sharded tables reduce-scattered / routed at world > 1 / routed at
       world 1 too).  Read at finish (sparse_finish): sp_walk=0 (the
       key-list passes instead of the fused first-base walks),
       sp_walk_rows=N / sp_walk_glist=N (the walks' row and general-tile
       list capacities: tests of the restart), sp_walk_dbg=1 (every tile
       through k_sp_gtiles) */
    uint64_t kv = 0;
    if (tune_knob("no_mixed", &kv)) e->no_mixed = kv == 1;
    /* k_count takes a couple of general tiles per range (the stream start, an
       isolated comment line) and leaves denser ones to k_resume's mixed tiles */
    if (!e->no_mixed) e->general_tiles = 2;
    if (tune_knob("pairs_kmax", &kv)) e->part_pairs_kmax = (int)std::min<uint64_t>(kv, 12u);
    if (tune_knob("route", &kv)) e->route_mode = (int)std::min<uint64_t>(kv, 2u);
    if (tune_knob("part_general", &kv)) e->part_general = (uint32_t)kv;
    if (tune_knob("glist_cap", &kv)) e->glist_force = kv;
    if (tune_knob("w16", &kv)) e->w16_ks = ((uint32_t)kv & 0x3000u) | (1u << 14);   /* k = 12, 13 (14 always) */
    if (tune_knob("events", &kv)) e->timing = kv != 0;
    if (tune_knob("static_pct", &kv)) e->static_pct = (uint32_t)std::min<uint64_t>(100u, std::max<uint64_t>(1u, kv));
    if (tune_knob("dyn_min_chunks", &kv)) e->dyn_min_chunks = kv;
    if (tune_knob("sp_pass", &kv)) e->sp_pass = kv;
    if (e->opts.timing_every > 1) e->timing_every = (uint32_t)e->opts.timing_every;
    e->sparse = k > FK_K_MAX_DENSE;
    e->nbins = e->sparse ? 0 : 1ull << (2 * k);
    /* 8 <= k <= 16 partitioned (k = 15, 16 with a second level, k_repart) */
    e->part = k >= 8 && k <= 16;
    e->maskk = (1ull << (2 * k)) - 1;
    /* the short walks' counts serve nodeCounter alone (depth-1 touches are
       counters): an engine without it keeps none (k = 16: 5.7 GB less to
       zero per step) */
    e->nshort = k > 1 && !e->sparse && e->opts.want_nodes ? ((1ull << (2 * k)) - 4) / 3 : 0;
    if (e->opts.stream) {
        e->stream = (hipStream_t)e->opts.stream;
    } else {
        /* a blocking stream: feeds of device buffers order after work on the
           device's legacy default stream (where PyTorch's default stream
           runs), so a buffer just filled there is complete when read */
        if (hipStreamCreateWithFlags(&e->stream, hipStreamDefault) != hipSuccess) { delete e; return FK_E_HIP; }
        e->own_stream = true;
    }
#define ALLOC(p, bytes)                                                         \
    if (hipMalloc((void **)&(p), (bytes)) != hipSuccess) { fk_engine_destroy(e); return FK_E_OOM; }
    ALLOC(e->d_table, std::max<uint64_t>(e->nbins, 4) * sizeof(uint32_t));
    if (hist_mode(e) != H_GLOBAL) {
        ALLOC(e->d_sub, FK_SUBTABLES * e->nbins * sizeof(uint32_t));
        if (hipMemsetAsync(e->d_sub, 0, FK_SUBTABLES * e->nbins * sizeof(uint32_t), e->stream) != hipSuccess) {
            fk_engine_destroy(e);
            return FK_E_HIP;
        }
    }
    if (e->nshort) { ALLOC(e->d_short, e->nshort * sizeof(uint32_t)); }
    ALLOC(e->d_acc, (1 + FK_ACC_COPIES) * ACC_N * sizeof(unsigned long long));
    e->d_facc = e->d_acc + ACC_N;
    ALLOC(e->d_opc, sizeof(OnePassCfg));
    ALLOC(e->d_ctl, FK_CTL_WORDS * sizeof(uint32_t));   /* [0] k_tail's block count; k_count's pool heads */
    /* the feed accumulators are zero between feeds (a fresh one-pass feed
       does not launch k_zero) */
    if (hipMemsetAsync(e->d_acc, 0, (1 + FK_ACC_COPIES) * ACC_N * sizeof(unsigned long long), e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_ctl, 0, FK_CTL_WORDS * sizeof(uint32_t), e->stream) != hipSuccess) {
        fk_engine_destroy(e);
        return FK_E_HIP;
    }
    ALLOC(e->d_res, sizeof(DevRes));
    if (hipMemsetAsync(e->d_res, 0, sizeof(DevRes), e->stream) != hipSuccess) {
        fk_engine_destroy(e);
        return FK_E_HIP;
    }
    ALLOC(e->d_tmp, 8 * sizeof(unsigned long long));
    ALLOC(e->d_state, sizeof(XState));
    ALLOC(e->d_tf, sizeof(TF));
#undef ALLOC
    /* lds_add addresses the bins from LDS address 0: the kernels that count
       in LDS must not have static LDS (a build invariant, checked once) */
    if (!lds_layout_ok()) { fk_engine_destroy(e); return FK_E_HIP; }
    /* the LDS bins and slices need more than the default dynamic-LDS limit */
    if (scan_kernels_init(lds_bytes(e)) != FK_OK || (e->part && part_kernels_init() != FK_OK)) {
        fk_engine_destroy(e);
        return FK_E_HIP;
    }
    for (int i = 0; i < 3; i++)
        /* timing only (results travel through mapped memory): no system-scope
           fence, which costs a cache writeback + invalidate and a gap of
           several us around each recorded launch */
        if (hipEventCreateWithFlags(&e->ev[i], hipEventDisableSystemFence) != hipSuccess) {
            fk_engine_destroy(e);
            return FK_E_HIP;
        }
    if (hipHostMalloc((void **)&e->h_res, sizeof(DevRes), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&e->h_res_dev, e->h_res, 0) != hipSuccess ||
        hipMalloc((void **)&e->d_done, sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&e->d_tpart, (size_t)e->cus * 4 * 10 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemsetAsync(e->d_done, 0, sizeof(uint32_t), e->stream) != hipSuccess) {
        fk_engine_destroy(e);
        return FK_E_OOM;
    }
    memset(e->h_res, 0, sizeof(DevRes));
    rc = zero_all(e);
    if (rc == FK_OK && hipStreamSynchronize(e->stream) != hipSuccess) rc = FK_E_HIP;
    if (rc) { fk_engine_destroy(e); return rc; }
    *out = e;
    return FK_OK;
}

extern "C" int fk_engine_reset(fk_engine *e) {
    if (!e) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    return zero_all(e);
}

/* per-range arrays */
int grow_arrays(fk_engine *e, uint64_t nranges) {
    if (nranges > e->range_cap || !e->d_rr) {
        uint64_t nr = std::max<uint64_t>(nranges, 1024);
        hipFree(e->d_rr); hipFree(e->d_rtrue); hipFree(e->d_redo); hipFree(e->d_resume);
        hipFree(e->d_aggs); hipFree(e->d_flags); hipFree(e->d_bsum);
        e->d_rr = nullptr; e->d_rtrue = nullptr; e->d_redo = nullptr; e->d_resume = nullptr;
        e->d_aggs = nullptr; e->d_flags = nullptr; e->d_bsum = nullptr;
        if (hipMalloc((void **)&e->d_rr, nr * sizeof(RangeRec)) != hipSuccess) return FK_E_OOM;
        if (hipMalloc((void **)&e->d_rtrue, nr * sizeof(XState)) != hipSuccess) return FK_E_OOM;
        if (hipMalloc((void **)&e->d_redo, nr * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
        if (hipMalloc((void **)&e->d_resume, nr * sizeof(ResumeRec)) != hipSuccess) return FK_E_OOM;
        const size_t nb = nr / SCAN_THREADS + 1;
        if (hipMalloc((void **)&e->d_aggs, nb * sizeof(TF)) != hipSuccess) return FK_E_OOM;
        if (hipMalloc((void **)&e->d_flags, nb * sizeof(uint32_t) + 64) != hipSuccess) return FK_E_OOM;
        HIPCHK(hipMemsetAsync(e->d_flags, 0, nb * sizeof(uint32_t) + 64, e->stream));
        e->scan_epoch = 0;
        const size_t nblk = nr / FK_WAVES_PER_BLOCK + 1;
        if (hipMalloc((void **)&e->d_bsum, nblk * sizeof(BlockSum)) != hipSuccess) return FK_E_OOM;
        OnePassCfg c;
        c.bsum = e->d_bsum; c.rtrue = e->d_rtrue; c.acc_total = e->d_acc; c.host_res = e->h_res_dev;
        c.state = e->d_state;
        HIPCHK(hipMemcpy(e->d_opc, &c, sizeof c, hipMemcpyHostToDevice));
        e->range_cap = nr;
    }
    return FK_OK;
}


/* scan + redo (or the partitioned count) + table stats, then the results */
/* Can a run reach the reference's int32 seqSize zone (findKmer.cpp:977) in
   a segment of len bytes entered in state e->state? */
bool int32_zone_possible(const fk_engine *e, uint64_t len) {
    const uint64_t r0 = e->state.hdr ? 0 : (uint64_t)(uint32_t)e->state.R;
    return r0 + len + FK_CHUNK_BYTES > 0x7FFFFFFFull;
}

/* What the segment's device-side bound checks saw (DevRes::fault, k = 15,
   16).  A general-tile list that overflowed left windows out of a fresh
   table: the segment is the first since the reset (tab_fresh), so it is
   counted again over a zeroed table from the exact range states k_scan just
   computed, its general tiles' windows added by global atomics (launch_part
   with `exact` keeps no list).  Any other bit fails the feed. */
int check_fault(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
    const uint32_t f = e->last.fault;
    if (!f) return FK_OK;
    if (f != FK_FAULT_LIST || !e->seg_clean) return FK_E_INTERNAL;
    HIPCHK(hipMemsetAsync(e->d_table, 0, e->nbins * sizeof(uint32_t), e->stream));
    if (e->nshort) HIPCHK(hipMemsetAsync(e->d_short, 0, e->nshort * sizeof(uint32_t), e->stream));
    /* (k_table_stats cleared the feed counters when it folded them) */
    int rc = launch_part(e, buf, len, lo, g, 1, e->d_rtrue);
    if (rc) return rc;
    rc = launch_table_stats(e, false, tev(e, 2), true, true);   /* fresh: the counters start over */
    if (rc) return rc;
    rc = wait_results(e);
    if (rc) return rc;
    e->list_recounts++;
    e->redo += g.nranges;   /* (fk_result.redo_chunks: every range of the segment again) */
    return e->last.fault ? FK_E_INTERNAL : FK_OK;
}

int resolve_and_fetch(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
    int rc;
    if (e->op_pending) {
        /* a one-pass k_count published the results itself, or says what is
           left to do */
        e->op_pending = false;
        rc = wait_results(e);
        if (rc) return rc;
        const uint32_t need = e->last.need;
        if (need == 0) {
            e->stats_valid = true;
            return FK_OK;
        }
        if (need & ONE_RESUME) {
            rc = launch_resume(e, buf, len, lo, g);
            if (rc) return rc;
        }
        rc = launch_scan(e, g, 0);
        if (rc) return rc;
        rc = launch_redo(e, buf, len, lo, g, 0);
        if (rc) return rc;
        /* the tail folded the sub-tables already */
        rc = launch_table_stats(e, false, tev(e, 2), false, e->op_fresh);
        if (rc) return rc;
        rc = wait_results(e);
        if (rc) return rc;
        e->stats_valid = true;
        e->dev_ev = 2;
        e->redo += e->last.redo_n;
        return FK_OK;
    }
    e->dev_ev = 2;
    rc = launch_scan(e, g, 0);
    if (rc) return rc;
    if (e->part && int32_zone_possible(e, len)) {
        /* A run past 2^31-1 bases (the reference's seqSize turns negative,
           :977): every range in the negative zone was counted from a guess
           that says "deep in a run", and k_redo would cancel each one with
           global atomics (a 3 Gbase single-record FASTA at k=11: 36 ms).  If
           many guesses were wrong, undo the segment and count it again with
           the exact range states k_scan just computed (~2x one pass). */
        uint32_t n = 0;
        HIPCHK(hipMemcpyAsync(&n, &e->d_res->redo_n, sizeof n, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if ((uint64_t)n * 16 > g.nranges) {
            if (e->seg_snap) {
                HIPCHK(hipMemcpyAsync(e->d_table, e->d_snap, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                      e->stream));
                if (e->nshort)
                    HIPCHK(hipMemcpyAsync(e->d_short, e->d_snap + e->nbins, e->nshort * sizeof(uint32_t),
                                          hipMemcpyDeviceToDevice, e->stream));
            } else if (e->seg_clean) {
                HIPCHK(hipMemsetAsync(e->d_table, 0, e->nbins * sizeof(uint32_t), e->stream));
                if (e->nshort) HIPCHK(hipMemsetAsync(e->d_short, 0, e->nshort * sizeof(uint32_t), e->stream));
            } else {
                return FK_E_STATE;   /* cannot happen: a dirty table is snapshotted when the zone is possible */
            }
            HIPCHK(hipMemsetAsync(e->d_facc, 0, FK_ACC_COPIES * ACC_N * sizeof(unsigned long long), e->stream));
            rc = launch_part(e, buf, len, lo, g, 1, e->d_rtrue);
            if (rc) return rc;
            rc = launch_table_stats(e, false, tev(e, 2));
            if (rc) return rc;
            rc = wait_results(e);
            if (rc) return rc;
            if (e->last.fault) return FK_E_INTERNAL;   /* (no list: exact states) */
            e->stats_valid = true;
            e->redo += n;
            return FK_OK;
        }
    }
    rc = launch_redo(e, buf, len, lo, g, 0);
    if (rc) return rc;
    rc = launch_table_stats(e, false, tev(e, 2));
    if (rc) return rc;
    rc = wait_results(e);
    if (rc) return rc;
    e->redo += e->last.redo_n;
    rc = check_fault(e, buf, len, lo, g);
    if (rc) return rc;
    e->stats_valid = true;
    return FK_OK;
}

/* exact first 0xFF outside a header (range observations are exact after redo) */
__global__ void k_obs_eof(const RangeRec *rr, uint64_t n, unsigned long long *out) {
    unsigned long long eof = ~0ull;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x)
        if (rr[r].eof != FK_NO_EOF64) eof = min(eof, (unsigned long long)(rr[r].c0 * FK_CHUNK_BYTES + rr[r].eof));
    if (eof != ~0ull) atomicMin(out, eof);
}

int exact_eof(fk_engine *e, const Geo &g, unsigned long long &eof) {
    HIPCHK(hipMemsetAsync(e->d_tmp, 0xFF, sizeof(unsigned long long), e->stream));
    unsigned gr = (unsigned)std::min<uint64_t>(1024, g.nranges / 256 + 1);
    hipLaunchKernelGGL(k_obs_eof, dim3(gr), dim3(256), 0, e->stream, e->d_rr, g.nranges, e->d_tmp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&eof, e->d_tmp, sizeof eof, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* Collect the unknown bytes of the just-counted segment (stream order). */
int collect_unknown(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g) {
    if (!e->opts.collect_unknown) return FK_OK;
    std::vector<RangeRec> rr((size_t)g.nranges);
    HIPCHK(hipMemcpyAsync(rr.data(), e->d_rr, g.nranges * sizeof(RangeRec), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::vector<uint32_t> list;
    std::vector<uint64_t> offs;
    uint64_t acc = 0;
    for (uint64_t r = 0; r < g.nranges; r++)
        if (rr[(size_t)r].unknown) { list.push_back((uint32_t)r); offs.push_back(acc); acc += rr[(size_t)r].unknown; }
    if (!acc) return FK_OK;
    DevScratch s_list, s_offs, s_out, s_pos;
    if (!s_list.alloc(list.size() * 4) || !s_offs.alloc(offs.size() * 8) || !s_out.alloc(acc)) return FK_E_OOM;
    const bool want_pos = e->opts.collect_unknown == 2;
    if (want_pos && !s_pos.alloc(acc * 8)) return FK_E_OOM;
    uint32_t *d_list = s_list.as<uint32_t>();
    uint64_t *d_offs = s_offs.as<uint64_t>();
    uint8_t *d_out = s_out.as<uint8_t>();
    HIPCHK(hipMemcpyAsync(d_list, list.data(), list.size() * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(d_offs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, e->stream));
    unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((list.size() + 7) / 8, (uint64_t)e->cus * 2));
    hipLaunchKernelGGL(k_extract, dim3(gx), dim3(FK_BLOCK), 0, e->stream, dbuf, len, lo, e->d_rr, e->d_rtrue, d_list,
                       d_offs, (uint32_t)list.size(), d_out, want_pos ? s_pos.as<uint64_t>() : nullptr);
    HIPCHK(hipGetLastError());
    size_t old = e->unknown_bytes.size();
    e->unknown_bytes.resize(old + acc);
    HIPCHK(hipMemcpyAsync(e->unknown_bytes.data() + old, d_out, acc, hipMemcpyDeviceToHost, e->stream));
    if (want_pos) {
        e->unknown_pos.resize(old + acc);
        HIPCHK(hipMemcpyAsync(e->unknown_pos.data() + old, s_pos.p, acc * 8, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    if (want_pos) {
        /* buffer offsets -> stream offsets: every caller has just added this
           segment's `len` bytes to e->scanned */
        const uint64_t seg0 = e->scanned - len;
        for (size_t i = old; i < old + acc; i++) e->unknown_pos[i] += seg0;
    }
    return FK_OK;
}

/* Feed timings: k_count (ev0 -> ev1, recorded in its dispatch) and the whole
   device path (ev0 -> ev2, at the end of k_table_stats).  The host continues
   as soon as the result block is published, so ev2 may still be pending: it
   is read when the events are about to be reused, or at finish. */
void add_times(fk_engine *e) { e->times_pending = e->timing && e->cur_timed; }
void settle_times(fk_engine *e, bool wait) {
    if (!e->times_pending) return;
    hipEvent_t end = e->ev[e->dev_ev];
    if (!wait && hipEventQuery(end) != hipSuccess) {
        /* k_count's events completed long ago; the whole-path time is
           best effort here (finish() does not wait for it) */
        float a = 0;
        if (hipEventElapsedTime(&a, e->ev[0], e->ev[1]) == hipSuccess) { e->main_ms += a; e->timed_n++; }
        e->times_pending = false;
        return;
    }
    e->times_pending = false;
    float a = 0, b = 0;
    if (hipEventQuery(end) != hipSuccess) hipEventSynchronize(end);
    if (hipEventElapsedTime(&a, e->ev[0], e->ev[1]) == hipSuccess) { e->main_ms += a; e->timed_n++; }
    if (hipEventElapsedTime(&b, e->ev[0], end) == hipSuccess) e->dev_ms += b;
}

/*
 * Count one device-resident segment whose entering state is *d_state (exact).
 * has_init = 0 is the shard case (entering state unknown; resolved later).
 */
int count_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, int has_init, Geo &g,
                         bool shard) {
    g = geometry(e, len);
    int rc = grow_arrays(e, g.nranges);
    if (rc) return rc;
    rc = flush_state(e);
    if (rc) return rc;
    settle_times(e, true);   /* before ev[] are reused */
    e->cur_timed = (e->launch_no++ % e->timing_every) == 0;
    /* one pass (k_count resolves, folds and publishes by itself) where the
       bins live in LDS and the entering state is known; it also does a
       pending reset (without nodeCounter, whose short-walk counts k_count
       adds to from every block) */
    bool op = e->onepass && !e->part && LDS_MODE(hist_mode(e)) && (has_init || shard);
    const bool fresh = op && e->zero_pending && !e->opts.want_nodes;
    /* k = 15, 16 right after a reset: k_count_parts writes every bin of the
       table, so the reset leaves the table out (16 GiB at k = 16); not where
       the int32 seqSize zone can be reached (its recount needs the zeroed
       table, and k_part<RES> counts such tiles with the general walk) */
    /* (k = 12..14 through k_bucket16 too, round 5) */
    e->tab_fresh = e->part && (e->k >= 15 || (e->k >= 12 && ((e->w16_ks >> e->k) & 1u))) && e->zero_pending &&
                   !e->no_mixed && !int32_zone_possible(e, len);
    if (fresh) {
        e->zero_pending = false;
    } else {
        rc = flush_zero(e, e->tab_fresh);      /* a pending reset, just before the first launch */
        if (rc) return rc;
    }
    e->op_pending = op;
    e->op_fresh = fresh;
    e->seg_clean = !e->dirty;
    e->dirty = true;
    e->seg_snap = false;
    if (e->part && !e->seg_clean && int32_zone_possible(e, len)) {
        /* the guessed count may have to be undone (resolve_and_fetch) */
        const uint64_t n = e->nbins + e->nshort;
        if (n > e->snap_cap) {
            hipFree(e->d_snap);
            e->d_snap = nullptr;
            e->snap_cap = 0;
            if (hipMalloc((void **)&e->d_snap, n * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
            e->snap_cap = n;
        }
        HIPCHK(hipMemcpyAsync(e->d_snap, e->d_table, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
        if (e->nshort)
            HIPCHK(hipMemcpyAsync(e->d_snap + e->nbins, e->d_short, e->nshort * sizeof(uint32_t),
                                  hipMemcpyDeviceToDevice, e->stream));
        e->seg_snap = true;
    }
    if (e->part) {
        /* 8 <= k <= 12: partitioned counting (k_part + k_bucket_count) */
        rc = launch_part(e, dbuf, len, lo, g, has_init);
        if (rc) return rc;
    } else {
        rc = launch_count(e, dbuf, len, lo, g, has_init, op, fresh, shard);
        if (rc) return rc;
        if (!op) {
            rc = launch_resume(e, dbuf, len, lo, g);
            if (rc) return rc;
        }
    }
    e->chunks += g.nchunks;
    return FK_OK;
}


/* After resolve: handle a 0xFF byte (recount the prefix) and unknown bytes. */
int finish_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g,
                          const XState &entering) {
    add_times(e);
    if (e->last.eof_cand != NO_EOF64) {
        unsigned long long eof = NO_EOF64;
        int rc = exact_eof(e, g, eof);
        if (rc) return rc;
        if (eof != NO_EOF64) {
            /* A 0xFF byte outside a header ends the reference's scan (:988):
               undo this segment and count only the bytes before it. */
            rc = launch_redo(e, dbuf, len, lo, g, 1);
            if (rc) return rc;
            HIPCHK(write_dstate(e, entering));
            e->ended = 1;
            e->scanned += eof;
            if (eof == 0) {
                rc = launch_table_stats(e, true);
                if (rc) return rc;
                rc = wait_results(e);
                if (rc) return rc;
                e->state = entering;
                return FK_OK;
            }
            Geo g2;
            rc = count_segment(e, dbuf, eof, lo, 1, g2);
            if (rc) return rc;
            rc = resolve_and_fetch(e, dbuf, eof, lo, g2);
            if (rc) return rc;
            add_times(e);
            e->state = e->last.exit;
            return collect_unknown(e, dbuf, eof, lo, g2);
        }
    }
    e->state = e->last.exit;
    e->scanned += len;
    return collect_unknown(e, dbuf, len, lo, g);
}

/* grow a retained device buffer to `need` bytes (geometrically, contents kept) */
int sp_grow(fk_engine *e, void **buf, uint64_t *cap, uint64_t used, uint64_t need) {
    if (need <= *cap && *buf) return FK_OK;
    const uint64_t c = std::max<uint64_t>(need, std::max<uint64_t>(*cap + *cap / 2, 1u << 20));
    void *p = nullptr;
    if (hipMalloc(&p, c) != hipSuccess) return FK_E_OOM;
    if (used) HIPCHK(hipMemcpyAsync(p, *buf, used, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    hipFree(*buf);
    *buf = p;
    *cap = c;
    return FK_OK;
}

/* keep a counted segment's bytes and its ranges' exact entering states
   (d_rtrue from the feed's k_scan) for finish's key-range passes */
int sp_retain(fk_engine *e, const uint8_t *dbuf, uint64_t len, const Geo &g) {
    /* borrowed (opts.borrow_input, a 16-B aligned device feed): finish reads
       the caller's bytes again; no copy (a 10 GB feed: 4.4 ms of a k = 17
       step) */
    const bool borrow = e->seg_borrow && ((uintptr_t)dbuf & 15) == 0;
    int rc = borrow ? FK_OK : sp_grow(e, (void **)&e->d_keep, &e->keep_cap, e->keep_len, e->keep_len + len + 16);
    if (rc) return rc;
    const uint64_t sb = g.nranges * sizeof(XState);
    rc = sp_grow(e, (void **)&e->d_kst, &e->kst_cap, e->kst_len * sizeof(XState), (e->kst_len + g.nranges) * sizeof(XState));
    if (rc) return rc;
    if (!borrow) HIPCHK(hipMemcpyAsync(e->d_keep + e->keep_len, dbuf, len, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->d_kst + e->kst_len, e->d_rtrue, sb, hipMemcpyDeviceToDevice, e->stream));
    e->spsegs.push_back({borrow ? 0 : e->keep_len, len, e->kst_len, g.nranges, g.cpw, g.nchunks, borrow ? dbuf : nullptr});
    /* segments start 16-B aligned in d_keep (load_lane's vector loads; it
       never reads past a segment's end), so small feeds cost little */
    if (!borrow) e->keep_len += (len + 15) / 16 * 16;
    e->kst_len += g.nranges;
    return FK_OK;
}

/*
 * A segment for 17 <= k <= 20: the state pass (k_count / k_resume in H_NONE
 * mode, k_scan) gives every range its exact entering state; k_redo mode 2
 * then takes the segment's counters and exact observations from those
 * states, and the segment's bytes and states are retained for finish.  A
 * 0xFF byte outside a header: cancel the counters and count the prefix again.
 */
int sparse_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, bool prefix) {
    const XState entering = e->state;
    Geo g;
    int rc = count_segment(e, dbuf, len, 0, 1, g);
    if (rc) return rc;
    rc = launch_scan(e, g, 0);
    if (rc) return rc;
    rc = launch_redo(e, dbuf, len, 0, g, 2);
    if (rc) return rc;
    rc = launch_table_stats(e, false, tev(e, 2));   /* no dense table: publishes counters and state */
    if (rc) return rc;
    rc = wait_results(e);
    if (rc) return rc;
    add_times(e);
    if (!prefix && e->last.eof_cand != NO_EOF64) {
        unsigned long long eof = NO_EOF64;
        rc = exact_eof(e, g, eof);
        if (rc) return rc;
        if (eof != NO_EOF64) {
            rc = launch_redo(e, dbuf, len, 0, g, 1);
            if (rc) return rc;
            HIPCHK(write_dstate(e, entering));
            e->state = entering;
            e->ended = 1;
            e->scanned += eof;
            if (eof == 0) {
                rc = launch_table_stats(e, true);
                if (rc) return rc;
                return wait_results(e);
            }
            return sparse_segment(e, dbuf, eof, true);
        }
    }
    e->state = e->last.exit;
    if (!prefix) e->scanned += len;
    rc = sp_retain(e, dbuf, len, g);
    if (rc) return rc;
    return collect_unknown(e, dbuf, len, 0, g);
}

int process_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len) {
    if (len == 0 || e->ended) return FK_OK;
    if (len < FK_LANE_BYTES && dbuf != e->d_stage) {
        /* too short for the clamped prefetch: copy into the staging buffer */
        if (!e->d_stage && hipMalloc((void **)&e->d_stage, STAGE_BYTES) != hipSuccess) return FK_E_OOM;
        HIPCHK(hipMemcpyAsync(e->d_stage, dbuf, len, hipMemcpyDeviceToDevice, e->stream));
        dbuf = e->d_stage;
    }
    if (e->sparse) return sparse_segment(e, dbuf, len);
    XState entering = e->state;
    Geo g;
    int rc = count_segment(e, dbuf, len, 0, 1, g);
    if (rc) return rc;
    rc = resolve_and_fetch(e, dbuf, len, 0, g);
    if (rc) return rc;
    return finish_segment(e, dbuf, len, 0, g, entering);
}

/* Segment length of a device feed.  8 <= k <= 12 allocates ~2 bytes of
   partition codes per input byte of a segment (k_part's rows, both
   regions): when free HBM cannot hold that for the whole feed (other
   processes on the GPU, k6thru11fullANDupstream.sh:16-24), the feed is cut
   into segments that fit -- segments carry the exact scan state, so the
   counts do not depend on the cut. */
uint64_t segment_budget(fk_engine *e, uint64_t len) {
    uint64_t seg = SEG_MAX_BYTES, kv = 0;
    if (tune_knob("seg_kb", &kv) && kv)   /* tests: segments of this many KiB */
        return std::max<uint64_t>(FK_CHUNK_BYTES, (kv << 10) / FK_CHUNK_BYTES * FK_CHUNK_BYTES);
    if (!e->part) return seg;
    /* codes (two row regions) + run index, bytes per input byte: 16-bit codes
       of 2 tiles per row, or 32-bit codes of one tile (k >= 15) */
    const uint64_t per = e->k >= 15 ? 2 * 2 * sizeof(uint32_t) + 2 + 1 : 2 * sizeof(uint16_t) + 1;   /* (+ the part streams) */
    if (std::min(len, seg) * per <= e->codes_cap * sizeof(uint16_t)) return seg;   /* already allocated */
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return seg;
    const uint64_t margin = 512ull << 20;
    const uint64_t avail = (uint64_t)fr + e->codes_cap * sizeof(uint16_t) + e->pidx_cap * sizeof(uint32_t);
    const uint64_t fit = avail > margin ? (avail - margin) / per : 0;
    const uint64_t floor_seg = 64ull << 20;
    if (fit < seg) seg = std::max(floor_seg, fit / FK_CHUNK_BYTES * FK_CHUNK_BYTES);
    return seg;
}

extern "C" int fk_engine_feed(fk_engine *e, const uint8_t *buf, uint64_t len, int on_device) {
    if (!e || (!buf && len)) return FK_E_INVALID;
    if (e->shard_pending) return FK_E_STATE;
    int rc = set_dev(e, false);   /* count_segment flushes a pending reset */
    if (rc) return rc;
    e->fed += len;
    if (e->ended || len == 0) return FK_OK;
    if (e->tail_added) return FK_E_STATE;     /* finish() already closed the stream */
    /* k_count's prefetch loads are clamped to [0, len-32]: inputs shorter
       than one lane go through the (larger) staging buffer */
    if (on_device && ((uintptr_t)buf & 15) == 0 && len >= FK_LANE_BYTES) {
        const uint64_t seg = segment_budget(e, len);
        e->seg_borrow = e->opts.borrow_input != 0;
        for (uint64_t off = 0; off < len && !e->ended; off += seg) {
            rc = process_segment(e, buf + off, std::min(seg, len - off));
            if (rc) { e->seg_borrow = false; return rc; }
        }
        e->seg_borrow = false;
        return FK_OK;
    }
    /* stage through pinned host memory (or realign device input) */
    if (!e->d_stage && hipMalloc((void **)&e->d_stage, STAGE_BYTES) != hipSuccess) return FK_E_OOM;
    if (!on_device && !e->h_stage &&
        hipHostMalloc((void **)&e->h_stage, STAGE_BYTES, hipHostMallocDefault) != hipSuccess)
        return FK_E_OOM;
    for (uint64_t off = 0; off < len && !e->ended; off += STAGE_BYTES) {
        uint64_t n = std::min(STAGE_BYTES, len - off);
        if (on_device) {
            HIPCHK(hipMemcpyAsync(e->d_stage, buf + off, n, hipMemcpyDeviceToDevice, e->stream));
        } else {
            memcpy(e->h_stage, buf + off, n);
            HIPCHK(hipMemcpyAsync(e->d_stage, e->h_stage, n, hipMemcpyHostToDevice, e->stream));
        }
        rc = process_segment(e, e->d_stage, n);
        if (rc) return rc;
    }
    return FK_OK;
}

extern "C" int fk_engine_state(fk_engine *e, fk_state *out) {
    if (!e || !out) return FK_E_INVALID;
    out->run = e->state.R;
    out->code = fk_sigma(e->state.code);     /* API codes use A0 C1 G2 T3 */
    out->hdr = e->state.hdr;
    out->ended = e->ended ? 1u : 0u;
    return FK_OK;
}

/* ---- shards ---- */

extern "C" int fk_engine_feed_shard(fk_engine *e, const uint8_t *buf, uint64_t len, uint64_t halo,
                                    int on_device) {
    if (!e || !buf || !on_device) return FK_E_INVALID;   /* shards are device-resident */
    if (e->fed || e->shard_pending) return FK_E_STATE;
    if (len > SEG_MAX_BYTES || ((uintptr_t)buf & 15) || (halo & 15)) return FK_E_INVALID;
    if (len && len < FK_LANE_BYTES) return FK_E_INVALID;   /* shards are at least one lane */
    int rc = set_dev(e, false);
    if (rc) return rc;
    e->fed = len;
    e->shard_buf = buf;
    e->shard_len = len;
    e->shard_lo = -(int64_t)std::min<uint64_t>(halo, FK_HALO_BYTES);
    e->shard_pending = 1;
    e->shard_op = e->shard_waited = e->shard_full = e->shard_resumed = false;
    if (len == 0) return flush_zero(e);
    Geo g;
    rc = count_segment(e, buf, len, e->shard_lo, 0, g, true);
    if (rc) return rc;
    if (e->op_pending) {
        /* one pass: k_tail publishes a compact summary (fetched lazily) */
        e->op_pending = false;
        e->shard_op = true;
        return FK_OK;
    }
    return launch_scan(e, g, 1);
}

/* the one-pass shard's result block (once) */
int shard_wait(fk_engine *e) {
    if (!e->shard_op || e->shard_waited) return FK_OK;
    int rc = wait_results(e);
    if (rc) return rc;
    e->shard_waited = true;
    return FK_OK;
}

/* the full transfer function of a one-pass shard (k_resume if a range ran
   out of general tiles, then k_scan mode 1) into d_tf */
int shard_full_tf(fk_engine *e) {
    if (!e->shard_op || e->shard_full) return FK_OK;
    int rc = shard_wait(e);
    if (rc) return rc;
    const Geo g = geometry(e, e->shard_len);
    if ((e->last.need & ONE_RESUME) && !e->shard_resumed) {
        rc = launch_resume(e, e->shard_buf, e->shard_len, e->shard_lo, g);
        if (rc) return rc;
        e->shard_resumed = true;
    }
    rc = launch_scan(e, g, 1);
    if (rc) return rc;
    e->shard_full = true;
    return FK_OK;
}


extern "C" int fk_engine_summary(fk_engine *e, fk_summary *out) {
    if (!e || !out) return FK_E_INVALID;
    static_assert(sizeof(TF) <= sizeof(fk_summary) - 8, "summary too small");
    memset(out, 0, sizeof *out);
    if (e->shard_pending && e->shard_len && e->shard_op && !e->shard_full) {
        int rc = set_dev(e);
        if (rc) return rc;
        rc = shard_wait(e);
        if (rc) return rc;
        if (e->last.need == 0) {
            const ShardSum &ss = e->last.shard;
            out->w[0] = ss.g_code;
            out->w[1] = (uint64_t)ss.g_R | ((uint64_t)ss.g_hdr << 32);
            out->w[2] = ss.nvb0;
            out->w[3] = ss.c_R;
            out->w[4] = ss.c_code;
            out->w[5] = (uint64_t)ss.c_hdr | ((uint64_t)ss.absorb << 32);
            out->w[6] = ss.nv;
            out->w[7] = e->shard_len;
            out->w[8] = (uint64_t)e->k;
            /* the guesses hold for every equivalent entering state, so a 0xFF
               byte they saw outside a header ends the stream in this shard */
            out->w[9] = e->last.eof_cand != NO_EOF64 ? 1u : 0u;
            out->w[11] = FK_SUMMARY_COMPACT;
            return FK_OK;
        }
    }
    return fk_engine_summary_full(e, out);
}

extern "C" int fk_engine_summary_full(fk_engine *e, fk_summary *out) {
    if (!e || !out) return FK_E_INVALID;
    memset(out, 0, sizeof *out);
    TF t = fk_identity();
    if (e->shard_pending && e->shard_len) {
        int rc = set_dev(e);
        if (rc) return rc;
        rc = shard_full_tf(e);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(&t, e->d_tf, sizeof t, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    memcpy(out, &t, sizeof t);
    return FK_OK;
}

/* A compact summary applied to an entering state (false: it does not apply:
   the state would count the shard's first range differently from its guess,
   or a run could reach the int32 wrap, which its local checks exclude). */
bool compact_apply(const fk_summary *s, const XState &in, XState &out) {
    const DState g{s->w[0], (uint32_t)s->w[1], (uint32_t)(s->w[1] >> 32)};
    const int k = (int)s->w[8];
    if (!fk_equiv(g, in, k, s->w[2])) return false;
    if (!in.hdr && (uint64_t)(uint32_t)in.R + s->w[7] + FK_CHUNK_BYTES > 0x7FFFFFFFull) return false;
    const uint32_t c_hdr = (uint32_t)s->w[5], absorb = (uint32_t)(s->w[5] >> 32);
    if (absorb) {
        out = XState{s->w[3], s->w[4], c_hdr, 0};
    } else {
        /* no run break and no header in the shard: a shift */
        out = XState{in.R + s->w[6], fk_join(in.code, s->w[4], s->w[6]), c_hdr, 0};
    }
    return true;
}

extern "C" int fk_summary_is_full(const fk_summary *s) {
    if (!s) return FK_E_INVALID;
    return s->w[11] == FK_SUMMARY_COMPACT ? 0 : 1;
}

extern "C" int fk_summary_apply(const fk_summary *s, const fk_state *in, fk_state *out) {
    if (!s || !in || !out) return FK_E_INVALID;
    if (in->ended > 1) return FK_E_INVALID;   /* 0 or 1 only (the field was padding before ABI 1.1) */
    if (in->ended) {           /* absorbing: the stream ended before this span */
        *out = *in;
        return FK_OK;
    }
    XState x{in->run, fk_sigma(in->code), in->hdr, 0};
    XState y;
    uint32_t ended = 0;
    if (s->w[11] == FK_SUMMARY_COMPACT) {
        if (!compact_apply(s, x, y)) return FK_E_SUMMARY;
        ended = s->w[9] ? 1u : 0u;
    } else {
        TF t;
        memcpy(&t, s, sizeof t);
        y = fk_apply(t, x);
    }
    out->run = y.R;
    out->code = fk_sigma(y.code);
    out->hdr = y.hdr;
    out->ended = ended;
    return FK_OK;
}

extern "C" int fk_engine_resolve(fk_engine *e, const fk_state *entering) {
    if (!e || !entering) return FK_E_INVALID;
    if (!e->shard_pending) return FK_E_STATE;
    /* `ended` is 0 or 1: a caller that left the old padding word
       uninitialised gets an error, not a silently dropped shard */
    if (entering->ended > 1) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    XState in{entering->run, fk_sigma(entering->code), entering->hdr, 0};
    if (entering->ended == 1) {
        /* the stream ended before this shard (a 0xFF byte in an earlier one,
           :988): it counts nothing; the pending count is zeroed lazily */
        const uint64_t len = e->shard_len;
        zero_all(e);
        e->fed = len;
        e->ended = 1;
        e->state = in;
        return FK_OK;
    }
    if (e->sparse) {
        /* 17 <= k <= 20: the shard's state pass only fixed its transfer
           function; count it now from the exact entering state (and retain
           it for finish's key-range passes) */
        e->shard_pending = 0;
        e->state = in;
        HIPCHK(write_dstate(e, in));
        if (e->shard_len == 0) {
            HIPCHK(hipStreamSynchronize(e->stream));
            return FK_OK;
        }
        e->chunks -= geometry(e, e->shard_len).nchunks;   /* counted again below */
        e->seg_borrow = e->opts.borrow_input != 0;   /* (a shard is the caller's device buffer) */
        const int rc2 = sparse_segment(e, e->shard_buf, e->shard_len);
        e->seg_borrow = false;
        return rc2;
    }
    /* the shard's compact summary, taken while the shard is still pending
       (fk_engine_summary describes a pending shard only) */
    fk_summary s;
    bool compact = false;
    if (e->shard_len && e->shard_op) {
        rc = shard_wait(e);
        if (rc) return rc;
        if (e->last.need == 0 && !e->shard_full) {
            rc = fk_engine_summary(e, &s);
            if (rc) return rc;
            compact = s.w[11] == FK_SUMMARY_COMPACT;
        }
    }
    e->shard_pending = 0;
    e->state = in;
    if (e->shard_len == 0) {
        HIPCHK(write_dstate(e, in));
        HIPCHK(hipStreamSynchronize(e->stream));
        return FK_OK;
    }
    Geo g = geometry(e, e->shard_len);
    if (e->shard_op) {
        if (compact) {
            XState ex;
            if (compact_apply(&s, in, ex)) {
                /* the guessed states count exactly: nothing to recount */
                e->last.exit = ex;
                e->dstate_val = ex;
                e->dstate_pending = true;
                e->stats_valid = true;
                return finish_segment(e, e->shard_buf, e->shard_len, e->shard_lo, g, in);
            }
        }
        /* the multi-launch path from the exact entering state: k_scan lists
           the ranges whose guess counts differently, k_redo recounts them */
        if ((e->last.need & ONE_RESUME) && !e->shard_resumed) {
            rc = launch_resume(e, e->shard_buf, e->shard_len, e->shard_lo, g);
            if (rc) return rc;
            e->shard_resumed = true;
        }
        HIPCHK(write_dstate(e, in));
        HIPCHK(hipMemsetAsync(&e->d_res->redo_n, 0, sizeof(uint32_t), e->stream));
        HIPCHK(hipMemsetAsync(&e->d_res->eof_cand, 0xFF, sizeof(unsigned long long), e->stream));
        rc = launch_scan(e, g, 0);
        if (rc) return rc;
        rc = launch_redo(e, e->shard_buf, e->shard_len, e->shard_lo, g, 0);
        if (rc) return rc;
        /* k_tail folded the sub-tables, and merged the feed's counters if
           it published a complete result */
        rc = launch_table_stats(e, false, tev(e, 2), false, e->op_fresh && e->last.need != 0);
        if (rc) return rc;
        rc = wait_results(e);
        if (rc) return rc;
        e->stats_valid = true;
        e->redo += e->last.redo_n;
        return finish_segment(e, e->shard_buf, e->shard_len, e->shard_lo, g, in);
    }
    HIPCHK(write_dstate(e, in));
    rc = resolve_and_fetch(e, e->shard_buf, e->shard_len, e->shard_lo, g);
    if (rc) return rc;
    return finish_segment(e, e->shard_buf, e->shard_len, e->shard_lo, g, in);
}

extern "C" int fk_engine_finish(fk_engine *e, fk_result *res) {
    if (!e || !res) return FK_E_INVALID;
    if (e->shard_pending) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    memset(res, 0, sizeof *res);
    const int k = e->k;
    /* an input ending with a run of 1..k-1 bases leaves its prefix walk */
    int32_t seq = (int32_t)(uint32_t)e->state.R;
    if (e->sparse) {
        if (!e->sp_done) {
            rc = sparse_finish(e, seq);
            if (rc) return rc;
            e->sp_done = true;
        }
    } else if (!e->state.hdr && seq >= 1 && seq < k && e->opts.want_nodes && !e->tail_added) {
        uint64_t off = ((1ull << (2 * seq)) - 4) / 3;
        uint64_t idx = off + fk_sigma(e->state.code & ((1ull << (2 * seq)) - 1));
        hipLaunchKernelGGL(k_add_short, dim3(1), dim3(1), 0, e->stream, e->d_short, idx);
        HIPCHK(hipGetLastError());
    }
    e->tail_added = true;
    if (!e->stats_valid) {
        rc = launch_table_stats(e, true);
        if (rc) return rc;
        rc = wait_results(e);
        if (rc) return rc;
        e->stats_valid = true;
    }
    static_assert(offsetof(DevRes, acc) == offsetof(DevRes, tstat) + sizeof(((DevRes *)0)->tstat),
                  "tstat and acc are fetched with one copy");
    /* the table stats and the accumulator snapshot of the last feed (or of
       the call above) describe the engine: no device round trip here */
    settle_times(e, false);
    if (e->sparse) memcpy(e->last.tstat, e->sp_tstat, sizeof e->sp_tstat);
    const unsigned long long *acc = e->last.acc;
    const unsigned long long *ts = e->last.tstat;
    res->windows = acc[ACC_WIN];
    /* every window's last base is a base the reference counts; a run's first
       window also counts its first k-1 bases (:1035-1057) */
    for (int b = 0; b < 4; b++) {
        res->base_count[b] = ts[2 + b] + acc[ACC_BASE + b];
        res->depth1[b] = ts[6 + b] + acc[ACC_D1S + b];
        if (res->depth1[b] >= (1ull << 32)) res->rollover = 1;
    }
    /* a bin that wrapped past 2^32 loses 2^32 from the table total: some trie
       counter reached 2^32 -> the reference's rollover exit (:642) */
    if (ts[1] != res->windows) res->rollover = 1;
    if (e->sparse && e->sp_roll) res->rollover = 1;
    res->valid_bases = res->windows + acc[ACC_VALID];
    res->distinct = ts[0];
    res->unknown_chars = acc[ACC_UNK];
    res->scanned_bytes = e->ended ? e->scanned : e->fed;
    res->hit_eof_byte = e->ended;
    res->unterminated_header = e->state.hdr ? 1 : 0;
    res->chunks = e->chunks;
    res->redo_chunks = e->redo;
    res->device_ms = e->dev_ms;
    res->main_kernel_ms = e->main_ms;
    res->timed_kernels = e->timed_n;
    uint64_t any_walk = res->depth1[0] | res->depth1[1] | res->depth1[2] | res->depth1[3];
    if (e->opts.want_nodes && e->sparse) {
        res->nodes = e->sp_nodes;
        res->nodes_valid = 1;
    } else if (e->opts.want_nodes) {
        /* nodeCounter = head + distinct prefixes of every walk (:620) */
        uint64_t nodes = 0;
        if (any_walk) {
            nodes = 1 + res->distinct;
            if (k >= 2) {
                DevScratch sa, sb;
                uint64_t n1 = 1ull << (2 * (k - 1));
                if (!sa.alloc(n1) || !sb.alloc(std::max<uint64_t>(n1 / 4, 4))) return FK_E_OOM;
                uint8_t *cur = sa.as<uint8_t>(), *nxt = sb.as<uint8_t>();
                for (int d = k - 1; d >= 1; d--) {
                    uint64_t nd = 1ull << (2 * d);
                    uint64_t off = ((1ull << (2 * d)) - 4) / 3;
                    HIPCHK(hipMemsetAsync(e->d_tmp, 0, sizeof(unsigned long long), e->stream));
                    unsigned g = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 4, nd / 256 + 1);
                    if (d == k - 1)
                        hipLaunchKernelGGL(k_fold_from_table, dim3(g), dim3(256), 0, e->stream, e->d_table,
                                           e->d_short + off, cur, nd, e->d_tmp);
                    else
                        hipLaunchKernelGGL(k_fold_level, dim3(g), dim3(256), 0, e->stream, nxt,
                                           e->d_short + off, cur, nd, e->d_tmp);
                    HIPCHK(hipGetLastError());
                    unsigned long long c = 0;
                    HIPCHK(hipMemcpyAsync(&c, e->d_tmp, sizeof c, hipMemcpyDeviceToHost, e->stream));
                    HIPCHK(hipStreamSynchronize(e->stream));
                    nodes += c;
                    std::swap(cur, nxt);   /* this level becomes the child level */
                }
            }
        }
        res->nodes = nodes;
        res->nodes_valid = 1;
    }
    if (e->fed == 0) return FK_E_EMPTY;
    if (res->rollover) return FK_E_ROLLOVER;
    if (res->unterminated_header) return FK_E_UNTERMINATED_HEADER;
    return FK_OK;
}

extern "C" int fk_engine_progress(fk_engine *e, uint64_t *valid_bases, uint64_t *windows) {
    if (!e) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    unsigned long long acc[ACC_N];
    HIPCHK(hipMemcpyAsync(acc, e->d_acc, sizeof acc, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (valid_bases) *valid_bases = acc[ACC_WIN] + acc[ACC_VALID];
    if (windows) *windows = acc[ACC_WIN];
    return FK_OK;
}

extern "C" int fk_engine_table(fk_engine *e, uint32_t *counts) {
    if (!e || !counts) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: fk_engine_sparse */
    int rc = set_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(counts, e->d_table, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_table_range(fk_engine *e, uint64_t first, uint64_t n, uint32_t *counts) {
    if (!e || (!counts && n) || first > e->nbins || n > e->nbins - first) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: fk_engine_sparse */
    int rc = set_dev(e);
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpyAsync(counts, e->d_table + first, n * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_table_device(fk_engine *e, uint32_t **dev_counts) {
    if (!e || !dev_counts) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: fk_engine_sparse */
    int rc = set_dev(e);
    if (rc) return rc;
    *dev_counts = e->d_table;
    return FK_OK;
}

extern "C" int fk_engine_table_to_device(fk_engine *e, void *dst) {
    if (!e || !dst) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: fk_engine_sparse */
    int rc = set_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(dst, e->d_table, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_table_from_device(fk_engine *e, const void *src) {
    if (!e || !src) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: fk_engine_sparse */
    int rc = set_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(e->d_table, src, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->stats_valid = false;
    return FK_OK;
}

extern "C" int fk_engine_unknown(fk_engine *e, uint8_t *out, uint64_t cap, uint64_t *n) {
    if (!e || !n) return FK_E_INVALID;
    *n = e->unknown_bytes.size();
    if (out) memcpy(out, e->unknown_bytes.data(), std::min<uint64_t>(cap, *n));
    return FK_OK;
}

/* The unknown bytes from index `first` on (stream order) and, with
   collect_unknown = 2, their stream offsets; *n receives the total so far. */
extern "C" int fk_engine_unknown_since(fk_engine *e, uint64_t first, uint8_t *out, uint64_t *pos, uint64_t cap,
                                       uint64_t *n) {
    if (!e || !n) return FK_E_INVALID;
    if (pos && e->opts.collect_unknown != 2) return FK_E_STATE;
    *n = e->unknown_bytes.size();
    if (first >= *n) return FK_OK;
    const uint64_t m = std::min<uint64_t>(cap, *n - first);
    if (out) memcpy(out, e->unknown_bytes.data() + first, m);
    if (pos) memcpy(pos, e->unknown_pos.data() + first, m * sizeof(uint64_t));
    return FK_OK;
}

__global__ void k_add_tables(uint32_t *dst, const uint32_t *src, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] += src[i];
}
__global__ void k_add_acc(unsigned long long *dst, const unsigned long long *src, int n) {
    int i = threadIdx.x;
    if (i < n) dst[i] += src[i];
}

extern "C" int fk_engine_merge_from(fk_engine *dst, fk_engine *src) {
    if (!dst || !src || dst->k != src->k) return FK_E_INVALID;
    if (dst->sparse || src->sparse) return FK_E_INVALID;
    /* both keep short-walk counts (nodeCounter) or neither: a merge would
       otherwise peer-copy from a null d_short */
    if (dst->nshort != src->nshort) return FK_E_INVALID;
    int rc = set_dev(src);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(src->stream));
    rc = set_dev(dst);
    if (rc) return rc;
    DevScratch s_tab, s_short, s_acc;
    if (!s_tab.alloc(dst->nbins * sizeof(uint32_t))) return FK_E_OOM;
    if (dst->nshort && !s_short.alloc(dst->nshort * sizeof(uint32_t))) return FK_E_OOM;
    if (!s_acc.alloc(ACC_N * sizeof(unsigned long long))) return FK_E_OOM;
    uint32_t *tmp = s_tab.as<uint32_t>(), *tmps = s_short.as<uint32_t>();
    unsigned long long *tmpa = s_acc.as<unsigned long long>();
    HIPCHK(hipMemcpyPeerAsync(tmp, dst->dev, src->d_table, src->dev, dst->nbins * sizeof(uint32_t), dst->stream));
    if (dst->nshort) HIPCHK(hipMemcpyPeerAsync(tmps, dst->dev, src->d_short, src->dev, dst->nshort * sizeof(uint32_t), dst->stream));
    HIPCHK(hipMemcpyPeerAsync(tmpa, dst->dev, src->d_acc, src->dev, ACC_N * sizeof(unsigned long long), dst->stream));
    unsigned g = (unsigned)std::min<uint64_t>((uint64_t)dst->cus * 8, dst->nbins / 256 + 1);
    hipLaunchKernelGGL(k_add_tables, dim3(g), dim3(256), 0, dst->stream, dst->d_table, tmp, dst->nbins);
    if (dst->nshort) {
        unsigned gs = (unsigned)std::min<uint64_t>((uint64_t)dst->cus * 8, dst->nshort / 256 + 1);
        hipLaunchKernelGGL(k_add_tables, dim3(gs), dim3(256), 0, dst->stream, dst->d_short, tmps, dst->nshort);
    }
    hipLaunchKernelGGL(k_add_acc, dim3(1), dim3(64), 0, dst->stream, dst->d_acc, tmpa, (int)ACC_N);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(dst->stream));
    dst->stats_valid = false;
    dst->unknown_bytes.insert(dst->unknown_bytes.end(), src->unknown_bytes.begin(), src->unknown_bytes.end());
    dst->unknown_pos.insert(dst->unknown_pos.end(), src->unknown_pos.begin(), src->unknown_pos.end());   /* (shard-relative) */
    dst->chunks += src->chunks;
    dst->redo += src->redo;
    dst->dev_ms += src->dev_ms;
    dst->main_ms += src->main_ms;
    dst->timed_n += src->timed_n;
    return FK_OK;
}

/* ---- one-shot helpers ---- */

extern "C" int fk_count(const uint8_t *buf, uint64_t len, int k, const fk_opts *opts, uint32_t *counts,
                        fk_result *res) {
    if (k > FK_K_MAX_DENSE) return FK_E_K_UNSUPPORTED;   /* a dense table out: engine + fk_engine_sparse */
    fk_engine *e = nullptr;
    int rc = fk_engine_create(k, opts, &e);
    if (rc) return rc;
    fk_result tmp;
    if (!res) res = &tmp;
    rc = fk_engine_feed(e, buf, len, 0);
    if (rc == FK_OK) {
        rc = fk_engine_finish(e, res);
        if (counts && (rc == FK_OK || rc == FK_E_UNTERMINATED_HEADER)) {
            int r2 = fk_engine_table(e, counts);
            if (r2) rc = r2;
        }
    }
    fk_engine_destroy(e);
    return rc;
}

/*
 * One process, ngpu devices: contiguous shards (chunk-aligned), each counted
 * on its own GPU from a guessed entry state, stitched in order with the shard
 * transfer functions, re-counted where the guess was wrong, then the tables
 * are merged into device 0 (peer copies over xGMI).
 */
extern "C" int fk_count_multi(const uint8_t *buf, uint64_t len, int k, int ngpu, const fk_opts *opts,
                              uint32_t *counts, fk_result *res) {
    if (k > FK_K_MAX_DENSE) return FK_E_K_UNSUPPORTED;
    int ndev = fk_device_count();
    if (ngpu <= 0 || ngpu > ndev) ngpu = ndev;
    if (ngpu <= 1 || len < (uint64_t)ngpu * FK_CHUNK_BYTES) return fk_count(buf, len, k, opts, counts, res);
    std::vector<fk_engine *> eng((size_t)ngpu, nullptr);
    std::vector<uint8_t *> dbuf((size_t)ngpu, nullptr);
    int rc = FK_OK;
    uint64_t per = ((len / (uint64_t)ngpu) / FK_CHUNK_BYTES) * FK_CHUNK_BYTES;
    std::vector<uint64_t> off((size_t)ngpu + 1);
    for (int g = 0; g < ngpu; g++) off[(size_t)g] = (uint64_t)g * per;
    off[(size_t)ngpu] = len;
    for (int g = 0; g < ngpu && rc == FK_OK; g++) {
        fk_opts o = opts ? *opts : fk_opts{};
        o.device = g;
        o.stream = nullptr;
        rc = fk_engine_create(k, &o, &eng[(size_t)g]);
        if (rc) break;
        uint64_t halo = g ? FK_HALO_BYTES : 0;
        uint64_t n = off[(size_t)g + 1] - off[(size_t)g];
        if (hipSetDevice(g) != hipSuccess) { rc = FK_E_HIP; break; }
        if (hipMalloc((void **)&dbuf[(size_t)g], n + halo + 16) != hipSuccess) { rc = FK_E_OOM; break; }
        if (hipMemcpy(dbuf[(size_t)g], buf + off[(size_t)g] - halo, n + halo, hipMemcpyHostToDevice) != hipSuccess) {
            rc = FK_E_HIP;
            break;
        }
        rc = fk_engine_feed_shard(eng[(size_t)g], dbuf[(size_t)g] + halo, n, halo, 1);
    }
    int last = ngpu - 1;
    if (rc == FK_OK) {
        fk_state s{0, 0, 0, 0};
        for (int g = 0; g < ngpu && rc == FK_OK; g++) {
            rc = fk_engine_resolve(eng[(size_t)g], &s);
            if (rc) break;
            rc = fk_engine_state(eng[(size_t)g], &s);
            if (rc) break;
            if (eng[(size_t)g]->ended) {          /* a 0xFF byte: later shards do not count */
                for (int h = g + 1; h < ngpu; h++) fk_engine_reset(eng[(size_t)h]);
                last = g;
                break;
            }
        }
    }
    if (rc == FK_OK) {
        for (int g = 1; g < ngpu && rc == FK_OK; g++) rc = fk_engine_merge_from(eng[0], eng[(size_t)g]);
        if (rc == FK_OK) {
            fk_engine *e0 = eng[0];
            e0->state = eng[(size_t)last]->state;
            uint64_t sc = 0;
            for (int g = 0; g <= last; g++) sc += eng[(size_t)g]->ended ? eng[(size_t)g]->scanned : eng[(size_t)g]->fed;
            e0->fed = len;
            e0->scanned = sc;
            e0->ended = eng[(size_t)last]->ended;
            fk_result tmp;
            if (!res) res = &tmp;
            rc = fk_engine_finish(e0, res);
            if (counts && (rc == FK_OK || rc == FK_E_UNTERMINATED_HEADER)) {
                int r2 = fk_engine_table(e0, counts);
                if (r2) rc = r2;
            }
        }
    }
    for (int g = 0; g < ngpu; g++) {
        if (dbuf[(size_t)g]) { hipSetDevice(g); hipFree(dbuf[(size_t)g]); }
        fk_engine_destroy(eng[(size_t)g]);
    }
    return rc;
}

extern "C" int fk_synth_device(uint8_t *dev_out, uint64_t cap, uint64_t n_bases, uint64_t seed,
                               int fasta_line, void *stream, uint64_t *written) {
    uint64_t hlen = fasta_line > 0 ? 11 : 0;
    int L = fasta_line < 0 ? -fasta_line : fasta_line;
    uint64_t total = hlen + n_bases + (L > 0 ? n_bases / (uint64_t)L : 0);
    if (total > cap) total = cap;
    uint64_t threads = (total + 15) / 16;
    unsigned blocks = (unsigned)((threads + 255) / 256);
    if (blocks)
        hipLaunchKernelGGL(k_synth, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dev_out, total, seed,
                           L, hlen);
    HIPCHK(hipGetLastError());
    if (written) *written = total;
    return FK_OK;
}

extern "C" int fk_synth_upstream_device(uint8_t *dev_out, uint64_t cap, uint64_t first_rec, uint64_t n_records,
                                        uint64_t seed, void *stream, uint64_t *written) {
    if (!dev_out && cap) return FK_E_INVALID;
    if (first_rec + n_records > 99999999999ull) return FK_E_INVALID;   /* 11 digits */
    const uint64_t total = std::min<uint64_t>(cap, n_records * FK_UPSTREAM_REC);
    const uint64_t blocks = (total + 16 * 256 - 1) / (16 * 256);
    if (blocks)
        hipLaunchKernelGGL(k_synth_upstream, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dev_out,
                           total, first_rec, seed);
    HIPCHK(hipGetLastError());
    if (written) *written = total;
    return FK_OK;
}
