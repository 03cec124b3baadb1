/*
 * findkmer.h — C-ABI of the MI355X k-mer counting engine (libfindkmer_hip.so).
 *
 * Drop-in boundary.  The reference (soundude462/findKmer) has no plugin or FFI
 * API: its hot path is the in-process call
 *
 *     node_t* findKmer(node_t* headNode, unsigned long long* baseCounter,
 *                      statistics_t* baseStatistics,
 *                      unsigned long long* TotalNumSequencesN);
 *                                             (findKmer/src/findKmer.cpp:962-964)
 *
 * which scans config.sequence_file_pointer byte by byte and grows a 4-ary
 * trie (:107-111, :612-690) whose depth-k leaves hold the k-mer counts, read
 * back by statistics() (:491-565) and histo_recursive() (:699-942).  This
 * header replaces that call with plain pointers and sizes: the trie becomes a
 * dense table of 4^k uint32 counters (the reference's `unsigned int
 * frequency`, :110) indexed by the 2-bit packing A=0 C=1 G=2 T=3, first base
 * most significant (base2int, :567-589), i.e. the trie's DFS order
 * (:719-724).  Errors are returned, never exit()ed; the host main
 * (./findKmer) maps them onto the reference's messages and exit codes.
 *
 * Threading: an engine is bound to one HIP device and is driven from one host
 * thread.  Multi-GPU runs use one engine per device (one process per GPU in
 * bench.py; fk_count_multi below fans out inside one process).
 */
#ifndef FINDKMER_H
#define FINDKMER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): fk_engine_shard_exchange's merge buffer is the table padded
   to a multiple of `world` plus FK_PACK_STATS words (fk_merge_layout), and
   fk_state.ended is checked (it was padding in 1) */
#define FK_ABI_VERSION 2
#define FK_K_MIN 1
#define FK_K_MAX_DENSE 16   /* 4^16 uint32 = 16 GiB table on one 288 GB GPU */
#define FK_K_MAX_REF 20     /* the reference accepts k <= 20 (:438) */

/* status codes (all < 0 are errors) */
enum {
    FK_OK = 0,
    FK_E_INVALID = -1,          /* bad argument */
    FK_E_K_UNSUPPORTED = -2,    /* a dense-table entry point (fk_count*) with
                                   17 <= k <= 20: use an engine and
                                   fk_engine_sparse */
    FK_E_NO_DEVICE = -3,        /* no HIP device / extension cannot run */
    FK_E_HIP = -4,              /* a HIP runtime call failed */
    FK_E_OOM = -5,              /* device or host allocation failed */
    FK_E_EMPTY = -6,            /* empty input: ref prints "Sequence File Is
                                   Empty, Ending Program" and exits (:982-985) */
    FK_E_UNTERMINATED_HEADER = -7, /* input ends inside a '>' line: the ref
                                      spins forever in the loop at :1005 */
    FK_E_ROLLOVER = -8,         /* a trie counter would wrap: ref prints
                                   COUNTER ROLLOVER and exits (:642-648) */
    FK_E_STATE = -9,            /* API called out of order */
    FK_E_IO = -10,              /* host file I/O failed */
    FK_E_RCCL = -11,            /* a collective failed */
    FK_E_SUMMARY = -12,         /* a compact shard summary does not apply to
                                   this entering state: exchange the full ones
                                   (fk_engine_summary_full) */
    FK_E_INTERNAL = -13         /* a device-side bound check failed: a kernel's
                                   output would have passed the end of its
                                   buffer.  Nothing was written past it; the
                                   feed's counts are not valid (reset) */
};

/* Scan state carried between byte ranges (exact; used for streaming feeds and
 * for stitching GPU shards).  `run` is the number of valid bases since the
 * last run break (the ref's seqSize, an int that wraps: we keep it exact and
 * apply the 32-bit wrap where the ref would); `code` holds the last bases,
 * first base most significant; `hdr` = inside a '>' comment line; `ended` = a
 * 0xFF byte outside a header already ended the stream (the reference's
 * signed-char EOF test, findKmer.cpp:988): an absorbing state, nothing after
 * it counts.  `ended` must be 0 or 1 (it was a padding word before): any
 * other value makes fk_engine_resolve / fk_summary_apply return
 * FK_E_INVALID. */
typedef struct {
    uint64_t run;
    uint64_t code;
    uint32_t hdr;
    uint32_t ended;
} fk_state;

typedef struct {
    uint64_t base_count[4];   /* baseStatistics[b].Count, exact (the ref keeps
                                 it in a u32 that wraps silently, :94) */
    uint64_t valid_bases;     /* baseCounter */
    uint64_t windows;         /* TotalNumSequencesN */
    uint64_t distinct;        /* k-mers with count >= 1 */
    uint64_t depth1[4];       /* depth-1 trie node frequencies (rollover) */
    uint64_t nodes;           /* nodeCounter incl. head (0 if not computed) */
    uint64_t unknown_chars;   /* bytes that print "Unknown character" */
    uint64_t scanned_bytes;   /* bytes consumed (stops at a 0xFF byte) */
    int32_t  hit_eof_byte;    /* a 0xFF byte outside a header ended the scan */
    int32_t  unterminated_header;
    int32_t  rollover;
    int32_t  nodes_valid;     /* `nodes` was computed */
    /* instrumentation (not part of parity) */
    uint64_t chunks;          /* 64 KiB scan chunks processed */
    uint64_t redo_chunks;     /* chunks re-counted after the state scan */
    double   device_ms;       /* HIP-event time of all scan kernels */
    double   main_kernel_ms;  /* HIP-event time of the main count kernel ... */
    uint64_t timed_kernels;   /* ... over this many launches (see fk_opts.timing_every) */
} fk_result;

typedef struct {
    int32_t device;           /* HIP device ordinal; -1 = current device */
    int32_t want_nodes;       /* compute nodeCounter (stdout "tree density") */
    void   *stream;           /* hipStream_t to use; NULL = an engine-owned
                                 blocking stream (orders after the device's
                                 legacy default stream) */
    int32_t collect_unknown;  /* keep the unknown bytes for stderr replay (2: and
                                 their stream offsets, fk_engine_unknown_since) */
    int32_t timing_every;     /* time the count kernel with HIP events on every
                                 Nth launch (0 or 1: every launch) */
    int32_t borrow_input;     /* 17 <= k <= 20: device feeds (16-B aligned, at
                                 least FK_LANE_BYTES) and shards are read again
                                 at finish from the caller's buffer instead of
                                 a copy the engine keeps: the caller leaves
                                 those bytes unchanged until fk_engine_finish
                                 (or reset / destroy) returns.  0: copy (round 6) */
    int32_t reserved[5];
} fk_opts;

typedef struct fk_engine fk_engine;

/* Library identity. */
int         fk_abi_version(void);
const char *fk_strerror(int status);
int         fk_device_count(void);   /* 0 when no GPU is visible */

/* Engine lifecycle: one engine per (device, k).  The device table lives in
 * HBM for the engine's lifetime. */
int  fk_engine_create(int k, const fk_opts *opts, fk_engine **out);
void fk_engine_destroy(fk_engine *e);
int  fk_engine_reset(fk_engine *e);     /* zero table, counters and state */

/* Feed a byte range of the stream.  `buf` is a device pointer when
 * on_device != 0, else host memory (staged through pinned buffers).  Feeds
 * continue the scan state of the previous feed exactly.  A device buffer
 * must be complete in the engine's stream order (see fk_opts.stream). */
int  fk_engine_feed(fk_engine *e, const uint8_t *buf, uint64_t len,
                    int on_device);

/* Shard entry (multi-GPU): feed bytes whose entering state is not known yet.
 * `halo` bytes immediately preceding buf (may be 0) are used to guess it;
 * fk_engine_resolve() later supplies the true entering state and re-counts
 * what the guess got wrong.  fk_engine_summary() returns the shard's effect
 * on the scan state as an opaque blob (fk_summary) that the caller exchanges
 * between shards: for a shard counted in one pass, a compact summary valid
 * for entering states equivalent to the shard's guess (fk_summary_apply then
 * returns FK_E_SUMMARY for any other state); otherwise, or from
 * fk_engine_summary_full(), the full transfer function, which applies to
 * every state.  A compact summary also records whether the shard ends the
 * stream (a 0xFF byte outside a header): fk_summary_apply sets out->ended.
 * A full summary does not know it (fk_summary_is_full): the caller learns
 * each shard's end from fk_engine_state(...).ended after fk_engine_resolve.
 * Applied to an ended state, any summary returns that state unchanged, and
 * fk_engine_resolve with an ended entering state drops the shard (its table
 * and counters stay zero). */
typedef struct { uint64_t w[12]; } fk_summary;
int  fk_engine_feed_shard(fk_engine *e, const uint8_t *buf, uint64_t len,
                          uint64_t halo, int on_device);
int  fk_engine_summary(fk_engine *e, fk_summary *out);
int  fk_engine_summary_full(fk_engine *e, fk_summary *out);
int  fk_summary_apply(const fk_summary *s, const fk_state *in, fk_state *out);
int  fk_summary_is_full(const fk_summary *s);   /* 1: full transfer function, 0: compact */
int  fk_engine_resolve(fk_engine *e, const fk_state *entering);

/* One-collective shard exchange (multi-GPU, findkmer_amd/dist.py).  After
 * fk_engine_feed_shard, enqueue on the engine's stream (no host wait) what
 * fk_engine_finish would report if the shard's guessed entering state holds,
 * into caller-owned device buffers that one collective then merges:
 *   table     4^k uint32: the shard's counts;
 *   counters  FK_PACK_COUNTERS u64 values, each as 4 little-endian 16-bit
 *             limbs in int32 slots (sums over ranks stay exact): windows,
 *             valid_bases, base_count[4], depth1[4], unknown_chars,
 *             scanned_bytes, ended (0), unterminated_header (only if
 *             is_last, else 0);
 *   rows      nrows x FK_PACK_ROW_WORDS uint32, zeroed except row `slot`:
 *             the shard's compact summary (fk_summary, words 0..23) and
 *             word 24 = 1 when the pack is valid (a one-pass shard whose
 *             range guesses held and that saw no 0xFF byte), else 0.
 * A sum of such row regions over ranks with distinct slots is an
 * all-gather, so with nrows = world the whole exchange is one all-reduce.
 * The shard stays pending: the caller composes the gathered rows
 * (fk_shard_rows_compose) and either calls fk_engine_resolve with the
 * entering state it returns (the merged buffer is then exact) or, if any
 * row is invalid, falls back to the fk_engine_summary exchange.  Replaces
 * no reference call (the reference is single-threaded, findKmer.cpp:962). */
#define FK_PACK_COUNTERS 14
#define FK_PACK_ROW_WORDS 32
int  fk_engine_shard_pack(fk_engine *e, uint32_t *table, int32_t *counters, uint32_t *rows, int nrows,
                          int slot, int is_last);
/* The engine's HIP stream (hipStream_t), for ordering a caller's collective
 * after fk_engine_shard_pack. */
int  fk_engine_stream(fk_engine *e, void **stream);
/* Compose gathered pack rows (host memory, `world` rows in rank order) from
 * the stream's initial state: FK_OK and *entering = the state entering
 * `rank`'s shard when every row is valid and every compact summary applies;
 * FK_E_SUMMARY otherwise (every rank gets the same answer: fall back). */
int  fk_shard_rows_compose(const uint32_t *rows, int world, int rank, fk_state *entering);

/* An RCCL communicator of the library (one rank per GPU; RCCL is loaded at
 * run time).  One rank creates the id, the caller hands it to every rank
 * (e.g. a torch.distributed broadcast), and every rank calls fk_comm_create
 * (collective: it returns when all have joined).  FK_E_RCCL when RCCL is
 * unavailable or fails. */
#define FK_COMM_ID_BYTES 128
typedef struct fk_comm fk_comm;
int  fk_comm_id(uint8_t *id /* FK_COMM_ID_BYTES */);
int  fk_comm_create(const uint8_t *id, int world, int rank, int device, fk_comm **out);
void fk_comm_destroy(fk_comm *c);
/* What RCCL reports for the communicator (ncclCommCount, ncclCommUserRank,
 * ncclCommCuDevice; -1 for a query this RCCL lacks): lets a sharded run's
 * output prove the world it ran in. */
int  fk_comm_info(fk_comm *c, int *nranks, int *rank, int *device);
/* The merge buffer of a sharded pass (int32 words, device memory for
 * fk_engine_shard_exchange):
 *   [0, TW)           the count table, TW = 4^k rounded up to a multiple of
 *                     `world` (zero padding after 4^k);
 *   [TW, +4*14)       the counter limbs (fk_engine_shard_pack's order);
 *   [.., +8)          FK_PACK_STATS: a sharded table's total u64 count and
 *                     distinct bins, as 16-bit limbs;
 *   [.., +world*32)   the pack rows.
 * fk_merge_layout gives TW and the total size for (k, world). */
#define FK_PACK_STATS 8
int  fk_merge_layout(int k, int world, uint64_t *table_words, uint64_t *total_words);

/* An RCCL communicator can be created on `device` in this process (RCCL
 * loads with every entry point, the device is usable) -- everything
 * fk_comm_create checks before its collective init, so ranks can agree on
 * it first and never leave one rank alone inside ncclCommInitRank. */
int  fk_comm_available(int device);

/* Flags of fk_engine_shard_exchange (info[0]). */
#define FK_XCHG_FAST 1          /* try the one-collective path */
#define FK_XCHG_SHARD_TABLE 2   /* stitched path: reduce-scatter the table
                                   instead of reducing it onto rank 0 */
#define FK_XCHG_TEST_INVALID 4  /* tests: mark this rank's pack row invalid
                                   (forces the fallback after the collective) */

/* A sharded pass's whole exchange on the engine's stream, after
 * fk_engine_feed_shard, with the library's communicator; `merge` is a device
 * buffer laid out as above (fk_merge_layout's total_words int32).
 *  - one collective (info == NULL, or FK_XCHG_FAST in info[0]): pack
 *    (fk_engine_shard_pack, slot = rank), an in-place all-reduce of the whole
 *    buffer, the rows published to host memory, one host wait,
 *    fk_shard_rows_compose, fk_engine_resolve.  Every rank's buffer then
 *    holds the merged table and counter limbs (info[0] = 1).
 *  - otherwise (the one-collective path is off, the shard was not counted in
 *    one pass -- 8 <= k <= 12 always --, or some guess did not hold; every
 *    rank takes this branch together): the shards' full transfer functions
 *    all-gathered and composed, fk_engine_resolve, the shards' end flags
 *    all-gathered (a 0xFF byte, findKmer.cpp:988), then the table and counter
 *    limbs -- zero on ranks after the first ending shard -- either reduced
 *    onto rank 0, or with FK_XCHG_SHARD_TABLE reduce-scattered: rank r owns
 *    bins [r*TW/world, (r+1)*TW/world) of the merged table (the table
 *    sharded by its top index bits, i.e. the k-mers' first bases, which is
 *    also the CSV's row order, findKmer.cpp:719-724), every rank gets the
 *    merged counters and the table's total and distinct bins.  info[0] = 0,
 *    info[1] = the first ending shard's rank or -1.
 * The shard is resolved either way (fk_engine_finish gives its own result),
 * and the call returns after the device work.  Replaces no reference call
 * (the reference is single-threaded, findKmer.cpp:962). */
int  fk_engine_shard_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *info /* [2], may be NULL */);

/* Routed sharded tables (round 5): for k >= FK_ROUTE_KMIN the stitched
 * exchange with FK_XCHG_SHARD_TABLE can send each owner only the nonzero bins
 * of its range instead of reduce-scattering the whole table: FINDKMER_TUNE
 * route=1 at world > 1, route=2 at world 1 too.  The default (route=0) is the
 * reduce-scatter until the grouped ncclSend/ncclRecv has run at world > 1 on
 * hardware (round 6); an RCCL without ncclSend/ncclRecv always reduce-scatters.
 * Every blob ends in a trailer (a magic word and the sum of its other words,
 * mod 2^32) that the owner checks: a blob that arrived short or corrupt makes
 * the exchange (and fk_engine_route_absorb) fail with FK_E_RCCL.
 * The same steps for a caller-driven transport (the gloo rehearsal):
 *  - fk_engine_route_pack: after fk_engine_finish, the finished table's blobs
 *    for owners 0..world-1 (words[d] int32 each, side by side; counting == 0:
 *    empty blobs, for a rank the stream never reached);
 *  - fk_engine_route_copy: that buffer into a caller-owned device buffer;
 *  - fk_engine_route_absorb: the blobs `rank` received (words[s] from source
 *    s, side by side at recv, device memory) counted into its slice of the
 *    merged table (device, bins [rank*TW/world, ...) of fk_merge_layout).
 * Replaces no reference call (the reference is single-threaded). */
#define FK_ROUTE_KMIN 15
int  fk_engine_route_pack(fk_engine *e, int world, int counting, uint64_t *words /* [world] */);
int  fk_engine_route_copy(fk_engine *e, void *dst);
int  fk_engine_route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words /* [world] */,
                            int32_t *slice);

/* Finish the stream (end-of-input rules) and fill *res.  Returns FK_OK or one
 * of FK_E_EMPTY / FK_E_UNTERMINATED_HEADER / FK_E_ROLLOVER (res is filled in
 * every case). */
int  fk_engine_finish(fk_engine *e, fk_result *res);

/* Copy the 4^k table to host memory (counts[4^k]) / borrow the device
 * pointer (valid until reset/destroy). */
int  fk_engine_table(fk_engine *e, uint32_t *counts);
int  fk_engine_table_device(fk_engine *e, uint32_t **dev_counts);
/* Copy bins [first, first+n) to host (stream a large-k table in pieces). */
int  fk_engine_table_range(fk_engine *e, uint64_t first, uint64_t n, uint32_t *counts);
/* Copy the table into a caller-owned device buffer (4^k uint32), e.g. a
 * torch tensor handed to an RCCL collective; and load it back. */
int  fk_engine_table_to_device(fk_engine *e, void *dst);
int  fk_engine_table_from_device(fk_engine *e, const void *src);
int  fk_engine_state(fk_engine *e, fk_state *out);

/* Running counters without finishing the stream (the -q 0 "Read %llu bases"
 * lines print baseCounter at every header, :996-997). */
int  fk_engine_progress(fk_engine *e, uint64_t *valid_bases, uint64_t *windows);

/* Add another engine's table and counters into this one (same k) — the
 * single-process multi-GPU merge when RCCL is not used. */
int  fk_engine_merge_from(fk_engine *dst, fk_engine *src);

/* Unknown bytes in stream order (collect_unknown=1): *n receives the number
 * available; copies min(cap, n). */
int  fk_engine_unknown(fk_engine *e, uint8_t *out, uint64_t cap, uint64_t *n);
/* The unknown bytes from index `first` on, at most cap of them, and (opts
 * collect_unknown = 2 only, else FK_E_STATE; pos may be NULL) their stream
 * offsets -- what a caller needs to print the warnings between the -q 0
 * progress lines in stream order, as the reference does (:582-584 during
 * the scan at :997).  *n receives the total so far. */
int  fk_engine_unknown_since(fk_engine *e, uint64_t first, uint8_t *out, uint64_t *pos, uint64_t cap,
                             uint64_t *n);

/* 17 <= k <= 20 (the reference's k limit, :438): the table is sparse.  After
 * fk_engine_finish, the distinct k-mer indices in ascending order (= the
 * CSV's row order) and their u32 frequencies; keys and counts may be NULL to
 * ask for *n.  The dense table calls (fk_engine_table...) return
 * FK_E_INVALID for these k.  Device memory: the input fed (1 byte per byte,
 * kept until reset: fk_engine_finish builds the table from it in key-range
 * passes sized to the free HBM) plus 12 bytes per distinct k-mer. */
int  fk_engine_sparse(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n);
/* The runs with keys in [key_lo, key_hi) (a contiguous piece of the table,
 * found by binary search): *n = their number, min(cap, *n) copied to host
 * memory -- a 10 GB input's table (~90 GB at k = 17) read piece by piece. */
int  fk_engine_sparse_range(fk_engine *e, uint64_t key_lo, uint64_t key_hi, uint64_t *keys, uint32_t *counts,
                            uint64_t cap, uint64_t *n);
/* The same into device buffers. */
int  fk_engine_sparse_device(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n);

/* Multi-GPU merge of sparse tables (replaces the reduce of dense ones): the
 * ranks' runs go to their owners -- rank r owns indices [r*S, (r+1)*S),
 * S = ceil(4^k / world), a contiguous run of CSV rows -- with one
 * all-to-all.  fk_engine_sparse_split: the finished table's run count per
 * owner (counts[world]; the runs are contiguous in owner order).
 * fk_engine_sparse_adopt: replace the table by the runs received (device
 * pointers, any order, repeated keys summed); stats[0] = distinct k-mers,
 * stats[1] = the sum of their u32 counts (short of the windows when a sum
 * reached 2^32: the reference's rollover exit, :642). */
int  fk_engine_sparse_split(fk_engine *e, int world, uint64_t *counts);
int  fk_engine_sparse_adopt(fk_engine *e, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                            uint64_t *stats /* [2] */);
/* The same merge over the library's communicator (round 6): this rank's
 * finished table cut at the owners' bounds, sent to its owners (grouped
 * ncclSend / ncclRecv, sizes as a world x world matrix of 16-bit limbs in
 * one all-reduce), the received runs adopted, then `limbs` (device, the
 * FK_PACK_COUNTERS counters as 4 16-bit limbs each, filled by the caller)
 * completed with this slice's (total, distinct) limbs (FK_PACK_STATS) and
 * all-reduced -- every collective on the engine's stream.  stats[0] =
 * distinct k-mers of this rank's slice, stats[1] = the sum of their u32
 * counts.  counting = 0: this rank sends nothing (a rank after the shard
 * that ended the stream).  Collective: every rank of comm calls it.
 * Replaces no reference call (the reference is single-threaded). */
int  fk_engine_sparse_exchange(fk_engine *e, fk_comm *comm, int counting, int32_t *limbs, uint64_t *stats /* [2] */);

/* One-shot convenience: count a whole buffer on one device. */
int  fk_count(const uint8_t *buf, uint64_t len, int k, const fk_opts *opts,
              uint32_t *counts /* host, 4^k */, fk_result *res);

/* One-shot multi-GPU: split buf (host) into ngpu contiguous shards, count
 * each on its own device, stitch the states, merge the tables. */
int  fk_count_multi(const uint8_t *buf, uint64_t len, int k, int ngpu,
                    const fk_opts *opts, uint32_t *counts, fk_result *res);

/* Deterministic on-device synthetic input (same bytes as the oracle's
 * fko_synth): n_bases uniform ACGT from `seed`, optional FASTA framing
 * (">synthetic\n" + '\n' every fasta_line bases; fasta_line < 0: '\n' every
 * -fasta_line bases and no header — a later shard of the same file).  Bytes
 * are those of base index >= 0 of the stream seeded `seed`; a shard starting
 * at base b (b a multiple of 32) uses seed + b/32.  Returns bytes written. */
int  fk_synth_device(uint8_t *dev_out, uint64_t cap, uint64_t n_bases,
                     uint64_t seed, int fasta_line, void *stream,
                     uint64_t *written);

/* Deterministic on-device upstream-regions-like FASTA (BASELINE.json
 * configs[4]; what get_upstreams.pl writes, findKmer/get_upstreams.pl:82-91):
 * records ">ENST%011u\n" + 1001 bases + "\n" (FK_UPSTREAM_REC bytes), record
 * r numbered first_rec + r; its bases uniform ACGT from splitmix64 of (seed,
 * record, word), and with probability 1/100 (from splitmix64 of (seed,
 * record)) a run of 50 'N' at an offset in [0, 951) drawn from the same
 * word.  Writes min(cap, n_records * FK_UPSTREAM_REC) bytes of records
 * [first_rec, first_rec + n_records) into dev_out on `stream`; the bytes
 * depend only on (seed, record number), so shards of one file are
 * generated independently. */
#define FK_UPSTREAM_REC 1019
int  fk_synth_upstream_device(uint8_t *dev_out, uint64_t cap, uint64_t first_rec, uint64_t n_records,
                              uint64_t seed, void *stream, uint64_t *written);

/* ---- file ingest (replaces the reference's per-byte fgetc reads of
 * config.sequence_file_pointer, findKmer.cpp:988, with a device-resident
 * copy of the whole file) --------------------------------------------------
 * fk_input_load: `threads` host threads (<= 0: up to 8) pread() the regular
 * file at `path` in 32 MiB chunks into pinned buffers and copy them
 * asynchronously into one device buffer on `device` (-1: current device),
 * overlapping reads with copies.  The buffer is 16-B aligned and can be fed
 * to any number of engines on that device (fk_engine_feed(..., 1)).
 * Returns FK_E_IO for unreadable or non-regular files (pipes: stream with
 * fk_engine_feed instead). */
typedef struct fk_input fk_input;
int  fk_input_load(const char *path, int device, int threads, fk_input **out);
int  fk_input_info(const fk_input *in, const uint8_t **dev_ptr, uint64_t *len,
                   int *device, double *seconds /* load wall time */);
void fk_input_destroy(fk_input *in);
/* The comment lines of the loaded file, for the reference's -q 0 progress
 * output (findKmer.cpp:996-1002): the offset of every '>' that starts one, and
 * baseCounter (valid bases counted so far, at k) as of that byte.  Computed
 * on the device (k_hdr_traj / k_hdr_list).  *n = how many; at most cap are
 * written.  FK_E_STATE when the counts are not expressible this way (a 0xFF
 * byte ends the scan, or a run reaches the reference's int32 seqSize wrap):
 * feed the file in pieces and use fk_engine_progress instead. */
int  fk_input_headers(fk_input *in, int k, uint64_t *pos, uint64_t *bases, uint64_t cap, uint64_t *n);

/* ---- device choice (several ./findKmer processes on one node) -----------
 * The reference's sweep driver starts 24 processes at once
 * (k6thru11fullANDupstream.sh:16-24).  fk_device_select makes the chosen
 * device current and returns it: FINDKMER_DEVICE=<ordinal> if set (else
 * FK_E_INVALID for a bad value); otherwise, among the devices whose free HBM
 * is >= need bytes, the one at (pid mod their count), so processes started
 * together spread over the GPUs; if none has enough, the one with the most
 * free HBM.  Free HBM is read from sysfs (no HIP context on the other
 * GPUs); where sysfs has no VRAM counters, the choice is pid mod ndev.  fk_device_policy is that rule alone (free_bytes[ndev] given):
 * returns the ordinal. */
int  fk_device_select(uint64_t need, int *device);
int  fk_device_policy(int ndev, const uint64_t *free_bytes, uint64_t need, uint32_t salt);

/* ---- host side of the boundary: byte-identical output writers ---------- */

/* statistics() (:491-565): writes "<k>mer_Base_Stats_Of_<file>.txt" content to
 * stats_path and the stdout lines to `log` (may be NULL).  Returns FK_OK, or 1
 * when a base probability is 0 ("Division overflow", ref exits 1 after
 * writing the earlier lines, :522-525). */
int  fk_write_stats(const char *stats_path, int k, const fk_result *res,
                    void *log /* FILE* */, double prob_out[4]);

/* histo_recursive() rows (:699-942) for all k-mers with count >= 1, in
 * ascending index order, appended to `out` (FILE*, header already written).
 * z filtering as -z (:852-854).  threads <= 0: use all host cores. */
int  fk_write_rows(void *out, int k, const uint32_t *counts,
                   const double prob[4], uint64_t windows, int z_enable,
                   double z_threshold, int threads);
/* the same rows for a sparse table (fk_engine_sparse's keys and counts) */
int  fk_write_rows_sparse(void *out, int k, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                          const double prob[4], uint64_t windows, int z_enable,
                          double z_threshold, int threads);
int  fk_write_csv_sparse(const char *csv_path, int k, const uint64_t *keys, const uint32_t *counts,
                         uint64_t n, const double prob[4], uint64_t windows, int z_enable,
                         double z_threshold, int threads);

/* Path-based variant for bindings: writes header + rows to csv_path. */
int  fk_write_csv(const char *csv_path, int k, const uint32_t *counts,
                  const double prob[4], uint64_t windows, int z_enable,
                  double z_threshold, int threads);

#ifdef __cplusplus
}
#endif
#endif /* FINDKMER_H */
