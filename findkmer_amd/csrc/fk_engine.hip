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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <type_traits>
#include <vector>

#include "findkmer.h"
#include "fk_comm.h"
#include "fk_device.h"
#include "fk_sparse.h"


/* ------------------------------------------------------------------------- */
/* device helpers                                                             */
/* ------------------------------------------------------------------------- */

__device__ __forceinline__ uint32_t fk_byte(const uint32_t w[4], int j) {
    return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
}

/* byte j (runtime) of a 16-byte lane without indexing the register array */
__device__ __forceinline__ uint32_t fk_byte_rt(const uint32_t w[4], uint32_t j) {
    uint32_t d = j >> 2;
    uint32_t v = d == 0 ? w[0] : d == 1 ? w[1] : d == 2 ? w[2] : w[3];
    return (v >> (8 * (j & 3))) & 0xFFu;
}

/* Internal base encoding A=0 C=1 T=2 G=3, i.e. (byte >> 1) & 3, so the fast
 * path needs no arithmetic beyond a shift and a mask; fk_sigma() maps indices
 * to the reference's A=0 C=1 G=2 T=3 (base2int :567-589).  -1: not a base. */
__device__ __forceinline__ int fk_sym(uint32_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'T' ? 2 : c == 'G' ? 3 : -1;
}

/* A use of a tile buffer on every path (even where its tile is not
   counted): the waitcnt bookkeeping then sees one consistent pending-load
   state at each merge and waits for exactly the tile being used. */
__device__ __forceinline__ void consume(const uint32_t w[8]) {
    asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]));
}

/* wave index inside the block, provably wave-uniform (lives in an SGPR, so
   the loops it bounds stay scalar) */
__device__ __forceinline__ uint32_t wave_in_block() {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

__device__ __forceinline__ uint32_t shup(uint32_t v, int d) { return __shfl_up(v, (unsigned)d, 64); }

/* Wave-wide reductions through DPP moves (quad_perm [1,0,3,2], [2,3,0,1],
 * row_ror:4, row_ror:8, row_bcast:15, row_bcast:31): lane 63 ends with the
 * result, read back as a wave-uniform value.  A butterfly of __shfl_xor is a
 * chain of 6 dependent ds_bpermute round trips per 32-bit value; a wave's
 * counter flush reduces 13 of them.  Every lane must be active (the callers
 * are wave-uniform). */
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <class Op>
__device__ __forceinline__ uint32_t wred32(uint32_t v, Op op) {
    v = op(v, dpp_mov32<0xb1>(v));
    v = op(v, dpp_mov32<0x4e>(v));
    v = op(v, dpp_mov32<0x124>(v));
    v = op(v, dpp_mov32<0x128>(v));
    v = op(v, dpp_mov32<0x142>(v));
    v = op(v, dpp_mov32<0x143>(v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
/* inclusive wave scan (sum) through DPP: row_shr 1/2/4/8 within each row of
   16 lanes, then row_bcast:15 and row_bcast:31 across rows (rocPRIM's
   sequence); every lane must be active */
__device__ __forceinline__ uint32_t wscan_incl32(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63, rl = lane & 15;
    uint32_t t;
    t = dpp_mov32<0x111>(v); if (rl >= 1) v += t;
    t = dpp_mov32<0x112>(v); if (rl >= 2) v += t;
    t = dpp_mov32<0x114>(v); if (rl >= 4) v += t;
    t = dpp_mov32<0x118>(v); if (rl >= 8) v += t;
    t = dpp_mov32<0x142>(v); if ((lane & 31) >= 16) v += t;
    t = dpp_mov32<0x143>(v); if (lane >= 32) v += t;
    return v;
}
/* inclusive wave scan (max), the same DPP sequence */
__device__ __forceinline__ uint32_t wscan_max32(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63, rl = lane & 15;
    uint32_t t;
    t = dpp_mov32<0x111>(v); if (rl >= 1) v = max(v, t);
    t = dpp_mov32<0x112>(v); if (rl >= 2) v = max(v, t);
    t = dpp_mov32<0x114>(v); if (rl >= 4) v = max(v, t);
    t = dpp_mov32<0x118>(v); if (rl >= 8) v = max(v, t);
    t = dpp_mov32<0x142>(v); if ((lane & 31) >= 16) v = max(v, t);
    t = dpp_mov32<0x143>(v); if (lane >= 32) v = max(v, t);
    return v;
}
struct OpAdd32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMin32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; } };
__device__ __forceinline__ uint32_t wsum32(uint32_t v) { return wred32(v, OpAdd32{}); }
__device__ __forceinline__ uint32_t wmin32(uint32_t v) { return wred32(v, OpMin32{}); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    return ((uint64_t)rdlane((uint32_t)(v >> 32), l) << 32) | rdlane((uint32_t)v, l);
}

__device__ __forceinline__ uint64_t comp_packed(uint64_t x, int k, uint64_t maskk) {
    /* counts of A,C,G,T among the k digits of x, packed 16 bits each */
    const uint64_t m5 = 0x5555555555555555ull & maskk;
    uint64_t lo = x & m5, hi = (x >> 1) & m5;
    uint32_t nT = __popcll(lo & hi);
    uint32_t nG = __popcll(hi) - nT;
    uint32_t nC = __popcll(lo) - nT;
    uint32_t nA = (uint32_t)k - nT - nG - nC;
    return (uint64_t)nA | ((uint64_t)nC << 16) | ((uint64_t)nG << 32) | ((uint64_t)nT << 48);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Counters {       /* per lane; flushed per range */
    uint64_t base;      /* 4 x 16-bit: first-window extra bases (first k-1 digits) */
    uint64_t d1s;       /* 4 x 16-bit: depth-1 trie touches of short walks */
    uint32_t valid;     /* baseCounter beyond one per window ((k-1) per first window) */
    uint32_t win;       /* windows counted */
    uint32_t unknown;
    uint32_t eof;       /* range-relative offset of first 0xFF, or FK_NO_EOF */
    uint32_t win_u;     /* windows counted, wave-uniform (an SGPR; lane 0 flushes it) */
};

/* Where windows are accumulated. */
enum HistMode {
    H_PAIRS = 0,    /* k <= 6: LDS bins of (k+1)-mers at every other base + LDS k-mer singles */
    H_LDS = 1,      /* k == 7: LDS k-mer bins */
    H_GLOBAL = 2,   /* k >= 14, and cancellations: global u32 atomics */
    H_NONE = 3,     /* 8 <= k <= 13, state pass: count nothing, only the scan state */
    H_EMIT = 4,     /* 8 <= k <= 13, k_part: fast tiles hand their windows to the
                       partition, general tiles use global atomics */
    H_SPARSE = 5    /* 17 <= k <= 20: general tiles from exact states write every
                       window's index (and every short walk) at its byte's slot */
};

/* sparse slots (H_SPARSE, k_sp_emit: one u64 per byte of the tile, in LDS):
   a window's reference-order index (< 2^40), a short walk (tag | depth << 40
   | its code), or empty.  Byte p of the tile (lane p / 32, byte p % 32) sits
   at column-major slot (p % 32) * 64 + p / 32: the 64 lanes writing their
   j-th bytes hit 64 consecutive slots (no bank conflicts). */
#define SP_SHORT (1ull << 62)
#define SP_EMPTY (~0ull)
__device__ __forceinline__ uint32_t sp_slot(uint32_t pos) { return ((pos & 31u) << 6) | (pos >> 5); }

/* a fast tile's windows for the partition (k_part): per half, the context
   word, the 16-slot word and whether slot 0 is not a window */
/* the modes that keep bins in LDS (zeroed at start, flushed at the end) */
#define LDS_MODE(hm) ((hm) == H_PAIRS || (hm) == H_LDS)

struct Emit {
    uint32_t AC, A2, BC, B2;
    bool h0, h1, deep;
    bool masked;        /* a mixed tile (tile_mixed): cm says which slots end a window */
    uint32_t cm;        /* half 0 in bits 15:0, half 1 in 31:16; bit 15 - s = slot s */
};

struct Ctx {            /* kernel-wide constants */
    const uint8_t *buf;
    uint64_t len;
    int64_t lo;         /* lowest readable offset (negative: halo before buf) */
    uint32_t *table;    /* global 4^k */
    uint32_t *lds;      /* LDS bins or nullptr */
    uint32_t *shortcnt; /* sum_{d<k} 4^d */
    unsigned long long *acc;
    DevRes *res;
    uint64_t maskk;
    uint32_t single_off;/* H_PAIRS: offset of the k-mer singles in LDS (4^(k+1)) */
    int k;
    uint32_t *flush;    /* where lds_flush adds the bins (nullptr: table) */
    uint64_t *slots;    /* H_SPARSE: the tile's slots in LDS (k_sp_emit), or nullptr (counting only) */
};

/* LDS atomic add at a byte offset into the bins.  The kernels that count
   in LDS (k_count, k_resume, k_redo) have no static LDS, so their dynamic
   bins start at LDS address 0 (checked on the host, lds_layout_ok): the
   address is the offset itself, with no base add per atomic (a generic
   pointer costs one v_add each, 16 per tile). */
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void lds_add(const Ctx &, uint32_t byte_off, uint32_t v) {
    lds_u32 *p = (lds_u32 *)(uintptr_t)byte_off;
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* idx in the internal encoding (A0 C1 T2 G3) */
template <int HM>
__device__ __forceinline__ void hist_add(const Ctx &cx, uint64_t idx, uint32_t w) {
    if (HM == H_NONE) return;
    if (HM == H_EMIT && cx.flush) {
        /* k_part over a fresh k = 15, 16 table (not zeroed: k_count_parts
           writes every bin): the window to the list k_list_add adds after
           it (cx.flush: [0] count, [1] capacity, then the indices) */
        const uint32_t i = atomicAdd(cx.flush, 1u);
        if (i < cx.flush[1]) cx.flush[2 + i] = (uint32_t)fk_sigma(idx);
    } else if (HM == H_GLOBAL || HM == H_EMIT) {
        atomicAdd(&cx.table[fk_sigma(idx)], w);
    } else if (HM == H_LDS) {
        lds_add(cx, (uint32_t)idx * 4u, w);
    } else {
        lds_add(cx, (cx.single_off + (uint32_t)idx) * 4u, w);
    }
}

__device__ __forceinline__ void short_run(const Ctx &cx, int seq, uint64_t code, uint32_t w) {
    /* a run ended with 1 <= seqSize < k: its prefix-only trie walk left nodes
       for nodeCounter (:1059-1062).  Offset of depth d: (4^d - 4) / 3. */
    uint64_t off = ((1ull << (2 * seq)) - 4) / 3;
    uint64_t m = (1ull << (2 * seq)) - 1;
    if (cx.shortcnt) atomicAdd(&cx.shortcnt[off + fk_sigma(code & m)], w);   /* (none without nodeCounter) */
}

/* Load lane bytes [off, off+nbytes) (nbytes = 16 or 32, relative to cx.buf;
 * may start below 0 down to cx.lo).  Fully-inside lanes use 16-B loads; the
 * stream's last partial lane loads bytewise.  Returns the valid byte count. */
template <int NB>
__device__ __forceinline__ int load_lane(const Ctx &cx, int64_t off, uint32_t w[NB / 4]) {
#pragma unroll
    for (int d = 0; d < NB / 4; d++) w[d] = 0;
    if (off < cx.lo || off >= (int64_t)cx.len) return 0;
    if (off + NB <= (int64_t)cx.len) {
#pragma unroll
        for (int q = 0; q < NB / 16; q++) {
            u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(cx.buf + off) + q);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        return NB;
    }
    /* the stream's last partial lane: independent (clamped) byte loads, all
       in flight together */
    int nb = (int)((int64_t)cx.len - off);
#pragma unroll
    for (int j = 0; j < NB; j++) {
        uint32_t b = cx.buf[min(off + j, (int64_t)cx.len - 1)];
        w[j >> 2] |= (j < nb ? b : 0u) << (8 * (j & 3));
    }
    return nb;
}

/* byte j (runtime) of a lane's 32 bytes without indexing the register array */
__device__ __forceinline__ uint32_t lane_word(const uint32_t w[8], uint32_t d) {
    uint32_t lo = d == 0 ? w[0] : d == 1 ? w[1] : d == 2 ? w[2] : w[3];
    uint32_t hi = d == 4 ? w[4] : d == 5 ? w[5] : d == 6 ? w[6] : w[7];
    return d < 4 ? lo : hi;
}

__device__ __forceinline__ uint32_t lane_byte(const uint32_t w[8], uint32_t j) {
    uint32_t d = j >> 2;
    uint32_t lo = d == 0 ? w[0] : d == 1 ? w[1] : d == 2 ? w[2] : w[3];
    uint32_t hi = d == 4 ? w[4] : d == 5 ? w[5] : d == 6 ? w[6] : w[7];
    return ((d < 4 ? lo : hi) >> (8 * (j & 3))) & 0xFFu;
}

/*
 * General tile (one wave, FK_LANE_BYTES per lane, `nb` valid): any bytes,
 * any state.  COUNT=false only advances the wave state (halo guess).
 * `tile_off` is the tile's byte offset inside its range.
 */
template <bool COUNT, int HM>
__device__ __forceinline__ void tile_general(const Ctx &cx, const uint32_t w[8], int nb,
                                             uint32_t tile_off, DState &st, Facts &f,
                                             Counters &cnt, uint32_t weight) {
    const int lane = threadIdx.x & 63;
    const int k = cx.k;
    const uint32_t LB = FK_LANE_BYTES;

    /* -- 1. header flag at each lane start: last '>' vs last '\n' before it */
    uint32_t lastGT = 0, lastNL = 0, firstSp = 0xFFFFu, firstGT = 0;
#pragma unroll 1
    for (int d_ = 0; d_ < 8 && 4 * d_ < nb; d_++) {
        const uint32_t wd_ = lane_word(w, (uint32_t)d_);   /* one word select per 4 bytes */
    #pragma unroll
        for (int b_ = 0; b_ < 4; b_++) {
        const int j = 4 * d_ + b_;
        if (j >= nb) break;
        uint32_t c = (wd_ >> (8 * b_)) & 0xFFu;
        uint32_t pos = (uint32_t)lane * LB + (uint32_t)j + 1u;
        bool gt = c == '>';
        bool nl = c == '\n';
        if (gt) lastGT = pos;
        if (nl) lastNL = pos;
        if ((gt || nl) && firstSp == 0xFFFFu) { firstSp = pos - 1; firstGT = gt; }
    }
    }
    uint32_t g = lastGT, n = lastNL;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t tg = shup(g, d), tn = shup(n, d);
        if (lane >= d) { g = max(g, tg); n = max(n, tn); }
    }
    uint32_t gx = shup(g, 1), nx = shup(n, 1);
    if (lane == 0) { gx = 0; nx = 0; }
    const uint32_t hdr0 = (gx | nx) ? (gx > nx ? 1u : 0u) : st.hdr;

    /* -- 2. per-lane run summary under hdr0: (reset?, bases since, code) */
    uint32_t hdr = hdr0, rs = 0, nv = 0, hdr_end;
    uint64_t code = 0;
#pragma unroll 1
    for (int d_ = 0; d_ < 8 && 4 * d_ < nb; d_++) {
        const uint32_t wd_ = lane_word(w, (uint32_t)d_);   /* one word select per 4 bytes */
    #pragma unroll
        for (int b_ = 0; b_ < 4; b_++) {
        const int j = 4 * d_ + b_;
        if (j >= nb) break;
        uint32_t c = (wd_ >> (8 * b_)) & 0xFFu;
        /* branch-free: every lane takes the same instructions (selects) */
        const int s = fk_sym(c);
        const bool in = hdr != 0, nl = c == '\n', base = s >= 0;
        const bool brk = !in && !nl && !base;          /* '>', N, any other byte */
        const bool take = !in && base;
        rs |= brk ? 1u : 0u;
        nv = brk ? 0u : nv + (take ? 1u : 0u);
        code = take ? (code << 2) | (uint32_t)s : code;
        hdr = in ? (nl ? 0u : 1u) : (c == '>' ? 1u : 0u);
    }
    }
    hdr_end = hdr;

    /* -- 3. inclusive scan of run summaries across the wave */
    uint32_t p = (rs << 31) | nv;
    uint64_t cd = code;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t tp = shup(p, d);
        uint32_t tlo = shup((uint32_t)cd, d), thi = shup((uint32_t)(cd >> 32), d);
        if (lane >= d && !(p >> 31)) {
            uint32_t mynv = p & 0x7FFFFFFFu;
            uint64_t tc = ((uint64_t)thi << 32) | tlo;
            cd = fk_join(tc, cd, mynv);
            p = (tp & 0x80000000u) | ((tp & 0x7FFFFFFFu) + mynv);
        }
    }
    /* wave exit state from lane 63's inclusive summary */
    const uint32_t p63 = rdlane(p, 63);
    const uint64_t cd63 = rdlane64(cd, 63);
    const uint32_t hdr63 = rdlane(hdr_end, 63);
    DState nst;
    nst.hdr = hdr63;
    nst.R = (p63 >> 31) ? (p63 & 0x7FFFFFFFu) : st.R + (p63 & 0x7FFFFFFFu);
    nst.code = (p63 >> 31) ? cd63 : fk_join(st.code, cd63, p63 & 0x7FFFFFFFu);

    if (COUNT) {
        /* exclusive summary -> this lane's entering state */
        uint32_t ep = shup(p, 1);
        uint32_t elo = shup((uint32_t)cd, 1), ehi = shup((uint32_t)(cd >> 32), 1);
        if (lane == 0) { ep = 0; elo = 0; ehi = 0; }
        uint64_t ecd = ((uint64_t)ehi << 32) | elo;
        uint32_t R = (ep >> 31) ? (ep & 0x7FFFFFFFu) : st.R + (ep & 0x7FFFFFFFu);
        uint64_t lc = (ep >> 31) ? ecd : fk_join(st.code, ecd, ep & 0x7FFFFFFFu);
        hdr = hdr0;

        /* first special byte of the chunk ('\n' or '>') */
        uint64_t spm = __ballot(firstSp != 0xFFFFu);
        uint32_t p1 = 0xFFFFFFFFu;
        int p1_lane = -1;
        if (f.found_p1) {
            p1 = 0;
        } else if (spm) {
            p1_lane = __ffsll((long long)spm) - 1;
            p1 = rdlane(firstSp, p1_lane);
        }
        const bool p1_here = !f.found_p1 && spm;
        uint32_t r_at = 0, lane_reset = 0, lane_reset_after = 0;
        const uint64_t maskk1 = cx.maskk >> 2;

#pragma unroll 1
        for (int d_ = 0; d_ < 8 && 4 * d_ < nb; d_++) {
            const uint32_t wd_ = lane_word(w, (uint32_t)d_);   /* one word select per 4 bytes */
        #pragma unroll
            for (int b_ = 0; b_ < 4; b_++) {
            const int j = 4 * d_ + b_;
            if (j >= nb) break;
            uint32_t c = (wd_ >> (8 * b_)) & 0xFFu;
            uint32_t pos = (uint32_t)lane * LB + (uint32_t)j;
            if (p1_here && pos == p1) r_at = R;
            if (hdr) {
                if (c == '\n') hdr = 0;
                continue;
            }
            if (c == '\n') continue;
            int s = fk_sym(c);
            if (s < 0) {                      /* run break: '>', N, other */
                int seq = (int)R;
                if (HM == H_SPARSE) {
                    if (cx.slots && seq >= 1 && seq < k)
                        cx.slots[sp_slot(pos)] =
                            SP_SHORT | ((uint64_t)seq << 40) | fk_sigma(lc & ((1ull << (2 * seq)) - 1));
                } else if (HM != H_NONE && seq >= 1 && seq < k) {
                    short_run(cx, seq, lc, weight);
                }
                R = 0;
                lane_reset = 1;
                if (f.found_p1 || (p1_here && pos > p1)) lane_reset_after = 1;
                if (c == '>') {
                    hdr = 1;
                } else if (c == 0xFFu) {
                    uint32_t o = tile_off + pos;
                    cnt.eof = min(cnt.eof, o);
                } else if (c != 'N') {
                    cnt.unknown++;
                }
                continue;
            }
            lc = (lc << 2) | (uint32_t)s;
            R += 1;
            int seq = (int)R;
            if (seq >= k) {
                uint64_t idx = lc & cx.maskk;
                if (HM == H_SPARSE) { if (cx.slots) cx.slots[sp_slot(pos)] = fk_sigma(idx); }
                else hist_add<HM>(cx, idx, weight);
                cnt.win += 1;
                if (seq == k) {               /* first window: its first k-1 bases */
                    cnt.base += comp_packed(fk_sigma(idx) >> 2, k - 1, maskk1);
                    cnt.valid += (uint32_t)(k - 1);
                }
            } else if (seq >= 1) {
                uint32_t d0 = (uint32_t)((lc >> (2 * seq - 2)) & 3);
                cnt.d1s += 1ull << (16 * (d0 ^ (d0 >> 1)));
            }
        }
        }

        /* chunk facts */
        if (__ballot(lane_reset)) f.any_reset = 1;
        if (__ballot(lane_reset_after)) f.reset_after_p1 = 1;
        if (!(p63 >> 31)) f.nv_total += p63 & 0x7FFFFFFFu;
        if (p1_here) {
            f.found_p1 = 1;
            f.p1_gt = rdlane(firstGT, p1_lane);
            f.R_at_p1 = rdlane(r_at, p1_lane);
        }
    }
    st = nst;
}


/* byte-wise "is non-zero" mask (bit 7 of each byte), exact per byte */
__device__ __forceinline__ uint32_t nz_bytes(uint32_t d) {
    return (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
}

/* previous lane's value (DPP wave_shr:1); lane 0 receives `carry` */
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t carry) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)v, 0x138, 0xF, 0xF, false);
}

/* 16 bases -> 32-bit word, first base in bits 31:30 (v_dot4_u32_u8 x4) */
__device__ __forceinline__ uint32_t pack16(const uint32_t *x) {
    uint32_t P = __builtin_amdgcn_udot4(x[0], 0x01041040u, 0u, false);
    P = __builtin_amdgcn_udot4(x[1], 0x01041040u, P << 8, false);
    P = __builtin_amdgcn_udot4(x[2], 0x01041040u, P << 8, false);
    return __builtin_amdgcn_udot4(x[3], 0x01041040u, P << 8, false);
}

/* The newline code of a half (tile_fast): 0 = no '\n'; 73 * (16 + j) = one
   '\n' at byte j; anything >= NL_TWO = more than one.  nl_byte decodes j + 16
   (exact for 16..31: 73 t * 899 >> 16 = t). */
#define NL_TWO (73u * 33u)
__device__ __forceinline__ uint32_t nl_byte(uint32_t c) { return __umul24(c, 899u) >> 16; }

/* drop digit j (the '\n' byte; first digit in bits 31:30) -> 15 bases
   right-aligned: the digits after j stay, those before it move down one.
   t = 16 + j. */
__device__ __forceinline__ uint32_t squeeze(uint32_t P, uint32_t t) {
    const uint32_t keep = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, 62u - 2u * t);   /* (1 << (30-2j)) - 1 */
    return (P & keep) | ((P >> 2) & ~keep);
}

/* Count the 16 windows ending in one half: {C, S2} is a contiguous base
 * stream with S2 holding this half's 16 slots (slot 0 belongs to the previous
 * half when `skip0`). */
template <int HM>
__device__ __forceinline__ void half_windows(const Ctx &cx, uint32_t C, uint32_t S2, bool skip0,
                                             uint32_t weight) {
    const uint32_t m2 = (uint32_t)cx.maskk << 2;
    if (HM == H_PAIRS) {
        /* (k+1)-mers ending at odd slots 1,3,..,15 cover the k-mers at slots
           (0,1),(2,3),...; without a real slot 0 the first pair becomes the
           single k-mer at slot 1 */
        const uint32_t m3 = (uint32_t)((cx.maskk << 2) | 3u) << 2;
#define FK_LDS_ADD(a_) lds_add(cx, (a_), weight)
        {
            uint32_t v = __builtin_amdgcn_alignbit(C, S2, 26u);
            uint32_t addr = skip0 ? (cx.single_off * 4u + (v & m2)) : (v & m3);
            FK_LDS_ADD(addr);
        }
#pragma unroll
        for (int j = 1; j < 7; j++) {
            uint32_t a = __builtin_amdgcn_alignbit(C, S2, (uint32_t)(26 - 4 * j)) & m3;
            FK_LDS_ADD(a);
        }
        FK_LDS_ADD((S2 << 2) & m3);
#undef FK_LDS_ADD
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t sh = 2u * (15u - (uint32_t)i);
            uint32_t v = i < 15 ? __builtin_amdgcn_alignbit(C, S2, sh) : S2;
            uint32_t idx = v & (uint32_t)cx.maskk;
            if (i > 0 || !skip0) {
                if (HM == H_LDS) lds_add(cx, idx * 4u, weight);
                else atomicAdd(&cx.table[fk_sigma(idx)], weight);
            }
        }
    }
}

/*
 * Fast tile: every byte is A/C/G/T except at most one '\n' per 16-byte half
 * lane, the wave is outside a header and deep inside a run (every window
 * counts as seqSize > k).  Returns false (without side effects) when the
 * tile does not qualify; the caller then runs tile_general.
 *
 * Per lane (32 bytes): bases -> 2-bit codes (A0 C1 T2 G3 = (byte>>1)&3, a
 * v_perm checks them against the bytes), two 32-bit words via
 * v_dot4_u32_u8; the previous lane's last word arrives by DPP wave_shr:1;
 * each window is one v_alignbit of a 64-bit {context, word} pair.
 */
/* The part of a fast tile after classification.  NL: some lane has a '\n'
 * (nl0/nl1 per half: 0, or 16 + its byte); without one every half holds 16
 * bases and all of the newline handling folds away. */
template <bool COUNT, int HM, bool INTER, bool NL>
__device__ __forceinline__ bool tile_finish(const Ctx &cx, const uint32_t x[8], uint32_t nl0, uint32_t nl1,
                                            DState &st, Facts &f, Counters &cnt, uint32_t weight, Emit *em,
                                            bool *kind) {
    const int k = cx.k;
    if (kind) *kind = true;   /* bases only (the state may still not be deep) */
    /* deep: every window of the tile counts (seq > k throughout); neg: the
       reference's int32 seqSize stays negative for the whole tile (a run
       past 2^31-1 bases, :977), so the tile only advances the state */
    const bool deep = (int32_t)st.R >= k && st.R <= 0x7FFFFFFFu - FK_TILE_BYTES;
    const bool neg = (int32_t)st.R < 0 && st.R <= 0xFFFFFFFFu - FK_TILE_BYTES;
    if (COUNT && !deep && !neg) return false;

    uint32_t S0 = pack16(x), S1 = pack16(x + 4);
    const bool h0 = NL && nl0 != 0, h1 = NL && nl1 != 0;
    /* a half with a '\n' holds 15 bases, right-aligned (the next lane's
       context and the carried state read it as the stream's last digits) */
    if (NL) {
        S0 = h0 ? squeeze(S0, nl_byte(nl0)) : S0;
        S1 = h1 ? squeeze(S1, nl_byte(nl1)) : S1;
    }
    /* the 16-byte piece before each half: contiguous layout (lane = 32
       bytes) -> half 0 follows the previous lane's half 1 and half 1 its own
       half 0; interleaved layout (half h of lane L at h*1024 + 16L) -> each
       half follows the previous lane's same half, lane 0's half 1 follows
       lane 63's half 0 */
    const uint32_t P0 = INTER ? from_prev_lane(S0, (uint32_t)st.code) : from_prev_lane(S1, (uint32_t)st.code);
    const uint32_t P1 = INTER ? from_prev_lane(S1, rdlane(S0, 63)) : S0;
    /* make each {C, S2} one contiguous base stream with S2 holding 16 digits */
    const uint32_t A2 = h0 ? (S0 | (P0 << 30)) : S0;
    const uint32_t AC = h0 ? (P0 >> 2) : P0;
    const uint32_t B2 = h1 ? (S1 | (P1 << 30)) : S1;
    const uint32_t BC = h1 ? (P1 >> 2) : P1;

    const uint64_t nb0 = NL ? __ballot(h0) : 0ull, nb1 = NL ? __ballot(h1) : 0ull;
    const uint32_t nsym = NL ? FK_TILE_BYTES - (uint32_t)__popcll(nb0) - (uint32_t)__popcll(nb1) : FK_TILE_BYTES;
    if (COUNT) {
        if (HM == H_EMIT) {
            em->AC = AC; em->A2 = A2; em->BC = BC; em->B2 = B2;
            em->h0 = h0; em->h1 = h1; em->deep = deep;
            if (deep) cnt.win_u += nsym;
        } else if (HM == H_SPARSE) {   /* the sparse feed's counters (k_redo mode 2): windows, no slots */
            if (deep) cnt.win_u += nsym;
        } else if (HM == H_NONE) {
        } else if (deep) {
            half_windows<HM>(cx, AC, A2, h0, weight);
            half_windows<HM>(cx, BC, B2, h1, weight);
            cnt.win_u += nsym;
        }
        /* facts: the first '\n' of the span (all bytes before it are bases) */
        if (NL && !f.found_p1 && (nb0 | nb1)) {
            uint32_t before;
            if (INTER) {
                const bool in0 = nb0 != 0;
                const int L = __ffsll((long long)(in0 ? nb0 : nb1)) - 1;
                const uint32_t c = nl_byte(in0 ? rdlane(nl0, L) : rdlane(nl1, L));
                before = (in0 ? 0u : 1024u) + 16u * (uint32_t)L + (c - 16u);
            } else {
                const int L0 = __ffsll((long long)(nb0 | nb1)) - 1;
                const uint32_t a = nl_byte(rdlane(nl0, L0)), b = nl_byte(rdlane(nl1, L0));
                before = (uint32_t)L0 * FK_LANE_BYTES + (a ? a - 16u : b);
            }
            f.found_p1 = 1;
            f.p1_gt = 0;
            f.R_at_p1 = st.R + before;
        }
        f.nv_total += nsym;
    }
    st.R += nsym;
    /* the last 32 bases: lane 63's second half and its context (both layouts) */
    st.code = ((uint64_t)rdlane(BC, 63) << 32) | rdlane(B2, 63);
    return true;
}

/*
 * Fast tile: every byte is A/C/G/T except at most one '\n' per 16-byte half
 * lane, the wave is outside a header and deep inside a run (every window
 * counts as seqSize > k).  Returns false (without side effects) when the
 * tile does not qualify; the caller then runs tile_general.
 *
 * Per lane (32 bytes): bases -> 2-bit codes (A0 C1 T2 G3 = (byte>>1)&3, a
 * v_perm checks them against the bytes), two 32-bit words via
 * v_dot4_u32_u8; the previous lane's last word arrives by DPP wave_shr:1;
 * each window is one v_alignbit of a 64-bit {context, word} pair.  A tile
 * of bases only (wave-uniform test) takes tile_finish<NL = false>.
 */
template <bool COUNT, int HM, bool INTER>
__device__ __forceinline__ bool tile_fast(const Ctx &cx, const uint32_t w[8], DState &st, Facts &f,
                                          Counters &cnt, uint32_t weight, Emit *em = nullptr, bool *kind = nullptr) {
    uint32_t x[8], m[8];
    uint32_t mis = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        x[d] = (w[d] >> 1) & 0x03030303u;
        m[d] = __builtin_amdgcn_perm(0u, 0x47544341u, x[d]) ^ w[d];   /* byte != "ACTG"[x] */
        mis |= m[d];
    }
    if (!__ballot(mis != 0)) return tile_finish<COUNT, HM, INTER, false>(cx, x, 0u, 0u, st, f, cnt, weight, em, kind);
    /* some lane has a non-base byte: every lane classifies (the wave runs
       this once for all of them).  A byte is a base (m = 0) or '\n'
       (w ^ 0x0A = 0) iff the product of the two is 0, so dot4(m, w ^ 0x0A)
       checks four bytes exactly (short chains: the dot4 latency is long).
       On a lane without other bytes m = 0x49 exactly at the '\n's, and a
       dot4 with weights 16 + j gives the half's newline code (NL_TWO). */
    uint32_t bad4[4], nl0, nl1;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        bad4[c] = __builtin_amdgcn_udot4(m[2 * c], w[2 * c] ^ 0x0A0A0A0Au, 0u, false);
        bad4[c] = __builtin_amdgcn_udot4(m[2 * c + 1], w[2 * c + 1] ^ 0x0A0A0A0Au, bad4[c], false);
    }
    {
        uint32_t a0 = __builtin_amdgcn_udot4(m[0], 0x13121110u, 0u, false);
        uint32_t a1 = __builtin_amdgcn_udot4(m[2], 0x1B1A1918u, 0u, false);
        uint32_t b0 = __builtin_amdgcn_udot4(m[4], 0x13121110u, 0u, false);
        uint32_t b1 = __builtin_amdgcn_udot4(m[6], 0x1B1A1918u, 0u, false);
        a0 = __builtin_amdgcn_udot4(m[1], 0x17161514u, a0, false);
        a1 = __builtin_amdgcn_udot4(m[3], 0x1F1E1D1Cu, a1, false);
        b0 = __builtin_amdgcn_udot4(m[5], 0x17161514u, b0, false);
        b1 = __builtin_amdgcn_udot4(m[7], 0x1F1E1D1Cu, b1, false);
        nl0 = a0 + a1;
        nl1 = b0 + b1;
    }
    const bool lane_ok = (bad4[0] | bad4[1] | bad4[2] | bad4[3]) == 0 && nl0 < NL_TWO && nl1 < NL_TWO;
    if (__ballot(!lane_ok)) return false;
    return tile_finish<COUNT, HM, INTER, true>(cx, x, nl0, nl1, st, f, cnt, weight, em, kind);
}

/*
 * Mixed tile: any bytes (comment lines, run breaks, several newlines, N,
 * unknown bytes, 0xFF), interleaved layout, counted without a byte walk.  The
 * tile is two sub-tiles of 1 KiB (half h of every lane: the 16 bytes at
 * h*1024 + 16L), counted in stream order by sub_mixed.  Per lane, over its 16
 * bytes as bit masks (bit j = byte j):
 *   - byte classes ('\n', '>', not a base) by SWAR byte compares;
 *   - the comment flag entering each lane from two ballots (is the last '>'
 *     or '\n' before it a '>'), then the comment bytes by one add: a '>'
 *     starts a carry that runs through the bytes up to the next '\n'
 *     (findKmer.cpp:991-1008; a '>' inside a comment changes nothing);
 *   - takes (bases outside comments) and breaks (every other byte outside
 *     comments but '\n', :1011-1024), and run starts (a take whose last take
 *     or break before it is a break) by the same add;
 *   - the takes' 2-bit codes compacted (blocks of other bytes squeezed out),
 *     right-aligned: the lane's digit stream;
 *   - the wave scan of (reset, bases since, code) that tile_general uses gives
 *     each lane its entering run length R and last 32 bases;
 *   - the slots that end a window (R >= k, :1035-1057) form a 16-bit mask W;
 *     windows go to the bins as in half_windows (a (k+1)-mer pair where both
 *     of a pair's slots count, else a single k-mer), or to the partition with
 *     the mask (H_EMIT).
 * The rare parts -- a run's first window (its first k-1 bases), the depth-1
 * touches of a run's first k-1 bases, runs shorter than k (:1059-1062), N,
 * unknown and 0xFF bytes -- loop over set bits, only in lanes that have them.
 * Not for the sparse mode or near the reference's int32 seqSize wrap: the
 * caller runs tile_general then.
 */
__device__ __forceinline__ uint32_t zero_bytes(uint32_t d) {   /* bit 7 of each byte: byte == 0 */
    return ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
}
__device__ __forceinline__ uint32_t bits4(uint32_t m) {   /* bit 7 of byte j -> bit j */
    return __builtin_amdgcn_udot4((m >> 7) & 0x01010101u, 0x08040201u, 0u, false);
}
__device__ __forceinline__ uint32_t hibit(uint32_t v) { return 31u - (uint32_t)__clz((int)v); }   /* v != 0 */

/* One sub-tile (16 bytes per lane at byte sub_off + 16L of the range).  Out:
   the lane's window words {C, S2} (S2 = the 16 slots ending at its last
   base, C the 16 before) and the slot mask W (bit 15 - s = slot s). */
template <int HM>
__device__ __forceinline__ void sub_mixed(const Ctx &cx, const uint32_t q[4], uint32_t sub_off, DState &st,
                                          Facts &f, Counters &cnt, uint32_t weight, uint32_t &oC, uint32_t &oS2,
                                          uint32_t &oW, bool &plain) {
    const uint32_t lane = threadIdx.x & 63;
    const int k = cx.k;
    /* -- 1. classes */
    uint32_t x[4], nbm = 0, nlm = 0, gtm = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        x[d] = (q[d] >> 1) & 0x03030303u;
        const uint32_t mb = __builtin_amdgcn_perm(0u, 0x47544341u, x[d]) ^ q[d];   /* 0: A/C/G/T */
        nbm |= bits4(nz_bytes(mb)) << (4 * d);
        nlm |= bits4(zero_bytes(q[d] ^ 0x0A0A0A0Au)) << (4 * d);
        gtm |= bits4(zero_bytes(q[d] ^ 0x3E3E3E3Eu)) << (4 * d);
    }
    /* -- 2. comment flag entering each lane, and after the sub-tile */
    const uint32_t ev = nlm | gtm;
    const bool lgt = ev != 0 && ((gtm >> hibit(ev | 1u)) & 1u);
    const uint64_t bev = __ballot(ev != 0), bgt = __ballot(lgt);
    const uint64_t before = bev & ((1ull << lane) - 1ull);
    const uint32_t hin = before ? (uint32_t)(bgt >> (63 - __clzll((long long)before))) & 1u : st.hdr;
    const uint32_t hout = bev ? (uint32_t)(bgt >> (63 - __clzll((long long)bev))) & 1u : st.hdr;
    /* -- 3. comment bytes (bit j: inside a comment before byte j), takes, breaks */
    const uint32_t pm = ((~nlm & 0xFFFFu) << 1) | hin, am = (gtm << 1) | hin;
    const uint32_t hb = (((pm + am) ^ pm) | am) & ~(nlm << 1) & 0xFFFFu;
    const uint32_t T = ~nbm & ~hb & 0xFFFFu;
    const uint32_t K = nbm & ~nlm & ~hb & 0xFFFFu;
    const uint32_t oth = K & ~gtm;   /* N, 0xFF, unknown */
    if (__ballot(oth != 0)) {
        uint32_t nm = 0, fm = 0;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            nm |= bits4(zero_bytes(q[d] ^ 0x4E4E4E4Eu)) << (4 * d);
            fm |= bits4(zero_bytes(~q[d])) << (4 * d);
        }
        cnt.unknown += __popc(oth & ~nm & ~fm);
        const uint32_t ff = oth & fm;
        if (ff) cnt.eof = min(cnt.eof, sub_off + 16u * lane + (uint32_t)(__ffs((int)ff) - 1));
    }
    /* -- 4. run starts; trailk: a break after the lane's last take */
    const uint32_t pz = ~T & 0xFFFFu, zs = pz + K;
    const uint32_t rbb = ((zs ^ pz) | K) & T;
    const uint32_t trailk = zs >> 16;
    /* -- 5. compaction: digit j at bit 15 - j, blocks of non-takes squeezed out
       from the first one on (the digits before a block move down past it) */
    const uint32_t nt = __popc(T);
    uint32_t P = pack16(x);
    uint32_t U = __builtin_bitreverse32(pz) >> 16;
    uint32_t RB = __builtin_bitreverse32(rbb) >> 16;
    while (__ballot(U != 0)) {
        if (U) {
            const uint32_t hi = hibit(U);
            const uint32_t V = ~U & ((1u << hi) - 1u);
            const uint32_t lo = V ? hibit(V) + 1u : 0u;
            const uint32_t L = hi - lo + 1u;
            const uint32_t k2 = (1u << (2u * lo)) - 1u, k1 = (1u << lo) - 1u;
            P = (P & k2) | ((uint32_t)((uint64_t)P >> (2u * L)) & ~k2);
            RB = (RB & k1) | ((RB >> L) & ~k1);
            U &= k1;
        }
    }
    /* -- 6. scan of (reset, bases since the last break, code) */
    const uint32_t after_k = K ? ~((2u << hibit(K)) - 1u) : 0xFFFFFFFFu;
    uint32_t p = (K ? 0x80000000u : 0u) | (uint32_t)__popc(T & after_k);
    uint64_t cd = P;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t tp = shup(p, d);
        const uint32_t tlo = shup((uint32_t)cd, d), thi = shup((uint32_t)(cd >> 32), d);
        if (lane >= (uint32_t)d && !(p >> 31)) {
            const uint32_t mynv = p & 0x7FFFFFFFu;
            cd = fk_join(((uint64_t)thi << 32) | tlo, cd, mynv);
            p = (tp & 0x80000000u) | ((tp & 0x7FFFFFFFu) + mynv);
        }
    }
    const uint32_t p63 = rdlane(p, 63);
    const uint64_t cd63 = rdlane64(cd, 63);
    uint32_t ep = shup(p, 1);
    uint32_t elo = shup((uint32_t)cd, 1), ehi = shup((uint32_t)(cd >> 32), 1);
    if (lane == 0) { ep = 0; elo = 0; ehi = 0; }
    const uint64_t ecd = ((uint64_t)ehi << 32) | elo;
    const uint32_t Rin = (ep >> 31) ? (ep & 0x7FFFFFFFu) : st.R + (ep & 0x7FFFFFFFu);
    const uint64_t cin = (ep >> 31) ? ecd : fk_join(st.code, ecd, ep & 0x7FFFFFFFu);
    /* -- 7. facts (before the window work: what they need dies here): the span's first '\n' or '>' (any state), breaks, bases */
    const bool anyk = __ballot(K != 0) != 0;
    if (!f.found_p1 && bev) {
        const int L1 = __ffsll((long long)bev) - 1;
        const uint32_t jf = ev ? (uint32_t)(__ffs((int)ev) - 1) : 0u;
        const uint32_t below = (1u << jf) - 1u, kb = K & below;
        const uint32_t r = kb ? (uint32_t)__popc(T & below & ~((2u << hibit(kb)) - 1u)) : Rin + (uint32_t)__popc(T & below);
        const bool after = lane > (uint32_t)L1 ? K != 0 : (lane == (uint32_t)L1 && (K >> (jf + 1u)) != 0);
        if (__ballot(after)) f.reset_after_p1 = 1;
        f.found_p1 = 1;
        f.p1_gt = rdlane((gtm >> jf) & 1u, L1);
        f.R_at_p1 = rdlane(r, L1);
    } else if (f.found_p1 && anyk) {
        f.reset_after_p1 = 1;
    }
    if (anyk) f.any_reset = 1;
    else f.nv_total += p63 & 0x7FFFFFFFu;
    /* bases only, at most one '\n' per lane, outside comments: the fast path's kind */
    plain = !anyk && st.hdr == 0 && hout == 0 && !__ballot(gtm != 0 || __popc(nlm) > 1);
    /* -- 8. digits with 1 <= R < k (F) and the window slots (W) */
    const uint32_t vd = (1u << nt) - 1u;
    uint32_t F = 0;
    if (k > 1) {
        uint32_t s = RB;   /* each run start covers its first k-1 digits */
        for (int cov = 1; cov < k - 1;) {
            const int sh = min(cov, k - 1 - cov);
            s |= s >> sh;
            cov += sh;
        }
        F = s;
        if (Rin < (uint32_t)(k - 1)) {
            const uint32_t m = min(nt, (uint32_t)(k - 1) - Rin);
            F |= vd & ~((1u << (nt - m)) - 1u);
        }
        F &= vd;
    }
    const uint32_t W = vd & ~F;
    const uint64_t full = (cin << (2u * nt)) | P;   /* the last 32 bases up to the lane's last take */
    const uint32_t C = (uint32_t)(full >> 32), S2 = (uint32_t)full;
    cnt.win += __popc(W);
    if (HM == H_PAIRS) {
        /* pair j: slots 2j, 2j + 1; {C, S2} << 2 puts slot 15's pair at 0 */
        const uint32_t m2 = (uint32_t)cx.maskk << 2, m3 = (uint32_t)((cx.maskk << 2) | 3u) << 2;
        const uint32_t S4 = S2 << 2;
#pragma unroll 2
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t two = (W >> (14u - 2u * j)) & 3u;   /* bit 1: slot 2j, bit 0: slot 2j + 1 */
            const uint32_t odd = j < 7u ? __builtin_amdgcn_alignbit(C, S2, 26u - 4u * j) : S4;
            if (two == 3u) lds_add(cx, odd & m3, weight);
            if (two == 1u || two == 2u) {
                const uint32_t a = two == 1u ? odd : __builtin_amdgcn_alignbit(C, S2, 28u - 4u * j);
                lds_add(cx, cx.single_off * 4u + (a & m2), weight);
            }
        }
    } else if (HM == H_LDS || HM == H_GLOBAL) {
#pragma unroll 2
        for (uint32_t i = 0; i < 16; i++) {
            if ((W >> (15u - i)) & 1u) {
                const uint32_t v = i < 15u ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - i)) : S2;
                hist_add<HM>(cx, v & (uint32_t)cx.maskk, weight);
            }
        }
    }
    if (k > 1) {
        /* a run's first window adds its first k-1 bases (:1044-1057) */
        uint32_t fw = RB >> (k - 1);
        if (Rin < (uint32_t)k && (uint32_t)(k - 1) - Rin < nt) fw |= 1u << (nt - 1u - ((uint32_t)(k - 1) - Rin));
        fw &= W;
        const uint64_t maskk1 = cx.maskk >> 2;
        while (__ballot(fw != 0)) {
            if (fw) {
                const uint32_t b = (uint32_t)(__ffs((int)fw) - 1);
                fw &= fw - 1u;
                const uint64_t idx = (full >> (2u * b)) & cx.maskk;
                cnt.base += comp_packed(fk_sigma(idx) >> 2, k - 1, maskk1);
                cnt.valid += (uint32_t)(k - 1);
            }
        }
        /* depth-1 touches: every digit with R < k, for its run's first base */
        if (__ballot(F != 0)) {
            const uint32_t top = RB ? ~((2u << hibit(RB)) - 1u) : 0xFFFFFFFFu;   /* before the first start */
            const uint32_t c0 = __popc(F & top);
            if (c0) {
                const uint32_t d0 = Rin ? (uint32_t)(cin >> (2u * (Rin - 1u))) & 3u : (P >> (2u * (nt - 1u))) & 3u;
                cnt.d1s += (uint64_t)c0 << (16 * (d0 ^ (d0 >> 1)));
            }
            uint32_t rem = F ? RB : 0u;
            while (__ballot(rem != 0)) {
                if (rem) {
                    const uint32_t b = hibit(rem);
                    rem &= ~(1u << b);
                    const uint32_t seg = ((2u << b) - 1u) & (rem ? ~((2u << hibit(rem)) - 1u) : 0xFFFFFFFFu);
                    const uint32_t c = __popc(F & seg);
                    if (c) {
                        const uint32_t d0 = (P >> (2u * b)) & 3u;
                        cnt.d1s += (uint64_t)c << (16 * (d0 ^ (d0 >> 1)));
                    }
                }
            }
        }
        /* runs that a break ends before they reach k bases: their prefix walk */
        if (HM != H_NONE && __ballot(K != 0)) {
            const uint32_t top = RB ? ~((2u << hibit(RB)) - 1u) : 0xFFFFFFFFu;
            if (K) {
                const uint32_t n0 = __popc(vd & top);
                const uint32_t L0 = Rin + n0;
                if ((RB || trailk) && L0 >= 1u && L0 < (uint32_t)k)
                    short_run(cx, (int)L0, n0 ? (full >> (2u * (nt - n0))) : cin, weight);
            }
            uint32_t rem = K ? RB : 0u;
            while (__ballot(rem != 0)) {
                if (rem) {
                    const uint32_t b = hibit(rem);
                    rem &= ~(1u << b);
                    const uint32_t e = rem ? hibit(rem) + 1u : 0u;   /* the run's last digit */
                    if ((rem || trailk) && b - e + 1u < (uint32_t)k) short_run(cx, (int)(b - e + 1u), full >> (2u * e), weight);
                }
            }
        }
    }
    st.hdr = hout;
    st.R = (p63 >> 31) ? (p63 & 0x7FFFFFFFu) : st.R + (p63 & 0x7FFFFFFFu);
    st.code = (p63 >> 31) ? cd63 : fk_join(st.code, cd63, p63 & 0x7FFFFFFFu);
    oC = C;
    oS2 = S2;
    oW = W;
}

/* A tile by sub_mixed.  plain: the tile was of the fast path's kind (bases
   only, at most one '\n' per 16 bytes, outside comments) and ends deep in a
   run, so the next tile most likely is too. */
template <int HM>
__device__ __forceinline__ bool tile_mixed(const Ctx &cx, const uint32_t w[8], uint32_t tile_off, DState &st,
                                           Facts &f, Counters &cnt, uint32_t weight, bool &plain,
                                           Emit *em = nullptr) {
    plain = false;
    if (HM == H_SPARSE || st.R > 0x7FFFFFFFu - FK_TILE_BYTES) return false;
    uint32_t C0 = 0, S0 = 0, W0 = 0;
    bool pl = true;
#pragma unroll 1
    for (uint32_t h = 0; h < 2; h++) {   /* one copy of sub_mixed: register pressure */
        const uint32_t hm = 0u - h;   /* select without indexing the register array */
        uint32_t q[4];
#pragma unroll
        for (int d = 0; d < 4; d++) q[d] = (w[4 + d] & hm) | (w[d] & ~hm);
        uint32_t C, S2, W;
        bool p;
        sub_mixed<HM>(cx, q, tile_off + h * (FK_TILE_BYTES / 2), st, f, cnt, weight, C, S2, W, p);
        pl = pl && p;
        if (HM == H_EMIT) {
            if (h == 0) {
                C0 = C; S0 = S2; W0 = W;
            } else {
                em->AC = C0; em->A2 = S0; em->BC = C; em->B2 = S2;
                em->h0 = em->h1 = false;
                em->deep = true;
                em->masked = true;
                em->cm = W0 | (W << 16);
            }
        }
    }
    plain = pl && st.R >= (uint32_t)cx.k;
    return true;
}


__device__ __forceinline__ void acc_add(unsigned long long *a, uint64_t v, uint32_t weight) {
    if (v) atomicAdd(a, (unsigned long long)(weight == 1u ? v : (0ull - v)));
}

__device__ __forceinline__ void flush_counters(const Ctx &cx, Counters &cnt, uint32_t weight, bool to_acc = true) {
    const int lane = threadIdx.x & 63;
    uint32_t vals[11];
#pragma unroll
    for (int b = 0; b < 4; b++) {
        vals[b] = (uint32_t)((cnt.base >> (16 * b)) & 0xFFFF);
        vals[6 + b] = (uint32_t)((cnt.d1s >> (16 * b)) & 0xFFFF);
    }
    vals[4] = cnt.valid;
    vals[5] = cnt.win + (lane == 0 ? cnt.win_u : 0u);
    vals[10] = cnt.unknown;
#pragma unroll
    for (int i = 0; i < 11; i++) vals[i] = wsum32(vals[i]);
    if (lane == 0 && to_acc) {
        unsigned long long *a =
            cx.acc + ((blockIdx.x * FK_WAVES_PER_BLOCK + (threadIdx.x >> 6)) % FK_ACC_COPIES) * ACC_N;
#pragma unroll
        for (int i = 0; i < 4; i++) acc_add(&a[ACC_BASE + i], vals[i], weight);
        acc_add(&a[ACC_VALID], vals[4], weight);
        acc_add(&a[ACC_WIN], vals[5], weight);
#pragma unroll
        for (int i = 0; i < 4; i++) acc_add(&a[ACC_D1S + i], vals[6 + i], weight);
        acc_add(&a[ACC_UNK], vals[10], weight);
    }
    cnt.base = cnt.d1s = 0;
    cnt.valid = cnt.win = cnt.win_u = 0;
}

/* One tile of count_range (interleaved layout): the fast path when it
 * qualifies, else a mixed tile, else the general path on the tile reloaded
 * in the contiguous layout (which also takes a tile only partly inside the
 * input). */
template <int HM>
__device__ __forceinline__ void do_tile(const Ctx &cx, const uint32_t w[8], int64_t toff, uint32_t tile_off,
                                        bool full, DState &st, Facts &f, Counters &cnt, uint32_t weight,
                                        bool mixed) {
    /* (H_SPARSE: only when counting, without slots -- the sparse feed's
       counters; k_sp_emit takes fast tiles itself) */
    if ((HM != H_SPARSE || !cx.slots) && full && st.hdr == 0 && tile_fast<true, HM, true>(cx, w, st, f, cnt, weight))
        return;
    bool plain;
    if (HM != H_SPARSE && full && mixed && tile_mixed<HM>(cx, w, tile_off, st, f, cnt, weight, plain)) return;
    const int lane = threadIdx.x & 63;
    uint32_t v[8];
    const int nb = load_lane<FK_LANE_BYTES>(cx, toff + lane * (int64_t)FK_LANE_BYTES, v);
    tile_general<true, HM>(cx, v, nb, tile_off, st, f, cnt, weight);
}

/* Bytes [rbase, rend) of a range and its tile count. */
struct Span {
    uint64_t rbase, rend, ntiles, nfull;
};
__device__ __forceinline__ Span range_span(const RangeRec &r, uint64_t len) {
    Span s;
    s.rbase = r.c0 * FK_CHUNK_BYTES;
    s.rend = min(r.c1 * FK_CHUNK_BYTES, len);
    s.ntiles = (s.rend - s.rbase + FK_TILE_BYTES - 1) / FK_TILE_BYTES;
    s.nfull = (s.rend - s.rbase) / FK_TILE_BYTES;
    return s;
}

/* Count tiles [t0, sp.ntiles) of a range from state st (weight 1, or
 * 0xFFFFFFFF to cancel), any bytes.  Tile t+1's loads stay in flight while
 * tile t is counted (A/B ping-pong). */
template <int HM>
__device__ void count_range(const Ctx &cx, const Span &sp, uint64_t t0, DState &st, Facts &f,
                            Counters &cnt, uint32_t weight, bool mixed) {
    const int lane = threadIdx.x & 63;
    uint32_t A[8], B[8];
    /* interleaved tiles (lane L: bytes 16L.. and 1024 + 16L..); unconditional
       loads clamped into the range keep the vmcnt accounting static (a full
       tile is never clamped); a tile only partly inside the input is
       reloaded by do_tile */
#define FK_LOADT(dst, t_)                                                            \
    {                                                                                \
        const uint64_t tb_ = sp.rbase + (uint64_t)(t_) * FK_TILE_BYTES + 16u * (uint64_t)lane; \
        const uint64_t o0_ = min(tb_, sp.rend - 16u), o1_ = min(tb_ + 1024u, sp.rend - 16u); \
        u32x4 v0_ = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(cx.buf + o0_)); \
        u32x4 v1_ = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(cx.buf + o1_)); \
        dst[0] = v0_.x; dst[1] = v0_.y; dst[2] = v0_.z; dst[3] = v0_.w;               \
        dst[4] = v1_.x; dst[5] = v1_.y; dst[6] = v1_.z; dst[7] = v1_.w;               \
    }
#define FK_DOT(buf_, t_)                                                             \
    {                                                                                \
        do_tile<HM>(cx, buf_, (int64_t)(sp.rbase + (uint64_t)(t_) * FK_TILE_BYTES),  \
                    (uint32_t)((t_) * FK_TILE_BYTES), (t_) < sp.nfull, st, f, cnt, weight, mixed); \
    }
    FK_LOADT(A, t0);
    for (uint64_t t = t0; t < sp.ntiles; t += 2) {
        FK_LOADT(B, t + 1);
        FK_DOT(A, t);
        if (t + 1 >= sp.ntiles) break;
        FK_LOADT(A, t + 2);
        FK_DOT(B, t + 1);
    }
#undef FK_DOT
    (void)lane;
}

/* Flush a range's counters; lane 0 records its observations in rr. */
__device__ __forceinline__ void range_obs(const Ctx &cx, Counters &cnt, uint32_t weight, const Span &sp, RangeRec *r,
                          bool write, bool to_acc = true) {
    flush_counters(cx, cnt, weight, to_acc);
    const uint32_t unk = wsum32(cnt.unknown);
    const uint32_t eof = wmin32(cnt.eof);
    if ((threadIdx.x & 63) == 0 && weight == 1u) {
        if (eof != FK_NO_EOF) atomicMin(&cx.res->eof_cand, (unsigned long long)(sp.rbase + eof));
        if (write) {
            r->eof = eof == FK_NO_EOF ? FK_NO_EOF64 : (uint64_t)eof;
            r->unknown = unk;
        }
    }
}

/* Guess the state entering a range from the FK_HALO_BYTES before it (lanes
 * 0..7 hold them, 32 contiguous bytes each; `valid` = this lane's bytes are
 * readable input).  All bases (the common case): R = 256 and the last 32
 * bases, packed as the fast path packs them; otherwise the general walk. */
template <int HM>
__device__ __forceinline__ DState halo_guess(const Ctx &cx, const uint32_t w[8], bool valid) {
    const uint32_t hl = FK_HALO_BYTES / FK_LANE_BYTES;
    uint32_t x[8];
    uint32_t mis = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        x[d] = (w[d] >> 1) & 0x03030303u;
        mis |= __builtin_amdgcn_perm(0u, 0x47544341u, x[d]) ^ w[d];
    }
    const uint64_t vm = __ballot(valid), bad = __ballot(valid && mis);
    if (vm == (1ull << hl) - 1 && bad == 0) {
        const uint32_t hi = rdlane(pack16(x), hl - 1), lo32 = rdlane(pack16(x + 4), hl - 1);
        return DState{((uint64_t)hi << 32) | lo32, FK_HALO_BYTES, 0};
    }
    uint32_t v[8];
#pragma unroll
    for (int d = 0; d < 8; d++) v[d] = valid ? w[d] : 0u;
    DState st{0, 0, 0};
    Facts f{0, 0, 0, 0, 0, 0};
    Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
    tile_general<false, HM>(cx, v, valid ? (int)FK_LANE_BYTES : 0, 0, st, f, cnt, 1u);
    return st;
}

__device__ uint32_t lds_words(int HM, int k) {
    return HM == H_PAIRS ? (1u << (2 * k + 2)) + (1u << (2 * k)) : HM == H_LDS ? (1u << (2 * k)) : 0u;
}

__device__ void lds_zero(uint32_t *lds, uint32_t nw) {
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) lds[i] = 0;
    __syncthreads();
}

/* fold the block's LDS bins into the global table */
template <int HM>
__device__ void lds_flush(const Ctx &cx) {
    __syncthreads();
    const uint32_t nk = 1u << (2 * cx.k);
    for (uint32_t i = threadIdx.x; i < nk; i += blockDim.x) {
        uint32_t v;
        if (HM == H_PAIRS) {
            const uint32_t *pr = cx.lds;
            v = cx.lds[cx.single_off + i];
            /* k-mer i is the prefix of (k+1)-mers 4i+a and the suffix of a*4^k+i */
            v += pr[4 * i] + pr[4 * i + 1] + pr[4 * i + 2] + pr[4 * i + 3];
            v += pr[i] + pr[nk + i] + pr[2 * nk + i] + pr[3 * nk + i];
        } else {
            v = cx.lds[i];
        }
        if (v) atomicAdd(&(cx.flush ? cx.flush : cx.table)[fk_sigma(i)], v);
    }
}

/* transfer-function wave scans (k_count's one-pass tail, k_scan) */
__device__ __forceinline__ uint64_t shup64(uint64_t v, int d) {
    return ((uint64_t)shup((uint32_t)(v >> 32), d) << 32) | shup((uint32_t)v, d);
}
__device__ __forceinline__ XState xs_shup(const XState &x, int d) {
    return XState{shup64(x.R, d), shup64(x.code, d), shup(x.hdr, d), 0};
}
__device__ __forceinline__ TF tf_shup(const TF &a, int d) {
    TF b;
    b.c1 = xs_shup(a.c1, d);
    b.c0 = xs_shup(a.c0, d);
    b.nv = shup64(a.nv, d);
    b.cs = shup64(a.cs, d);
    b.f0_const = shup(a.f0_const, d);
    b.pad = 0;
    return b;
}
__device__ __forceinline__ TF tf_rdlane(const TF &x, int l) {
    TF o;
    o.c1 = XState{rdlane64(x.c1.R, l), rdlane64(x.c1.code, l), rdlane(x.c1.hdr, l), 0};
    o.c0 = XState{rdlane64(x.c0.R, l), rdlane64(x.c0.code, l), rdlane(x.c0.hdr, l), 0};
    o.nv = rdlane64(x.nv, l);
    o.cs = rdlane64(x.cs, l);
    o.f0_const = rdlane(x.f0_const, l);
    o.pad = 0;
    return o;
}
/* inclusive scan of one TF per lane across the wave */
__device__ __forceinline__ TF tf_wave_scan(TF a) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        TF b = tf_shup(a, d);
        if (lane >= (uint32_t)d) a = fk_compose(b, a);
    }
    return a;
}

/* Wave-wide reductions of 64-bit values through DPP moves (quad_perm
 * [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8, row_bcast:15, row_bcast:31):
 * lane 63 ends with the result, read back as a wave-uniform value.  A
 * butterfly of __shfl_xor is 12 dependent ds_bpermute round trips per 64-bit
 * value (k_tail reduced 11 of them in ~3.4 us).  Every lane must be active. */
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_mov64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}
template <class Op>
__device__ __forceinline__ uint64_t wred64(uint64_t v, Op op) {
    v = op(v, dpp_mov64<0xb1>(v));
    v = op(v, dpp_mov64<0x4e>(v));
    v = op(v, dpp_mov64<0x124>(v));
    v = op(v, dpp_mov64<0x128>(v));
    v = op(v, dpp_mov64<0x142>(v));
    v = op(v, dpp_mov64<0x143>(v));
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}
struct OpAdd64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; } };
struct OpMin64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a < b ? a : b; } };
struct OpOr64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a | b; } };
struct OpMaxS64 {
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return (int64_t)a > (int64_t)b ? a : b; }
};

__device__ __forceinline__ unsigned long long wsum64(unsigned long long v) {
    return (unsigned long long)wred64((uint64_t)v, OpAdd64{});
}

/* Copy the result block to pinned host memory, sequence number last (the
 * host spins on it instead of a copy plus a stream synchronisation).  The
 * whole block calls. */
__device__ void publish_res_wave(const DevRes *res, DevRes *host_res, uint32_t seq) {
    /* one wave (which wrote *res itself); one system fence */
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(res);
    uint32_t *dst = reinterpret_cast<uint32_t *>(host_res);
    for (uint32_t i = lane; i < offsetof(DevRes, seq) / 4; i += 64) dst[i] = src[i];
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(&host_res->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void keep(uint32_t v) { asm volatile("" ::"v"(v)); }
template <typename T>
__device__ __forceinline__ uint32_t xput(T *p, T v) {
    /* returning exchange: the caller waits for it by keeping the result */
    return (uint32_t)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T xget(const T *p) {
    return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* LDS layout of k_tail's last block */
#define TAIL_BLOCKS 16u
#define FK_DYN_TARGET 16384u   /* k_count: at most ~this many dynamic ranges per segment */
#define FK_FLUSH_BYTES (1u << 20)   /* k_count: a wave flushes its counters after this many bytes */
/* k_count's dynamic-range pool heads (one per CU's pair of blocks), 64 B apart */
#define FK_HEAD_STRIDE 16u
#define FK_HEADS_OFF 64u
#define FK_MAX_POOLS 1024u
#define FK_CTL_WORDS (FK_HEADS_OFF + FK_MAX_POOLS * FK_HEAD_STRIDE)
#define TAIL_THREADS 512u

/*
 * One-pass feeds (LDS modes, entering state of the segment known): k_count
 * plus k_tail do what k_resume, k_scan, k_redo and k_table_stats did in four
 * launches, in two, and without a segment-wide scan of range states.
 *
 * In k_count, after its flush, wave 0 of every block (lane l = range 8b+l)
 *  - composes its ranges' transfer functions (the block aggregate);
 *  - checks each range's guessed entering state against the exit state of
 *    the range before it, counted from that range's own guess.  If the
 *    previous guess counts like the exact state, so does the exit state it
 *    reaches (same header flag and last bases; the same run length, or both
 *    deep in a run), so a guess equivalent to it is equivalent to the exact
 *    state -- provided no run length in the segment reaches the reference's
 *    int32 wrap, which k_tail checks.  By induction from range 0 (whose
 *    guess is the exact entering state), every guess is then exact enough;
 *  - writes a BlockSum: aggregate, first guess, last exit, flags.
 * k_tail (16 blocks) folds the sub-tables into the table with its
 * statistics, then its last block checks the block boundaries the same way,
 * reduces the aggregates to the exit state, merges the accumulators and
 * publishes the result block.  A failed check, a range that ran out of
 * general tiles, or a segment long enough for the int32 wrap: the result
 * block says so and the host runs k_resume / k_scan / k_redo /
 * k_table_stats as before.
 */
struct BlockSum {
    uint64_t e_R, e_code;    /* exit state of its last range, counted from that range's guess */
    uint64_t g_code;         /* guessed entering state of its first range */
    uint64_t nvb;            /* bytes of its first range */
    uint64_t eof;            /* smallest 0xFF candidate (segment offset) of its ranges */
    uint64_t nv;             /* bases of its ranges (the exit R shift, when not absorbing) */
    uint32_t e_hdr, g_R, g_hdr;
    uint32_t flags;          /* ONE_RESUME: a range has no transfer function yet; ONE_SCAN: a
                                local check failed; BS_ABSORB: the exit does not depend on the
                                block's entering state (a run break, or it enters a header) */
};
static_assert(sizeof(BlockSum) == 64, "BlockSums are 64 bytes");
#define BS_ABSORB 8u

/* k_count, one-pass mode: wave 0 of the block summarises its ranges (after
 * the flush, when their RangeRecs are written). */
__device__ __forceinline__ void block_summary(const Ctx &cx, const OnePassCfg *opc, RangeRec *rr, uint64_t nranges) {
    const uint32_t lane = threadIdx.x & 63, b = blockIdx.x;
    const uint64_t r = (uint64_t)b * FK_WAVES_PER_BLOCK + lane;
    const bool mine = lane < FK_WAVES_PER_BLOCK && r < nranges;
    TF x = fk_identity();
    uint64_t g_code = 0, nvb = 0, eof = ~0ull;
    uint32_t g_R = 0, g_hdr = 0;
    bool res_here = false;
    if (mine) {
        const RangeRec &q = rr[r];
        res_here = q.resume != 0;
        if (!res_here) {
            x = q.tf;
            g_code = q.a_code; g_R = q.a_R; g_hdr = q.a_hdr;
            nvb = (q.c1 - q.c0) * FK_CHUNK_BYTES;
            if (q.eof != FK_NO_EOF64) eof = q.c0 * FK_CHUNK_BYTES + q.eof;
        }
    }
    const XState g{g_R, g_code, g_hdr, 0};
    /* the exit state each range reached from its own guess; range l's guess
       is checked against range l-1's */
    const XState e = fk_apply(x, g);
    const XState e_prev = xs_shup(e, 1);
    const bool bad = mine && lane > 0 && !fk_equiv(DState{g_code, g_R, g_hdr}, e_prev, cx.k, nvb);
    /* a range whose transfer function is constant (a run break, or entering
       inside a header) decides the exit state's run length */
    const bool absorb = __ballot(mine && !res_here && x.f0_const) != 0;
    uint64_t nv = mine ? x.nv : 0;
#pragma unroll
    for (int d = 4; d >= 1; d >>= 1) {
        const uint64_t o = ((uint64_t)__shfl_xor((uint32_t)(nv >> 32), d, 64) << 32) |
                           (uint32_t)__shfl_xor((uint32_t)nv, d, 64);
        nv += o;
    }
    const uint32_t flags = (__ballot(mine && res_here) ? (uint32_t)ONE_RESUME : 0u) |
                           (__ballot(bad) ? (uint32_t)ONE_SCAN : 0u) | (absorb ? BS_ABSORB : 0u);
    if (mine && !res_here) opc->rtrue[r] = g;   /* equivalent to the exact state when the feed completes here */
#pragma unroll
    for (int d = 4; d >= 1; d >>= 1) {
        const uint64_t o = ((uint64_t)__shfl_xor((uint32_t)(eof >> 32), d, 64) << 32) |
                           (uint32_t)__shfl_xor((uint32_t)eof, d, 64);
        eof = min(eof, o);
    }
    const uint32_t lastl = (uint32_t)min((uint64_t)FK_WAVES_PER_BLOCK, nranges - (uint64_t)b * FK_WAVES_PER_BLOCK) - 1;
    const uint64_t el_R = rdlane64(e.R, lastl), el_code = rdlane64(e.code, lastl);
    const uint32_t el_hdr = rdlane(e.hdr, lastl);
    const uint64_t f_code = rdlane64(g_code, 0), f_nvb = rdlane64(nvb, 0);
    const uint32_t f_R = rdlane(g_R, 0), f_hdr = rdlane(g_hdr, 0);
    if (lane == 0) {
        BlockSum *bs = reinterpret_cast<BlockSum *>(opc->bsum) + b;
        bs->e_R = el_R; bs->e_code = el_code; bs->e_hdr = el_hdr;
        bs->g_code = f_code; bs->g_R = f_R; bs->g_hdr = f_hdr;
        bs->nvb = f_nvb;
        bs->eof = eof;
        bs->nv = nv;
        bs->flags = flags;
    }
}

/*
 * k_count: main pass, fast path only.  Wave w owns the chunk range
 * [w*cpw, (w+1)*cpw); its entering state is guessed from the halo before it
 * (or is the known stream state *d_init for chunk 0).  The wave streams the
 * range's tiles with three tiles in flight and counts them with tile_fast;
 * nothing else is in the loop (no byte walk, no stores), so the loads stay
 * in flight across chunk boundaries.  The first tile the fast path cannot
 * take (header, run break, several newlines per half, the input's ragged
 * end) ends the wave's work: it appends a ResumeRec and k_resume continues
 * the range from there.  A range counted to its end gets its RangeRec here.
 */


/* A wave's next dynamic range (wave-uniform), from its block's pool: pool
 * blockIdx % npools, whose ranges are d = p, p + npools, ... (largest first).
 * The pools are sized for the two blocks one CU holds (blocks b and
 * b + npools under the dispatcher's round-robin placement -- for speed only:
 * any placement drains every pool, since each pool's blocks exist).  The
 * waves of a CU run at different speeds (oldest-first issue: a SIMD's four
 * waves finish a static range at 113 / 126 / 138 / 160 us at 1 GB), and the
 * pool evens that out with a claim that only 16 waves contend for.
 * Returns dg.ndyn when the pool is empty. */
__device__ __forceinline__ uint32_t claim_dyn(uint32_t *heads, const DynGeo &dg) {
    const uint32_t p = blockIdx.x % dg.npools;
    const uint32_t np = dg.ndyn > p ? (dg.ndyn - 1 - p) / dg.npools + 1 : 0;
    uint32_t j = np;
    if ((threadIdx.x & 63) == 0) j = atomicAdd(&heads[p * FK_HEAD_STRIDE], 1u);
    j = (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
    return j < np ? j * dg.npools + p : dg.ndyn;
}

/* interleaved tile loads: lane L takes bytes [16L, 16L+16) and [1024+16L, ...)
   of a 2 KiB tile, so each instruction reads one contiguous KiB; the tile
   base is clamped into the range (a scalar), so prefetches past its end
   re-read its last full tile */
#define FK_LOADI(dst, t_)                                                            \
    {                                                                                \
        const uint64_t tb_ = min(sp.rbase + (uint64_t)(t_) * FK_TILE_BYTES, last_tile); \
        const u32x4 *p_ = reinterpret_cast<const u32x4 *>(cx.buf + tb_) + lane;      \
        u32x4 v0_ = __builtin_nontemporal_load(p_);                                  \
        u32x4 v1_ = __builtin_nontemporal_load(p_ + 64);                             \
        dst[0] = v0_.x; dst[1] = v0_.y; dst[2] = v0_.z; dst[3] = v0_.w;               \
        dst[4] = v1_.x; dst[5] = v1_.y; dst[6] = v1_.z; dst[7] = v1_.w;               \
    }

/* A range's prologue loads: the halo before it (lanes 0..7, 32 contiguous
   bytes each, clamped to valid memory), then its first three tiles. */
__device__ __forceinline__ void range_prologue(const Ctx &cx, const Span &sp, uint64_t last_tile, bool has,
                                               uint32_t (&hw)[8], bool &hv, uint32_t (&A)[8], uint32_t (&B)[8],
                                               uint32_t (&C)[8]) {
    const int lane = threadIdx.x & 63;
    const int64_t ho = (int64_t)sp.rbase - (int64_t)FK_HALO_BYTES + (int64_t)lane * FK_LANE_BYTES;
    hv = has && lane < (int)(FK_HALO_BYTES / FK_LANE_BYTES) && ho >= cx.lo;
    {
        /* inputs shorter than a lane are staged in a large buffer, so
           [lo, lo+32) is always readable */
        const int64_t hc = max(min(ho, (int64_t)cx.len - (int64_t)FK_LANE_BYTES), cx.lo);
        const u32x4 *hp = reinterpret_cast<const u32x4 *>(cx.buf + hc);
        u32x4 h0 = __builtin_nontemporal_load(hp), h1 = __builtin_nontemporal_load(hp + 1);
        hw[0] = h0.x; hw[1] = h0.y; hw[2] = h0.z; hw[3] = h0.w;
        hw[4] = h1.x; hw[5] = h1.y; hw[6] = h1.z; hw[7] = h1.w;
    }
    if (sp.nfull) {
        /* issue order A, B, C as in the loop (the barriers keep the compiler
           from reordering them, which would merge two different pending-load
           orders at the loop header) */
        asm volatile("" ::: "memory");
        FK_LOADI(A, 0);
        asm volatile("" ::: "memory");
        FK_LOADI(B, 1);
        asm volatile("" ::: "memory");
        FK_LOADI(C, 2);
    }
}

/* Count range `rid` (chunks [c0, c1)) whose prologue loads are in flight,
   and write its RangeRec (or, if it ran out of general tiles, a ResumeRec).
   The wave's counters accumulate across its ranges (`cnt`, flushed by the
   caller); `unk_seen` = the wave's unknown bytes counted before this range. */
template <int HM>
__device__ __forceinline__ void count_wave_range(const Ctx &cx, const Span &sp, uint64_t last_tile, uint64_t rid,
                                                 uint64_t c0, uint64_t c1, uint32_t (&hw)[8], bool hv,
                                                 uint32_t (&A)[8], uint32_t (&B)[8], uint32_t (&C)[8],
                                                 const XState *d_init, int has_init, uint32_t op_flags,
                                                 ResumeRec *resume, RangeRec *rr, uint32_t general_tiles,
                                                 Counters &cnt, uint32_t &unk_seen) {
    const int lane = threadIdx.x & 63;
    DState st;
    if (c0 == 0 && has_init) {
        const XState in = (op_flags & OP_FRESH) ? XState{0, 0, 0, 0} : *d_init;
        st.hdr = in.hdr;
        st.R = (uint32_t)in.R;
        st.code = in.code;
    } else {
        st = halo_guess<HM>(cx, hw, hv);
    }
    /* the halo words are waited for on every path (the d_init one too):
       a load left pending into the loop makes its first tile wait for
       vmcnt(0), i.e. for all three tiles in flight */
    consume(hw);
    const DState first = st;
    Facts f{0, 0, 0, 0, 0, 0};
    cnt.eof = FK_NO_EOF;
    uint64_t t = 0;
    uint32_t general_left = general_tiles;
    bool primed = sp.nfull > 0;
    for (;;) {
        if (primed) {
            /* one exit per group of three tiles and unconditional loads:
               every path into the latch has the same loads in flight, so each
               tile waits only for its own data */
            bool live = st.hdr == 0;
            for (uint64_t g = t; live; g += 3) {
                live = t < sp.nfull && tile_fast<true, HM, true>(cx, A, st, f, cnt, 1u);
                t += live;
                consume(A);
                FK_LOADI(A, g + 3);
                live = live && t < sp.nfull && tile_fast<true, HM, true>(cx, B, st, f, cnt, 1u);
                t += live;
                consume(B);
                FK_LOADI(B, g + 4);
                live = live && t < sp.nfull && tile_fast<true, HM, true>(cx, C, st, f, cnt, 1u);
                t += live;
                consume(C);
                FK_LOADI(C, g + 5);
            }
        }
        if (t >= sp.ntiles || general_left == 0) break;
        /* a tile the fast path cannot take (stream start, header, run
           break, the ragged end): general path, then back to streaming;
           past the budget k_resume takes the rest of the range, with mixed
           tiles */
        general_left--;
        uint32_t v[8];
        const int64_t toff = (int64_t)(sp.rbase + t * FK_TILE_BYTES);
        const int nb = load_lane<FK_LANE_BYTES>(cx, toff + lane * (int64_t)FK_LANE_BYTES, v);
        tile_general<true, HM>(cx, v, nb, (uint32_t)(t * FK_TILE_BYTES), st, f, cnt, 1u);
        consume(v);
        t++;
        primed = t < sp.nfull;
        if (primed) {
            asm volatile("" ::: "memory");
            FK_LOADI(A, t);
            asm volatile("" ::: "memory");
            FK_LOADI(B, t + 1);
            asm volatile("" ::: "memory");
            FK_LOADI(C, t + 2);
        }
    }
    const uint32_t unk_all = wsum32(cnt.unknown);
    const uint32_t unk = unk_all - unk_seen;
    unk_seen = unk_all;
    const uint32_t eof = wmin32(cnt.eof);
    if (lane == 0) {
        if (t < sp.ntiles) {
            ResumeRec q;
            q.tile = t;
            q.code = st.code; q.R = st.R; q.hdr = st.hdr;
            q.a_code = first.code; q.a_R = first.R; q.a_hdr = first.hdr;
            q.range = (uint32_t)rid;
            q.unknown = unk;
            q.eof = eof;
            q.pad = 0;
            q.f = f;
            resume[rid] = q;
            RangeRec &r = rr[rid];
            r.c0 = c0; r.c1 = c1;
            r.resume = 1;
        } else {
            RangeRec r;
            r.tf = fk_tf_span(first, st, f);
            r.a_code = first.code; r.a_R = first.R; r.a_hdr = first.hdr;
            r.c0 = c0; r.c1 = c1;
            r.eof = eof == FK_NO_EOF ? FK_NO_EOF64 : (uint64_t)eof;
            r.unknown = unk;
            r.resume = 0;
            rr[rid] = r;
        }
    }
}

template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 2)
k_count(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
        uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr,
        uint64_t nchunks, const XState *d_init, int has_init, uint64_t cpw, ResumeRec *resume,
        uint32_t general_tiles, uint32_t *subs, const OnePassCfg *opc, uint32_t op_flags,
        uint64_t nstatic, DynGeo dg, uint32_t *heads) {
    extern __shared__ uint32_t lds_bins[];
    /* open the feed's result block (the kernels after this one in the
       stream accumulate into it) */
    if (blockIdx.x == 0) {
        if (!(op_flags & OP_ON)) {
            if (threadIdx.x < 10) res->tstat[threadIdx.x] = 0;
            if (threadIdx.x == 10) res->eof_cand = ~0ull;
            if (threadIdx.x == 11) res->redo_n = 0;
        }
        /* one pass: k_tail writes the whole result block, and does a
           pending reset (table = 0 + the sub-tables) */
    }
    const uint32_t nw = lds_words(HM, k);
    /* the 509-odd blocks flush their bins into FK_SUBTABLES copies of the
       table (fewer same-address atomics at the end of the kernel);
       k_table_stats folds them into the table */
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k,
           subs ? subs + (size_t)(blockIdx.x % FK_SUBTABLES) * ((size_t)1 << (2 * k)) : nullptr};
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    /* the wave's static range; the static ranges end where the dynamic ones
       begin */
    const uint64_t send = dg.ndyn ? dg.base : nchunks;
    uint64_t rid = wave;
    uint64_t c0 = wave * cpw, c1 = min(c0 + cpw, send);
    if (dg.ndyn) static_span(dg, wave, c0, c1);
    bool has = wave < nstatic && c0 < c1;
    RangeRec hdr_r;
    hdr_r.c0 = has ? c0 : 0;
    hdr_r.c1 = has ? c1 : 0;
    Span sp = range_span(hdr_r, len);
    uint64_t last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
    /* prologue, all loads first; LDS is zeroed and the halo state computed
       while they fly */
    uint32_t hw[8], A[8], B[8], C[8];
    bool hv;
    range_prologue(cx, sp, last_tile, has, hw, hv, A, B, C);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    /* the wave's counters, flushed once per FK_FLUSH_BYTES of its ranges
       (packed 16-bit fields per lane) and at the end: one set of
       accumulator atomics per wave, not per range */
    Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
    uint32_t unk_seen = 0;
    uint64_t since = 0;
    for (;;) {
        if (has) {
            count_wave_range<HM>(cx, sp, last_tile, rid, c0, c1, hw, hv, A, B, C, d_init, has_init, op_flags,
                                 resume, rr, general_tiles, cnt, unk_seen);
            since += sp.rend - sp.rbase;
            if (since >= FK_FLUSH_BYTES) {
                flush_counters(cx, cnt, 1u, HM != H_NONE);
                cnt.unknown = 0;
                unk_seen = 0;
                since = 0;
            }
        }
        if (dg.ndyn == 0) break;
        const uint32_t d = claim_dyn(heads, dg);
        if (d >= dg.ndyn) break;
        rid = nstatic + d;
        dyn_span(dg, d, c0, c1);
        hdr_r.c0 = c0;
        hdr_r.c1 = c1;
        sp = range_span(hdr_r, len);
        last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
        has = true;
        range_prologue(cx, sp, last_tile, has, hw, hv, A, B, C);
    }
    flush_counters(cx, cnt, 1u, HM != H_NONE);
    if (LDS_MODE(HM)) {
        lds_flush<HM>(cx);
        if ((op_flags & OP_ON) && threadIdx.x < 64) block_summary(cx, opc, rr, nstatic);
    }
}
#undef FK_LOADI
#undef FK_LOADT

/*
 * k_resume: finish the ranges k_count stopped in (one wave per range, as in
 * k_count), with the general path wherever the fast path does not apply, and
 * write their RangeRecs.  Blocks without such a range exit at once.
 */
template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 4)   /* 4 waves per SIMD (<= 128 VGPRs): two blocks per CU */
k_resume(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
         uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr, uint64_t nranges,
         const ResumeRec *resume, uint32_t *heads, int mixed) {
    extern __shared__ uint32_t lds_bins[];
    /* k_scan lists the ranges to redo after this kernel (a one-pass k_count
       that gave up may have listed some already) */
    if (blockIdx.x == 0 && threadIdx.x == 0) res->redo_n = 0;
    /* k_count is done: reset its dynamic-range pools for the next launch */
    if (blockIdx.x == 0)
        for (uint32_t q = threadIdx.x; q < FK_MAX_POOLS; q += blockDim.x) heads[q * FK_HEAD_STRIDE] = 0;
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    const bool mine = wave < nranges && rr[wave].resume;
    /* uniform per block; in the LDS modes through the first bin (before the
       bins are zeroed): __syncthreads_or keeps its reduction in static LDS,
       which would move the bins off address 0 (lds_add) */
    bool any;
    if (LDS_MODE(HM)) {
        if (threadIdx.x == 0) lds_bins[0] = 0;
        __syncthreads();
        if (mine) lds_bins[0] = 1;
        __syncthreads();
        any = lds_bins[0] != 0;
        __syncthreads();
    } else {
        any = __syncthreads_or(mine);
    }
    if (!any) return;
    const uint32_t nw = lds_words(HM, k);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k};
    if (mine) {
        const ResumeRec q = resume[wave];
        RangeRec r = rr[wave];
        const Span sp = range_span(r, len);
        DState st{q.code, q.R, q.hdr};
        const DState a{q.a_code, q.a_R, q.a_hdr};
        Facts f = q.f;
        Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
        count_range<HM>(cx, sp, q.tile, st, f, cnt, 1u, mixed);
        r.tf = fk_tf_span(a, st, f);
        r.a_code = a.code; r.a_R = a.R; r.a_hdr = a.hdr;
        range_obs(cx, cnt, 1u, sp, &r, true, HM != H_NONE);
        if ((threadIdx.x & 63) == 0) {
            /* plus what k_count observed before the resume point */
            r.unknown += q.unknown;
            if (q.eof != FK_NO_EOF) r.eof = min(r.eof, (uint64_t)q.eof);
            rr[wave] = r;
        }
    }
    if (LDS_MODE(HM)) lds_flush<HM>(cx);
}

/*
 * k_redo, mode 0: each listed range (its guessed entering state would count
 * differently from the exact one) is counted again with weight -1 from the
 * guess, cancelling k_count + k_resume exactly, and with weight +1 from the
 * exact state, which also replaces its observations.  mode 1: cancel every
 * range from its exact state (a 0xFF byte truncates the input and the
 * segment is recounted).
 */
template <int HM>
__global__ void __launch_bounds__(FK_BLOCK, 4)
k_redo(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
       uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr,
       const XState *rtrue, const uint32_t *list, uint64_t nranges, int mode, int mixed) {
    extern __shared__ uint32_t lds_bins[];
    const uint64_t n = mode != 0 ? nranges : (uint64_t)res->redo_n;
    if ((uint64_t)blockIdx.x * FK_WAVES_PER_BLOCK >= n) return;   /* uniform per block */
    const uint32_t nw = lds_words(HM, k);
    if (LDS_MODE(HM)) lds_zero(lds_bins, nw);
    Ctx cx{buf, len, lo, table, LDS_MODE(HM) ? lds_bins : nullptr, shortcnt, acc, res, maskk,
           1u << (2 * k + 2), k};
    const uint64_t wave = blockIdx.x * FK_WAVES_PER_BLOCK + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * FK_WAVES_PER_BLOCK;
    for (uint64_t i = wave; i < n; i += nwaves) {
        const uint64_t r = mode != 0 ? i : list[i];
        RangeRec q = rr[r];
        const Span sp = range_span(q, len);
        const XState t = rtrue[r];
        DState ts{t.code, (uint32_t)t.R, t.hdr};
        /* passes over the range (one inlined count_range: its register
           footprint decides this kernel's occupancy):
           mode 0: -1 from the guess, then +1 from the exact state -- except
                   when the whole range lies in the reference's negative
                   int32 zone (seqSize < 0 from its first base to its last,
                   no run break: a run longer than 2^31 bases, :977), where
                   the exact state counts nothing: one read instead of two;
           mode 1: -1 from the exact state;
           mode 2: +1 from the exact state (H_SPARSE: counters and
                   observations only; k_sp_emit emits the windows at finish). */
        const bool neg_zone = mode == 0 && !t.hdr && !q.tf.f0_const && (int32_t)(uint32_t)t.R < 0 &&
                              (uint64_t)(uint32_t)t.R + (sp.rend - sp.rbase) <= 0xFFFFFFFFull;
        const int npass = mode == 0 && !neg_zone ? 2 : 1;
#pragma unroll 1
        for (int pass = 0; pass < npass; pass++) {
            const bool cancel = mode == 1 || (mode == 0 && pass == 0);
            const uint32_t wt = cancel ? 0xFFFFFFFFu : 1u;
            DState st = (mode == 0 && pass == 0) ? DState{q.a_code, q.a_R, q.a_hdr} : ts;
            Facts f{0, 0, 0, 0, 0, 0};
            Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
            count_range<HM>(cx, sp, 0, st, f, cnt, wt, mixed);
            if (cancel) {
                flush_counters(cx, cnt, wt);
            } else {
                /* exact observations replace the guessed trajectory's */
                range_obs(cx, cnt, 1u, sp, &q, true);
                if ((threadIdx.x & 63) == 0) { rr[r].eof = q.eof; rr[r].unknown = q.unknown; }
            }
        }
    }
    if (LDS_MODE(HM)) lds_flush<HM>(cx);
}

/*
 * 17 <= k <= 20: the table is built at finish by key-range passes over the
 * input the engine retained (1 byte per input byte, plus every range's exact
 * entering state from the feed's k_scan), never by materialising a slot per
 * byte.  k_sp_emit walks every range from its exact state, one 2 KiB tile at
 * a time, with tile_general -- the same per-byte rules as every other count
 * (findKmer.cpp:962-1069) -- writing each byte's window index (reference
 * order, :719-724) or short walk (:1059-1062) into the wave's LDS slots, and
 * then, per mode:
 *   SP_HIST  every window's bucket (key >> shift) into an LDS histogram
 *            (flushed with one atomic per bucket and block), every short
 *            walk to a global list;
 *   SP_KEYS  the windows with lo <= key < hi to a compact global list (one
 *            atomic per tile and wave for the space, ballot-ordered writes),
 *            and the short walks too when one pass takes every window (the
 *            feed counted them; no SP_HIST launch then);
 *   SP_DENSE the windows with lo <= key < hi counted in a dense u64 table
 *            (one bucket too large for a sorted pass: few distinct keys).
 */
/* SP_KEYS: one key range [lo, hi) of a walk and its list */
#define SP_MAXP 4u                  /* key ranges (passes) one SP_KEYS walk emits (round 5) */
struct SpPass {
    uint64_t lo, hi;
    uint64_t *out;                  /* the keys, or */
    uint32_t *out32;                /* ... (a range of <= 2^32 keys) key - lo as 32 bits */
    uint64_t cap;                   /* slots of the list */
    unsigned long long *ctr;        /* [0] slots claimed (whole SP_CHUNKs), [1] windows written (the rest: pads) */
};
struct SpEmit {
    int mode;
    uint32_t shift;                 /* bucket of a key: key >> shift */
    uint64_t lo, hi;                /* SP_DENSE: the key range [lo, hi) */
    unsigned long long *bhist;      /* SP_HIST: window count per bucket */
    uint32_t nbuckets;
    uint64_t *shorts;               /* SP_HIST: the short walks */
    unsigned long long *nshort;
    uint64_t short_cap;
    uint32_t np;                    /* SP_KEYS: the walk's key ranges, ascending (unused: lo = ~0) */
    uint64_t gend;                  /* ... the last range's hi */
    SpPass ps[SP_MAXP];
    unsigned long long *dense;      /* SP_DENSE: count of key lo + i */
};
enum { SP_HIST = 1, SP_KEYS = 2, SP_DENSE = 3 };
#define SP_WAVES 4u
#define SP_BUCKET_BITS 12u
/* SP_KEYS output: each wave claims SP_CHUNK slots at a time from the pass's
   counter and fills them in order; the unfilled end of its last chunk holds
   pads (4^k - 1, the largest key -- 0xFFFFFFFF in a 32-bit pass -- so the
   sort puts them last, and their number is taken off the last run).  Round 4: one claim per
   tile and wave -- 5 M same-address atomics per 10 GB pass -- made each keys
   pass take 60 ms against 10 ms for the histogram pass of the same walk. */
#define SP_CHUNK 8192u
struct SpOut {
    uint64_t base;    /* the wave's current chunk (wave-uniform) */
    uint32_t fill;    /* slots of it used (SP_CHUNK: none claimed yet) */
    uint64_t real;    /* windows written by the wave */
};
/* One window per lane (v, or SP_EMPTY / a short walk: none) into its key
   range's list, every lane of the wave calling together.  The ranges are
   told apart by a wave multisplit (3 ballots: range bits 0 and 1, and
   "in a range"), each range's entries placed at its chunk's fill point in
   lane order; a range claims a new SP_CHUNK (one atomic) when this step's
   entries run past its chunk.  One walk thus emits every range's keys:
   round 4 walked the input once per range, computing every window's key
   twice each time. */
static_assert(SP_MAXP == 4u, "sp_range compares three range starts");
/* the range of key v (SP_MAXP: none).  The host groups consecutive passes
   only: between two ranges lie empty buckets, which hold no key */
__device__ __forceinline__ uint32_t sp_range(const SpEmit &em, uint64_t v) {
    if (v < em.ps[0].lo || v >= em.gend) return SP_MAXP;
    return (uint32_t)(v >= em.ps[1].lo) + (uint32_t)(v >= em.ps[2].lo) + (uint32_t)(v >= em.ps[3].lo);
}
__device__ __forceinline__ void sp_place(const SpEmit &em, SpOut (&so)[SP_MAXP], uint64_t v, uint32_t lane) {
    const uint32_t q = sp_range(em, v);
    const unsigned long long bv = __ballot(q < SP_MAXP);
    if (!bv) return;
    const unsigned long long b0 = __ballot((q & 1u) != 0u), b1 = __ballot((q & 2u) != 0u);
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t i = 0; i < SP_MAXP; i++) {
        if (i >= em.np) break;
        const unsigned long long mi = bv & ((i & 1u) ? b0 : ~b0) & ((i & 2u) ? b1 : ~b1);
        if (!mi) continue;
        const uint32_t cnt = (uint32_t)__popcll(mi);
        const uint32_t rem = SP_CHUNK - so[i].fill;
        uint64_t nb = 0;
        if (cnt > rem) {
            unsigned long long c = 0;
            if (lane == 0) c = atomicAdd(em.ps[i].ctr, (unsigned long long)SP_CHUNK);
            nb = rdlane64(c, 0);
        }
        if (q == i) {
            const uint64_t p = (uint64_t)__popcll(mi & lt);
            const uint64_t at = p < rem ? so[i].base + so[i].fill + p : nb + (p - rem);
#ifndef SPX_NOSTORE
            if (at < em.ps[i].cap) {
                if (em.ps[i].out32) em.ps[i].out32[at] = (uint32_t)(v - em.ps[i].lo);
                else em.ps[i].out[at] = v;
            }
#endif
        }
        if (cnt > rem) { so[i].base = nb; so[i].fill = cnt - rem; }
        else so[i].fill += cnt;
        so[i].real += cnt;
    }
}
/* the end of the wave's walk: pad each range's chunk (4^k - 1, or
   0xFFFFFFFF in a 32-bit list), count its windows */
__device__ __forceinline__ void sp_close(const SpEmit &em, const SpOut (&so)[SP_MAXP], uint64_t pad) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t q = 0; q < SP_MAXP; q++) {
        if (q >= em.np) break;
        const SpPass &ps = em.ps[q];
        if (so[q].fill < SP_CHUNK)
            for (uint32_t i = so[q].fill + lane; i < SP_CHUNK; i += 64u) {
                if (so[q].base + i >= ps.cap) continue;
                if (ps.out32) ps.out32[so[q].base + i] = 0xFFFFFFFFu;
                else ps.out[so[q].base + i] = pad;
            }
        if (lane == 0 && so[q].real) atomicAdd(ps.ctr + 1, (unsigned long long)so[q].real);
    }
}

/* The windows of a fast tile (contiguous layout, tile_fast's Emit) as
 * reference-order keys, handed to the pass's mode.  Half h of a lane holds D
 * = 16 digits (15 with a '\n', right-aligned in its word R); the 32 digits
 * before the half are the previous half's {C, S2} (half 1: this lane's half
 * 0; half 0: the previous lane's half 1, lane 0: the tile's entering code),
 * so the window ending at digit j of the half is
 *   ((prev << 2(j+1)) | (R >> 2(D-1-j))) & (4^k - 1)
 * -- up to 20 bases from two words, which the 16-base {C, S2} of the dense
 * path cannot give. */
__device__ __forceinline__ void sp_fast_emit(const SpEmit &em, const Emit &fe, uint64_t c0, uint64_t maskk,
                                             uint32_t *bh, uint32_t lane, SpOut (&so)[SP_MAXP], uint64_t *stg) {
    const uint64_t pv0 = ((uint64_t)from_prev_lane(fe.BC, (uint32_t)(c0 >> 32)) << 32) |
                         from_prev_lane(fe.B2, (uint32_t)c0);
    const uint64_t pv1 = ((uint64_t)fe.AC << 32) | fe.A2;
    const uint32_t R0 = fe.h0 ? fe.A2 & 0x3FFFFFFFu : fe.A2, R1 = fe.h1 ? fe.B2 & 0x3FFFFFFFu : fe.B2;
    const uint32_t D0 = fe.h0 ? 15u : 16u, D1 = fe.h1 ? 15u : 16u;
    /* window jj (half jj / 16, digit jj % 16), or SP_EMPTY past the half's digits */
    auto key = [&](uint32_t jj) -> uint64_t {
        const bool h = jj >= 16u;
        const uint32_t j = jj & 15u, D = h ? D1 : D0, R = h ? R1 : R0;
        const uint64_t pv = h ? pv1 : pv0;
        if (j >= D) return SP_EMPTY;
        return fk_sigma(((pv << (2u * (j + 1u))) | (uint64_t)(R >> (2u * (D - 1u - j)))) & maskk);
    };
    if (em.mode == SP_KEYS) {
        /* the tile's <= 2048 windows staged in the wave's slots, grouped by
           range (a wave scan of each lane's per-range counts, packed two
           16-bit fields a word), then copied out range by range, 64
           consecutive entries a store */
        uint64_t kv[32];
        uint32_t c01 = 0, c23 = 0;
#pragma unroll
        for (uint32_t jj = 0; jj < 32u; jj++) {
            kv[jj] = key(jj);
            const uint32_t q = sp_range(em, kv[jj]), inc = 1u << (16u * (q & 1u));
            c01 += q < 2u ? inc : 0u;
            c23 += (q - 2u) < 2u ? inc : 0u;
        }
        const uint32_t i01 = wscan_incl32(c01), i23 = wscan_incl32(c23);
        const uint32_t t01 = rdlane(i01, 63), t23 = rdlane(i23, 63);
        const uint32_t T[4] = {t01 & 0xFFFFu, t01 >> 16, t23 & 0xFFFFu, t23 >> 16};
        const uint32_t S[4] = {0u, T[0], T[0] + T[1], T[0] + T[1] + T[2]};
        const uint32_t e01 = i01 - c01, e23 = i23 - c23;
        uint32_t p0 = e01 & 0xFFFFu, p1 = S[1] + (e01 >> 16), p2 = S[2] + (e23 & 0xFFFFu), p3 = S[3] + (e23 >> 16);
#pragma unroll
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint32_t q = sp_range(em, kv[jj]);
            if (q < SP_MAXP) {
                const uint32_t at = q == 0u ? p0 : q == 1u ? p1 : q == 2u ? p2 : p3;
                stg[at] = kv[jj];
                p0 += q == 0u; p1 += q == 1u; p2 += q == 2u; p3 += q == 3u;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (uint32_t q = 0; q < SP_MAXP; q++) {
            if (q >= em.np) break;
            const uint32_t t = T[q];
            if (!t) continue;
            const SpPass &ps = em.ps[q];
            const uint32_t rem = SP_CHUNK - so[q].fill;
            uint64_t nb = 0;
            if (t > rem) {   /* (t <= 2048 < SP_CHUNK: one new chunk at most) */
                unsigned long long c = 0;
                if (lane == 0) c = atomicAdd(ps.ctr, (unsigned long long)SP_CHUNK);
                nb = rdlane64(c, 0);
            }
            for (uint32_t j = lane; j < t; j += 64u) {
                const uint64_t v = stg[S[q] + j];
                const uint64_t at = j < rem ? so[q].base + so[q].fill + j : nb + (j - rem);
#ifndef SPX_NOSTORE
                if (at < ps.cap) {
                    if (ps.out32) ps.out32[at] = (uint32_t)(v - ps.lo);
                    else ps.out[at] = v;
                }
#endif
            }
            if (t > rem) { so[q].base = nb; so[q].fill = t - rem; }
            else so[q].fill += t;
            so[q].real += t;
        }
        __builtin_amdgcn_wave_barrier();
    } else if (em.mode == SP_DENSE) {
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint64_t v = key(jj);
            if (v >= em.lo && v < em.hi) atomicAdd(&em.dense[v - em.lo], 1ull);
        }
    } else {
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32u; jj++) {
            const uint64_t v = key(jj);
            if (v != SP_EMPTY) atomicAdd(&bh[v >> em.shift], 1u);
        }
    }
}

__global__ void __launch_bounds__(SP_WAVES * 64u)
k_sp_emit(const uint8_t *buf, uint64_t len, int k, uint64_t maskk, const XState *rst, uint64_t nranges,
          uint64_t cpw, uint64_t nchunks, SpEmit em) {
    extern __shared__ uint64_t sp_lds[];   /* SP_WAVES x 2048 slots, then (SP_HIST) the buckets */
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t *slots = sp_lds + (size_t)wv * FK_TILE_BYTES;
    uint32_t *bh = reinterpret_cast<uint32_t *>(sp_lds + (size_t)SP_WAVES * FK_TILE_BYTES);
    if (em.mode == SP_HIST) {
        for (uint32_t i = threadIdx.x; i < em.nbuckets; i += blockDim.x) bh[i] = 0;
        __syncthreads();
    }
    Ctx cx{buf, len, 0, nullptr, nullptr, nullptr, nullptr, nullptr, maskk, 0, k, nullptr, slots};
    const uint64_t nw = (uint64_t)gridDim.x * SP_WAVES;
    SpOut so[SP_MAXP];          /* SP_KEYS: the wave's output chunk in each range's list */
#pragma unroll
    for (uint32_t q = 0; q < SP_MAXP; q++) so[q] = SpOut{0, SP_CHUNK, 0};
    for (uint64_t r = (uint64_t)blockIdx.x * SP_WAVES + wv; r < nranges; r += nw) {
        const uint64_t c0 = r * cpw, c1 = min(c0 + cpw, nchunks);
        const uint64_t rb = c0 * FK_CHUNK_BYTES, re = min(c1 * FK_CHUNK_BYTES, len);
        const XState x = rst[r];
        DState st{x.code, (uint32_t)x.R, x.hdr};
        /* the next full tile's words load while this one is counted */
        uint32_t wn[8];
        auto load_full = [&](uint64_t at) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(buf + at + (uint64_t)lane * FK_LANE_BYTES);
            const u32x4 a = __builtin_nontemporal_load(p), c = __builtin_nontemporal_load(p + 1);
            wn[0] = a.x; wn[1] = a.y; wn[2] = a.z; wn[3] = a.w;
            wn[4] = c.x; wn[5] = c.y; wn[6] = c.z; wn[7] = c.w;
        };
        if (rb + FK_TILE_BYTES <= re) load_full(rb);
        for (uint64_t tb = rb; tb < re; tb += FK_TILE_BYTES) {
            uint32_t w[8];
            int nb = (int)FK_LANE_BYTES;
            if (tb + FK_TILE_BYTES <= re) {
#pragma unroll
                for (int d = 0; d < 8; d++) w[d] = wn[d];
            } else {
                nb = load_lane<FK_LANE_BYTES>(cx, (int64_t)(tb + (uint64_t)lane * FK_LANE_BYTES), w);
            }
            if (tb + 2 * FK_TILE_BYTES <= re) load_full(tb + FK_TILE_BYTES);
            Facts f{0, 0, 0, 0, 0, 0};
            Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF, 0};
            /* a fast tile (bases and at most one '\n' per half, deep in a run,
               outside a header: no short walks, every base ends a window)
               computes its 40-bit windows in registers: no byte walk, no
               slots */
            {
                const uint64_t c0 = st.code;
                Emit fe{0, 0, 0, 0, false, false, false};
                if (tb + FK_TILE_BYTES <= re && st.hdr == 0 &&
                    tile_fast<true, H_EMIT, false>(cx, w, st, f, cnt, 1u, &fe)) {
                    if (fe.deep) sp_fast_emit(em, fe, c0, maskk, bh, lane, so, slots);
                    continue;
                }
            }
            /* a lane reads back only the slots of its own 32 bytes */
#pragma unroll 8
            for (uint32_t j = 0; j < FK_LANE_BYTES; j++) slots[j * 64u + lane] = SP_EMPTY;
            tile_general<true, H_SPARSE>(cx, w, nb, 0u, st, f, cnt, 1u);
            if (em.mode == SP_KEYS) {
                if (em.shorts) {   /* (a single pass: no SP_HIST) */
#pragma unroll 8
                    for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                        const uint64_t v = slots[j * 64u + lane];
                        if (v >= SP_SHORT && v != SP_EMPTY) {
                            const unsigned long long i = atomicAdd(em.nshort, 1ull);
                            if (i < em.short_cap) em.shorts[i] = v;
                        }
                    }
                }
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) sp_place(em, so, slots[j * 64u + lane], lane);
            } else if (em.mode == SP_DENSE) {
#pragma unroll 8
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v >= em.lo && v < em.hi) atomicAdd(&em.dense[v - em.lo], 1ull);
                }
            } else {
                for (uint32_t j = 0; j < FK_LANE_BYTES; j++) {
                    const uint64_t v = slots[j * 64u + lane];
                    if (v < SP_SHORT) {
                        atomicAdd(&bh[v >> em.shift], 1u);
                    } else if (v != SP_EMPTY) {
                        const unsigned long long i = atomicAdd(em.nshort, 1ull);
                        if (i < em.short_cap) em.shorts[i] = v;
                    }
                }
            }
        }
    }
    if (em.mode == SP_KEYS) sp_close(em, so, (1ull << (2 * k)) - 1);
    if (em.mode == SP_HIST) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < em.nbuckets; i += blockDim.x)
            if (bh[i]) atomicAdd(&em.bhist[i], (unsigned long long)bh[i]);
    }
}

/*
 * Partitioned counting for 8 <= k <= 12 (the 4^k table does not fit in LDS,
 * and global atomics top out near 27 G/s on this chip).  The state pass
 * (k_count / k_resume in H_NONE mode, then k_scan) gives every range its
 * exact entering state; then:
 *
 * k_part: one wave per range, three interleaved tiles in flight as in
 *   k_count.  Each round, every wave counts one tile: a fast tile hands its
 *   windows to the block's batch, any other tile is counted by the general
 *   path with global atomics.  The block counting-sorts the round's windows
 *   (up to 8 x 2048) by table slice (the top index bits) in LDS, writes the
 *   sorted batch contiguously to its code region (the low `sh` index bits,
 *   u16 each) and records each slice's run (start, count) in a slice-major
 *   index.
 * k_bucket_count: one block per slice (and group of rows) counts its runs in
 *   an LDS slice of 2^sh bins and adds the slice into the table.
 */
/* Waves per k_part block (template parameter W, 8 or 16; part_waves_of()).
   Larger blocks make k_part itself slower (more waves per barrier) but its
   batches larger, so k_bucket_count reads longer runs: one block per CU for
   the 512-slice tables (k = 11, 12: 16 waves, 132 KiB of LDS), two 8-wave
   blocks per CU for k <= 10 (<= 128 slices, long runs already).  Round 2:
   16-wave blocks took the k=11 FASTA step from 1.12 to 1.08 ms and k=12
   from 1.85 to 1.73 ms against 8-wave ones; 4-wave blocks made k=11 5 %
   slower and k=12 30 % slower. */
#define PART_BLOCK_W(W) ((W) * 64u)
/* tiles per wave per batch: 2 single-window tiles or 4 pair tiles fill the
   same LDS batch (a pair tile hands over half as many entries) */
#define PART_TILES(PAIRS) ((PAIRS) ? 4u : 2u)
#define PART_MAX_BATCH_W(W) (2u * (W) * FK_TILE_BYTES)   /* entries per batch */
/* k = 15, 16 (C32): 32-bit codes under 2048 coarse slices, one tile per wave
   per batch (W x 2048 entries, the same 128 KiB of LDS and row slot) */
#define PART_TILES3(PAIRS, C32) ((C32) ? 1u : PART_TILES(PAIRS))
#define PART_ROW_BYTES(W) (4u * (W) * FK_TILE_BYTES)   /* one batch's row slot in d_codes */
static_assert(PART_MAX_BATCH_W(16u) <= 65536u, "run index words hold 16-bit starts and counts - 1");
/* slices of a batch: k = 11 pairs 2^24 / 2^15 (the single k-mers fold into
   them, flagged), k = 12 2^24 / 2^15, k = 13 2^26 / 2^15; k <= 10 at most 128 */
#define PART_SM(W) ((W) >= 16u ? 2048u : 128u)   /* k = 13: 2^26 / 2^15 slices */
/* k = 14: 2^28 / 2^16 = 4096 slices of 16-bit codes (k_bucket_count counts a
   slice as two halves of 2^15 bins, PartGeo::split).  Their run cursors are
   packed two per word (16 KiB of counts + 8 KiB of cursors + the 128 KiB
   batch fit the 160 KiB of LDS): a cursor only reaches 2^16 at the batch's
   very end, where the carry lands on a slice with an empty run. */
#define PART_BIG 4096u
/* Measured and not kept (round 3): pairs mode keeping 8 batches' run words
   per slice in LDS and writing them as one 32-B piece (each scattered 4-B word
   costs a ~40-B write-back, 1.6 GB per 10 GB step): k_part 5.54 -> 5.67 ms,
   k=11 10 GB step 8.08 -> 8.21 ms (the flush and the extra LDS cost more). */
#define PART_SINGLE 0x8000u   /* a stored code with this bit: a single k-mer (pairs mode) */

/* A run index word: (start << 16) | (count - 1) for a run of count >= 1
   codes (a batch holds up to 2^16 of them, all possibly in one slice), and
   PART_NO_RUN for an empty one (start + count <= 2^16 never encodes to it) */
#define PART_NO_RUN 0xFFFFFFFFu
__device__ __forceinline__ uint32_t run_word(uint32_t start, uint32_t count) {
    return count ? (start << 16) | (count - 1u) : PART_NO_RUN;
}
__device__ __forceinline__ uint32_t run_count(uint32_t e) { return e == PART_NO_RUN ? 0u : (e & 0xFFFFu) + 1u; }

struct PartGeo {
    uint16_t *codes;       /* per row (batch): `batch` entries at row * batch */
    uint32_t batch;        /* entries per row slot: PART_MAX_BATCH_W of k_part's block size (+ 8 per slice
                              of pad pieces for PART_PAD) */
    uint32_t *idx;         /* [row][slice]: run_word(start, count) (row-major: one contiguous row of
                              words per batch; round 3: the slice-major layout's scattered 4-B writes
                              cost ~1.6 GB of write-backs per 10 GB step) */
    uint32_t rounds;       /* rows per block */
    uint32_t rows;         /* rows in all: grid * rounds */
    uint32_t nslices;      /* a multiple of 8 */
    uint32_t sh;           /* slice index = code >> sh; stored code = code & (2^sh - 1) */
    uint32_t npair;        /* pairs mode: slices [0, npair) hold (k+1)-mer pairs */
    /* pairs mode, a single k-mer x (a '\n' half's slot 1): slice sbase + ((x << slsh) >> sh), stored
       ((x << slsh) & lowm) | sflag.  2^15-bin slices: x filed under the pair code x << 2 with
       PART_SINGLE set (sbase 0, slsh 2); 2^16-bin slices (W16, k_bucket16): the singles' own slices
       [npair, npair + 4^k / 2^16) (sbase npair, slsh 0, sflag 0) */
    uint32_t sbase, slsh, sflag;
    uint32_t w16;          /* 2^16-bin slices counted in packed 16-bit LDS bins (k_bucket16): k = 11..14 */
    uint32_t nbk;          /* W16: slices k_bucket16 counts ([0, nbk): the index row may be wider) */
    uint32_t *pairs;       /* pairs mode: 4^(k+1) pair bins (k_bucket_count -> k_pair_fold) */
    uint32_t *singles;     /* pairs mode: 4^k single k-mer bins */
    uint32_t nomix;        /* no_mixed: tiles the fast path cannot take go to tile_general */
    uint32_t general;      /* general tiles (other than bases-only ones) k_part takes per range
                              before k_part<RES> takes the rest */
    uint32_t stride;       /* index row stride: rows of both regions (k_part, then k_part<RES>) */
    uint32_t *flag;        /* [0] != 0: some range went to k_part<RES>, region 2 holds rows */
    uint32_t split;        /* k = 15, 16: a coarse slice holds 2^split parts of 2^15 bins */
    uint32_t *glist;       /* k = 15, 16 over a fresh table: the general tiles' windows (hist_add), or nullptr */
    unsigned long long *fz;/* ... and the table statistics k_count_parts takes of it: FZ_SLOTS x 10 partials */
    uint32_t kk;           /* k */
};
#define FZ_SLOTS 1024u   /* (spread: 128 same-address atomics each at k = 16, not 2048) */

/* Every entry a fast tile's Emit hands to the partition, as f(slice, low).
 * Single windows: the 16 windows ending in each half (15 when slot 0 is not
 * a window).  PAIRS (as half_windows<H_PAIRS> does in LDS): the (k+1)-mers
 * ending at the odd slots 1, 3, .., 15 of each half, each standing for the
 * two k-mers ending at slots (2j, 2j+1); without a real slot 0 the first one
 * is the single k-mer x at slot 1, filed under the pair code x << 2 (its
 * slice) with PART_SINGLE set in the stored low bits. */
/* where a pairs-mode single k-mer goes (PartGeo::sbase, slsh, sflag) */
struct SingleEnc {
    uint32_t sbase, slsh, sflag;
};
template <bool PAIRS, bool MIX, typename F>
__device__ __forceinline__ void part_entries(const Emit &em, uint32_t mk, uint32_t m1, uint32_t sh, uint32_t lowm,
                                             const SingleEnc &se, F &&f) {
    if (MIX && em.masked) {
        /* a mixed tile: only the slots in the mask end windows; a pair where
           both of its slots do, else the single k-mer of the one that does */
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
            const uint32_t cm = (em.cm >> (16 * h)) & 0xFFFFu;
            if (PAIRS) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t two = (cm >> (14 - 2 * j)) & 3u;
                    if (two == 3u) {
                        const uint32_t v = (j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2) & m1;
                        f(v >> sh, v & lowm);
                    } else if (two) {
                        const uint32_t s = 2u * (uint32_t)j + (two == 1u ? 1u : 0u);
                        const uint32_t v = ((s < 15u ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - s)) : S2) & mk) << se.slsh;
                        f(se.sbase + (v >> sh), (v & lowm) | se.sflag);
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    if ((cm >> (15 - i)) & 1u) {
                        const uint32_t v = (i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2) & mk;
                        f(v >> sh, v & lowm);
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
        if (PAIRS) {
            const uint32_t v0 = __builtin_amdgcn_alignbit(C, S2, 28u);
            const uint32_t c0 = skip0 ? (v0 & mk) << se.slsh : (v0 & m1);
            f((skip0 ? se.sbase : 0u) + (c0 >> sh), (c0 & lowm) | (skip0 ? se.sflag : 0u));
#pragma unroll
            for (int j = 1; j < 8; j++) {
                const uint32_t v = (j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2) & m1;
                f(v >> sh, v & lowm);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t v = (i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2) & mk;
                if (i > 0 || !skip0) f(v >> sh, v & lowm);
            }
        }
    }
}

/*
 * Padded runs (PART_PAD: the k_part instances of at most 512 slices, i.e.
 * 8 <= k <= 11 in pairs mode).  A batch's runs start on 16-B pieces in LDS
 * and in its row (the up to 7 codes after a run's last one are whatever the
 * LDS held: k_bucket_count<BK_PAD> masks them by the run's count), so that
 * k_bucket_count reads a run as whole aligned pieces with one mask for its
 * last piece instead of a bounds check per code.  The row slot grows by 16 B
 * per slice (<= 1 pad piece per run).  Measured and dropped (round 4):
 * appending each slice's runs to its own 4 KiB chunks (tools/chunk_probe.hip:
 * whole-chunk reads at 6.1 TB/s): k_bucket_count 2.46 -> 1.93 ms at k = 11
 * over 10 G bases, but k_part 4.40 -> 6.75 ms -- the runs' scattered,
 * line-unaligned stores cost 1.6 ms and the per-slice chunk bookkeeping 0.8.
 */
#define PART_PAD_MAX_SM 512u
#define PART_ROW_PAD(SM) (16u * (SM))   /* bytes of pad pieces a row slot adds */

/* The block-wide batch of one round: windows of the waves whose tile was
 * fast (have), counting-sorted by slice.  Every thread of the block calls
 * this the same number of times (it contains barriers).
 *
 * Round 3 measured (tools/exp_part_probe.py: s_memtime per phase, k=11,
 * 10 GB FASTA, cycles per wave and batch of 16 waves x 4 tiles): tiles 11.4 K,
 * histogram atomics 2.7 K + barrier 5.7 K, wave 0's scan 5.2 K (the others
 * wait 3.2 K), placement 14.3 K + barrier 3.0 K, write-out 2.4 K: the LDS
 * atomics bind.  Spreading each slice's counters over 8 lane buckets (2-way
 * instead of ~3.5-way bank conflicts) with a scan split over all waves did
 * not make the atomic phases cheaper (the atomic instructions' issue, not
 * the banks, sets their cost) and its extra barrier made the batch slower
 * (47.0 K vs 45.7 K cycles), so the scan stays on wave 0. */
template <bool PAIRS, bool MIX, uint32_t W, uint32_t SM, typename CT>
__device__ __forceinline__ bool part_batch(const Ctx &cx, const PartGeo &pg, const Emit *es, const bool *haves,
                                           bool more, uint32_t row, uint32_t *hist,
                                           uint32_t *cur, uint32_t *total, CT *ent, uint32_t *scr) {
    constexpr bool C32 = sizeof(CT) == 4;
    constexpr bool PAD = !C32 && SM <= PART_PAD_MAX_SM;   /* runs padded to 16-B pieces (PART_PAD) */
    constexpr int NT = PART_TILES3(PAIRS, C32);
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint32_t mk = (uint32_t)cx.maskk, sh = pg.sh, lowm = (1u << sh) - 1u;
    const uint32_t m1 = (mk << 2) | 3u;
    const SingleEnc se{pg.sbase, pg.slsh, pg.sflag};
    /* 1: slice histogram */
#pragma unroll
    for (int i = 0; i < NT; i++)
        if (haves[i]) part_entries<PAIRS, MIX>(es[i], mk, m1, sh, lowm, se, [&](uint32_t b, uint32_t) { atomicAdd(&hist[b], 1u); });
    /* (the barrier also tells whether any wave has tiles left) */
    const bool any_more = __syncthreads_or(more);
    /* 2: exclusive scan of the slice counts, index row: wave 0 alone for up
       to 512 slices; k = 13's 2048 slices split over all waves (each sums
       its contiguous share, one more barrier, then scans it from the sum of
       the shares before it) */
    if (!PAIRS && W >= 16u && pg.nslices > 512u) {
        const uint32_t per_w = pg.nslices / W, ppl = per_w / 64u;   /* multiples of 64 */
        const uint32_t wv = t >> 6, b0 = wv * per_w + lane * ppl;
        uint32_t mine = 0;
        for (uint32_t j = 0; j < ppl; j++) mine += hist[b0 + j];
        const uint32_t wt = wsum32(mine);
        if (lane == 0) scr[wv] = wt;
        __syncthreads();
        const uint32_t off = wsum32(lane < wv ? scr[lane] : 0u);
        const uint32_t inc = wscan_incl32(mine);
        uint32_t run = off + inc - mine;
        uint32_t lo16 = 0;
        for (uint32_t j = 0; j < ppl; j++) {
            const uint32_t b = b0 + j, c = hist[b];
            if (SM > 2048u) {   /* packed cursors (b0 and ppl are even) */
                if ((b & 1u) == 0) lo16 = run & 0xFFFFu;
                else cur[b >> 1] = lo16 | (run << 16);
            } else {
                cur[b] = run;
            }
            pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
            hist[b] = 0;
            run += c;
        }
        if (wv == W - 1u && lane == 63) *total = run;
    } else if (PAD && t < 64) {
        /* runs start on 16-B pieces; cursors and run index in entries / pieces */
        const uint32_t per = (pg.nslices + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) sum += (hist[b] + 7u) >> 3;
        }
        const uint32_t inc = wscan_incl32(sum);
        uint32_t run = inc - sum;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) {
                const uint32_t c = hist[b];
                cur[b] = 8u * run;
                pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
                hist[b] = 0;
                run += (c + 7u) >> 3;
            }
        }
        if (lane == 63) *total = 8u * inc;
    } else if (t < 64) {
        const uint32_t per = (pg.nslices + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) sum += hist[b];
        }
        const uint32_t inc = wscan_incl32(sum);
        uint32_t run = inc - sum;
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t b = lane * per + j;
            if (b < pg.nslices) {
                const uint32_t c = hist[b];
                cur[b] = run;
                pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
                hist[b] = 0;
                run += c;
            }
        }
        if (lane == 63) *total = inc;
    }
    __syncthreads();
    /* 3: place each entry at its slot.  The codes are recomputed from the
       Emit words (laundered, so the compiler cannot keep phase 1's codes
       live across the barriers: that costs more VGPRs than it saves VALU) */
    auto place = [&](uint32_t b, uint32_t low) {
        uint32_t p;
        if (SM > 2048u) {
            const uint32_t h = (b & 1u) * 16u;
            p = (atomicAdd(&cur[b >> 1], 1u << h) >> h) & 0xFFFFu;
        } else {
            p = atomicAdd(&cur[b], 1u);
        }
        ent[p] = (CT)low;
    };
#pragma unroll
    for (int i = 0; i < NT; i++) {
        Emit f = es[i];
        asm volatile("" : "+v"(f.AC), "+v"(f.A2), "+v"(f.BC), "+v"(f.B2));
        if (haves[i]) part_entries<PAIRS, MIX>(f, mk, m1, sh, lowm, se, place);
    }
    __syncthreads();
    /* 4: the sorted batch into its row's fixed slot (pg.batch entries: a
       run's position needs no per-row base), as 16-B pieces; the up to 7
       codes past the batch's end are padding no run covers */
    const uint32_t n8 = (*total * (uint32_t)sizeof(CT) + 15u) >> 4;
    uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(pg.codes) + (size_t)row * pg.batch * sizeof(CT));
    const uint4 *src = reinterpret_cast<const uint4 *>(ent);
    for (uint32_t i = t; i < n8; i += PART_BLOCK_W(W)) dst[i] = src[i];
    return any_more;
}

/*
 * Pipelined batches (PIPE: the main pass of tables of at most 512 slices,
 * whose scan wave 0 runs alone, and of k = 13's 2048, whose scan all waves
 * share: part_scan_sum).  part_batch runs its phases one after
 * another on every wave -- tiles (VALU), histogram atomics, barrier, scan,
 * barrier, placement atomics (LDS), barrier, write-out -- so the CU's VALU
 * idles while its LDS works and the other way round.  Here batch j's
 * entries are placed while the waves count batch j+1's tiles: each round a
 * wave counts one tile, adds its entries to the histogram of batch j+1 and
 * places the entries of the tile it stashed in the same slot during batch j
 * (every tile of a batch sits in its own stash slot, so one stash serves
 * both batches).  At the end of a batch's tiles, one barrier (batch j's
 * placement and batch j+1's histogram done), then wave 0 scans batch j+1's
 * histogram (cursors, run index, total) while the other waves write batch j
 * out, then a second barrier: two barriers per batch instead of three, and
 * the tiles' VALU work overlaps the placement atomics across the waves.
 */
/* A fast tile's entries (as part_entries without mixed tiles) placed at
   their slices' cursors, eight at a time: the eight returning cursor
   atomics are issued back to back and only then the eight code stores.
   (One entry at a time -- atomic, wait, store -- the compiler cannot move
   the next atomic above the previous store into the same LDS, so every
   entry waited out a whole LDS round trip.) */
/* Entry j of group g of half h of a fast tile (as part_entries without
   mixed tiles): its slice (one bit-field extract: the code's bits [sh, sh +
   wsl), wsl = the slice bits) and its stored low bits (PAIRS: a single k-mer
   x at slot 1 of a '\n' half is the pair code x << 2 with PART_SINGLE) */
template <bool PAIRS>
__device__ __forceinline__ void part_entry(uint32_t C, uint32_t S2, bool skip0, int g, int j, uint32_t sh,
                                           uint32_t wsl, uint32_t lowm, const SingleEnc &se, uint32_t &b,
                                           uint32_t *low) {
    if (PAIRS) {
        const uint32_t v = j < 7 ? __builtin_amdgcn_alignbit(C, S2, 28u - 4u * (uint32_t)j) : S2;
        if (j == 0 && skip0) {   /* x = v & mk, as (x << slsh): its slice is v's bits [sh - slsh, 2k) */
            b = se.sbase + __builtin_amdgcn_ubfe(v, sh - se.slsh, wsl - 2u + se.slsh);
            if (low) *low = ((v << se.slsh) & lowm) | se.sflag;
        } else {
            b = __builtin_amdgcn_ubfe(v, sh, wsl);
            if (low) *low = v & lowm;
        }
    } else {
        const int i = 8 * g + j;
        const uint32_t v = i < 15 ? __builtin_amdgcn_alignbit(C, S2, 2u * (15u - (uint32_t)i)) : S2;
        b = __builtin_amdgcn_ubfe(v, sh, wsl);
        if (low) *low = v & lowm;
    }
}

/* A fast tile's entries into the batch's slice histogram */
template <bool PAIRS>
__device__ __forceinline__ void part_hist8(const Emit &em, uint32_t sh, uint32_t wsl, const SingleEnc &se,
                                           uint32_t *hist) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
#pragma unroll
        for (int g = 0; g < (PAIRS ? 1 : 2); g++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;   /* slot 0 is not a window */
                uint32_t b;
                part_entry<PAIRS>(C, S2, skip0, g, j, sh, wsl, 0u, se, b, nullptr);
                atomicAdd(&hist[b], 1u);
            }
    }
}

/* A fast tile's entries placed at their slices' cursors (byte offsets into
   the batch), eight at a time: the eight returning cursor atomics are issued
   back to back and only then the eight code stores.  (One entry at a time --
   atomic, wait, store -- the compiler cannot move the next atomic above the
   previous store into the same LDS, so every entry waited out a whole LDS
   round trip.) */
typedef __attribute__((address_space(3))) uint16_t lds_u16;
template <bool PAIRS>
__device__ __forceinline__ void part_place8(const Emit &em, uint32_t sh, uint32_t wsl, uint32_t lowm,
                                            const SingleEnc &se, uint32_t *cur) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t C = h ? em.BC : em.AC, S2 = h ? em.B2 : em.A2;
        const bool skip0 = h ? em.h1 : em.h0;
#pragma unroll
        for (int g = 0; g < (PAIRS ? 1 : 2); g++) {
            uint32_t b[8], low[8], p[8];
#pragma unroll
            for (int j = 0; j < 8; j++) part_entry<PAIRS>(C, S2, skip0, g, j, sh, wsl, lowm, se, b[j], &low[j]);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;   /* slot 0 is not a window */
                p[j] = atomicAdd(&cur[b[j]], 2u);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (!PAIRS && g == 0 && j == 0 && skip0) continue;
                *(lds_u16 *)(uintptr_t)p[j] = (uint16_t)low[j];
            }
        }
    }
}

/* PAD: runs start on 16-B pieces (PART_PAD), the run index and the total in
   pieces / entries (8 per piece) */
template <bool PAD>
__device__ __forceinline__ void part_scan_w0(const PartGeo &pg, uint32_t row, uint32_t *hist, uint32_t *cur,
                                             uint32_t *tot, uint32_t ent_lds) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t per = (pg.nslices + 63) / 64;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; j++) {
        const uint32_t b = lane * per + j;
        if (b < pg.nslices) sum += PAD ? (hist[b] + 7u) >> 3 : hist[b];
    }
    const uint32_t inc = wscan_incl32(sum);
    uint32_t run = inc - sum;
    for (uint32_t j = 0; j < per; j++) {
        const uint32_t b = lane * per + j;
        if (b < pg.nslices) {
            const uint32_t c = hist[b];
            cur[b] = ent_lds + (PAD ? 16u : 2u) * run;   /* LDS byte addresses (part_place8) */
            pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
            hist[b] = 0;
            run += PAD ? (c + 7u) >> 3 : c;
        }
    }
    if (lane == 63) *tot = PAD ? 8u * inc : inc;
}

/* The same for 2048 slices (k = 13), over all W waves: each wave sums its
   contiguous share (part 1, beside the write-out), one more barrier, then
   scans its share from the sum of the shares before it (part 2) */
__device__ __forceinline__ uint32_t part_scan_sum(const PartGeo &pg, const uint32_t *hist, uint32_t nw, uint32_t *scr) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t per_w = pg.nslices / nw, ppl = per_w / 64u, b0 = wv * per_w + lane * ppl;
    uint32_t mine = 0;
    for (uint32_t j = 0; j < ppl; j++) mine += hist[b0 + j];
    const uint32_t wt = wsum32(mine);
    if (lane == 0) scr[wv] = wt;
    return mine;
}
__device__ __forceinline__ void part_scan_place(const PartGeo &pg, uint32_t row, uint32_t *hist, uint32_t *cur,
                                                uint32_t nw, const uint32_t *scr, uint32_t mine, uint32_t *tot,
                                                uint32_t ent_lds) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t per_w = pg.nslices / nw, ppl = per_w / 64u, b0 = wv * per_w + lane * ppl;
    const uint32_t off = wsum32(lane < wv ? scr[lane] : 0u);
    uint32_t run = off + wscan_incl32(mine) - mine;
    for (uint32_t j = 0; j < ppl; j++) {
        const uint32_t b = b0 + j, c = hist[b];
        cur[b] = ent_lds + 2u * run;
        pg.idx[(size_t)row * pg.nslices + b] = run_word(run, c);
        hist[b] = 0;
        run += c;
    }
    if (wv == nw - 1u && lane == 63) *tot = run;
}

template <uint32_t W>
__device__ __forceinline__ void part_writeout(const PartGeo &pg, uint32_t row, uint32_t total, const uint16_t *ent,
                                              uint32_t t0, uint32_t nt) {
    const uint32_t n8 = (total * (uint32_t)sizeof(uint16_t) + 15u) >> 4;
    uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(pg.codes) + (size_t)row * pg.batch * 2u);
    const uint4 *src = reinterpret_cast<const uint4 *>(ent);
    for (uint32_t i = t0; i < n8; i += nt) dst[i] = src[i];
}

/* RES = false: the main pass.  With mixed tiles on, a range that needs more
 * than pg.general general tiles stops there (ResumeRec) and
 * RES = true -- the same blocks and ranges, their rows in region 2 -- counts
 * the rest of it, each tile fast, mixed (the masked entries of tile_mixed)
 * or general.  Two kernels: tile_mixed's registers stay out of the main
 * pass.  k_part<RES> returns at once unless some range stopped. */
template <bool PAIRS, bool RES, uint32_t W, uint32_t SM = PART_SM(W), bool C32 = false, bool PIPE = false,
          uint32_t KC = 0>
__global__ void __launch_bounds__(PART_BLOCK_W(W), 4) /* 4 waves per SIMD (<= 128 VGPRs): 16 waves per CU */
k_part(const uint8_t *buf, uint64_t len, int64_t lo, int k, uint64_t maskk, uint32_t *table,
       uint32_t *shortcnt, unsigned long long *acc, DevRes *res, RangeRec *rr, uint64_t nchunks, uint64_t cpw,
       const XState *d_init, int has_init, PartGeo pg, ResumeRec *resume, const XState *exact) {
    static_assert(!PIPE || (!RES && !C32 && SM <= 2048u), "PIPE: the main pass, 16-bit codes, unpacked cursors");
    /* one LDS object: the histogram and the cursors first (below 64 KiB, so
       their base folds into the LDS instructions' offset field), then the
       batch */
    using CT = typename std::conditional<C32, uint32_t, uint16_t>::type;
    /* runs padded to 16-B pieces (PART_PAD) for the tables of at most 512 slices */
    constexpr bool PAD = !C32 && SM <= PART_PAD_MAX_SM;
    constexpr uint32_t CURW = SM > 2048u ? SM / 2u : SM;
    constexpr uint32_t ENT_OFF = (SM + CURW + 4u + W + 15u) & ~15u;   /* words, 64-B aligned */
    constexpr uint32_t ENT_BYTES = PART_ROW_BYTES(W) + (PAD ? PART_ROW_PAD(SM) : 0u);
    __shared__ __attribute__((aligned(64))) uint32_t lds_part[ENT_OFF + ENT_BYTES / 4u];
    uint32_t *const hist = lds_part, *const cur = lds_part + SM, &total = lds_part[SM + CURW],
                    *const tot = lds_part + SM + CURW + 1u, *const scr = lds_part + SM + CURW + 4u;
    CT *const ent = reinterpret_cast<CT *>(lds_part + ENT_OFF);
    if (RES && *(volatile uint32_t *)pg.flag == 0) return;   /* uniform: no range stopped */
    /* open the feed's result block (the kernels after this one accumulate
       into it) */
    if (!RES && blockIdx.x == 0) {
        if (threadIdx.x < 10) res->tstat[threadIdx.x] = 0;
        if (threadIdx.x == 10) res->eof_cand = ~0ull;
        if (threadIdx.x == 11) res->redo_n = 0;
    }
    for (uint32_t i = threadIdx.x; i < pg.nslices; i += PART_BLOCK_W(W)) hist[i] = 0;
    Ctx cx{buf, len, lo, table, nullptr, shortcnt, acc, res, maskk, 0, k, pg.glist};
    const int lane = threadIdx.x & 63;
    const uint64_t wave = blockIdx.x * W + wave_in_block();
    const uint64_t c0 = wave * cpw, c1 = min(c0 + cpw, nchunks);
    const bool has = c0 < c1 && (!RES || rr[wave].resume);
    RangeRec hdr_r;
    hdr_r.c0 = has ? c0 : 0;
    hdr_r.c1 = has ? c1 : 0;
    const Span sp = range_span(hdr_r, len);
    const uint64_t last_tile = sp.nfull ? sp.rend - FK_TILE_BYTES : 0;
    const bool ld = sp.nfull > 0;
    const ResumeRec *qr = resume + wave;   /* k_part<RES>: where k_part stopped (fields read where used) */
    uint64_t t = RES && has ? qr->tile : 0;
#define FK_LOADP(dst, t_)                                                            \
    if (ld) {                                                                        \
        const uint64_t tb_ = min(sp.rbase + (uint64_t)(t_) * FK_TILE_BYTES, last_tile); \
        const u32x4 *p_ = reinterpret_cast<const u32x4 *>(cx.buf + tb_) + lane;      \
        u32x4 v0_ = __builtin_nontemporal_load(p_);                                  \
        u32x4 v1_ = __builtin_nontemporal_load(p_ + 64);                             \
        dst[0] = v0_.x; dst[1] = v0_.y; dst[2] = v0_.z; dst[3] = v0_.w;               \
        dst[4] = v1_.x; dst[5] = v1_.y; dst[6] = v1_.z; dst[7] = v1_.w;               \
    }
    /* halo (lanes 0..7) and the first three tiles in flight before anything
       waits (as in k_count) */
    uint32_t hw[8] = {};
    const int64_t ho = (int64_t)sp.rbase - (int64_t)FK_HALO_BYTES + (int64_t)lane * FK_LANE_BYTES;
    const bool hv = has && lane < (int)(FK_HALO_BYTES / FK_LANE_BYTES) && ho >= lo;
    if (!RES) {
        const int64_t hc = max(min(ho, (int64_t)len - (int64_t)FK_LANE_BYTES), lo);
        const u32x4 *hp = reinterpret_cast<const u32x4 *>(buf + hc);
        u32x4 h0 = __builtin_nontemporal_load(hp), h1 = __builtin_nontemporal_load(hp + 1);
        hw[0] = h0.x; hw[1] = h0.y; hw[2] = h0.z; hw[3] = h0.w;
        hw[4] = h1.x; hw[5] = h1.y; hw[6] = h1.z; hw[7] = h1.w;
    }
    uint32_t A[8] = {}, B[8] = {}, C[8] = {};
    asm volatile("" ::: "memory");
    FK_LOADP(A, t);
    asm volatile("" ::: "memory");
    FK_LOADP(B, t + 1);
    asm volatile("" ::: "memory");
    FK_LOADP(C, t + 2);
    /* entering state: the known stream state for chunk 0, else a guess from
       the halo (k_scan checks it, k_redo recounts a range it got wrong);
       k_part<RES>: where k_part stopped */
    DState st{0, 0, 0}, first{0, 0, 0};
    Facts f{0, 0, 0, 0, 0, 0};
    if (RES) {
        if (has) {
            st = DState{qr->code, qr->R, qr->hdr};
            first = DState{qr->a_code, qr->a_R, qr->a_hdr};
            f = qr->f;
        }
    } else if (has) {
        if (exact) {
            /* a recount from the exact range states (resolve_and_fetch) */
            const XState x = exact[wave];
            st = DState{x.code, (uint32_t)x.R, x.hdr};
        } else if (c0 == 0 && has_init) {
            st = DState{d_init->code, (uint32_t)d_init->R, d_init->hdr};
        } else {
            st = halo_guess<H_EMIT>(cx, hw, hv);
        }
        first = st;
    }
    consume(hw);   /* waited on every path (see k_count) */
    Counters cnt{0, 0, 0, 0, 0, FK_NO_EOF};
    bool done = !has || t >= sp.ntiles, stopped = false;
    uint32_t general_left = pg.nomix ? 0xFFFFFFFFu : pg.general;
    uint32_t round = 0;
    const uint32_t row0 = (RES ? pg.rows : 0u) + blockIdx.x * pg.rounds;
    constexpr uint32_t NT = PART_TILES3(PAIRS, C32);
    Emit stash[NT];
    bool have_stash[NT];
#pragma unroll
    for (uint32_t i = 0; i < NT; i++) {
        stash[i] = Emit{0, 0, 0, 0, false, false, false};
        have_stash[i] = false;
    }
    /* PIPE: the codes of an entry and its placement (unpacked cursors) */
    /* KC: k as a compile-time constant (the headline k = 11), so that the
       slice and low-bit extracts fold into single bit-field ops */
    constexpr uint32_t KBC = KC ? (PAIRS ? KC + 1u : KC) : 0u;
    /* (KC: 2^15-bin slices, singles filed under their pair code, PART_SINGLE) */
    const uint32_t shv = KC ? (2u * KBC - 6u < 15u ? 2u * KBC - 6u : 15u) : pg.sh;
    const uint32_t lowm = (1u << shv) - 1u;
    const SingleEnc se = KC ? SingleEnc{0u, 2u, PART_SINGLE} : SingleEnc{pg.sbase, pg.slsh, pg.sflag};
    /* the batch's LDS byte address (the PIPE cursors hold LDS addresses) */
    const uint32_t ent_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) CT *)ent;
    const uint32_t wsl = 2u * (KC ? KBC : (uint32_t)(PAIRS ? k + 1 : k)) - shv;   /* slice bits of a code */
    __syncthreads();
    /* PIPE: the stashed entry of this round's slot (batch j) to its place; odd
       waves place before their tile, even waves after it, so that the waves
       of a SIMD tend to be in different phases (VALU / LDS) */
    const bool early = PIPE && ((wave_in_block() >> 1) & 1u);
#define FK_PLACE_OLD()                                                               \
    {                                                                                \
        const uint32_t ph_ = round % NT;                                             \
        Emit old_ = stash[0];                                                        \
        bool hold_ = have_stash[0];                                                  \
        _Pragma("unroll") for (uint32_t i_ = 1; i_ < NT; i_++) if (ph_ == i_) {      \
            old_ = stash[i_];                                                        \
            hold_ = have_stash[i_];                                                  \
        }                                                                            \
        if (hold_) part_place8<PAIRS>(old_, shv, wsl, lowm, se, cur); \
    }
/* (a macro, not a lambda: the same body as an always-inline lambda called
   three times gave the compiler a different register allocation -- 107
   VGPRs and 256 SGPR spills instead of 123 and 207 -- and k_part at k = 11
   over 10 G bases 4.41 -> 4.85 ms, round 4) */
#define FK_ROUND(X)                                                                  \
    {                                                                                \
        Emit em{0, 0, 0, 0, false, false, false};                                    \
        if (PIPE && early) FK_PLACE_OLD();                                           \
        bool have = false, plain_ = false, kind_ = false;                            \
        if (!done) {                                                                 \
            if (t < sp.nfull && st.hdr == 0 && tile_fast<true, H_EMIT, true>(cx, X, st, f, cnt, 1u, &em, &kind_)) { \
                have = em.deep;                                                      \
                t++;                                                                 \
            } else if (RES && t < sp.nfull &&                                        \
                       tile_mixed<H_EMIT>(cx, X, (uint32_t)(t * FK_TILE_BYTES), st, f, cnt, 1u, plain_, &em)) { \
                have = true;                                                         \
                t++;                                                                 \
            } else if (!RES && !kind_ && general_left == 0) {                        \
                /* k_part<RES> counts this tile and the rest of the range (the  \
                   tile is skipped here: t advances on every path) */           \
                stopped = true;                                                      \
                t++;                                                                 \
            } else {                                                                 \
                general_left -= kind_ ? 0u : 1u;                                     \
                uint32_t v_[8];                                                      \
                const int64_t toff_ = (int64_t)(sp.rbase + t * FK_TILE_BYTES);       \
                const int nb_ = load_lane<FK_LANE_BYTES>(cx, toff_ + lane * (int64_t)FK_LANE_BYTES, v_); \
                tile_general<true, H_EMIT>(cx, v_, nb_, (uint32_t)(t * FK_TILE_BYTES), st, f, cnt, 1u); \
                consume(v_);                                                         \
                t++;                                                                 \
            }                                                                        \
            done = stopped || t >= sp.ntiles;                                        \
        }                                                                            \
        consume(X);                                                                  \
        FK_LOADP(X, t + 2);                                                          \
        if (PIPE) {   /* batch j+1's histogram, batch j's placement (see part_scan_w0) */ \
            const uint32_t ph_ = round % NT;                                         \
            if (have) part_hist8<PAIRS>(em, shv, wsl, se, hist);                   \
            if (!early) FK_PLACE_OLD();                                              \
            _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++) if (ph_ == i_) {  \
                stash[i_] = em;                                                      \
                have_stash[i_] = have;                                               \
            }                                                                        \
            if (ph_ == NT - 1) {                                                     \
                const uint32_t j_ = round / NT;                                      \
                const bool more_ = __syncthreads_or(!done);                          \
                if (KC == 0 && pg.nslices > 512u) {   /* 2048 slices: the scan over all waves */ \
                    const uint32_t mine_ = part_scan_sum(pg, hist, W, scr);          \
                    if (j_ > 0) part_writeout<W>(pg, row0 + j_ - 1, tot[(j_ - 1) & 1u], (const uint16_t *)ent, \
                                                 threadIdx.x, PART_BLOCK_W(W));       \
                    __syncthreads();                                                 \
                    part_scan_place(pg, row0 + j_, hist, cur, W, scr, mine_, &tot[j_ & 1u], ent_lds); \
                } else if (threadIdx.x < 64) {                                       \
                    part_scan_w0<PAD>(pg, row0 + j_, hist, cur, &tot[j_ & 1u], ent_lds); \
                } else if (j_ > 0) {                                                 \
                    part_writeout<W>(pg, row0 + j_ - 1, tot[(j_ - 1) & 1u], (const uint16_t *)ent, \
                                     threadIdx.x - 64u, PART_BLOCK_W(W) - 64u);       \
                }                                                                    \
                __syncthreads();                                                     \
                if (!more_ || j_ + 1 >= pg.rounds) {                                 \
                    /* the last batch: placed, then written out */                  \
                    _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++)           \
                        if (have_stash[i_]) part_place8<PAIRS>(stash[i_], shv, wsl, lowm, se, cur); \
                    __syncthreads();                                                 \
                    part_writeout<W>(pg, row0 + j_, tot[j_ & 1u], (const uint16_t *)ent, threadIdx.x, PART_BLOCK_W(W)); \
                    round++;                                                         \
                    break;                                                           \
                }                                                                    \
            }                                                                        \
        } else {   /* static stash slots (no dynamic register indexing) */          \
            const uint32_t ph_ = round % NT;                                         \
            _Pragma("unroll") for (uint32_t i_ = 0; i_ < NT; i_++) if (ph_ == i_) {  \
                stash[i_] = em;                                                      \
                have_stash[i_] = have;                                               \
            }                                                                        \
            if (ph_ == NT - 1) {                                                     \
                const bool more_ = part_batch<PAIRS, RES, W, SM, CT>(cx, pg, stash, have_stash, !done, \
                                                          row0 + round / NT, hist, cur, &total, ent, scr); \
                if (!more_ || round / NT + 1 >= pg.rounds) { round++; break; }       \
            }                                                                        \
        }                                                                            \
        round++;                                                                     \
    }
    for (;;) {
        FK_ROUND(A);
        FK_ROUND(B);
        FK_ROUND(C);
    }
#undef FK_ROUND
#undef FK_PLACE_OLD
#undef FK_LOADP
    /* rows the block did not reach are empty */
    for (uint32_t r = (round + NT - 1) / NT; r < pg.rounds; r++) {
        const uint32_t row = row0 + r;
        for (uint32_t b = threadIdx.x; b < pg.nslices; b += PART_BLOCK_W(W)) pg.idx[(size_t)row * pg.nslices + b] = PART_NO_RUN;
    }
    if (!has) {
        flush_counters(cx, cnt, 1u);
        return;
    }
    if (!RES && stopped) {
        /* k_part<RES> counts the rest of the range */
        flush_counters(cx, cnt, 1u);
        const uint32_t unk = wsum32(cnt.unknown), eof = wmin32(cnt.eof);
        if (lane == 0) {
            ResumeRec w;
            w.tile = t - 1;   /* the tile it stopped at */
            w.code = st.code; w.R = st.R; w.hdr = st.hdr;
            w.a_code = first.code; w.a_R = first.R; w.a_hdr = first.hdr;
            w.range = (uint32_t)wave;
            w.unknown = unk;
            w.eof = eof;
            w.pad = 0;
            w.f = f;
            resume[wave] = w;
            RangeRec &r = rr[wave];
            r.c0 = c0; r.c1 = c1;
            r.resume = 1;
            atomicOr(pg.flag, 1u);
        }
        return;
    }
    /* the range's record: transfer function, guess, observations */
    RangeRec r;
    r.tf = fk_tf_span(first, st, f);
    r.a_code = first.code; r.a_R = first.R; r.a_hdr = first.hdr;
    r.c0 = c0; r.c1 = c1;
    r.resume = 0;
    range_obs(cx, cnt, 1u, sp, &r, true);
    if (lane == 0) {
        if (RES) {   /* plus what k_part observed before it stopped */
            r.unknown += qr->unknown;
            if (qr->eof != FK_NO_EOF) r.eof = min(r.eof, (uint64_t)qr->eof);
        }
        rr[wave] = r;
    }
}

/* k_bucket_count's first loads per quad: BUCKET_ROWS rows at once, each
   with BUCKET_U 16-B pieces per lane (64 B per quad each).  2 x 4 (256 B
   of a ~200-B run, k=11 with 16-wave k_part blocks) beat 4 x 2 by ~1 %
   (k=11 step 1.082 -> 1.070 ms); 3 x 3, 3 x 4 and 1 x 8 fell in between.
   2 x 5 (95 VGPRs, still 4 waves per SIMD): a k=11 pair run is ~120 codes,
   so 4 pieces per lane (128 codes from the aligned-down start) sent a third
   of the runs -- and so nearly every wave of 16 runs -- through the
   long-run loop for a few codes; k_bucket_count 334 -> 325 us, k=11 step
   1.081 -> 1.074 ms, k=12 1.684 -> 1.669 ms, k=8 unchanged (2 x 6: the
   same within noise; 3 x 5 at 128 VGPRs 331 -> 351 us, 1 x 10 -> 341 us). */
#ifndef BUCKET_U
#define BUCKET_U 5
#endif
#ifndef BUCKET_ROWS
#define BUCKET_ROWS 2
#endif
/* MODE (a template parameter, so that the hot loop of the common k carries
   no test of it: a runtime flag there cost ~0.9 ms of a k=11 10 GB step):
   BK_PLAIN 16-bit codes, one block per slice (and row group).  (Round 4's
            BK_SPLIT, k = 14 counted as two blocks per 2^16-bin slice that
            each read all of its codes, is k_bucket16's now.) */
/* BK_PAD: BK_PLAIN over padded runs (PART_PAD: a run starts on a 16-B
            piece, its index word holds that piece; only its last piece
            needs a mask) */
enum { BK_PLAIN = 0, BK_PAD = 2 };
template <int MODE>
__global__ void __launch_bounds__(1024)
k_bucket_count(PartGeo pg, uint32_t groups, uint32_t *table) {
    extern __shared__ uint32_t slice[];
    constexpr bool PADDED = MODE == BK_PAD;
    constexpr uint32_t CPP = 8u;   /* 16-bit codes per 16-B piece */
    constexpr uint32_t PSH = 3u;
    const uint32_t nb = 1u << pg.sh;
    /* pairs mode: the slice's 2^sh pair bins, then the 2^(sh-2) bins of the
       single k-mers filed under it (PART_SINGLE codes) */
    const uint32_t ns = pg.pairs ? nb >> 2 : 0u;
    /* consecutive slices on one XCD (blocks b, b + 8, .. share an XCD): the
       128-B line two neighbouring runs of a row share is fetched once into
       that XCD's L2 (k=11: 1 GB step 1.085 -> 1.065 ms, 10 GB 8.10 -> 8.04) */
    const uint32_t b = groups == 1 && (pg.nslices & 7u) == 0 ? (blockIdx.x & 7u) * (pg.nslices >> 3) + (blockIdx.x >> 3)
                                                             : blockIdx.x % pg.nslices;
    const uint32_t g = blockIdx.x / pg.nslices;
    for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) slice[i] = 0;
    __syncthreads();
    const uint32_t *ix = pg.idx + b;
    /* region 2 (k_part<RES>) holds rows only if some range went there */
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    /* four lanes share a run and read it as contiguous 64-byte pieces (one
       request per quad instead of one per lane).  (k = 14, round 4: a lane
       per run with 4 rows and 3 pieces each in flight fetched 19.4 GB per
       G-base instead of 5.3 -- 33 MB of lines in flight per XCD evict the
       lines the slice's other half and its neighbours would read from L2 --
       and took 3.46 ms instead of 2.86.)  A quad takes BUCKET_ROWS
       rows at once: their first 64 * BUCKET_U bytes of codes and the next
       rows' index words are all in flight together (a run is ~50-250 codes, so one
       dependent chain per run would leave the CU waiting on latency; rows
       sit at fixed offsets, so a run's position needs no further load) */
    constexpr uint32_t QL = 4u;   /* lanes per run */
    const uint32_t sub = threadIdx.x & (QL - 1u);
    const uint32_t quads = blockDim.x / QL, step = groups * quads;
    auto add16 = [&](const uint4 &v, uint64_t q, uint64_t s0, uint64_t s1) {
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const uint32_t nv = PADDED ? (uint32_t)min<uint64_t>(CPP, s1 - q * CPP) : 0u;   /* codes of the run in q */
#pragma unroll
        for (int h = 0; h < (int)CPP; h++) {
            const uint64_t at = q * CPP + h;
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            if (PADDED) {   /* the run starts on this lane's first piece: only its end bounds it */
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if ((uint32_t)h < nv) atomicAdd(&slice[a], 1u);
            } else {
                const uint32_t a = c & PART_SINGLE ? nb + ((c & ~PART_SINGLE) >> 2) : c;
                if (at >= s0 && at < s1) atomicAdd(&slice[a], 1u);
            }
        }
    };
    uint32_t en[BUCKET_ROWS];   /* the next iteration's index words, loaded with this one's codes */
    const uint32_t r00 = g * quads + threadIdx.x / QL;
#pragma unroll
    for (int j = 0; j < BUCKET_ROWS; j++) en[j] = r00 + j * step < nrows ? ix[(size_t)(r00 + j * step) * pg.nslices] : PART_NO_RUN;
    for (uint32_t r = r00; r < nrows; r += BUCKET_ROWS * step) {
        uint32_t e[BUCKET_ROWS];
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) e[j] = en[j];
        const uint32_t rn = r + BUCKET_ROWS * step;
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) en[j] = rn + j * step < nrows ? ix[(size_t)(rn + j * step) * pg.nslices] : PART_NO_RUN;
        uint64_t s0[BUCKET_ROWS], s1[BUCKET_ROWS];
        uint4 v[BUCKET_ROWS][BUCKET_U];
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) {
            s0[j] = (uint64_t)(r + j * step) * pg.batch + (e[j] == PART_NO_RUN ? 0u : (e[j] >> 16) * (PADDED ? CPP : 1u));
            s1[j] = s0[j] + run_count(e[j]);
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (int u = 0; u < BUCKET_U; u++) v[j][u] = q0 + QL * u < q1 ? g4[q0 + QL * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BUCKET_ROWS; j++) {
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (int u = 0; u < BUCKET_U; u++)
                if (q0 + QL * u < q1) add16(v[j][u], q0 + QL * u, s0[j], s1[j]);
            /* the rest of a long run */
            for (uint64_t q = q0 + QL * BUCKET_U; q < q1; q += 4 * QL) {
                uint4 w[4];
#pragma unroll
                for (int u = 0; u < 4; u++) w[u] = q + QL * u < q1 ? g4[q + QL * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (q + QL * u < q1) add16(w[u], q + QL * u, s0[j], s1[j]);
            }
        }
    }
    __syncthreads();
    if (pg.pairs) {
        /* pairs mode: the slice's bins, in kernel index order, into the pair
           and single bins (k_pair_fold reduces them into the table) */
        uint32_t *dp = pg.pairs + ((size_t)b << pg.sh), *ds = pg.singles + ((size_t)b << (pg.sh - 2));
        for (uint32_t i = threadIdx.x; i < nb + ns; i += blockDim.x) {
            const uint32_t v = slice[i];
            uint32_t *dst = i < nb ? dp + i : ds + (i - nb);
            if (groups == 1) *dst = v;   /* this block owns the slice: every bin written */
            else if (v) atomicAdd(dst, v);
        }
        return;
    }
    const uint64_t base = (uint64_t)b << pg.sh;
    if (groups != 1) {
        for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
            const uint32_t v = slice[i];
            if (v) atomicAdd(&table[fk_sigma(base | i)], v);
        }
        return;
    }
    /* this block owns the slice: eight loads in flight per lane before the
       adds and stores (one load-add-store chain at a time is latency-bound) */
    constexpr uint32_t U = 8u;
    for (uint32_t i0 = threadIdx.x; i0 < nb; i0 += U * blockDim.x) {
        uint32_t v[U], o[U];
#pragma unroll
        for (uint32_t j = 0; j < U; j++) {
            const uint32_t i = i0 + j * blockDim.x;
            v[j] = i < nb ? slice[i] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < U; j++) o[j] = v[j] ? table[fk_sigma(base | (i0 + j * blockDim.x))] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < U; j++)
            if (v[j]) table[fk_sigma(base | (i0 + j * blockDim.x))] = o[j] + v[j];
    }
}

/*
 * W16 (k = 11..14): slices of 2^16 bins counted in 16-bit LDS bins, two per
 * word (128 KiB for the whole slice).  Against 2^15-bin slices in 32-bit bins
 * that halves the slices, so every run a block reads is twice as long (k =
 * 11: ~240 codes, 480 B) and the reads of a run's partial first and last
 * lines are half as many; k = 14 counts a slice in one block instead of two
 * blocks that each read all of its codes.  A code c adds 1 << 16 (c & 1) to
 * word c >> 1 (non-returning, as the 32-bit bins).  A 16-bit bin that wraps
 * carries into its neighbour (low half) or out of the word (high half): both
 * make the sum of the halves fall short of the codes counted, and nothing
 * else does, so the block checks that sum against its exact count and, only
 * if it fell short (a bin past 65535 codes in one slice: poly-A stretches),
 * counts the slice again as two halves of 2^15 32-bit bins.  (Round 2 tried
 * 16-bit bins with returning atomics to catch wraps as they happen: 20 %
 * slower; the sum check costs one add per word.)
 *
 * Blocks: pairs mode puts the single k-mers (a '\n' half's slot 1) in their
 * own slices [npair, nbk), lightly loaded: they come first, so the pair
 * slices -- consecutive ones on one XCD, as k_bucket_count -- start at most
 * one light block late.
 */
/* Every code of slice b's runs (index column ix) as f(code): QL lanes per
   run reading 16-B pieces (QL x 16 B contiguous per request), ROWS rows per
   lane group in flight with U pieces each, the next rows' index words loaded
   with this iteration's codes (k_bucket_count's shape) */
template <uint32_t QL, uint32_t ROWS, uint32_t U, bool PADDED, typename F>
__device__ __forceinline__ void walk_runs(const PartGeo &pg, const uint32_t *ix, uint32_t nrows, F &&f) {
    constexpr uint32_t CPP = 8u, PSH = 3u;
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    const uint32_t sub = threadIdx.x & (QL - 1u), groups = blockDim.x / QL;
    auto add16 = [&](const uint4 &v, uint64_t q, uint64_t s0, uint64_t s1) {
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const uint32_t nv = PADDED ? (uint32_t)min<uint64_t>(CPP, s1 - q * CPP) : 0u;
#pragma unroll
        for (int h = 0; h < (int)CPP; h++) {
            const uint64_t at = q * CPP + h;
            const uint32_t c = (w4[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
            if (PADDED ? (uint32_t)h < nv : (at >= s0 && at < s1)) f(c);
        }
    };
    uint32_t en[ROWS];
    const uint32_t r00 = threadIdx.x / QL;
#pragma unroll
    for (uint32_t j = 0; j < ROWS; j++)
        en[j] = r00 + j * groups < nrows ? ix[(size_t)(r00 + j * groups) * pg.nslices] : PART_NO_RUN;
    for (uint32_t r = r00; r < nrows; r += ROWS * groups) {
        uint32_t e[ROWS];
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) e[j] = en[j];
        const uint32_t rn = r + ROWS * groups;
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++)
            en[j] = rn + j * groups < nrows ? ix[(size_t)(rn + j * groups) * pg.nslices] : PART_NO_RUN;
        uint64_t s0[ROWS], s1[ROWS];
        uint4 v[ROWS][U];
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) {
            s0[j] = (uint64_t)(r + j * groups) * pg.batch + (e[j] == PART_NO_RUN ? 0u : (e[j] >> 16) * (PADDED ? CPP : 1u));
            s1[j] = s0[j] + run_count(e[j]);
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (uint32_t u = 0; u < U; u++) v[j][u] = q0 + QL * u < q1 ? g4[q0 + QL * u] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t j = 0; j < ROWS; j++) {
            const uint64_t q0 = (s0[j] >> PSH) + sub, q1 = (s1[j] + CPP - 1) >> PSH;
#pragma unroll
            for (uint32_t u = 0; u < U; u++)
                if (q0 + QL * u < q1) add16(v[j][u], q0 + QL * u, s0[j], s1[j]);
            for (uint64_t q = q0 + QL * U; q < q1; q += 4 * QL) {
                uint4 w[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) w[u] = q + QL * u < q1 ? g4[q + QL * u] : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    if (q + QL * u < q1) add16(w[u], q + QL * u, s0[j], s1[j]);
            }
        }
    }
}

/* the heavy (pair or plain) slices' walk shape: 4 lanes per run, 2 rows x 3
   pieces in flight (QL 1, 2, 8 and U 4, 5 measured slower); the singles' slices hold a few codes
   per run, so a lane per run and 4 rows in flight (their walk is a chain of
   index and code loads: with the heavy shape the 64 single-slice blocks of
   k = 11 took ~0.3 ms, which the pair slices' last blocks waited out) */
/* W16 for k = 12, 13, 14 (1 G-base FASTA steps, round 5: k = 12 1.33 ->
   1.22 ms, k = 13 2.12 -> 1.84 ms, k = 14 4.4 -> 3.35 ms).  Not k = 11:
   its runs are long already (~120 codes), and with half the slices k_part's
   histogram and cursor atomics collide more often within a wave (k_part
   4.40 -> 4.51 ms per 10 G bases) while k_bucket16's 256 heavy blocks run
   as one round (k_bucket 2.31 -> 2.6-3.0 ms over the shapes tried): step
   6.79 -> 7.2-7.7 ms.  k = 14 has no other path (2^16-bin slices). */
#define W16_KS_DEFAULT ((1u << 12) | (1u << 13) | (1u << 14))
#ifndef B16_QL
#define B16_QL 4
#endif
#ifndef B16_ROWS
#define B16_ROWS 2
#endif
#ifndef B16_U
#define B16_U 3   /* (5: k = 12 1.250, 13 1.837, 14 3.348 ms per G-base; 3: 1.228, 1.820, 3.294) */
#endif
#ifndef B16L_QL
#define B16L_QL 1
#endif
#ifndef B16L_ROWS
#define B16L_ROWS 4
#endif
#ifndef B16L_U
#define B16L_U 1
#endif
template <bool PADDED>
__global__ void __launch_bounds__(1024)
k_bucket16(PartGeo pg, uint32_t *table) {
    extern __shared__ uint32_t bins[];
    constexpr uint32_t NW = 1u << 15;   /* words: 2^16 16-bit bins, or 2^15 32-bit ones */
    const uint32_t nsing = pg.pairs ? pg.nbk - pg.npair : 0u;
    uint32_t b;
    if (blockIdx.x < nsing) {
        b = pg.npair + blockIdx.x;
    } else {
        const uint32_t j = blockIdx.x - nsing, nh = pg.nbk - nsing;   /* (nh a multiple of 8) */
        b = (j & 7u) * (nh >> 3) + (j >> 3);
    }
    const bool light = b >= pg.npair && nsing;
    const uint32_t *ix = pg.idx + b;
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    auto walk = [&](auto &&f) {
        if (light) walk_runs<B16L_QL, B16L_ROWS, B16L_U, PADDED>(pg, ix, nrows, f);
        else walk_runs<B16_QL, B16_ROWS, B16_U, PADDED>(pg, ix, nrows, f);
    };
    /* where bin i of the slice goes: pairs mode -> the pair or single bins
       (k_pair_fold reduces them, this block owns them: stored), else the
       table (added, reference index order) */
    uint32_t *dst = nullptr;
    if (pg.pairs) dst = b < pg.npair ? pg.pairs + ((size_t)b << 16) : pg.singles + ((size_t)(b - pg.npair) << 16);
    const uint64_t base = (uint64_t)b << 16;
    /* fresh (round 5: the segment's k_zero left the table out, the general
       tiles' windows wait in pg.glist): every bin of the slice written, no
       read, and the table statistics taken here (pg.fz, as k_count_parts) */
    const bool fresh = pg.glist != nullptr && !pg.pairs;
    unsigned long long sd = 0, l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    auto out2 = [&](uint32_t i2, uint32_t lo, uint32_t hi) {   /* bins 2 i2, 2 i2 + 1 */
        if (!(lo | hi) && !pg.pairs && !fresh) return;
        if (pg.pairs) {
            reinterpret_cast<uint2 *>(dst)[i2] = make_uint2(lo, hi);
        } else {
            /* sigma maps the last digit 0 1 2 3 -> 0 1 3 2: the pair stays
               adjacent, swapped when the last digit of 2 i2 is 2 */
            uint2 *t2 = reinterpret_cast<uint2 *>(table + (fk_sigma(base | (2u * i2)) & ~1ull));
            if (fresh) {   /* (streaming stores, as the sparse outputs: not read back soon) */
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 ov = (i2 & 1u) ? u32x2{hi, lo} : u32x2{lo, hi};
                __builtin_nontemporal_store(ov, reinterpret_cast<u32x2 *>(t2));
                sd += (lo != 0u) + (hi != 0u);
                if (i2 & 1u) { l3 += lo; l2 += hi; } else { l0 += lo; l1 += hi; }
                return;
            }
            uint2 o = *t2;
            if (i2 & 1u) { o.x += hi; o.y += lo; } else { o.x += lo; o.y += hi; }
            *t2 = o;
        }
    };
    /* the block's statistics into one of the FZ_SLOTS partials: distinct,
       sum, last-base marginals, and the sum under the slice's first base
       (the slice's bins share their top 16 index bits) */
    __shared__ unsigned long long fzw[16][6];
    auto fz_flush = [&]() {
        if (!fresh) return;
        unsigned long long v6[6] = {sd, l0 + l1 + l2 + l3, l0, l1, l2, l3};
#pragma unroll
        for (int q = 0; q < 6; q++) v6[q] = wsum64(v6[q]);
        if ((threadIdx.x & 63) == 0)
#pragma unroll
            for (int q = 0; q < 6; q++) fzw[threadIdx.x >> 6][q] = v6[q];
        __syncthreads();
        if (threadIdx.x < 10) {
            const uint32_t q = threadIdx.x;
            unsigned long long t = 0;
            for (uint32_t w = 0; w < 16; w++) t += fzw[w][q < 6 ? q : 1u];
            if (q >= 6 && (uint32_t)((fk_sigma(base) >> (2 * pg.kk - 2)) & 3u) != q - 6u) t = 0;
            if (t) atomicAdd(&pg.fz[(blockIdx.x % FZ_SLOTS) * 10u + q], t);
        }
    };
    for (uint32_t i = threadIdx.x; i < NW / 4u; i += blockDim.x) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    uint32_t n = 0;
    walk([&](uint32_t c) {
        atomicAdd(&bins[c >> 1], 1u << ((c & 1u) << 4));
        n++;
    });
    __syncthreads();
    /* the wrap check: sum of the halves == codes counted */
    unsigned long long hs = 0;
    for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) hs += (bins[i] & 0xFFFFu) + (bins[i] >> 16);
    __shared__ unsigned long long red[2][16];
    {
        const unsigned long long a = wsum64(hs), c = wsum64((unsigned long long)n);
        if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = c; }
    }
    __syncthreads();
    unsigned long long sa = 0, sc = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) { sa += red[0][w]; sc += red[1][w]; }
    if (sa == sc) {
        for (uint32_t i = threadIdx.x; i < NW; i += blockDim.x) out2(i, bins[i] & 0xFFFFu, bins[i] >> 16);
        fz_flush();
        return;
    }
    /* a 16-bit bin wrapped: the slice again, as two halves of 2^15 32-bit bins */
    for (uint32_t h = 0; h < 2u; h++) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < NW / 4u; i += blockDim.x) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        walk([&](uint32_t c) {
            if ((c >> 15) == h) atomicAdd(&bins[c & 0x7FFFu], 1u);
        });
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < NW / 2u; i += blockDim.x) {
            const uint32_t i2 = (h << 14) + i;   /* bins (h << 15) + 2 i, + 1 */
            out2(i2, bins[2u * i], bins[2u * i + 1u]);
        }
    }
    fz_flush();
}

/*
 * k = 15, 16: the second partition level.  k_part leaves each of the 2048
 * coarse slices as runs of 32-bit codes (low 2k - 11 index bits) in every
 * batch row; a slice holds 2^(2k-26) parts of 2^15 bins (16 at k = 15, 64 at
 * k = 16).  k_repart (one block per REPART_G consecutive coarse slices)
 * reads the slices' runs -- counting their entries per part, then writing
 * each entry's low 15 bits as a 16-bit code into its part's contiguous
 * stream -- after taking the group's region of the output with one global
 * atomic.  k_count_parts (one block per part) then reads one contiguous
 * stream into 2^15 LDS bins and adds them to the table.
 *
 * Round 4 (k = 15 / 16, 1 G bases): one block per coarse slice, a lane per
 * row, and the entries stored one at a time at a per-part cursor moved 68-70
 * GB of HBM per step for ~14 GB of codes (10.3 / 11.8 ms): each lane's 64-B
 * run straddled lines no neighbour shared, and every 2-B store wrote back a
 * partial line.  Now the lanes of a row take the group's adjacent runs (one
 * contiguous span per row) and each round's entries are counting-sorted by
 * part in LDS and written out as contiguous segments.
 */
struct PartMeta {
    unsigned long long off;   /* first code of the part's stream (a multiple of 8) */
    uint32_t n, pad;
};
#define REPART_MAXP 64u       /* parts per coarse slice (k = 16) */
/* coarse slices per k_repart block, and (16-bit parts) two blocks per CU:
   <= 64 VGPRs (a few spill) beside 72 KiB of LDS each.  k = 16 1 G-base
   step 11.5 -> 10.5 ms, k = 17 10 G-base 204 -> 195 ms against G = 8 with
   one block per CU (G = 4 alone: 10.8 / 198) */
#ifndef REPART_G
#define REPART_G 4u
#endif
#ifndef REPART_MINW
#define REPART_MINW 8
#endif
/* parts per block: G x parts per slice (16-bit parts: up to REPART_MAXP a
   slice; the wide sparse passes' 32-bit parts: REPART_METAP) */
#define REPART_GP(OT, G) ((G) * (sizeof(OT) == 2 ? REPART_MAXP : REPART_METAP))
#define REPART_METAP 128u     /* meta entries per coarse slice (wide sparse passes: 128 parts, G = 4) */
#define REPART_CAP 32768u     /* entries per pass-B round: a batch (16 waves x 2048), the longest run */
static_assert(16u * FK_TILE_BYTES <= REPART_CAP, "a C32 row's run fits one k_repart round");

/* OT = uint16_t: a code's part is its bits [15, 15 + split), stored as its
   low 15 bits (k = 15, 16; k = 17 passes, psh = 15).  OT = uint32_t (wide
   sparse passes): part bits [psh, psh + 6), stored as the low psh bits. */
template <typename OT, uint32_t G = REPART_G>
__global__ void __launch_bounds__(1024, sizeof(OT) == 2 && G == REPART_G ? REPART_MINW : 1)
k_repart(PartGeo pg, OT *out, unsigned long long *alloc, PartMeta *meta, uint64_t cap,
         unsigned long long *err, uint32_t psh, unsigned long long *pmax) {
    /* (G coarse slices of 2^split parts: G << split <= GP, else nothing is
       done and the pass fails -- the arrays below are sized by GP) */
    constexpr uint32_t GP = REPART_GP(OT, G);
    /* per (slice in the group, part): entries, round count / offset /
       cursor, written so far, stream start */
    __shared__ uint32_t cnt[GP], hc[GP], ho[GP], cur[GP], wr[GP];
    __shared__ unsigned long long poff[GP];
    if ((G << pg.split) > GP) {
        if (threadIdx.x == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
        return;
    }
    __shared__ uint32_t scn[17];
    __shared__ __attribute__((aligned(16))) OT rbuf[REPART_CAP];
    const uint32_t pmask = (1u << psh) - 1u;
    const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const uint32_t np = 1u << pg.split, gp = G * np;   /* parts of the block */
    const uint32_t b0 = blockIdx.x * G;                /* its first coarse slice */
    for (uint32_t i = t; i < gp; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint32_t nrows = pg.flag && *pg.flag ? 2u * pg.rows : pg.rows;
    const uint32_t nitems = nrows * G;   /* (row, slice) pairs, row-major: a row's runs side by side */
    const uint4 *g4 = reinterpret_cast<const uint4 *>(pg.codes);
    /* item i: row i / G, slice b0 + i % G; its codes as 16-B pieces (4 each)
       -- the G lanes of a row read one contiguous span */
    auto each_code = [&](uint32_t i, auto &&f) {
        const uint32_t r = i / G, sl = i % G;
        const uint32_t e = pg.idx[(size_t)r * pg.nslices + b0 + sl];
        if (e == PART_NO_RUN) return;
        const uint64_t s0 = (uint64_t)r * pg.batch + (e >> 16), s1 = s0 + run_count(e);
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
        auto piece = [&](const uint4 &v, uint64_t q) {
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int h = 0; h < 4; h++)
                if (q * 4 + h >= s0 && q * 4 + h < s1) f(sl * np + (w4[h] >> psh), w4[h]);
        };
        /* the pieces of a run of up to 17 codes in flight together (one
           load at a time left the kernel latency-bound) */
        uint4 v[5];
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++) v[u] = q0 + u < q1 ? g4[q0 + u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++)
            if (q0 + u < q1) piece(v[u], q0 + u);
        for (uint64_t q = q0 + 5u; q < q1; q++) piece(g4[q], q);
    };
    /* pass A: entries per part */
    for (uint32_t i = t; i < nitems; i += blockDim.x)
        each_code(i, [&](uint32_t p, uint32_t) { atomicAdd(&cnt[p], 1u); });
    __syncthreads();
    if (t < 64) {   /* the parts' 8-aligned stream starts in the group's region */
        uint32_t carry = 0;
        for (uint32_t p0 = 0; p0 < gp; p0 += 64u) {
            const uint32_t p = p0 + lane;
            const uint32_t sz = p < gp ? (cnt[p] + 7u) & ~7u : 0u;
            const uint32_t inc = wscan_incl32(sz);
            if (p < gp) ho[p] = carry + inc - sz;   /* (ho: scratch here) */
            carry += rdlane(inc, 63);
        }
        unsigned long long g0 = 0;
        if (lane == 0) g0 = atomicAdd(alloc, (unsigned long long)carry);
        g0 = rdlane64(g0, 0);
        /* bound check: the group's region inside the `cap` codes of `out`
           (the host sizes it for every entry a segment can hold); past it,
           nothing is written, the parts read as empty and the feed fails */
        const bool over = g0 + carry > cap;
        if (over && lane == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
        for (uint32_t p = lane; p < gp; p += 64u) {
            poff[p] = over ? ~0ull : g0 + ho[p];
            wr[p] = 0;
            /* slice-major: (b0 + p / np) * np + p % np */
            meta[(size_t)b0 * np + p] = over ? PartMeta{0, 0, 0} : PartMeta{g0 + ho[p], cnt[p], 0};
        }
        if (pmax) {   /* the largest part (k_kp_sort's LDS size) */
            uint32_t mx = 0;
            for (uint32_t p = lane; p < gp; p += 64u) mx = max(mx, cnt[p]);
            mx = wscan_max32(mx);
            if (lane == 63) atomicMax(pmax, (unsigned long long)mx);
        }
    }
    /* pass B: rounds of whole runs (a lane per item) holding up to
       REPART_CAP entries: counted by part, placed in LDS by part, and each
       part's segment written after the part's earlier rounds */
    uint32_t base = 0;
    __syncthreads();
    /* one item per lane and round, software-pipelined: the next round's
       items are known once this round's are taken, so their index words
       load during this round's count and their first pieces during its
       placement and write-out (each round was a chain of an index load, a
       code load and five barriers: k_repart latency-bound) */
    auto idx_word = [&](uint32_t i) -> uint32_t {
        return i < nitems ? pg.idx[(size_t)(i / G) * pg.nslices + b0 + i % G] : PART_NO_RUN;
    };
    auto span = [&](uint32_t i, uint32_t e, uint64_t &s0, uint64_t &s1) {
        /* (an empty run -- PART_NO_RUN, count 0 -- reads nothing) */
        s0 = (uint64_t)(i / G) * pg.batch + (e == PART_NO_RUN ? 0u : e >> 16);
        s1 = s0 + run_count(e);
    };
    auto load5 = [&](uint64_t s0, uint64_t s1, uint4 *v) {
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
#pragma unroll
        for (uint32_t u = 0; u < 5u; u++) v[u] = q0 + u < q1 ? g4[q0 + u] : make_uint4(0, 0, 0, 0);
    };
    uint32_t ie = idx_word(base + t);
    uint4 pv[5];
    {
        uint64_t a0, a1;
        span(base + t, ie, a0, a1);
        load5(a0, a1, pv);
    }
    for (;;) {
        const uint32_t i = base + t;
        const uint32_t c = run_count(ie);
        const uint32_t wi = wscan_incl32(c);
        if (lane == 63) scn[wv] = wi;
        for (uint32_t p = t; p < gp; p += blockDim.x) hc[p] = 0;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += scn[w];
        /* the leading items whose runs fit (item `base`'s always does: a
           run holds at most one batch) */
        const bool take = i < nitems && before + wi <= REPART_CAP;
        const uint32_t ntake = (uint32_t)__syncthreads_count(take);
        const uint32_t nbase = base + ntake;
        const uint32_t ien = idx_word(nbase + t);   /* the next round's item */
        uint64_t s0, s1;
        span(i, take ? ie : PART_NO_RUN, s0, s1);
        const uint32_t sl = i % G;
        const uint64_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
        auto codes = [&](auto &&f) {
            auto piece = [&](const uint4 &v, uint64_t q) {
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int h = 0; h < 4; h++)
                    if (q * 4 + h >= s0 && q * 4 + h < s1) f(sl * np + (w4[h] >> psh), w4[h]);
            };
#pragma unroll
            for (uint32_t u = 0; u < 5u; u++)
                if (q0 + u < q1) piece(pv[u], q0 + u);
            for (uint64_t q = q0 + 5u; q < q1; q++) piece(g4[q], q);
        };
        codes([&](uint32_t p, uint32_t) { atomicAdd(&hc[p], 1u); });
        __syncthreads();
        if (t < 64) {
            uint32_t carry = 0;
            for (uint32_t p0 = 0; p0 < gp; p0 += 64u) {
                const uint32_t p = p0 + lane;
                const uint32_t n = p < gp ? hc[p] : 0u;
                const uint32_t inc = wscan_incl32(n);
                if (p < gp) { ho[p] = carry + inc - n; cur[p] = carry + inc - n; }
                carry += rdlane(inc, 63);
            }
        }
        __syncthreads();
        codes([&](uint32_t p, uint32_t v) {
            const uint32_t at = atomicAdd(&cur[p], 1u);
            rbuf[at] = (OT)(v & pmask);
        });
        /* the next round's first pieces (this round's are consumed) */
        {
            uint64_t a0, a1;
            span(nbase + t, ien, a0, a1);
            load5(a0, a1, pv);
        }
        ie = ien;
        __syncthreads();
        /* a wave per part: consecutive entries to consecutive 2-B slots */
        for (uint32_t p = wv; p < gp; p += 16u) {
            const uint32_t n = poff[p] == ~0ull ? 0u : hc[p], o = ho[p];
            OT *dst = out + poff[p] + wr[p];
            for (uint32_t j = lane; j < n; j += 64u) dst[j] = rbuf[o + j];
        }
        __syncthreads();
        for (uint32_t p = t; p < gp; p += blockDim.x) wr[p] += hc[p];
        base = nbase;
        if (base >= nitems || ntake == 0) break;
        __syncthreads();
    }
}

/* one block per part: its stream into 2^15 LDS bins, then into the table */
__global__ void __launch_bounds__(1024)
k_count_parts(PartGeo pg, const uint16_t *in, const PartMeta *meta, uint32_t *table, uint64_t cap,
              unsigned long long *err) {
    extern __shared__ uint32_t slice[];
    const uint32_t np = 1u << pg.split;
    const uint32_t b = blockIdx.x / np, part = blockIdx.x % np;
    for (uint32_t i = threadIdx.x; i < (1u << 13); i += blockDim.x)
        reinterpret_cast<uint4 *>(slice)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    PartMeta m = meta[blockIdx.x];
    if (m.off + m.n > cap) {   /* bound check: a stream past the parts buffer is not read */
        if (threadIdx.x == 0) atomicOr(err, (unsigned long long)FK_FAULT_META);
        m.n = 0;
        m.off = 0;
    }
    const uint4 *g4 = reinterpret_cast<const uint4 *>(in + m.off);   /* 16-B aligned: off % 8 == 0 */
    const uint32_t nq = (m.n + 7u) >> 3;
    for (uint32_t q = threadIdx.x; q < nq; q += blockDim.x) {
        const uint4 v = g4[q];
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 8; h++)
            if (q * 8u + (uint32_t)h < m.n) atomicAdd(&slice[(w4[h >> 1] >> (16 * (h & 1))) & 0x7FFFu], 1u);
    }
    __syncthreads();
    /* the part's bins into the table (the block owns them), eight loads in
       flight per lane before the adds and stores: one load-add-store chain
       at a time left this loop latency-bound (k = 16: 13.3 ms per G-base) */
    const uint64_t base = ((uint64_t)b << pg.sh) | ((uint64_t)part << 15);
    if (pg.glist) {
        /* a fresh table (the segment's k_zero left it out): every bin of
           the part written, no read (k = 16: 17 GB of zeroing and 17 GB of
           reads less per step); the general tiles' windows follow
           (k_list_add) */
        /* with the statistics k_table_stats would read the table for
           (distinct, sum, last- and first-base marginals): they stand unless
           the general tiles' list or k_redo adds to the table afterwards */
        const int fs = 2 * pg.kk - 2;
        /* a lane's bins i = lane + 1024 j all end in the same base (sigma
           maps digits one by one, and i & 3 = lane & 3): its sum is its
           last-base marginal */
        /* four bins per lane: kernel bins 4m + d land at reference index
           sigma(base | 4m) + sigma(d), i.e. the last digits 0 1 3 2 (sigma
           maps digit by digit): one 16-B store */
        uint32_t dist = 0;
        unsigned long long last[4] = {0, 0, 0, 0};
        const uint4 *s4 = reinterpret_cast<const uint4 *>(slice);
        uint4 *t4 = reinterpret_cast<uint4 *>(table);
        for (uint32_t m = threadIdx.x; m < (1u << 13); m += 1024u) {
            const uint4 q = s4[m];
            const uint4 o = make_uint4(q.x, q.y, q.w, q.z);
            {   /* streaming stores: the 16 GiB table is not read back soon
                   (k = 16 1 G-base step 10.74 -> 10.42 ms) */
                const u32x4 ov = {o.x, o.y, o.z, o.w};
                __builtin_nontemporal_store(ov, reinterpret_cast<u32x4 *>(t4) + (fk_sigma(base | ((uint64_t)m << 2)) >> 2));
            }
            dist += (o.x != 0) + (o.y != 0) + (o.z != 0) + (o.w != 0);
            last[0] += o.x; last[1] += o.y; last[2] += o.z; last[3] += o.w;
        }
        const unsigned long long sum = last[0] + last[1] + last[2] + last[3];
        unsigned long long v10[6] = {dist, sum, last[0], last[1], last[2], last[3]};
#pragma unroll
        for (int q = 0; q < 6; q++) v10[q] = wsum64(v10[q]);
        /* the wave sums in the bins' LDS, once every lane has read its bins
           (no static LDS: the kernel's dynamic maximum is the whole 160 KiB) */
        __syncthreads();
        unsigned long long *wp = reinterpret_cast<unsigned long long *>(slice);
        const uint32_t wv = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0)
#pragma unroll
            for (int q = 0; q < 6; q++) wp[wv * 6u + q] = v10[q];
        __syncthreads();
        if (threadIdx.x < 10) {
            unsigned long long t = 0;
            const uint32_t q = threadIdx.x;
            if (q < 6) {
                for (uint32_t w = 0; w < 16; w++) t += wp[w * 6u + q];
            } else {   /* the first base of every bin of the part: one digit */
                for (uint32_t w = 0; w < 16; w++) t += wp[w * 6u + 1u];
                if ((uint32_t)((fk_sigma(base) >> fs) & 3u) != q - 6u) t = 0;
            }
            if (t) atomicAdd(&pg.fz[(blockIdx.x % FZ_SLOTS) * 10u + q], t);
        }
        return;
    }
    constexpr uint32_t U = 8u;
    for (uint32_t i0 = threadIdx.x; i0 < (1u << 15); i0 += U * 1024u) {
        uint32_t v[U], o[U];
#pragma unroll
        for (uint32_t j = 0; j < U; j++) v[j] = slice[i0 + j * 1024u];
#pragma unroll
        for (uint32_t j = 0; j < U; j++) o[j] = v[j] ? table[fk_sigma(base | (i0 + j * 1024u))] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < U; j++)
            if (v[j]) table[fk_sigma(base | (i0 + j * 1024u))] = o[j] + v[j];
    }
}

/* the general tiles' windows of a fresh two-level table (hist_add's list) */
__global__ void k_list_init(uint32_t *list, uint32_t cap, unsigned long long *fz) {
    if (threadIdx.x == 0) { list[0] = 0; list[1] = cap; }
    for (uint32_t i = threadIdx.x; i < FZ_SLOTS * 10u; i += blockDim.x) fz[i] = 0;
}
__global__ void __launch_bounds__(256)
k_list_add(const uint32_t *list, uint32_t *table, int k, unsigned long long *fz) {
    const uint32_t n = min(list[0], list[1]);
    const int fs = 2 * k - 2;
    /* with what each window changes in the statistics k_count_parts took
       (the old value of its bin tells whether it was distinct before) */
    unsigned long long v10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t x = list[2 + i];
        const uint32_t old = atomicAdd(&table[x], 1u);
        v10[0] += old == 0;
        v10[1] += 1;
        v10[2 + (x & 3u)] += 1;
        v10[6 + ((x >> fs) & 3u)] += 1;
    }
#pragma unroll
    for (int q = 0; q < 10; q++) {
        const unsigned long long t = wsum64(v10[q]);
        if ((threadIdx.x & 63) == 0 && t) atomicAdd(&fz[((blockIdx.x * 4u + (threadIdx.x >> 6)) % FZ_SLOTS) * 10u + q], t);
    }
}

/* pairs mode: every k-mer x (kernel order) is the prefix of the pairs
 * 4x + b and the suffix of the pairs b*4^k + x (a pair stands for both of
 * its k-mers), plus the single windows counted at x */
__global__ void __launch_bounds__(256)
k_pair_fold(const uint32_t *pairs, const uint32_t *singles, uint64_t nbins, uint32_t *table, int fresh) {
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < nbins; x += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 pre = reinterpret_cast<const uint4 *>(pairs)[x];
        uint32_t v = pre.x + pre.y + pre.z + pre.w + singles[x];
#pragma unroll
        for (int b = 0; b < 4; b++) v += pairs[(uint64_t)b * nbins + x];
        if (fresh) table[fk_sigma(x)] = v;   /* (a fresh table: k_zero left it out) */
        else if (v) table[fk_sigma(x)] += v;
    }
}

/*
 * k_scan: exact entering state of every range, one thread per range.  Each
 * 256-thread block scans its ranges' transfer functions (wave shuffles, then
 * the four wave aggregates), publishes the block aggregate with an
 * epoch-tagged flag, waits for the flags of all blocks before it and
 * composes their aggregates with one wave scan (all predecessors publish at
 * about the same time, so this is one round trip, not a chain).
 * mode 0: resolve from *d_state, list the ranges whose guess is not
 * equivalent, write the exit state back to *d_state and res->exit.
 * mode 1: only the total transfer function (shard summary) into *tf_total.
 * Every block reads *d_state before publishing its flag; the last block
 * writes it only after seeing every flag.  All blocks are co-resident (a
 * handful), and a block only waits on blocks dispatched before it.
 */
#define SCAN_THREADS 256
#define SCAN_WAVES (SCAN_THREADS / 64)

__global__ void __launch_bounds__(SCAN_THREADS)
k_scan(const RangeRec *rr, uint64_t n, XState *d_state, XState *rtrue, uint32_t *redo_list,
       DevRes *res, int k, int mode, TF *tf_total, TF *aggs, uint32_t *flags, uint32_t epoch) {
    __shared__ TF wincl[SCAN_WAVES];   /* inclusive wave aggregates */
    __shared__ TF bprefix;
    __shared__ unsigned long long eof_min;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, b = blockIdx.x;
    const uint64_t r = (uint64_t)b * SCAN_THREADS + t;
    const XState init = *d_state;
    if (t == 0) eof_min = ~0ull;
    TF a = fk_identity();
    unsigned long long em = ~0ull;
    if (r < n) {
        a = rr[r].tf;
        const uint64_t e = rr[r].eof;
        if (e != FK_NO_EOF64) em = rr[r].c0 * FK_CHUNK_BYTES + e;
    }
    a = tf_wave_scan(a);
    if (lane == 63) wincl[w] = a;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        unsigned long long o = ((unsigned long long)__shfl_xor((unsigned)(em >> 32), d, 64) << 32) |
                               (unsigned)__shfl_xor((unsigned)em, d, 64);
        em = min(em, o);
    }
    __syncthreads();
    if (lane == 0 && em != ~0ull) atomicMin(&eof_min, em);
    if (t == 0) {
        for (int i = 1; i < SCAN_WAVES; i++) wincl[i] = fk_compose(wincl[i - 1], wincl[i]);
        aggs[b] = wincl[SCAN_WAVES - 1];
        __threadfence();
        __hip_atomic_store(&flags[b], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    /* prefix of all blocks before this one (wave 0) */
    if (w == 0) {
        TF carry = fk_identity();
        for (uint32_t base = 0; base < b; base += 64) {
            const uint32_t i = base + lane;
            TF x = fk_identity();
            if (i < b) {
                while (__hip_atomic_load(&flags[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch)
                    __builtin_amdgcn_s_sleep(1);
                x = aggs[i];
            }
            x = tf_wave_scan(x);
            /* lane 63 holds the chunk's aggregate (identity padding is neutral) */
            const TF chunk = tf_rdlane(x, 63);
            carry = fk_compose(carry, chunk);
        }
        if (lane == 0) bprefix = carry;
    }
    __syncthreads();
    if (mode == 1) {
        if (b == gridDim.x - 1 && t == 0) *tf_total = fk_compose(bprefix, wincl[SCAN_WAVES - 1]);
        return;
    }
    /* exclusive prefix of this thread's range */
    TF ex = tf_shup(a, 1);
    if (lane == 0) ex = fk_identity();
    if (w > 0) ex = fk_compose(wincl[w - 1], ex);
    ex = fk_compose(bprefix, ex);
    if (r < n) {
        const RangeRec &q = rr[r];
        const XState s = fk_apply(ex, init);
        rtrue[r] = s;
        DState as{q.a_code, q.a_R, q.a_hdr};
        if (!fk_equiv(as, s, k, (q.c1 - q.c0) * FK_CHUNK_BYTES)) {
            uint32_t slot = atomicAdd(&res->redo_n, 1u);
            redo_list[slot] = (uint32_t)r;
        }
        if (r == n - 1) {
            const XState fin = fk_apply(q.tf, s);
            *d_state = fin;
            res->exit = fin;
        }
    }
    if (t == 0 && eof_min != ~0ull) atomicMin(&res->eof_cand, eof_min);
}

/*
 * k_tail (one-pass feeds, after k_count; TAIL_BLOCKS x TAIL_THREADS).  Block
 * j takes 1/B of the table and 1/B of k_count's BlockSums:
 *  - table bins: table = (fresh ? 0 : table) + the FK_SUBTABLES sub-tables
 *    (zeroed), and their statistics;
 *  - BlockSums: each block's first guess against the previous block's last
 *    exit (the local check of block_summary, across blocks), flags, 0xFF
 *    candidates, and for the exit state's run length the last absorbing
 *    block (its exit R is exact) plus the bases of the blocks after it.
 * The last block to finish combines the B partial results (a segmented
 * reduction for the run length), merges the feed's accumulators and
 * publishes the result block.
 */
struct TailPart {
    unsigned long long st[10];   /* table statistics of the bin slice */
    uint64_t eof;                /* smallest 0xFF candidate */
    uint64_t Rj;                 /* exit R of the slice's last absorbing block */
    uint64_t nv_after;           /* bases of the slice's blocks after it (all, if none) */
    uint32_t need;               /* ONE_* bits */
    int32_t j;                   /* the slice's last absorbing block, or -1 */
};

__device__ __forceinline__ unsigned long long wmax64s(long long v) {
    return (unsigned long long)wred64((uint64_t)v, OpMaxS64{});
}

/* Item i of k_tail's chain: a k_count block's BlockSum (i < G), else the
 * dynamic range nstatic + (i - G), summarised here from its RangeRec as a
 * block of one range would be (block_summary). */
__device__ __forceinline__ BlockSum tail_item(const BlockSum *bsum, const RangeRec *rr, uint32_t G,
                                              uint64_t nstatic, uint32_t i) {
    if (i < G) return bsum[i];
    const RangeRec q = rr[nstatic + (i - G)];
    BlockSum b;
    if (q.resume) {
        b.e_R = 0; b.e_code = 0; b.e_hdr = 0;
        b.g_code = 0; b.g_R = 0; b.g_hdr = 0;
        b.nvb = 0; b.eof = ~0ull; b.nv = 0;
        b.flags = ONE_RESUME;
        return b;
    }
    const XState g{q.a_R, q.a_code, q.a_hdr, 0};
    const XState e = fk_apply(q.tf, g);
    b.e_R = e.R; b.e_code = e.code; b.e_hdr = e.hdr;
    b.g_code = q.a_code; b.g_R = q.a_R; b.g_hdr = q.a_hdr;
    b.nvb = (q.c1 - q.c0) * FK_CHUNK_BYTES;
    b.eof = q.eof != FK_NO_EOF64 ? q.c0 * FK_CHUNK_BYTES + q.eof : ~0ull;
    b.nv = q.tf.nv;
    b.flags = q.tf.f0_const ? BS_ABSORB : 0u;
    return b;
}

#define TAIL_KEEP 2
/* k_tail: bin i of the table, and zeros where the sub-tables held counts
   (streaming stores: no dirty L2 lines for a system fence to write back) */
__device__ __forceinline__ void tail_store(uint32_t *table, uint32_t *subs, uint32_t nbins, uint32_t i, uint32_t v,
                                           uint32_t m) {
#pragma unroll
    for (int j = 0; j < FK_SUBTABLES; j++)
        if (m & (1u << j)) __builtin_nontemporal_store(0u, &subs[(size_t)j * nbins + i]);
    __builtin_nontemporal_store(v, &table[i]);
}

__global__ void __launch_bounds__(TAIL_THREADS)
k_tail(const OnePassCfg *opc, uint32_t flags, uint32_t seq, uint32_t *table, int k, uint32_t *subs,
       unsigned long long *facc, DevRes *res, const XState *d_init, uint32_t G0, uint64_t seg_len,
       TailPart *part, uint32_t *done, const RangeRec *rr, uint64_t nstatic, uint32_t ndyn) {
    __shared__ unsigned long long sh[TAIL_THREADS / 64][16];
    __shared__ uint32_t bc[4];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, B = gridDim.x, jb = blockIdx.x;
    const uint32_t nbins = 1u << (2 * k);
    const bool fresh = (flags & OP_FRESH) != 0;
    const BlockSum *bsum = reinterpret_cast<const BlockSum *>(opc->bsum);
    /* the chain: G0 block summaries, then the dynamic ranges */
    const uint32_t G = G0 + ndyn;
    /* every load of the slice phase first (one round trip): this block's
       BlockSums [b0, b1) and their predecessors' exits, one per thread, and
       its table bins with the sub-tables (bins strided over the threads) */
    const uint32_t b0 = (uint32_t)((uint64_t)G * jb / B), b1 = (uint32_t)((uint64_t)G * (jb + 1) / B);
    const uint32_t lo = (uint32_t)((uint64_t)nbins * jb / B), hi = (uint32_t)((uint64_t)nbins * (jb + 1) / B);
    const uint32_t bi = b0 + t;
    const bool hb = bi < b1;   /* G <= B x TAIL_THREADS (host): one item per thread at most */
    BlockSum bs;
    uint64_t pe_R = 0, pe_code = 0;
    uint32_t pe_hdr = 0;
    if (hb) {
        bs = tail_item(bsum, rr, G0, nstatic, bi);
        if (bi > 0) {
            const BlockSum pb = tail_item(bsum, rr, G0, nstatic, bi - 1);
            pe_R = pb.e_R; pe_code = pb.e_code; pe_hdr = pb.e_hdr;
        }
        /* a dynamic range's guess is its exact entering state when the feed
           completes here (block_summary does this for the static ranges) */
        if (bi >= G0 && !(bs.flags & ONE_RESUME))
            opc->rtrue[nstatic + (bi - G0)] = XState{bs.g_R, bs.g_code, bs.g_hdr, 0};
    }
    const int fs = 2 * (k - 1);
    unsigned long long v10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    /* The stores (the table bins, zeros into the sub-tables) wait until this
       block has reported its partial record: a wave's returning atomics come
       back in order behind its earlier stores, so storing first made every
       block's report wait for its stores to complete (~5 us).  A thread
       keeps up to TAIL_KEEP bins (k <= 7: at most 2 with 16 blocks). */
    uint32_t keep_v[TAIL_KEEP], keep_m[TAIL_KEEP], nkeep = 0;
    for (uint32_t i = lo + t; i < hi; i += blockDim.x) {
        uint32_t a[FK_SUBTABLES];
#pragma unroll
        for (int j = 0; j < FK_SUBTABLES; j++) a[j] = subs[(size_t)j * nbins + i];
        uint32_t v = fresh ? 0u : table[i];
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < FK_SUBTABLES; j++) {
            v += a[j];
            m |= a[j] ? 1u << j : 0u;
        }
        if (nkeep < TAIL_KEEP) {
            keep_v[nkeep] = v;
            keep_m[nkeep] = m;
            nkeep++;
        } else {
            tail_store(table, subs, nbins, i, v, m);
        }
        v10[0] += v != 0;
        v10[1] += v;
        const uint32_t ld = i & 3u, fd = k == 1 ? ld : (i >> fs) & 3u;
        v10[2] += ld == 0 ? v : 0; v10[3] += ld == 1 ? v : 0; v10[4] += ld == 2 ? v : 0; v10[5] += ld == 3 ? v : 0;
        v10[6] += fd == 0 ? v : 0; v10[7] += fd == 1 ? v : 0; v10[8] += fd == 2 ? v : 0; v10[9] += fd == 3 ? v : 0;
    }
    /* BlockSum i: its first guess against block i-1's last exit (the local
       check of block_summary, across blocks), flags, 0xFF candidate */
    uint32_t need = 0;
    uint64_t eof = ~0ull;
    long long jmax = -1;
    if (hb) {
        need = bs.flags & (ONE_RESUME | ONE_SCAN);
        if (bi > 0 && !fk_equiv(DState{bs.g_code, bs.g_R, bs.g_hdr}, XState{pe_R, pe_code, pe_hdr, 0}, k, bs.nvb))
            need |= ONE_SCAN;
        eof = bs.eof;
        if (bs.flags & BS_ABSORB) jmax = bi;
    }
    /* the slice's last absorbing block, then the bases after it */
    const long long jw = (long long)wmax64s(jmax);
    if (lane == 0) sh[w][10] = (unsigned long long)jw;
    __syncthreads();
    long long js = -1;
    for (uint32_t q = 0; q < blockDim.x / 64; q++) js = max(js, (long long)sh[q][10]);
    uint64_t nv_after = hb && (long long)bi > js ? bs.nv : 0;
    if (hb && (long long)bi == js) sh[0][11] = bs.e_R;   /* the owner publishes its R */
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(v10[q]);
    nv_after = wsum64(nv_after);
    need = (uint32_t)wred64(need, OpOr64{});
    eof = wred64(eof, OpMin64{});
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 10; q++) sh[w][q] = v10[q];
        sh[w][12] = nv_after;
        sh[w][13] = need;
        sh[w][14] = eof;
    }
    __syncthreads();
    if (w == 0) {
        /* the partial record, with returning exchanges (waited for before
           the count below: no release fence) */
        uint32_t sink = 0;
        if (t < 16) {
            unsigned long long a = t == 14 ? ~0ull : 0ull;
            for (uint32_t q = 0; q < blockDim.x / 64; q++) {
                const unsigned long long v = sh[q][t];
                if (t < 10 || t == 12) a += v;
                else if (t == 13) a |= v;
                else if (t == 14) a = min(a, v);
            }
            TailPart &P = part[jb];
            if (t < 10) sink = xput(&P.st[t], a);
            if (t == 12) sink = xput(&P.nv_after, (uint64_t)a);
            if (t == 13) sink = xput(&P.need, (uint32_t)a);
            if (t == 14) sink = xput(&P.eof, (uint64_t)a);
            if (t == 15) sink = xput(&P.j, (int32_t)js) | xput(&P.Rj, (uint64_t)(js >= 0 ? sh[0][11] : 0));
        }
        keep(sink);
        /* 2. the last block to finish combines */
        if (t == 0) bc[0] = atomicAdd(done, 1u) == B - 1;
    }
    __syncthreads();
    /* k_count is done: block 0 resets its dynamic-range pools for the next
       launch (after its report, like the bin stores) */
    if (jb == 0)
        for (uint32_t q = t; q < FK_MAX_POOLS; q += blockDim.x) done[FK_HEADS_OFF + q * FK_HEAD_STRIDE] = 0;
    if (!bc[0]) {
        for (uint32_t q = 0; q < nkeep; q++) tail_store(table, subs, nbins, lo + t + q * blockDim.x, keep_v[q], keep_m[q]);
        return;
    }
    if (t < 64) {
        if (t == 0) *done = 0;
        /* every load of the combine first: partial `lane`, the last
           BlockSum, the entering state, the accumulators */
        const bool have = lane < B;
        uint32_t nd = 0;
        uint64_t ef = ~0ull, pR = 0, pn = 0;
        int32_t pj = -1;
        unsigned long long st[10];
        if (have) {
            const TailPart &P = part[lane];   /* device-coherent loads (other XCDs wrote them) */
            nd = xget(&P.need); ef = xget(&P.eof); pj = xget(&P.j); pR = xget(&P.Rj); pn = xget(&P.nv_after);
#pragma unroll
            for (int q = 0; q < 10; q++) st[q] = xget(&P.st[q]);
        } else {
#pragma unroll
            for (int q = 0; q < 10; q++) st[q] = 0;
        }
        const BlockSum lb = tail_item(bsum, rr, G0, nstatic, G - 1);
        /* a shard's entering state is unknown: count from its first guess
           (the host checks it against the stitched state at resolve) */
        const bool shard = (flags & OP_SHARD) != 0;
        const BlockSum b0s = bsum[0];
        const XState init = shard ? XState{b0s.g_R, b0s.g_code, b0s.g_hdr, 0}
                                  : fresh ? XState{0, 0, 0, 0} : *d_init;
        unsigned long long fa = 0;
        if (lane < ACC_N)
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) fa += facc[c * ACC_N + lane];
        const unsigned long long ta = lane < ACC_N && !fresh ? opc->acc_total[lane] : 0ull;
#pragma unroll
        for (int q = 0; q < 10; q++) st[q] = wsum64(st[q]);
        nd = (uint32_t)wred64(nd, OpOr64{});
        ef = wred64(ef, OpMin64{});
        /* exit run length: the last slice with an absorbing block, its R,
           plus the bases after it */
        const uint64_t hasj = __ballot(have && pj >= 0);
        const int sstar = hasj ? 63 - __builtin_clzll(hasj) : -1;
        const uint64_t add = wsum64((have && (int)lane > sstar) ? pn : 0);
        const uint64_t base = sstar >= 0 ? rdlane64(pR, sstar) + rdlane64(pn, sstar) : init.R;
        uint32_t need_all = nd;
        /* no run length in the segment reaches the int32 wrap (the local
           checks rely on it) */
        if (!shard && (uint64_t)(uint32_t)init.R + seg_len + FK_CHUNK_BYTES > 0x7FFFFFFFull) need_all |= ONE_SCAN;
        /* the exit state: header flag and last bases of the last block's
           exit (identical trajectories), exact when it absorbs or holds at
           least 32 bases; else the host path */
        if (!(lb.flags & BS_ABSORB) && lb.nv < 32) need_all |= ONE_SCAN;
#pragma unroll
        for (int q = 0; q < 10; q++)
            if (lane == (uint32_t)q) res->tstat[q] = st[q];
        if (need_all == 0 && lane < ACC_N) {
            const unsigned long long v = ta + fa;
            opc->acc_total[lane] = v;
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) facc[c * ACC_N + lane] = 0;
            res->acc[lane] = v;
        }
        if (lane == 0) {
            if (need_all == 0) {
                const uint64_t fR = base + add;
                XState *ps = opc->state;
                ps->R = fR; ps->code = lb.e_code; ps->hdr = lb.e_hdr; ps->pad = 0;
                res->exit.R = fR; res->exit.code = lb.e_code; res->exit.hdr = lb.e_hdr; res->exit.pad = 0;
            } else if (fresh) {
                XState *ps = opc->state;   /* k_scan starts from it */
                ps->R = 0; ps->code = 0; ps->hdr = 0; ps->pad = 0;
            }
            res->eof_cand = need_all ? ~0ull : ef;
            res->redo_n = 0;
            res->need = need_all;
            if (shard) {
                ShardSum &ss = res->shard;
                ss.g_code = b0s.g_code; ss.g_R = b0s.g_R; ss.g_hdr = b0s.g_hdr;
                ss.nvb0 = b0s.nvb;
                ss.absorb = sstar >= 0;
                ss.c_R = sstar >= 0 ? base + add : 0;
                ss.nv = add;
                ss.c_code = lb.e_code; ss.c_hdr = lb.e_hdr;
            }
        }
        publish_res_wave(res, opc->host_res, seq);
    }
    for (uint32_t q = 0; q < nkeep; q++) tail_store(table, subs, nbins, lo + t + q * blockDim.x, keep_v[q], keep_m[q]);
}

/* Sum the per-block partials of k_table_stats into res->tstat and publish
   the result block (one block of 256 threads). */
__device__ void stats_publish(DevRes *res, DevRes *host_res, const unsigned long long *part, uint32_t nparts,
                              uint32_t seq) {
    __shared__ unsigned long long wq[4][10];
    const uint32_t wv = threadIdx.x >> 6;
    unsigned long long acc10[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nparts; b += blockDim.x)
#pragma unroll
        for (int q = 0; q < 10; q++) acc10[q] += part[(size_t)b * 10 + q];
#pragma unroll
    for (int q = 0; q < 10; q++) acc10[q] = wsum64(acc10[q]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wq[wv][q] = acc10[q];
    __syncthreads();
    if (threadIdx.x < 10) {
        unsigned long long s = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) s += wq[w][threadIdx.x];
        res->tstat[threadIdx.x] = s;
    }
    __syncthreads();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(res);
    uint32_t *dst = reinterpret_cast<uint32_t *>(host_res);
    for (uint32_t i = threadIdx.x; i < offsetof(DevRes, seq) / 4; i += blockDim.x) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&host_res->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* One pass over the final table: distinct k-mers, total, and the first- and
 * last-base marginals (-> depth-1 trie frequencies and base composition). */
__global__ void __launch_bounds__(256)
k_table_stats(uint32_t *table, uint64_t n, int k, DevRes *res,
              unsigned long long *acc, unsigned long long *facc, int fresh, DevRes *host_res, uint32_t *done,
              uint32_t seq, uint32_t *subs, int nsub, unsigned long long *part, int split,
              const unsigned long long *fz, const uint32_t *glist, const unsigned long long *perr) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            /* the segment's bound checks (k = 15, 16): the general tiles'
               list past its capacity, k_repart / k_count_parts past theirs */
            uint32_t f = perr ? (uint32_t)*perr : 0u;
            if (glist && glist[0] > glist[1]) f |= FK_FAULT_LIST;
            res->fault = f;
        }
        /* the feed's counters (facc, zero between feeds) join the engine's */
        if (threadIdx.x < ACC_N) {
            unsigned long long v = fresh ? 0ull : acc[threadIdx.x];
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) v += facc[c * ACC_N + threadIdx.x];
            acc[threadIdx.x] = v;
#pragma unroll
            for (int c = 0; c < FK_ACC_COPIES; c++) facc[c * ACC_N + threadIdx.x] = 0;
            res->acc[threadIdx.x] = v;
        }
        if (threadIdx.x == 0) res->need = 0;
    }
    unsigned long long dist = 0, sum = 0, last[4] = {0, 0, 0, 0}, first[4] = {0, 0, 0, 0};
    uint64_t n4 = n / 4;
    /* a fresh k = 15, 16 table whose statistics k_count_parts and
       k_list_add took: they stand unless k_redo changed it since */
    if (fz && res->redo_n == 0) {
        n4 = 0;
        if (threadIdx.x == 0) {
            for (uint32_t sl = blockIdx.x; sl < FZ_SLOTS; sl += gridDim.x) {
                const unsigned long long *z = fz + sl * 10u;
                dist += z[0]; sum += z[1];
                last[0] += z[2]; last[1] += z[3]; last[2] += z[4]; last[3] += z[5];
                first[0] += z[6]; first[1] += z[7]; first[2] += z[8]; first[3] += z[9];
            }
        }
    }
    uint4 *t4 = reinterpret_cast<uint4 *>(table);
    const int fs = 2 * (k - 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = t4[i];
        if (nsub) {
            /* fold k_count's sub-tables into the table (and clear them); all
               FK_SUBTABLES loads in flight at once */
            uint4 a[FK_SUBTABLES];
#pragma unroll
            for (int s = 0; s < FK_SUBTABLES; s++) a[s] = reinterpret_cast<uint4 *>(subs + (size_t)s * n)[i];
#pragma unroll
            for (int s = 0; s < FK_SUBTABLES; s++) {
                v.x += a[s].x; v.y += a[s].y; v.z += a[s].z; v.w += a[s].w;
                reinterpret_cast<uint4 *>(subs + (size_t)s * n)[i] = make_uint4(0, 0, 0, 0);
            }
            t4[i] = v;
        }
        dist += (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
        unsigned long long s4 = (unsigned long long)v.x + v.y + v.z + v.w;
        sum += s4;
        last[0] += v.x; last[1] += v.y; last[2] += v.z; last[3] += v.w;
        if (k == 1) {
            first[0] += v.x; first[1] += v.y; first[2] += v.z; first[3] += v.w;
        } else {
            uint32_t fd = (uint32_t)(((i * 4) >> fs) & 3);
            first[0] += fd == 0 ? s4 : 0; first[1] += fd == 1 ? s4 : 0;
            first[2] += fd == 2 ? s4 : 0; first[3] += fd == 3 ? s4 : 0;
        }
    }
    /* block partials (no same-address atomics across hundreds of blocks:
       the last block adds them up) */
    __shared__ unsigned long long wp[4][10];
    unsigned long long v10[10] = {dist, sum, last[0], last[1], last[2], last[3], first[0], first[1], first[2], first[3]};
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(v10[q]);
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wp[wv][q] = v10[q];
    __syncthreads();
    if (threadIdx.x < 10) {
        unsigned long long s = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) s += wp[w][threadIdx.x];
        part[(size_t)blockIdx.x * 10 + threadIdx.x] = s;
    }
    /* the last block to finish sums the partials, then publishes the whole
       result block to pinned host memory, sequence number last: the host
       spins on it instead of a copy plus a stream synchronisation.  With
       `split` (large tables: hundreds of blocks, whose release fences would
       each write back the L2 the table was just written into) the blocks
       stop here and k_table_final does that in a second launch. */
    if (split) return;
    __shared__ uint32_t is_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) is_last = atomicAdd(done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    stats_publish(res, host_res, part, gridDim.x, seq);
    if (threadIdx.x == 0) *done = 0;
}

__global__ void __launch_bounds__(256)
k_table_final(DevRes *res, DevRes *host_res, const unsigned long long *part, uint32_t nparts, uint32_t seq) {
    stats_publish(res, host_res, part, nparts, seq);
}

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

/* ------------------------------------------------------------------------- */
/* host engine                                                                */
/* ------------------------------------------------------------------------- */

#define HIPCHK(x)                                                               \
    do {                                                                        \
        hipError_t _e = (x);                                                    \
        if (_e != hipSuccess) {                                                 \
            fprintf(stderr, "findkmer: %s failed: %s (%s:%d)\n", #x,             \
                    hipGetErrorString(_e), __FILE__, __LINE__);                 \
            return FK_E_HIP;                                                    \
        }                                                                       \
    } while (0)

/* A scratch device allocation, freed on every return path (hipFree waits for
   the work queued on it). */
struct DevScratch {
    void *p = nullptr;
    size_t bytes = 0;
    DevScratch() = default;
    DevScratch(const DevScratch &) = delete;
    DevScratch &operator=(const DevScratch &) = delete;
    ~DevScratch() { release(); }
    bool alloc(size_t n) {
        release();
        if (hipMalloc(&p, n) != hipSuccess) { p = nullptr; return false; }
        bytes = n;
        return true;
    }
    void release() { if (p) hipFree(p); p = nullptr; bytes = 0; }
    template <class T> T *as() const { return (T *)p; }
};

static const uint64_t SEG_MAX_BYTES = 1ull << 34;                 /* 16 GiB per segment */
static const uint64_t STAGE_BYTES = 256ull << 20;                 /* host feed staging */
static const unsigned long long NO_EOF64 = ~0ull;

struct fk_engine {
    int dev = 0, k = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    fk_opts opts{};
    uint64_t nbins = 0, nshort = 0, maskk = 0;
    int cus = 256;
    uint32_t ts_blocks = 0;                   /* k_table_stats grid override (0 = default) */
    bool part = false;                        /* 8 <= k <= 13: partitioned counting (k_part) */
    bool sparse = false;                      /* 17 <= k <= 20: key-range passes at finish (k_sp_emit) */
    uint8_t *d_keep = nullptr;                /* sparse: the input fed so far */
    XState *d_kst = nullptr;                  /* sparse: every retained range's exact entering state */
    uint64_t keep_len = 0, keep_cap = 0, kst_len = 0, kst_cap = 0;
    struct SpSeg { uint64_t off, len, st, nranges, cpw, nchunks; };
    std::vector<SpSeg> spsegs;                /* the retained segments */
    /* the finished table, contiguous (the passes append in key order): keys
       ascending + u32 counts; kept across steps (grown, never shrunk), as are
       a pass's emitted keys and the dense bucket table */
    uint64_t *d_spk = nullptr;
    uint32_t *d_spc = nullptr;
    uint64_t spk_cap = 0, spc_cap = 0;
    uint64_t *d_emit = nullptr;
    uint64_t emit_cap = 0;
    unsigned long long *d_spdense = nullptr;
    uint64_t spdense_cap = 0;
    uint64_t sp_distinct = 0;
    uint64_t sp_pass = 0;                     /* FINDKMER_TUNE sp_pass: window keys per pass (0: by free HBM) */
    FksState fks;
    bool sp_done = false;                     /* d_spk / d_spc hold the finished table */
    unsigned long long sp_nodes = 0, sp_roll = 0, sp_tstat[10] = {};
    uint16_t *d_codes = nullptr;              /* k_part: block code regions */
    uint32_t *d_pflag = nullptr;              /* k_part: a range went to k_part<RES> */
    uint32_t *d_pidx = nullptr;               /* k_part: slice-major run index */
    uint64_t codes_cap = 0, pidx_cap = 0;
    uint32_t *d_pairs = nullptr;              /* k_part pairs mode: 4^(k+1) pair bins + 4^k single bins */
    uint16_t *d_parts = nullptr;              /* k = 15, 16: the second level's part streams (k_repart) */
    uint64_t parts_cap = 0;
    void *d_pmeta = nullptr;                  /* k = 15, 16: PartMeta per part + the allocation counter */
    int32_t *d_rsend = nullptr, *d_rrecv = nullptr;   /* routed sharded tables: blobs out / in (fk_engine_route_*) */
    uint64_t rsend_cap = 0, rrecv_cap = 0, rsend_words = 0;
    void *d_raux = nullptr;                   /* ... their per-destination geometry and slot offsets */
    uint64_t raux_cap = 0;
    int route_mode = 1;                       /* FINDKMER_TUNE route: 0 = reduce-scatter the table, 1 = route it
                                                 when world > 1 (at world 1 the reduce-scatter is a local copy,
                                                 ~11 ms less per k = 16 step), 2 = route at any world (tests) */
    uint64_t pair_cap = 0;
    uint32_t w16_ks = W16_KS_DEFAULT;         /* k (bits) counted through k_bucket16 (FINDKMER_TUNE w16=mask) */
    int part_pairs_kmax = 12;                 /* pairs mode for k <= this (FINDKMER_TUNE pairs_kmax; k = 12 pairs:
                                                 2048 slices of 32-code runs, half the entries of
                                                 512 single-window slices: 1 G-base step 1.63 -> 1.36 ms) */
    uint32_t general_tiles = FK_COUNT_GENERAL_TILES;   /* per range in k_count */
    /* device state */
    uint32_t *d_table = nullptr, *d_short = nullptr;
    uint32_t *d_sub = nullptr;                /* FK_SUBTABLES table copies k_count flushes into (LDS modes) */
    unsigned long long *d_acc = nullptr;      /* ACC_N, engine lifetime (+ ACC_N: d_facc) */
    unsigned long long *d_facc = nullptr;     /* FK_ACC_COPIES x ACC_N the counting kernels of a feed add into;
                                                 merged into d_acc by the feed's publisher, zero between feeds */
    /* one-pass k_count (k <= 7, entering state known) */
    bool onepass = true;                      /* k <= 7: k_count + k_tail in one pass */
    BlockSum *d_bsum = nullptr;               /* per block of k_count */
    uint32_t *d_ctl = nullptr;                /* k_tail's finished-block count */
    uint32_t ranges_per_wave = 1;             /* k <= 7: ranges per k_count wave slot */
    bool no_mixed = false;                    /* FINDKMER_TUNE no_mixed=1: no mixed tiles (general byte walk) */
    uint32_t part_general = 1;                /* k_part: general tiles per range (FINDKMER_TUNE part_general) */
    uint32_t static_pct = 100;                /* k <= 7: % of a large segment in static ranges (FINDKMER_TUNE static_pct;
                                                 100 = no dynamic ranges: on a plain stream the waves that
                                                 finish early hand their bandwidth to the others, so
                                                 balancing gains nothing -- 1 GB k=6 0.174 ms either way --
                                                 while header-dense input gains 9 % at 75) */
    uint32_t cls_w[4] = {1000, 1000, 1000, 1000};   /* static share per wave class, per mille */
    uint64_t dyn_min_chunks = 0;              /* segments with dynamic ranges: >= this many chunks (0: 8 per
                                                 wave slot; FINDKMER_TUNE dyn_min_chunks, tests) */
    OnePassCfg *d_opc = nullptr;
    bool op_pending = false;                  /* the last count_segment launched a one-pass k_count */
    bool op_fresh = false;                    /* ... which did a pending reset itself */
    /* a shard counted in one pass: its k_tail result (compact summary) */
    bool shard_op = false, shard_waited = false, shard_full = false, shard_resumed = false;
    int dev_ev = 2;                           /* event that ends the last feed's device path */
    DevRes *d_res = nullptr;                  /* per feed */
    unsigned long long *d_tmp = nullptr;      /* scratch counters */
    XState *d_state = nullptr;                /* entering state of the next feed */
    RangeRec *d_rr = nullptr;
    XState *d_rtrue = nullptr;
    uint32_t *d_redo = nullptr;
    ResumeRec *d_resume = nullptr;            /* ranges k_count hands to k_resume */
    TF *d_aggs = nullptr;                     /* k_scan block aggregates */
    uint32_t *d_flags = nullptr;              /* ... and their epoch flags */
    uint32_t scan_epoch = 0;
    TF *d_tf = nullptr;
    uint64_t range_cap = 0;
    uint8_t *d_stage = nullptr, *h_stage = nullptr;
    hipEvent_t ev[3] = {};
    bool times_pending = false;               /* ev[] of the last feed not yet read */
    bool timing = true;                       /* record ev[] (FINDKMER_TUNE events=0: off) */
    bool zero_pending = false;                /* reset() not yet issued to the device */
    DevRes *h_res = nullptr, *h_res_dev = nullptr;   /* pinned, mapped result block */
    uint32_t *d_done = nullptr;               /* k_table_stats finished-block count */
    unsigned long long *d_tpart = nullptr;    /* k_table_stats per-block partial sums */
    uint32_t res_seq = 0;
    /* host bookkeeping */
    XState state{0, 0, 0, 0};
    DevRes last{};                            /* last feed's results */
    bool stats_valid = false;                 /* last.tstat describes the table */
    bool tail_added = false;                  /* end-of-input short run recorded */
    uint64_t fed = 0, scanned = 0, chunks = 0, redo = 0;
    int ended = 0;                            /* a 0xFF byte ended the input */
    int shard_pending = 0;
    const uint8_t *shard_buf = nullptr;
    uint64_t shard_len = 0;
    int64_t shard_lo = 0;
    double dev_ms = 0, main_ms = 0;
    uint64_t timed_n = 0;                     /* launches main_ms covers */
    uint64_t launch_no = 0;                   /* counting launches, for timing_every */
    uint32_t timing_every = 1;
    bool cur_timed = true;                    /* the current feed's launches record events */
    std::vector<uint8_t> unknown_bytes;
    std::vector<uint64_t> unknown_pos;        /* collect_unknown = 2: their stream offsets */
    /* partitioned path near the reference's int32 seqSize zone: a segment
       whose guessed range states are mostly wrong is recounted from the exact
       states instead of cancelled range by range (resolve_and_fetch) */
    XState dstate_val{0, 0, 0, 0};            /* d_state to write before the next kernel that reads it */
    bool dstate_pending = false;
    bool dirty = false;                       /* table / short walks changed since the last reset */
    bool seg_clean = true;                    /* ... not before the current segment */
    bool tab_fresh = false;                   /* k = 15, 16: this segment's k_zero left the table out
                                                 (k_count_parts writes every bin, k_list_add the rest) */
    uint32_t *d_glist = nullptr;              /* ... the general tiles' windows: [0] count, [1] cap, indices */
    uint64_t glist_cap = 0;
    unsigned long long *d_fz = nullptr;       /* ... and its statistics from k_count_parts (FZ_SLOTS x 10) */
    bool fz_ready = false;                    /* the next launch_table_stats may take them */
    bool glist_live = false;                  /* ... and must check the general tiles' list for overflow */
    unsigned long long *d_perr = nullptr;     /* k = 15, 16: k_repart / k_count_parts bound-check bits */
    bool perr_live = false;                   /* ... set by the last launch_part, for the next statistics */
    uint64_t glist_force = 0;                 /* FINDKMER_TUNE glist_cap=N: the list's capacity (tests) */
    uint64_t list_recounts = 0;               /* segments counted again after the list overflowed */
    bool seg_snap = false;                    /* d_snap holds them as before the current segment */
    uint32_t *d_snap = nullptr;
    uint64_t snap_cap = 0;
    /* fk_engine_shard_exchange: gathered pack rows, pinned and mapped (word
       0: sequence number, rows from word 32) */
    uint32_t *h_rows = nullptr, *h_rows_dev = nullptr;
    uint32_t *d_rows = nullptr;               /* the stitched exchange's rows (device) */
    uint32_t rows_cap = 0, rows_seq = 0;
};

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
static int flush_state(fk_engine *e) {
    if (!e->dstate_pending) return FK_OK;
    e->dstate_pending = false;
    hipLaunchKernelGGL(k_set_state, dim3(1), dim3(1), 0, e->stream, e->d_state, e->dstate_val);
    HIPCHK(hipGetLastError());
    return FK_OK;
}
static hipError_t write_dstate(fk_engine *e, const XState &x) {
    e->dstate_pending = false;
    return hipMemcpyAsync(e->d_state, &x, sizeof x, hipMemcpyHostToDevice, e->stream);
}

static int flush_zero(fk_engine *e, bool keep_table = false) {
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
static int set_dev(fk_engine *e, bool flush = true) {
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

static int hist_mode(const fk_engine *e) {
    return e->sparse ? H_SPARSE : e->k <= 6 ? H_PAIRS : e->k == 7 ? H_LDS : H_GLOBAL;
}

/* 128 VGPRs -> 4 waves/SIMD = two 512-thread blocks per CU */
static uint64_t blocks_per_cu(const fk_engine *) { return 2; }

static size_t lds_bytes(const fk_engine *e) {
    int m = hist_mode(e);
    if (m == H_PAIRS) return ((size_t)e->nbins * 4 + e->nbins) * sizeof(uint32_t);
    if (m == H_LDS) return (size_t)e->nbins * sizeof(uint32_t);
    return 0;
}

/* Zero table, counters and the stream state (asynchronous, stream-ordered). */
/* a sparse buffer of at least `n` elements of `sz` bytes (contents dropped) */
static int sp_ensure(void **p, uint64_t *cap, uint64_t n, size_t sz) {
    if (*p && *cap >= n) return FK_OK;
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t c = std::max<uint64_t>(n, 1024);
    if (hipMalloc(p, c * sz) != hipSuccess) return FK_E_OOM;
    *cap = c;
    return FK_OK;
}

static int zero_all(fk_engine *e) {
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
    hipFree(e->d_parts); hipFree(e->d_pmeta); hipFree(e->d_glist); hipFree(e->d_fz);
    hipFree(e->d_rsend); hipFree(e->d_rrecv); hipFree(e->d_raux);
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

/* the LDS-counting kernels keep their bins at LDS address 0 (lds_add) */
static bool lds_layout_ok() {
    static int ok = -1;
    if (ok < 0) {
        const void *fns[] = {(const void *)k_count<H_PAIRS>, (const void *)k_count<H_LDS>,
                             (const void *)k_resume<H_PAIRS>, (const void *)k_resume<H_LDS>,
                             (const void *)k_redo<H_PAIRS>, (const void *)k_redo<H_LDS>};
        int good = 1;
        for (const void *f : fns) {
            hipFuncAttributes a;
            if (hipFuncGetAttributes(&a, f) != hipSuccess || a.sharedSizeBytes != 0) good = 0;
        }
        ok = good;
    }
    return ok == 1;
}

/* One knob of FINDKMER_TUNE ("name=value,name=value"): true and *v = value
   when `name` is set. */
static bool tune_knob(const char *name, uint64_t *v) {
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
       ones take the dense path) */
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
    /* the LDS bins need more than the default dynamic-LDS limit */
    size_t sh = lds_bytes(e);
    if (sh > 65536) {
        hipFuncSetAttribute((const void *)k_count<H_PAIRS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipFuncSetAttribute((const void *)k_redo<H_PAIRS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        hipFuncSetAttribute((const void *)k_resume<H_PAIRS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    }
    if (e->part)   /* k_bucket_count: one 2^15-bin slice + its 2^13 single bins (160 KiB) in LDS */
        for (const void *f : {(const void *)k_bucket_count<BK_PLAIN>, (const void *)k_count_parts,
                              (const void *)k_bucket_count<BK_PAD>, (const void *)k_bucket16<true>,
                              (const void *)k_bucket16<false>})
            /* (k_bucket16: 128 KiB of bins beside its static reduction words) */
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (f == (const void *)k_bucket16<true> || f == (const void *)k_bucket16<false>)
                                        ? 1 << 17 : 5 << 15) != hipSuccess) {
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
static int grow_arrays(fk_engine *e, uint64_t nranges) {
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

/* A segment's decomposition into per-wave chunk ranges. */
struct Geo {
    uint64_t nchunks, cpw, nranges;
    uint64_t nstatic;     /* static ranges (one per k_count wave) */
    DynGeo dg;            /* the dynamic ranges after them (k <= 7) */
    unsigned grid;        /* k_count's blocks */
    unsigned rgrid;       /* blocks of the one-wave-per-range kernels (k_resume, k_redo) */
};
/* k_part's waves per block: 16 for the tables of 512 slices or more (one
   block per CU: only 16-wave blocks have the LDS for their cursors, PART_SM),
   else 8 (two per CU; 16 measured 1-5 % slower for k = 8..10, rounds 2, 3) */
static uint32_t part_waves_of(const fk_engine *e) { return e->k >= 11 ? 16u : 8u; }

static Geo geometry(const fk_engine *e, uint64_t len) {
    Geo g;
    g.nchunks = (len + FK_CHUNK_BYTES - 1) / FK_CHUNK_BYTES;
    uint64_t max_waves = (uint64_t)e->cus * blocks_per_cu(e) * FK_WAVES_PER_BLOCK;
    /* k_part: one range per wave of its blocks, the blocks one round over the CUs */
    if (e->part) max_waves = (uint64_t)e->cus * part_waves_of(e) * (part_waves_of(e) >= 16u ? 1u : 2u);
    /* k <= 7 (k_count counts in LDS): ranges_per_wave ranges per wave slot
       of the chip, i.e. that many rounds of blocks (experiment knob, default
       1).  Equal static ranges finish up to 35 % apart (tools/wave_times.py:
       per-XCD means differ by ~18 %), but more rounds of smaller blocks do
       not fix it -- the dispatcher deals blocks to the XCDs round-robin --
       and cost LDS zero/flush per block: 4 rounds 0.29 ms vs 0.18 ms. */
    if (!e->part && !e->sparse && LDS_MODE(hist_mode(e))) max_waves *= e->ranges_per_wave;
    memset(&g.dg, 0, sizeof g.dg);
    g.dg.nchunks = g.nchunks;
    const uint64_t min_chunks = e->dyn_min_chunks ? e->dyn_min_chunks : 8 * max_waves;
    const bool dyn = !e->part && !e->sparse && LDS_MODE(hist_mode(e)) && e->static_pct < 100 &&
                     g.nchunks >= std::max<uint64_t>(min_chunks, 4);
    if (dyn) {
        /* static ranges cover static_pct % of the segment (one per wave, or
           fewer for a short segment); the rest is cut into dynamic ranges of
           4u, 2u and u chunks (half, a quarter and a quarter of it), u chosen
           so that there are at most ~16 K of them */
        const uint64_t sc = std::max<uint64_t>(1, g.nchunks * e->static_pct / 100);
        g.cpw = std::max<uint64_t>(1, sc / max_waves);
        g.nstatic = std::min<uint64_t>(max_waves, sc / g.cpw);
        DynGeo &d = g.dg;
        const uint64_t grid = (g.nstatic + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK;
        /* one pool per pair of k_count blocks (the blocks one CU holds) */
        d.npools = (uint32_t)std::min<uint64_t>(FK_MAX_POOLS, std::max<uint64_t>(1, grid / blocks_per_cu(e)));
        for (int c = 0; c < 4; c++) d.cls[c] = (uint32_t)g.cpw;
        if (g.nstatic == max_waves && grid == 2ull * d.npools) {
            /* weighted static ranges per wave class (cls_w, per mille) */
            const uint64_t wsum = e->cls_w[0] + e->cls_w[1] + e->cls_w[2] + e->cls_w[3];
            const uint64_t avg = sc / max_waves;
            uint64_t tot = 0;
            for (int c = 0; c < 4; c++) {
                d.cls[c] = (uint32_t)std::max<uint64_t>(1, avg * e->cls_w[c] * 4 / wsum);
                tot += d.cls[c];
            }
            if (tot * (max_waves / 4) >= g.nchunks)
                for (int c = 0; c < 4; c++) d.cls[c] = (uint32_t)g.cpw;   /* keep a dynamic part */
        }
        const uint64_t stot = (uint64_t)d.npools * (4ull * d.cls[0] + 4ull * d.cls[1]) +
                              (grid - std::min<uint64_t>(grid, d.npools)) * (4ull * d.cls[2] + 4ull * d.cls[3]);
        const bool uniform = d.cls[0] == d.cls[1] && d.cls[1] == d.cls[2] && d.cls[2] == d.cls[3];
        d.base = uniform ? g.nstatic * g.cpw : stot;
        const uint64_t D = g.nchunks - d.base;
        const uint64_t u = std::max<uint64_t>(1, (D + 2 * FK_DYN_TARGET - 1) / (2 * FK_DYN_TARGET));
        d.sz[0] = (uint32_t)(4 * u); d.sz[1] = (uint32_t)(2 * u); d.sz[2] = (uint32_t)u;
        d.n[0] = (uint32_t)(D / 2 / d.sz[0]);
        d.n[1] = (uint32_t)(D / 4 / d.sz[1]);
        const uint64_t rem = D - (uint64_t)d.n[0] * d.sz[0] - (uint64_t)d.n[1] * d.sz[1];
        d.n[2] = (uint32_t)((rem + u - 1) / u);
        d.ndyn = d.n[0] + d.n[1] + d.n[2];
    } else {
        g.cpw = std::max<uint64_t>(1, (g.nchunks + max_waves - 1) / max_waves);
        g.nstatic = (g.nchunks + g.cpw - 1) / g.cpw;
    }
    g.nranges = g.nstatic + g.dg.ndyn;
    g.grid = (unsigned)std::max<uint64_t>(1, (g.nstatic + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK);
    g.rgrid = (unsigned)std::max<uint64_t>(1, (g.nranges + FK_WAVES_PER_BLOCK - 1) / FK_WAVES_PER_BLOCK);
    return g;
}

#define FK_DISPATCH(HMV, ...)                                                   \
    switch (HMV) {                                                              \
    case H_PAIRS: { constexpr int HM = H_PAIRS; __VA_ARGS__; } break;          \
    case H_LDS: { constexpr int HM = H_LDS; __VA_ARGS__; } break;              \
    case H_SPARSE: { constexpr int HM = H_SPARSE; __VA_ARGS__; } break;        \
    default: { constexpr int HM = H_GLOBAL; __VA_ARGS__; } break;              \
    }
/* the counting passes of k_count / k_resume: state only (H_NONE) when the
   partitioned path (k_part) does the counting */
#define FK_DISPATCH_COUNT(e, ...)                                               \
    if ((e)->part || (e)->sparse) { constexpr int HM = H_NONE; __VA_ARGS__; }   \
    else FK_DISPATCH(hist_mode(e), __VA_ARGS__)

/* the timing events of a launch (none when timing is off) */
static hipEvent_t tev(const fk_engine *e, int i) { return e->timing && e->cur_timed ? e->ev[i] : nullptr; }

static int launch_count(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g,
                        int has_init, bool onepass = false, bool fresh = false, bool shard = false) {
    size_t sh = lds_bytes(e);
    const uint32_t flags = (onepass ? (OP_ON | (fresh ? OP_FRESH : 0u) | (shard ? OP_SHARD : 0u)) : 0u) |
                           (e->no_mixed ? (uint32_t)OP_NOMIX : 0u);
    FK_DISPATCH_COUNT(e,
                hipExtLaunchKernelGGL((k_count<HM>), dim3(g.grid), dim3(FK_BLOCK), sh, e->stream, tev(e, 0), tev(e, 1),
                                      0, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr,
                                   g.nchunks, e->d_state, has_init, g.cpw, e->d_resume, e->general_tiles,
                                   e->d_sub, e->d_opc, flags, g.nstatic, g.dg, e->d_ctl + FK_HEADS_OFF));
    HIPCHK(hipGetLastError());
    if (onepass) {
        if (++e->res_seq == 0) e->res_seq = 1;
        /* one chain item per thread: the block summaries, then the dynamic ranges */
        const uint64_t items = (uint64_t)g.grid + g.dg.ndyn;
        const unsigned tb = (unsigned)std::max<uint64_t>(TAIL_BLOCKS, (items + TAIL_THREADS - 1) / TAIL_THREADS);
        hipExtLaunchKernelGGL(k_tail, dim3(tb), dim3(TAIL_THREADS), 0, e->stream, nullptr, tev(e, 2), 0,
                              e->d_opc, flags, e->res_seq, e->d_table, e->k, e->d_sub, e->d_facc, e->d_res,
                              e->d_state, g.grid, len, reinterpret_cast<TailPart *>(e->d_tpart), e->d_ctl,
                              e->d_rr, g.nstatic, g.dg.ndyn);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

static int launch_resume(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
    size_t sh = lds_bytes(e);
    FK_DISPATCH_COUNT(e,
                hipLaunchKernelGGL((k_resume<HM>), dim3(g.rgrid), dim3(FK_BLOCK), sh, e->stream, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nranges,
                                   e->d_resume, e->d_ctl + FK_HEADS_OFF, e->no_mixed ? 0 : 1));
    HIPCHK(hipGetLastError());
    return FK_OK;
}

static int launch_redo(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int mode) {
    size_t sh = lds_bytes(e);
    FK_DISPATCH(hist_mode(e),
                hipLaunchKernelGGL((k_redo<HM>), dim3(g.rgrid), dim3(FK_BLOCK), sh, e->stream, buf, len, lo, e->k,
                                   e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr,
                                   e->d_rtrue, e->d_redo, g.nranges, mode, e->no_mixed ? 0 : 1));
    HIPCHK(hipGetLastError());
    return FK_OK;
}


static int launch_scan(fk_engine *e, const Geo &g, int mode) {
    {
        const int rc = flush_state(e);
        if (rc) return rc;
    }
    const unsigned blocks = (unsigned)((g.nranges + SCAN_THREADS - 1) / SCAN_THREADS);
    if (++e->scan_epoch == 0) {   /* flags hold epochs; never reuse 0 */
        HIPCHK(hipMemsetAsync(e->d_flags, 0, e->range_cap / SCAN_THREADS * sizeof(uint32_t) + 64, e->stream));
        e->scan_epoch = 1;
    }
    hipLaunchKernelGGL(k_scan, dim3(blocks), dim3(SCAN_THREADS), 0, e->stream, e->d_rr, g.nranges, e->d_state,
                       e->d_rtrue, e->d_redo, e->d_res, e->k, mode, e->d_tf, e->d_aggs, e->d_flags, e->scan_epoch);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* Table statistics and an accumulator snapshot into d_res, published to the
   pinned host copy (e->h_res) with a new sequence number.  The feed path's
   k_count has zeroed the sums already; other callers ask for a memset.
   `stop` (optional) is recorded when the kernel completes. */
static int launch_table_stats(fk_engine *e, bool zero_first, hipEvent_t stop = nullptr, bool subs = true,
                              bool fresh = false) {
    if (zero_first) HIPCHK(hipMemsetAsync(e->d_res->tstat, 0, sizeof(e->d_res->tstat), e->stream));
    unsigned gd = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 4, (e->nbins / 4 + 255) / 256 + 1);
    if (e->ts_blocks) gd = std::min<unsigned>(e->ts_blocks, (unsigned)e->cus * 4);
    const int split = gd > 16;   /* large tables: partials, then k_table_final */
    if (++e->res_seq == 0) e->res_seq = 1;
    const bool fz = e->fz_ready;   /* only for the statistics right after a fresh two-level count */
    e->fz_ready = false;
    const bool gl = fz || e->glist_live;
    e->glist_live = false;
    unsigned long long *perr = e->perr_live ? e->d_perr : nullptr;
    e->perr_live = false;
    hipExtLaunchKernelGGL(k_table_stats, dim3(gd), dim3(256), 0, e->stream, nullptr, split ? nullptr : stop, 0,
                          e->d_table, e->nbins, e->k, e->d_res, e->d_acc, e->d_facc, fresh ? 1 : 0, e->h_res_dev,
                          e->d_done, e->res_seq, e->d_sub, (subs && e->d_sub) ? FK_SUBTABLES : 0, e->d_tpart, split,
                          fz ? (const unsigned long long *)e->d_fz : nullptr, gl ? (const uint32_t *)e->d_glist : nullptr,
                          (const unsigned long long *)perr);
    HIPCHK(hipGetLastError());
    if (split) {
        hipExtLaunchKernelGGL(k_table_final, dim3(1), dim3(256), 0, e->stream, nullptr, stop, 0, e->d_res,
                              e->h_res_dev, e->d_tpart, gd, e->res_seq);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

/* Wait for the result block published by the last launch_table_stats() and
   copy it to e->last: spin on its sequence number in pinned memory, checking
   the stream for errors now and then. */
static int wait_results(fk_engine *e) {
    const uint32_t want = e->res_seq;
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&e->h_res->seq, __ATOMIC_ACQUIRE) == want) break;
        if ((spin & 4095) == 0) {
            hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(&e->h_res->seq, __ATOMIC_ACQUIRE) == want) break;
                return FK_E_HIP;   /* stream drained without publishing */
            }
            if (q != hipErrorNotReady) return FK_E_HIP;
        }
        __builtin_ia32_pause();
    }
    memcpy(&e->last, e->h_res, sizeof(DevRes));
    return FK_OK;
}

/* k_part + k_bucket_count over a resolved segment (exact range states in
   d_rtrue): the counting of the partitioned path */
static int launch_part(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g, int has_init,
                       const XState *exact = nullptr) {
    PartGeo pg;
    const int k = e->k;
    /* k <= 12: (k+1)-mer pairs at every other base (half the entries), plus
       the single k-mers at the first slot of halves with a '\n' */
    const bool pairs = k <= e->part_pairs_kmax;
    const int kb = pairs ? k + 1 : k;                      /* bits of a pair (or window) code: 2 kb */
    /* >= 64 slices, <= 2^15 bins (128 KiB) each; k = 14: 2^16 codes per slice,
       counted as two halves (PART_BIG); k = 15, 16: 2048 coarse slices of
       2^19 / 2^21 32-bit codes, counted in 2^15-bin parts */
    const bool c32 = k >= 15;
    /* 2^16-bin slices counted in 16-bit LDS bins (k_bucket16) for the k in
       e->w16_ks (12 <= k <= 14) */
    const bool w16 = !c32 && k >= 12 && ((e->w16_ks >> k) & 1u);
    pg.w16 = w16 ? 1u : 0u;
    pg.sh = c32 ? 2 * k - 11 : w16 ? 16 : std::min(15, 2 * kb - 6);
    pg.split = c32 ? (uint32_t)(pg.sh - 15) : 0u;
    pg.npair = pairs ? 1u << (2 * kb - pg.sh) : 0u;
    if (pairs && w16) {
        /* the single k-mers in their own 2^16-bin slices after the pair slices */
        pg.sbase = pg.npair;
        pg.slsh = 0;
        pg.sflag = 0;
        pg.nbk = pg.npair + (1u << (2 * k - 16));
        /* (k = 12: 1280 slices in an index row of 2048, the width k_part's
           all-wave scan divides among its 16 waves) */
        pg.nslices = pg.nbk <= 512u ? pg.nbk : (pg.nbk + 1023u) & ~1023u;
    } else {
        /* singles filed under the pair code x << 2 (PART_SINGLE) */
        pg.sbase = 0;
        pg.slsh = 2;
        pg.sflag = PART_SINGLE;
        pg.nslices = pairs ? pg.npair : 1u << (2 * k - pg.sh);
        pg.nbk = pg.nslices;
    }
    pg.pairs = pg.singles = nullptr;
    pg.nomix = e->no_mixed ? 1u : 0u;
    pg.glist = nullptr;
    pg.fz = nullptr;
    pg.kk = (uint32_t)k;
    e->fz_ready = false;
    e->glist_live = false;
    if ((c32 || w16) && e->tab_fresh && !exact) {
        /* the general tiles' windows go to a list (hist_add): at most
           part_general + 3 general tiles per range (the comment lines or run
           breaks k_part takes and the bases-only tiles around them, the
           ragged last tile in k_part<RES>; tile_mixed takes every other tile
           outside the int32 zone, which tab_fresh excludes, and with
           no_mixed there is no fresh table).  Should a segment hold more,
           hist_add drops what does not fit and k_table_stats flags it
           (FK_FAULT_LIST): resolve_and_fetch counts the segment again */
        uint64_t cap = (uint64_t)g.nranges * (e->part_general + 3u) * FK_TILE_BYTES + 4096u;
        if (e->glist_force) cap = e->glist_force;
        if (cap + 2 > e->glist_cap) {
            hipFree(e->d_glist);
            e->d_glist = nullptr;
            e->glist_cap = 0;
            if (hipMalloc((void **)&e->d_glist, (cap + 2) * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
            e->glist_cap = cap + 2;
        }
        if (!e->d_fz && hipMalloc((void **)&e->d_fz, FZ_SLOTS * 10 * sizeof(unsigned long long)) != hipSuccess)
            return FK_E_OOM;
        hipLaunchKernelGGL(k_list_init, dim3(1), dim3(256), 0, e->stream, e->d_glist, (uint32_t)cap, e->d_fz);
        HIPCHK(hipGetLastError());
        pg.glist = e->d_glist;
        pg.fz = e->d_fz;
        /* the statistics: k_count_parts / k_bucket16 take them (pairs mode:
           k_table_stats reads the folded table) */
        e->fz_ready = !pairs;
        e->glist_live = true;
    }
    e->tab_fresh = false;
    if (pairs) {
        const uint64_t need = e->nbins * 5;                 /* 4^(k+1) pair bins + 4^k single bins */
        if (need > e->pair_cap) {
            hipFree(e->d_pairs);
            e->d_pairs = nullptr;
            if (hipMalloc((void **)&e->d_pairs, need * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
            e->pair_cap = need;
        }
        pg.pairs = e->d_pairs;
        pg.singles = e->d_pairs + e->nbins * 4;
    }
    pg.rounds = (uint32_t)((g.cpw * FK_CHUNK_TILES + 2) / PART_TILES3(pairs, c32) + 2);   /* rows (batches) per block */
    /* block size: 16 waves (larger batches, longer runs for k_bucket_count)
       for the tables of 512 slices or more, else 8 */
    const uint32_t W = part_waves_of(e);
    pg.batch = c32 ? W * FK_TILE_BYTES : PART_MAX_BATCH_W(W);   /* entries per row slot */
    const unsigned pgrid = (unsigned)((g.nranges + W - 1) / W);   /* the same ranges as k_count's waves */
    pg.rows = pgrid * pg.rounds;
    /* mixed tiles: ranges past their general tiles go to k_part<RES>, whose
       rows (region 2, as many as k_part's) follow k_part's */
    const bool mixed = !e->no_mixed;
    /* one comment line (or run break) per range stays here; a second one
       sends the range to k_part<RES>, whose block-wide rounds only pay off
       when many ranges go there */
    pg.general = e->part_general;
    pg.stride = mixed ? 2 * pg.rows : pg.rows;
    if (!e->d_pflag && hipMalloc((void **)&e->d_pflag, 64) != hipSuccess) return FK_E_OOM;
    pg.flag = e->d_pflag;
    HIPCHK(hipMemsetAsync(e->d_pflag, 0, sizeof(uint32_t), e->stream));
    /* runs padded to 16-B pieces (PART_PAD: the instances of at most 512
       slices, i.e. the 8-wave blocks of k <= 10 and k = 11's pairs): the row
       slot grows by one pad piece per slice */
    const bool padded = !c32 && k != 14 && (W == 8u || (k == 11 && pairs));
    if (padded) pg.batch += PART_ROW_PAD(W == 8u ? PART_SM(8u) : PART_PAD_MAX_SM) / 2u;
    const uint64_t ncodes = (uint64_t)pg.stride * pg.batch * (c32 ? 2u : 1u),
                   nidx = (uint64_t)pg.nslices * pg.stride;
    if (ncodes > e->codes_cap) {
        hipFree(e->d_codes);
        e->d_codes = nullptr;
        if (hipMalloc((void **)&e->d_codes, ncodes * sizeof(uint16_t)) != hipSuccess) return FK_E_OOM;
        e->codes_cap = ncodes;
    }
    if (nidx > e->pidx_cap) {
        hipFree(e->d_pidx);
        e->d_pidx = nullptr;
        if (hipMalloc((void **)&e->d_pidx, nidx * sizeof(uint32_t)) != hipSuccess) return FK_E_OOM;
        e->pidx_cap = nidx;
    }
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    /* the main pass: pipelined batches (PIPE) for k = 8..13 (<= 512 slices,
       wave 0 scanning alone; k = 12 pairs and k = 13: 2048 slices, the scan
       over all waves), phase by phase for k = 14 (PART_BIG) and k = 15, 16
       (C32); the headline k = 11 with k a compile-time constant */
    auto kmain = c32 ? k_part<false, false, 16u, PART_SM(16u), true>
                 : k == 14 ? k_part<false, false, 16u, PART_BIG>
                 : W == 16u ? (pairs ? (k == 11 ? k_part<true, false, 16u, PART_PAD_MAX_SM, false, true, 11u>
                                                : k_part<true, false, 16u, PART_SM(16u), false, true>)
                                     : k_part<false, false, 16u, PART_SM(16u), false, true>)
                            : (pairs ? k_part<true, false, 8u, PART_SM(8u), false, true>
                                     : k_part<false, false, 8u, PART_SM(8u), false, true>);
    hipExtLaunchKernelGGL(kmain, dim3(pgrid), dim3(PART_BLOCK_W(W)), 0, e->stream, tev(e, 0), tev(e, 1), 0, buf, len,
                          lo, e->k, e->maskk, e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nchunks, g.cpw,
                          e->d_state, has_init, pg, e->d_resume, exact);
    HIPCHK(hipGetLastError());
    if (mixed) {
        auto kres = c32 ? k_part<false, true, 16u, PART_SM(16u), true>
                    : k == 14 ? k_part<false, true, 16u, PART_BIG>
                    : W == 16u ? (pairs ? (k == 11 ? k_part<true, true, 16u, PART_PAD_MAX_SM> : k_part<true, true, 16u>)
                                        : k_part<false, true, 16u>)
                               : (pairs ? k_part<true, true, 8u> : k_part<false, true, 8u>);
        hipLaunchKernelGGL(kres, dim3(pgrid), dim3(PART_BLOCK_W(W)), 0, e->stream, buf, len, lo, e->k, e->maskk,
                           e->d_table, e->d_short, e->d_facc, e->d_res, e->d_rr, g.nchunks, g.cpw, e->d_state,
                           has_init, pg, e->d_resume, exact);
        HIPCHK(hipGetLastError());
    } else {
        pg.flag = nullptr;
    }
    const uint32_t groups = w16 ? 1u : std::max<uint32_t>(1, (uint32_t)e->cus / pg.nslices);
    if (pairs && groups > 1) HIPCHK(hipMemsetAsync(e->d_pairs, 0, e->nbins * 5 * sizeof(uint32_t), e->stream));
    const size_t bc_lds = ((size_t)1 << (pg.sh - pg.split)) * sizeof(uint32_t) * (pairs ? 5 : 4) / 4;   /* + single bins */
    if (c32) {
        /* the second partition level: each coarse slice's runs into one
           contiguous 16-bit stream per part, then one block per part */
        const uint64_t nparts = (uint64_t)pg.nslices << pg.split;
        const uint64_t need = len + 8 * nparts + 16;   /* (entries <= bytes; 8-aligned parts) */
        if (need > e->parts_cap) {
            hipFree(e->d_parts);
            e->d_parts = nullptr;
            e->parts_cap = 0;
            if (hipMalloc((void **)&e->d_parts, need * sizeof(uint16_t)) != hipSuccess) return FK_E_OOM;
            e->parts_cap = need;
        }
        if (!e->d_pmeta &&
            hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
            return FK_E_OOM;
        PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
        /* [0]: the output claim, [1]: bound-check bits (DevRes::fault) */
        unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
        e->d_perr = alloc + 1;
        e->perr_live = true;
        HIPCHK(hipMemsetAsync(alloc, 0, 2 * sizeof(unsigned long long), e->stream));
        /* k = 15 (16 parts a slice): 8 slices per block, one block per CU
           (4.27 ms per G-base against 4.68 with two blocks of 4) */
        if (pg.split <= 4)
            hipLaunchKernelGGL((k_repart<uint16_t, 8u>), dim3(pg.nslices / 8u), dim3(1024), 0, e->stream, pg,
                               e->d_parts, alloc, meta, (uint64_t)e->parts_cap, e->d_perr, 15u, nullptr);
        else
            hipLaunchKernelGGL(k_repart<uint16_t>, dim3(pg.nslices / REPART_G), dim3(1024), 0, e->stream, pg,
                               e->d_parts, alloc, meta, (uint64_t)e->parts_cap, e->d_perr, 15u, nullptr);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_count_parts, dim3((unsigned)nparts), dim3(1024), (size_t)1 << 17, e->stream, pg,
                           (const uint16_t *)e->d_parts, (const PartMeta *)meta, e->d_table, (uint64_t)e->parts_cap,
                           e->d_perr);
        if (pg.glist) {
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
        }
    } else if (w16) {
        if (padded)
            hipLaunchKernelGGL(k_bucket16<true>, dim3(pg.nbk), dim3(1024), (size_t)1 << 17, e->stream, pg, e->d_table);
        else
            hipLaunchKernelGGL(k_bucket16<false>, dim3(pg.nbk), dim3(1024), (size_t)1 << 17, e->stream, pg, e->d_table);
        if (pg.glist && !pairs) {   /* (pairs mode: after k_pair_fold below) */
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
        }
    } else if (padded) {
        hipLaunchKernelGGL(k_bucket_count<BK_PAD>, dim3(pg.nslices * groups), dim3(1024), bc_lds, e->stream, pg,
                           groups, e->d_table);
    } else
        hipLaunchKernelGGL(k_bucket_count<BK_PLAIN>, dim3(pg.nslices * groups), dim3(1024), bc_lds, e->stream, pg,
                           groups, e->d_table);
    HIPCHK(hipGetLastError());
    if (pairs) {
        const unsigned fg = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 4, (e->nbins + 255) / 256);
        hipLaunchKernelGGL(k_pair_fold, dim3(fg), dim3(256), 0, e->stream, e->d_pairs, e->d_pairs + e->nbins * 4,
                           e->nbins, e->d_table, pg.glist ? 1 : 0);
        HIPCHK(hipGetLastError());
        if (pg.glist) {
            hipLaunchKernelGGL(k_list_add, dim3((unsigned)e->cus * 4), dim3(256), 0, e->stream, pg.glist, e->d_table,
                               k, pg.fz);
            HIPCHK(hipGetLastError());
        }
    }
    return FK_OK;
}

/* scan + redo (or the partitioned count) + table stats, then the results */
/* Can a run reach the reference's int32 seqSize zone (findKmer.cpp:977) in
   a segment of len bytes entered in state e->state? */
static bool int32_zone_possible(const fk_engine *e, uint64_t len) {
    const uint64_t r0 = e->state.hdr ? 0 : (uint64_t)(uint32_t)e->state.R;
    return r0 + len + FK_CHUNK_BYTES > 0x7FFFFFFFull;
}

/* What the segment's device-side bound checks saw (DevRes::fault, k = 15,
   16).  A general-tile list that overflowed left windows out of a fresh
   table: the segment is the first since the reset (tab_fresh), so it is
   counted again over a zeroed table from the exact range states k_scan just
   computed, its general tiles' windows added by global atomics (launch_part
   with `exact` keeps no list).  Any other bit fails the feed. */
static int check_fault(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
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

static int resolve_and_fetch(fk_engine *e, const uint8_t *buf, uint64_t len, int64_t lo, const Geo &g) {
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

static int exact_eof(fk_engine *e, const Geo &g, unsigned long long &eof) {
    HIPCHK(hipMemsetAsync(e->d_tmp, 0xFF, sizeof(unsigned long long), e->stream));
    unsigned gr = (unsigned)std::min<uint64_t>(1024, g.nranges / 256 + 1);
    hipLaunchKernelGGL(k_obs_eof, dim3(gr), dim3(256), 0, e->stream, e->d_rr, g.nranges, e->d_tmp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&eof, e->d_tmp, sizeof eof, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* Collect the unknown bytes of the just-counted segment (stream order). */
static int collect_unknown(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g) {
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
static void add_times(fk_engine *e) { e->times_pending = e->timing && e->cur_timed; }
static void settle_times(fk_engine *e, bool wait) {
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
static int count_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, int has_init, Geo &g,
                         bool shard = false) {
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
static int finish_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, int64_t lo, const Geo &g,
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
static int sp_grow(fk_engine *e, void **buf, uint64_t *cap, uint64_t used, uint64_t need) {
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
static int sp_retain(fk_engine *e, const uint8_t *dbuf, uint64_t len, const Geo &g) {
    int rc = sp_grow(e, (void **)&e->d_keep, &e->keep_cap, e->keep_len, e->keep_len + len + 16);
    if (rc) return rc;
    const uint64_t sb = g.nranges * sizeof(XState);
    rc = sp_grow(e, (void **)&e->d_kst, &e->kst_cap, e->kst_len * sizeof(XState), (e->kst_len + g.nranges) * sizeof(XState));
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(e->d_keep + e->keep_len, dbuf, len, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->d_kst + e->kst_len, e->d_rtrue, sb, hipMemcpyDeviceToDevice, e->stream));
    e->spsegs.push_back({e->keep_len, len, e->kst_len, g.nranges, g.cpw, g.nchunks});
    /* segments start 16-B aligned in d_keep (load_lane's vector loads; it
       never reads past a segment's end), so small feeds cost little */
    e->keep_len += (len + 15) / 16 * 16;
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
static int sparse_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len, bool prefix = false) {
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

static int process_segment(fk_engine *e, const uint8_t *dbuf, uint64_t len) {
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
static uint64_t segment_budget(fk_engine *e, uint64_t len) {
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
        for (uint64_t off = 0; off < len && !e->ended; off += seg) {
            rc = process_segment(e, buf + off, std::min(seg, len - off));
            if (rc) return rc;
        }
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
static int shard_wait(fk_engine *e) {
    if (!e->shard_op || e->shard_waited) return FK_OK;
    int rc = wait_results(e);
    if (rc) return rc;
    e->shard_waited = true;
    return FK_OK;
}

/* the full transfer function of a one-pass shard (k_resume if a range ran
   out of general tiles, then k_scan mode 1) into d_tf */
static int shard_full_tf(fk_engine *e) {
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

#define FK_SUMMARY_COMPACT 0x434F4D50414354ull   /* "COMPACT": tag in w[11] */

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
static bool compact_apply(const fk_summary *s, const XState &in, XState &out) {
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
        return sparse_segment(e, e->shard_buf, e->shard_len);
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

/* ---- one-collective shard exchange ---- */

/* The pending one-pass shard's result into a caller's merge buffer: the
 * table (every block, 16-B pieces), the counters as 16-bit limbs and the
 * pack rows (block 0).  `valid`: the host knows the shard went through
 * k_count + k_tail; the device adds k_tail's verdict (no ONE_* bits, no
 * 0xFF candidate).  The counter values are fk_engine_finish's formulas. */
__global__ void __launch_bounds__(1024)
k_shard_pack(const DevRes *res, const uint32_t *table, uint64_t nbins, uint32_t *dt, int32_t *dc, uint32_t *rows,
             int nrows, int slot, int is_last, int valid, uint64_t len, int k) {
    const bool ok = valid && res->need == 0 && res->eof_cand == ~0ull;
    if (valid) {
        /* nbins >= 4 (k >= 1); 16-B pieces while they fit, then words */
        const uint64_t n4 = nbins / 4;
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += stride)
            reinterpret_cast<uint4 *>(dt)[i] = reinterpret_cast<const uint4 *>(table)[i];
    }
    if (blockIdx.x != 0) return;
    const uint32_t t = threadIdx.x;
    if (t < FK_PACK_COUNTERS * 4) {
        const unsigned long long *acc = res->acc, *ts = res->tstat;
        const uint32_t c = t >> 2, limb = t & 3;
        unsigned long long v = 0;
        if (ok) {
            switch (c) {
            case 0: v = acc[ACC_WIN]; break;
            case 1: v = acc[ACC_WIN] + acc[ACC_VALID]; break;
            case 2: case 3: case 4: case 5: v = ts[2 + (c - 2)] + acc[ACC_BASE + (c - 2)]; break;
            case 6: case 7: case 8: case 9: v = ts[6 + (c - 6)] + acc[ACC_D1S + (c - 6)]; break;
            case 10: v = acc[ACC_UNK]; break;
            case 11: v = len; break;
            case 12: v = 0; break;                           /* ended: a 0xFF shard is never packed */
            default: v = is_last ? res->exit.hdr : 0u; break;   /* unterminated_header */
            }
        }
        dc[t] = (int32_t)((v >> (16 * limb)) & 0xFFFFu);
    }
    for (uint32_t i = t; i < (uint32_t)nrows * FK_PACK_ROW_WORDS; i += blockDim.x) {
        const uint32_t r = i / FK_PACK_ROW_WORDS, j = i % FK_PACK_ROW_WORDS;
        uint32_t v = 0;
        if ((int)r == slot && ok) {
            if (j < 24) {
                const ShardSum &ss = res->shard;
                uint64_t w = 0;
                switch (j >> 1) {
                case 0: w = ss.g_code; break;
                case 1: w = (uint64_t)ss.g_R | ((uint64_t)ss.g_hdr << 32); break;
                case 2: w = ss.nvb0; break;
                case 3: w = ss.c_R; break;
                case 4: w = ss.c_code; break;
                case 5: w = (uint64_t)ss.c_hdr | ((uint64_t)ss.absorb << 32); break;
                case 6: w = ss.nv; break;
                case 7: w = len; break;
                case 8: w = (uint64_t)k; break;
                case 11: w = FK_SUMMARY_COMPACT; break;
                default: w = 0; break;                        /* 9: no 0xFF byte; 10: unused */
                }
                v = (j & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
            } else if (j == 24) {
                v = 1u;
            }
        }
        rows[i] = v;
    }
}

extern "C" int fk_engine_shard_pack(fk_engine *e, uint32_t *table, int32_t *counters, uint32_t *rows, int nrows,
                                    int slot, int is_last) {
    if (!e || !table || !counters || !rows || nrows < 1 || slot < 0 || slot >= nrows) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;   /* 17 <= k <= 20: no dense table to merge */
    if (!e->shard_pending) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    /* packable: counted in one pass (k_count + k_tail, k <= 7), nothing of
       the multi-launch path run since */
    const int valid = e->shard_len && e->shard_op && !e->shard_full && !e->shard_resumed ? 1 : 0;
    const uint64_t n4 = e->nbins / 4;
    const unsigned grid = valid ? (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n4 + 1023) / 1024, 1024)) : 1u;
    hipLaunchKernelGGL(k_shard_pack, dim3(grid), dim3(1024), 0, e->stream, e->d_res, e->d_table, e->nbins, table,
                       counters, rows, nrows, slot, is_last ? 1 : 0, valid, e->shard_len, e->k);
    HIPCHK(hipGetLastError());
    return FK_OK;
}

/* The gathered rows to pinned host memory, sequence number last (one block,
   one system fence per thread, then a block barrier before thread 0's
   release store: every thread's row stores are ordered before the sequence
   number the host spins on, whatever the block size). */
__global__ void __launch_bounds__(64) k_rows_publish(const uint32_t *rows, uint32_t n, uint32_t *host, uint32_t seq) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) host[32 + i] = rows[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&host[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* One row of a rows region (zeros elsewhere): words [0, nsrc) from src (a
   device transfer function), or w0 in word 0; word 24 = 1 (a valid row). */
__global__ void __launch_bounds__(64) k_fill_row(uint32_t *rows, int nrows, int slot, const uint32_t *src,
                                                 uint32_t nsrc, uint32_t w0) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)nrows * FK_PACK_ROW_WORDS; i += 64) {
        const uint32_t r = i / FK_PACK_ROW_WORDS, j = i % FK_PACK_ROW_WORDS;
        uint32_t v = 0;
        if ((int)r == slot) v = j == 24 ? 1u : (src ? (j < nsrc ? src[j] : 0u) : (j == 0 ? w0 : 0u));
        rows[i] = v;
    }
}

/* pinned, mapped scratch of the exchange: [0] sequence number, rows from
   word 32, counter and slice-statistics limbs (staging) after the rows */
static int ensure_rows(fk_engine *e, uint32_t nrow) {
    if (e->rows_cap >= nrow) return FK_OK;
    if (e->h_rows) hipHostFree(e->h_rows);
    hipFree(e->d_rows);
    e->h_rows = e->h_rows_dev = nullptr;
    e->d_rows = nullptr;
    e->rows_cap = 0;
    const size_t words = 32 + nrow + 4 * FK_PACK_COUNTERS + FK_PACK_STATS;
    if (hipHostMalloc((void **)&e->h_rows, words * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&e->h_rows_dev, e->h_rows, 0) != hipSuccess ||
        hipMalloc((void **)&e->d_rows, nrow * sizeof(uint32_t)) != hipSuccess)
        return FK_E_OOM;
    memset(e->h_rows, 0, words * sizeof(uint32_t));
    e->rows_cap = nrow;
    return FK_OK;
}

/* The rows (device, already all-reduced on e->stream) into e->h_rows + 32;
   one host wait. */
static int rows_fetch(fk_engine *e, const uint32_t *rows, uint32_t nrow) {
    if (++e->rows_seq == 0) e->rows_seq = 1;
    const uint32_t want = e->rows_seq;
    hipLaunchKernelGGL(k_rows_publish, dim3(1), dim3(64), 0, e->stream, rows, nrow, e->h_rows_dev, want);
    HIPCHK(hipGetLastError());
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&e->h_rows[0], __ATOMIC_ACQUIRE) == want) break;
        if ((spin & 4095) == 0) {
            hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(&e->h_rows[0], __ATOMIC_ACQUIRE) == want) break;
                return FK_E_HIP;   /* stream drained without publishing */
            }
            if (q != hipErrorNotReady) return FK_E_HIP;
        }
        __builtin_ia32_pause();
    }
    return FK_OK;
}

/* The stitched exchange with the library's communicator (the shard is
   pending): the shards' full transfer functions all-gathered (an
   all-reduce of rows), composed on the host, the shard resolved; the shards'
   end flags all-gathered the same way (a 0xFF byte, :988, exact only after
   the resolve); then the table and counter limbs, zero for ranks after the
   first ending shard, reduced onto rank 0. */
/* merge buffer layout (include/findkmer.h, fk_merge_layout): the table
   padded to a multiple of the world size, the counter limbs, the slice
   statistics, the rows */
static uint64_t merge_table_words(uint64_t nbins, int world) {
    const uint64_t w = (uint64_t)std::max(1, world);
    return (nbins + w - 1) / w * w;
}

/* the u64 sum and the nonzero bins of one table slice (sharded table) */
__global__ void __launch_bounds__(256) k_slice_sum(const uint32_t *t, uint64_t n, unsigned long long *out2) {
    /* 16-B loads between a scalar head (to the first aligned word: a slice
       starts at rank * S) and tail; one 4-B load per lane left the k = 16
       slice at 2.2 TB/s */
    unsigned long long sum = 0, nz = 0;
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t head = std::min<uint64_t>(n, ((16u - ((uintptr_t)t & 15u)) & 15u) / 4u);
    const uint64_t n4 = (n - head) / 4;
    if (tid < head) { const uint32_t v = t[tid]; sum += v; nz += v != 0; }
    const u32x4 *t4 = reinterpret_cast<const u32x4 *>(t + head);
    for (uint64_t q = tid; q < n4; q += nth) {
        const u32x4 v = __builtin_nontemporal_load(t4 + q);
        sum += (unsigned long long)v.x + v.y + v.z + v.w;
        nz += (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
    }
    for (uint64_t i = head + n4 * 4 + tid; i < n; i += nth) { const uint32_t v = t[i]; sum += v; nz += v != 0; }
    sum = wsum64(sum);
    nz = wsum64(nz);
    if ((threadIdx.x & 63) == 0) {
        if (sum) atomicAdd(&out2[0], sum);
        if (nz) atomicAdd(&out2[1], nz);
    }
}

/* ... as 16-bit limbs in int32 words (sums over ranks stay exact) */
__global__ void k_slice_limbs(const unsigned long long *in2, int32_t *limbs8) {
    const uint32_t i = threadIdx.x;
    if (i < 8) limbs8[i] = (int32_t)((in2[i >> 2] >> (16 * (i & 3))) & 0xFFFFu);
}

/*
 * Routed sharded tables (k >= 15, FK_XCHG_SHARD_TABLE over RCCL or a gloo
 * rehearsal): instead of reduce-scattering the whole 4^k table (k = 16:
 * 16 GiB a rank, ~15 GiB of it over xGMI), each rank sends every owner only
 * the nonzero bins of the owner's range, as one blob of 4-B entries per
 * destination, and each owner counts the blobs it receives into its slice.
 * A shard of 1.25 G windows leaves ~1.1 G nonzero bins at k = 16: ~4.4 GB
 * sent instead of 15 GiB, and nothing sent for bins no rank saw.
 *
 * Parts: 2^15-bin blocks of the table (reference index order).  Owner d holds
 * bins [d S, min((d + 1) S, 4^k)), S = TW / world (fk_merge_layout), so a part
 * belongs to one owner or, at a range boundary, to two.  A (destination,
 * part) pair is a slot, slots destination-major.  Blob for destination d:
 *   [0, 4)           E_d (entries) and O_d (overflow pairs), u64 as 2 words
 *   [4, 4 + P_d)     entries per slot of d (P_d slots: its parts)
 *   [.., + E_d)      entries, slot by slot: (bin offset in the part << 17) | count
 *   [.., + 2 O_d)    overflow pairs (bin - d S, count): counts >= 2^17 - 1
 */
#define RT_SH 15u
#define RT_ESC 0x1FFFFu
#define RT_HDR 4u
#define RT_STAT_SLOTS 512u

/* per-destination arrays in one device buffer (u64 each, world W):
   p0 [0,W) first part, sb [W, 2W+1) first slot, np [2W+1, 3W+1) parts,
   bb [3W+1, 4W+1) blob start (words), ne [4W+1, 5W+1) entries,
   no [5W+1, 6W+1) overflow pairs, oc [6W+1, 7W+1) overflow cursor; then
   off[nslots + 1] (exclusive entry offset of each slot), then cnt[nslots] u32 */
struct RouteGeo {
    uint64_t nbins, S;
    uint32_t world, nparts;
    unsigned long long *aux;
    __device__ __forceinline__ unsigned long long *p0() const { return aux; }
    __device__ __forceinline__ unsigned long long *sb() const { return aux + world; }
    __device__ __forceinline__ unsigned long long *np() const { return aux + 2 * world + 1; }
    __device__ __forceinline__ unsigned long long *bb() const { return aux + 3 * world + 1; }
    __device__ __forceinline__ unsigned long long *ne() const { return aux + 4 * world + 1; }
    __device__ __forceinline__ unsigned long long *no() const { return aux + 5 * world + 1; }
    __device__ __forceinline__ unsigned long long *oc() const { return aux + 6 * world + 1; }
    __device__ __forceinline__ unsigned long long *off() const { return aux + 7 * world + 1; }
};

/* a part's owner(s): d0 and, when the part crosses d0's end b, d0 + 1 */
__device__ __forceinline__ void rt_owners(const RouteGeo &g, uint64_t x0, uint32_t &d0, uint64_t &b, bool &two) {
    d0 = (uint32_t)min<uint64_t>(x0 / g.S, (uint64_t)g.world - 1);
    b = (uint64_t)(d0 + 1) * g.S;
    two = d0 + 1 < g.world && b < x0 + (1ull << RT_SH);
}

/* one block per part: its entries and overflow bins per owner, and per wave
   (a quarter of the part each: k_route_write's start positions, wc) */
__global__ void __launch_bounds__(256)
k_route_count(const uint32_t *table, RouteGeo g, int counting, uint32_t *cnt, uint32_t *wc) {
    __shared__ uint32_t ws[4][4];
    const uint32_t p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t x0 = (uint64_t)p << RT_SH;
    uint32_t d0;
    uint64_t b;
    bool two;
    rt_owners(g, x0, d0, b, two);
    uint32_t c[4] = {0, 0, 0, 0};   /* entries lo / hi, overflow lo / hi */
    if (counting) {
        const u32x4 *t4 = reinterpret_cast<const u32x4 *>(table + x0) + (size_t)wv * ((1u << RT_SH) / 16u);
        for (uint32_t q = lane; q < (1u << RT_SH) / 16u; q += 64u) {
            const u32x4 v4 = __builtin_nontemporal_load(t4 + q);
            const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const bool hi = x0 + wv * ((1u << RT_SH) / 4u) + q * 4u + (uint32_t)h >= b;
                const uint32_t v = w[h];
                c[hi ? 1 : 0] += v != 0u && v < RT_ESC;
                c[hi ? 3 : 2] += v >= RT_ESC;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) c[i] = wsum32(c[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 4; i++) ws[wv][i] = c[i];
        wc[(size_t)p * 8u + wv * 2u] = c[0];
        wc[(size_t)p * 8u + wv * 2u + 1u] = c[1];
    }
    __syncthreads();
    if (t == 0) {
        uint32_t s[4] = {0, 0, 0, 0};
        for (int w = 0; w < 4; w++)
            for (int i = 0; i < 4; i++) s[i] += ws[w][i];
        cnt[g.sb()[d0] + p - g.p0()[d0]] = s[0];
        if (s[2]) atomicAdd(&g.no()[d0], (unsigned long long)s[2]);
        if (two) {
            cnt[g.sb()[d0 + 1] + p - g.p0()[d0 + 1]] = s[1];
            if (s[3]) atomicAdd(&g.no()[d0 + 1], (unsigned long long)s[3]);
        }
    }
}

/* exclusive prefix of cnt[0, n) into off[0, n], off[n] = the total (one
   block: a few hundred K slots at most) */
__global__ void __launch_bounds__(1024)
k_route_scan(const uint32_t *cnt, uint64_t n, unsigned long long *off) {
    __shared__ unsigned long long part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (n + 1023) / 1024, b0 = min<uint64_t>(n, per * t), b1 = min<uint64_t>(n, b0 + per);
    unsigned long long s = 0;
    for (uint64_t i = b0; i < b1; i++) s += cnt[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        unsigned long long run = 0;
        for (uint32_t i = 0; i < 1024u; i++) {
            const unsigned long long v = part[i];
            part[i] = run;
            run += v;
        }
        off[n] = run;
    }
    __syncthreads();
    unsigned long long run = part[t];
    for (uint64_t i = b0; i < b1; i++) {
        off[i] = run;
        run += cnt[i];
    }
}

/* one block per part: its entries in bin order into each owner's blob (a
   wave per quarter of the part, its start from the waves before it),
   overflow bins appended to the owner's pairs, the slot counts, and (block
   0) every blob's header */
__global__ void __launch_bounds__(256)
k_route_write(const uint32_t *table, RouteGeo g, int counting, const uint32_t *cnt, const uint32_t *wc,
              uint32_t *send) {
    const uint32_t p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (p == 0 && t < g.world) {
        const unsigned long long e = g.ne()[t], o = g.no()[t];
        uint32_t *h = send + g.bb()[t];
        h[0] = (uint32_t)e; h[1] = (uint32_t)(e >> 32); h[2] = (uint32_t)o; h[3] = (uint32_t)(o >> 32);
    }
    const uint64_t x0 = (uint64_t)p << RT_SH;
    uint32_t d0;
    uint64_t b;
    bool two;
    rt_owners(g, x0, d0, b, two);
    const uint32_t d1 = two ? d0 + 1 : d0;
    const uint64_t s0 = g.sb()[d0] + p - g.p0()[d0], s1 = g.sb()[d1] + p - g.p0()[d1];
    if (t == 0) {
        send[g.bb()[d0] + RT_HDR + (s0 - g.sb()[d0])] = cnt[s0];
        if (two) send[g.bb()[d1] + RT_HDR + (s1 - g.sb()[d1])] = cnt[s1];
    }
    if (!counting) return;
    constexpr uint32_t QW = (1u << RT_SH) / 4u;   /* bins per wave */
    const uint32_t *tw = table + x0 + (uint64_t)wv * QW;
    uint64_t pos0 = g.off()[s0] - g.off()[g.sb()[d0]], pos1 = g.off()[s1] - g.off()[g.sb()[d1]];
    for (uint32_t w = 0; w < wv; w++) { pos0 += wc[(size_t)p * 8u + w * 2u]; pos1 += wc[(size_t)p * 8u + w * 2u + 1u]; }
    uint32_t *e0 = send + g.bb()[d0] + RT_HDR + g.np()[d0], *e1 = send + g.bb()[d1] + RT_HDR + g.np()[d1];
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t i0 = 0; i0 < QW; i0 += 64u) {
        const uint32_t i = i0 + lane;
        const uint32_t v = tw[i];
        const uint64_t x = x0 + wv * QW + i;
        const bool hi = x >= b, nz = v != 0u && v < RT_ESC;
        const unsigned long long m0 = __ballot(nz && !hi), m1 = __ballot(nz && hi);
        const uint32_t ent = ((wv * QW + i) << 17) | v;
        if (nz) {
            if (hi) e1[pos1 + __popcll(m1 & lt)] = ent;
            else e0[pos0 + __popcll(m0 & lt)] = ent;
        }
        if (v >= RT_ESC) {
            const uint32_t d = hi ? d1 : d0;
            const unsigned long long at = atomicAdd(&g.oc()[d], 1ull);
            uint32_t *op = send + g.bb()[d] + RT_HDR + g.np()[d] + g.ne()[d] + 2 * at;
            op[0] = (uint32_t)(x - (uint64_t)d * g.S);
            op[1] = v;
        }
        pos0 += __popcll(m0);
        pos1 += __popcll(m1);
    }
}

/* the owner: one block per part of its range, every source's entries for
   the part into 2^15 LDS bins, then the part's owned bins into the slice
   (written, not added: the slice holds nothing before) */
__global__ void __launch_bounds__(1024)
k_route_absorb(const uint32_t *recv, const unsigned long long *rd, const unsigned long long *roff, uint32_t world,
               uint32_t np, uint64_t p0, uint64_t lo, uint64_t hi, uint32_t *out, unsigned long long *stats) {
    extern __shared__ uint32_t bins[];
    const uint32_t j = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = t; i < (1u << RT_SH) / 4u; i += 1024u) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t s = 0; s < world; s++) {
        const uint32_t *blob = recv + rd[s];
        const uint32_t n = blob[RT_HDR + j];
        const uint32_t *ent = blob + RT_HDR + np + roff[(uint64_t)s * (np + 1) + j];
        for (uint32_t i = t; i < n; i += 1024u) {
            const uint32_t e = ent[i];
            atomicAdd(&bins[e >> 17], e & RT_ESC);
        }
    }
    __syncthreads();
    const uint64_t x0 = (p0 + j) << RT_SH;
    unsigned long long sum = 0, nz = 0;
    for (uint32_t i = t; i < (1u << RT_SH); i += 1024u) {
        const uint64_t x = x0 + i;
        if (x >= lo && x < hi) {
            const uint32_t v = bins[i];
            out[x - lo] = v;
            sum += v;
            nz += v != 0;
        }
    }
    /* the slice's total and nonzero bins (k_slice_sum's), before the
       overflow pairs add theirs (k_route_overflow): a block's sums into one
       of RT_STAT_SLOTS slot pairs (per-wave atomics on one address took
       50 ms at k = 16), k_route_stats folds them */
    if (stats) {
        __shared__ unsigned long long bs[16][2];
        sum = wsum64(sum);
        nz = wsum64(nz);
        if ((t & 63) == 0) { bs[t >> 6][0] = sum; bs[t >> 6][1] = nz; }
        __syncthreads();
        if (t < 2) {
            unsigned long long a = 0;
            for (int w = 0; w < 16; w++) a += bs[w][t];
            if (a) atomicAdd(&stats[(j % RT_STAT_SLOTS) * 2 + t], a);
        }
    }
}

__global__ void __launch_bounds__(256) k_route_stats(const unsigned long long *slots, unsigned long long *out2) {
    unsigned long long a = 0, b = 0;
    for (uint32_t i = threadIdx.x; i < RT_STAT_SLOTS; i += 256u) { a += slots[2 * i]; b += slots[2 * i + 1]; }
    a = wsum64(a);
    b = wsum64(b);
    if ((threadIdx.x & 63) == 0) {
        if (a) atomicAdd(&out2[0], a);
        if (b) atomicAdd(&out2[1], b);
    }
}

/* every source's overflow pairs added into the slice */
__global__ void __launch_bounds__(256)
k_route_overflow(const uint32_t *recv, const unsigned long long *rd, uint32_t np, uint32_t *out,
                 unsigned long long *stats) {
    const uint32_t *blob = recv + rd[blockIdx.x];
    const uint64_t ne = blob[0] | ((uint64_t)blob[1] << 32), no = blob[2] | ((uint64_t)blob[3] << 32);
    const uint32_t *op = blob + RT_HDR + np + ne;
    for (uint64_t i = threadIdx.x; i < no; i += 256u) {
        const uint32_t old = atomicAdd(&out[op[2 * i]], op[2 * i + 1]);
        if (stats) {
            atomicAdd(&stats[0], (unsigned long long)op[2 * i + 1]);
            if (old == 0) atomicAdd(&stats[1], 1ull);
        }
    }
}

/* the owners' geometry for (nbins, world) on the host */
struct RouteHost {
    uint64_t S = 0, nslots = 0;
    uint32_t nparts = 0;
    std::vector<unsigned long long> p0, sb, np;
};
static RouteHost route_geometry(uint64_t nbins, int world) {
    RouteHost h;
    h.S = merge_table_words(nbins, world) / (uint64_t)world;
    h.nparts = (uint32_t)(nbins >> RT_SH);
    h.p0.assign(world, 0);
    h.sb.assign(world + 1, 0);
    h.np.assign(world, 0);
    for (int d = 0; d < world; d++) {
        const uint64_t a = (uint64_t)d * h.S, z = std::min<uint64_t>((uint64_t)(d + 1) * h.S, nbins);
        if (a < z) {
            h.p0[d] = a >> RT_SH;
            h.np[d] = ((z - 1) >> RT_SH) - h.p0[d] + 1;
        } else {
            h.p0[d] = h.nparts;
        }
        h.sb[d + 1] = h.sb[d] + h.np[d];
    }
    h.nslots = h.sb[world];
    return h;
}

/* fk_engine_route_pack: the finished table's blobs, one per destination,
   side by side in e->d_rsend (words[d] each) */
static int route_pack(fk_engine *e, int world, bool counting, uint64_t *words) {
    if (e->sparse || e->k < 8 || world < 1) return FK_E_INVALID;
    const RouteHost h = route_geometry(e->nbins, world);
    if (h.S < (1ull << RT_SH)) return FK_E_INVALID;   /* (a part spans at most two owners) */
    const uint64_t W = (uint64_t)world;
    const uint64_t naux = 7 * W + 1 + h.nslots + 1, aux_bytes = naux * 8 + h.nslots * 4 + (uint64_t)h.nparts * 32 + 16;
    int rc = sp_ensure(&e->d_raux, &e->raux_cap, aux_bytes, 1);
    if (rc) return rc;
    unsigned long long *aux = static_cast<unsigned long long *>(e->d_raux);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(aux + naux), *wcnt = cnt + h.nslots;
    std::vector<unsigned long long> ha(7 * W + 1, 0);
    for (int d = 0; d < world; d++) { ha[d] = h.p0[d]; ha[2 * W + 1 + d] = h.np[d]; }
    for (int d = 0; d <= world; d++) ha[W + d] = h.sb[d];
    HIPCHK(hipMemcpyAsync(aux, ha.data(), ha.size() * 8, hipMemcpyHostToDevice, e->stream));
    RouteGeo g{e->nbins, h.S, (uint32_t)world, h.nparts, aux};
    hipLaunchKernelGGL(k_route_count, dim3(h.nparts), dim3(256), 0, e->stream, (const uint32_t *)e->d_table, g,
                       counting ? 1 : 0, cnt, wcnt);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, e->stream, (const uint32_t *)cnt, h.nslots,
                       aux + 7 * W + 1);
    HIPCHK(hipGetLastError());
    std::vector<unsigned long long> off(h.nslots + 1), no(W);
    HIPCHK(hipMemcpyAsync(off.data(), aux + 7 * W + 1, (h.nslots + 1) * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(no.data(), aux + 5 * W + 1, W * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t total = 0;
    for (int d = 0; d < world; d++) {
        const uint64_t ne = off[h.sb[d + 1]] - off[h.sb[d]];
        words[d] = RT_HDR + h.np[d] + ne + 2 * no[d];
        ha[3 * W + 1 + d] = total;   /* bb */
        ha[4 * W + 1 + d] = ne;      /* ne */
        total += words[d];
    }
    rc = sp_ensure((void **)&e->d_rsend, &e->rsend_cap, total, sizeof(uint32_t));
    if (rc) return rc;
    e->rsend_words = total;
    HIPCHK(hipMemcpyAsync(aux + 3 * W + 1, ha.data() + 3 * W + 1, 2 * W * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemsetAsync(aux + 6 * W + 1, 0, W * 8, e->stream));
    hipLaunchKernelGGL(k_route_write, dim3(h.nparts), dim3(256), 0, e->stream, (const uint32_t *)e->d_table, g,
                       counting ? 1 : 0, (const uint32_t *)cnt, (const uint32_t *)wcnt,
                       reinterpret_cast<uint32_t *>(e->d_rsend));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* fk_engine_route_absorb: the blobs received from every source (words[s]
   each, side by side at recv) into this rank's slice of the merged table */
static int route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words, int32_t *slice,
                        unsigned long long *stats) {
    if (e->sparse || e->k < 8 || world < 1 || rank < 0 || rank >= world) return FK_E_INVALID;
    const RouteHost h = route_geometry(e->nbins, world);
    if (h.S < (1ull << RT_SH)) return FK_E_INVALID;
    const uint64_t np = h.np[rank];
    if (!np) return FK_OK;   /* (owns no bin) */
    const uint64_t W = (uint64_t)world;
    std::vector<unsigned long long> rd(W);
    uint64_t at = 0;
    for (int s = 0; s < world; s++) {
        rd[s] = at;
        if (words[s] < RT_HDR + np) return FK_E_INVALID;
        at += words[s];
    }
    /* every blob's header against its size */
    std::vector<uint32_t> hdr(4 * W);
    for (int s = 0; s < world; s++)
        HIPCHK(hipMemcpyAsync(&hdr[4 * s], recv + rd[s], 16, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int s = 0; s < world; s++) {
        const uint64_t ne = hdr[4 * s] | ((uint64_t)hdr[4 * s + 1] << 32),
                       no = hdr[4 * s + 2] | ((uint64_t)hdr[4 * s + 3] << 32);
        if (RT_HDR + np + ne + 2 * no != words[s]) return FK_E_INVALID;
    }
    const uint64_t aux_bytes = (W + W * (np + 1) + 2 * RT_STAT_SLOTS) * 8 + 16;
    int rc = sp_ensure(&e->d_raux, &e->raux_cap, aux_bytes, 1);
    if (rc) return rc;
    unsigned long long *drd = static_cast<unsigned long long *>(e->d_raux), *roff = drd + W,
                       *sslots = roff + W * (np + 1);
    if (stats) HIPCHK(hipMemsetAsync(sslots, 0, 2 * RT_STAT_SLOTS * 8, e->stream));
    HIPCHK(hipMemcpyAsync(drd, rd.data(), W * 8, hipMemcpyHostToDevice, e->stream));
    const uint32_t *r32 = reinterpret_cast<const uint32_t *>(recv);
    for (int s = 0; s < world; s++) {
        hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, e->stream, r32 + rd[s] + RT_HDR, np,
                           roff + (uint64_t)s * (np + 1));
        HIPCHK(hipGetLastError());
    }
    const uint64_t lo = (uint64_t)rank * h.S, hi = std::min<uint64_t>(lo + h.S, e->nbins);
    HIPCHK(hipFuncSetAttribute((const void *)k_route_absorb, hipFuncAttributeMaxDynamicSharedMemorySize, 1 << 17));
    uint32_t *out = reinterpret_cast<uint32_t *>(slice);
    hipLaunchKernelGGL(k_route_absorb, dim3((uint32_t)np), dim3(1024), (size_t)1 << 17, e->stream, r32,
                       (const unsigned long long *)drd, (const unsigned long long *)roff, (uint32_t)world, (uint32_t)np,
                       (uint64_t)h.p0[rank], lo, hi, out, stats ? sslots : nullptr);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_route_overflow, dim3((uint32_t)world), dim3(256), 0, e->stream, r32,
                       (const unsigned long long *)drd, (uint32_t)np, out, stats);
    HIPCHK(hipGetLastError());
    if (stats) {
        hipLaunchKernelGGL(k_route_stats, dim3(1), dim3(256), 0, e->stream, (const unsigned long long *)sslots, stats);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_route_pack(fk_engine *e, int world, int counting, uint64_t *words) {
    if (!e || !words) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    return route_pack(e, world, counting != 0, words);
}

extern "C" int fk_engine_route_copy(fk_engine *e, void *dst) {
    if (!e || !dst || !e->d_rsend) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(dst, e->d_rsend, e->rsend_words * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

extern "C" int fk_engine_route_absorb(fk_engine *e, int world, int rank, const int32_t *recv, const uint64_t *words,
                                      int32_t *slice) {
    if (!e || !recv || !words || !slice) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    return route_absorb(e, world, rank, recv, words, slice, nullptr);
}

/* the routed exchange over RCCL: blobs packed, their sizes all-reduced as a
   world x world matrix of 16-bit limbs, one grouped send/recv, the received
   blobs into this rank's slice */
static int route_exchange(fk_engine *e, fk_comm *comm, bool counting, int32_t *slice, unsigned long long *stats) {
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    const uint64_t W = (uint64_t)world;
    std::vector<uint64_t> sw(W), rw(W), sd(W), rdsp(W);
    int rc = route_pack(e, world, counting, sw.data());
    if (rc) return rc;
    DevScratch m;
    const uint64_t nm = W * W * 3;
    if (!m.alloc(nm * 4)) return FK_E_OOM;
    std::vector<int32_t> hm(nm, 0);
    for (uint64_t d = 0; d < W; d++)
        for (int j = 0; j < 3; j++) hm[((uint64_t)rank * W + d) * 3 + j] = (int32_t)((sw[d] >> (16 * j)) & 0xFFFFu);
    HIPCHK(hipMemcpyAsync(m.p, hm.data(), nm * 4, hipMemcpyHostToDevice, e->stream));
    rc = fkc_allreduce_i32(comm, m.as<int32_t>(), nm, e->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(hm.data(), m.p, nm * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t sat = 0, rat = 0;
    for (uint64_t s = 0; s < W; s++) {
        uint64_t v = 0;
        for (int j = 0; j < 3; j++) v |= (uint64_t)(uint32_t)hm[(s * W + (uint64_t)rank) * 3 + j] << (16 * j);
        rw[s] = v;
        rdsp[s] = rat;
        rat += v;
        sd[s] = sat;
        sat += sw[s];
    }
    rc = sp_ensure((void **)&e->d_rrecv, &e->rrecv_cap, rat, sizeof(int32_t));
    if (rc) return rc;
    rc = fkc_alltoallv_i32(comm, e->d_rsend, sw.data(), sd.data(), e->d_rrecv, rw.data(), rdsp.data(), e->stream);
    if (rc) return rc;
    return route_absorb(e, world, rank, e->d_rrecv, rw.data(), slice, stats);
}

static int stitched_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *first_end_out, bool scatter) {
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    const uint64_t tw = merge_table_words(e->nbins, world);
    const uint32_t nrow = (uint32_t)world * FK_PACK_ROW_WORDS;
    int rc = shard_full_tf(e);
    if (rc) return rc;
    if (e->shard_len == 0) {
        const TF id = fk_identity();
        HIPCHK(hipMemcpyAsync(e->d_tf, &id, sizeof id, hipMemcpyHostToDevice, e->stream));
    }
    hipLaunchKernelGGL(k_fill_row, dim3(1), dim3(64), 0, e->stream, e->d_rows, world, rank,
                       reinterpret_cast<const uint32_t *>(e->d_tf), (uint32_t)(sizeof(TF) / 4), 0u);
    HIPCHK(hipGetLastError());
    rc = fkc_allreduce_i32(comm, reinterpret_cast<int32_t *>(e->d_rows), nrow, e->stream);
    if (rc) return rc;
    rc = rows_fetch(e, e->d_rows, nrow);
    if (rc) return rc;
    XState s{0, 0, 0, 0}, in = s;   /* from the stream's initial state */
    for (int r = 0; r < world; r++) {
        TF t;
        memcpy(&t, e->h_rows + 32 + (size_t)r * FK_PACK_ROW_WORDS, sizeof t);
        if (r == rank) in = s;
        s = fk_apply(t, s);
    }
    fk_state ent{in.R, fk_sigma(in.code), in.hdr, 0};
    rc = fk_engine_resolve(e, &ent);
    if (rc) return rc;
    fk_result res;
    rc = fk_engine_finish(e, &res);
    if (rc != FK_OK && rc != FK_E_ROLLOVER && rc != FK_E_UNTERMINATED_HEADER && rc != FK_E_EMPTY) return rc;
    /* where the stream ends */
    hipLaunchKernelGGL(k_fill_row, dim3(1), dim3(64), 0, e->stream, e->d_rows, world, rank, (const uint32_t *)nullptr,
                       0u, res.hit_eof_byte ? 1u : 0u);
    HIPCHK(hipGetLastError());
    rc = fkc_allreduce_i32(comm, reinterpret_cast<int32_t *>(e->d_rows), nrow, e->stream);
    if (rc) return rc;
    rc = rows_fetch(e, e->d_rows, nrow);
    if (rc) return rc;
    int first_end = -1;
    for (int r = 0; r < world && first_end < 0; r++)
        if (e->h_rows[32 + (size_t)r * FK_PACK_ROW_WORDS]) first_end = r;
    const bool counting = first_end < 0 || rank <= first_end;
    const int last = first_end >= 0 ? first_end : world - 1;
    /* the table and the counters (fk_engine_finish's values, as 16-bit limbs) */
    uint64_t v[FK_PACK_COUNTERS] = {};
    if (counting) {
        v[0] = res.windows; v[1] = res.valid_bases;
        for (int b = 0; b < 4; b++) { v[2 + b] = res.base_count[b]; v[6 + b] = res.depth1[b]; }
        v[10] = res.unknown_chars; v[11] = res.scanned_bytes;
        v[12] = rank == first_end ? 1u : 0u;
        v[13] = rank == last ? (uint64_t)res.unterminated_header : 0u;
    }
    /* the reduce-scatter reads the engine's own table when its blocks divide
       it exactly (a power-of-two world): no copy of the whole table into
       the merge buffer first (k = 16: 16 GiB, ~5 ms per step); a rank whose
       shard the stream never reached sends zeros (its table, zeroed: the
       engine's count is discarded anyway) */
    const bool route = scatter && e->k >= FK_ROUTE_KMIN && fkc_has_alltoallv(comm) &&
                       (e->route_mode == 2 || (e->route_mode == 1 && world > 1));
    const bool direct = scatter && tw == e->nbins;
    if (route) {
        /* (the table stays where it is: route_pack reads it) */
    } else if (direct) {
        if (!counting) HIPCHK(hipMemsetAsync(e->d_table, 0, e->nbins * sizeof(uint32_t), e->stream));
    } else if (counting) {
        HIPCHK(hipMemcpyAsync(merge, e->d_table, e->nbins * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream));
    } else {
        HIPCHK(hipMemsetAsync(merge, 0, e->nbins * sizeof(uint32_t), e->stream));
    }
    if (!route && !direct && tw > e->nbins)
        HIPCHK(hipMemsetAsync(merge + e->nbins, 0, (tw - e->nbins) * sizeof(uint32_t), e->stream));
    uint32_t *limbs = e->h_rows + 32 + e->rows_cap;   /* pinned staging */
    for (int i = 0; i < FK_PACK_COUNTERS; i++)
        for (int j = 0; j < 4; j++) limbs[4 * i + j] = (uint32_t)((v[i] >> (16 * j)) & 0xFFFFu);
    for (int j = 0; j < FK_PACK_STATS; j++) limbs[4 * FK_PACK_COUNTERS + j] = 0;
    HIPCHK(hipMemcpyAsync(merge + tw, limbs, (4 * FK_PACK_COUNTERS + FK_PACK_STATS) * sizeof(uint32_t),
                          hipMemcpyHostToDevice, e->stream));
    if (scatter) {
        /* the table sharded by its top index bits (the first bases): rank r
           keeps bins [r * S, (r + 1) * S) of the sum, S = tw / world; the
           counters and every slice's (sum, distinct) are all-reduced */
        const uint64_t S = tw / (uint64_t)world;
        HIPCHK(hipMemsetAsync(e->d_tmp, 0, 2 * sizeof(unsigned long long), e->stream));
        if (route) {   /* (the slice's total and nonzero bins as it is absorbed) */
            rc = route_exchange(e, comm, counting, merge + (uint64_t)rank * S, e->d_tmp);
        } else {
            rc = direct ? fkc_reduce_scatter_from_i32(comm, reinterpret_cast<const int32_t *>(e->d_table), merge, S,
                                                      e->stream)
                        : fkc_reduce_scatter_i32(comm, merge, S, e->stream);
        }
        if (rc) return rc;
        const uint64_t lo = (uint64_t)rank * S, n = lo < e->nbins ? std::min(S, e->nbins - lo) : 0;
        if (n && !route) {
            const unsigned gr = (unsigned)std::min<uint64_t>((uint64_t)e->cus * 8, (n + 1023) / 1024);
            hipLaunchKernelGGL(k_slice_sum, dim3(gr), dim3(256), 0, e->stream,
                               reinterpret_cast<const uint32_t *>(merge) + lo, n, e->d_tmp);
        }
        hipLaunchKernelGGL(k_slice_limbs, dim3(1), dim3(64), 0, e->stream, e->d_tmp,
                           merge + tw + 4 * FK_PACK_COUNTERS);
        HIPCHK(hipGetLastError());
        rc = fkc_allreduce_i32(comm, merge + tw, 4 * FK_PACK_COUNTERS + FK_PACK_STATS, e->stream);
    } else {
        rc = fkc_reduce_i32(comm, merge, tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS, 0, e->stream);
    }
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (first_end_out) *first_end_out = first_end;
    return FK_OK;
}

extern "C" int fk_engine_shard_exchange(fk_engine *e, fk_comm *comm, int32_t *merge, int32_t *info) {
    if (!e || !comm || !merge) return FK_E_INVALID;
    if (e->sparse) return FK_E_INVALID;
    if (!e->shard_pending) return FK_E_STATE;
    const int world = fkc_world(comm), rank = fkc_rank(comm);
    if (fkc_device(comm) != e->dev) return FK_E_INVALID;
    const int32_t flags = info ? info[0] : FK_XCHG_FAST;
    const bool try_fast = (flags & FK_XCHG_FAST) != 0;
    const bool scatter = (flags & FK_XCHG_SHARD_TABLE) != 0;
    int rc = set_dev(e);
    if (rc) return rc;
    const uint32_t nrow = (uint32_t)world * FK_PACK_ROW_WORDS;
    rc = ensure_rows(e, nrow);
    if (rc) return rc;
    const uint64_t tw = merge_table_words(e->nbins, world);
    if (try_fast) {
        /* one collective: pack, all-reduce table + counters + rows, compose */
        int32_t *stats = merge + tw + 4 * FK_PACK_COUNTERS;
        uint32_t *rows = reinterpret_cast<uint32_t *>(stats + FK_PACK_STATS);
        rc = fk_engine_shard_pack(e, reinterpret_cast<uint32_t *>(merge), merge + tw, rows, world, rank,
                                  rank == world - 1);
        if (rc) return rc;
        if (tw > e->nbins) HIPCHK(hipMemsetAsync(merge + e->nbins, 0, (tw - e->nbins) * sizeof(uint32_t), e->stream));
        HIPCHK(hipMemsetAsync(stats, 0, FK_PACK_STATS * sizeof(int32_t), e->stream));
        if (flags & FK_XCHG_TEST_INVALID)   /* tests: this rank's pack row reads as invalid */
            HIPCHK(hipMemsetAsync(rows + (size_t)rank * FK_PACK_ROW_WORDS + 24, 0, sizeof(uint32_t), e->stream));
        rc = fkc_allreduce_i32(comm, merge, tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS + nrow, e->stream);
        if (rc) return rc;
        rc = rows_fetch(e, rows, nrow);
        if (rc) return rc;
        fk_state st;
        rc = fk_shard_rows_compose(e->h_rows + 32, world, rank, &st);
        if (rc == FK_OK) {
            rc = fk_engine_resolve(e, &st);
            if (rc) return rc;
            if (info) { info[0] = 1; info[1] = -1; }
            return FK_OK;
        }
        if (rc != FK_E_SUMMARY) return rc;
        /* some guess did not hold (every rank sees it): stitched, below */
    }
    int32_t first_end = -1;
    rc = stitched_exchange(e, comm, merge, &first_end, scatter);
    if (rc) return rc;
    if (info) { info[0] = 0; info[1] = first_end; }
    return FK_OK;
}

extern "C" int fk_merge_layout(int k, int world, uint64_t *table_words, uint64_t *total_words) {
    if (k < FK_K_MIN || k > FK_K_MAX_DENSE || world < 1) return FK_E_INVALID;
    const uint64_t tw = merge_table_words(1ull << (2 * k), world);
    if (table_words) *table_words = tw;
    if (total_words)
        *total_words = tw + 4 * FK_PACK_COUNTERS + FK_PACK_STATS + (uint64_t)world * FK_PACK_ROW_WORDS;
    return FK_OK;
}

extern "C" int fk_engine_stream(fk_engine *e, void **stream) {
    if (!e || !stream) return FK_E_INVALID;
    *stream = (void *)e->stream;
    return FK_OK;
}

extern "C" int fk_shard_rows_compose(const uint32_t *rows, int world, int rank, fk_state *entering) {
    if (!rows || world < 1 || rank < 0 || rank >= world || !entering) return FK_E_INVALID;
    XState s{0, 0, 0, 0};   /* the stream's initial state */
    XState mine = s;
    for (int r = 0; r < world; r++) {
        const uint32_t *row = rows + (size_t)r * FK_PACK_ROW_WORDS;
        if (row[24] != 1u) return FK_E_SUMMARY;
        fk_summary sm;
        for (int j = 0; j < 12; j++) sm.w[j] = (uint64_t)row[2 * j] | ((uint64_t)row[2 * j + 1] << 32);
        if (sm.w[11] != FK_SUMMARY_COMPACT || sm.w[9] != 0) return FK_E_SUMMARY;
        if (r == rank) mine = s;
        XState y;
        if (!compact_apply(&sm, s, y)) return FK_E_SUMMARY;
        s = y;
    }
    entering->run = mine.R;
    entering->code = fk_sigma(mine.code);
    entering->hdr = mine.hdr;
    entering->ended = 0;
    return FK_OK;
}

/* ---- finish ---- */

/* one k_sp_emit launch per retained segment */
static int sp_emit_all(fk_engine *e, const SpEmit &em) {
    const size_t lds = (size_t)SP_WAVES * FK_TILE_BYTES * sizeof(uint64_t) +
                       (em.mode == SP_HIST ? (size_t)em.nbuckets * sizeof(uint32_t) : 0);
    for (const auto &sg : e->spsegs) {
        if (!sg.nranges) continue;
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((sg.nranges + SP_WAVES - 1) / SP_WAVES,
                                                                                 (uint64_t)e->cus * 8));
        hipLaunchKernelGGL(k_sp_emit, dim3(grid), dim3(SP_WAVES * 64u), lds, e->stream, e->d_keep + sg.off, sg.len,
                           e->k, e->maskk, e->d_kst + sg.st, sg.nranges, sg.cpw, sg.nchunks, em);
        HIPCHK(hipGetLastError());
    }
    return FK_OK;
}

/*
 * A k = 17 key-range pass (keys lo + r, r < 2^32, emitted as 32-bit r) into
 * its runs without a sort (round 5; rocPRIM's radix sort and run-length
 * encode took 228 ms of a 10 G-base step's 390).  The pass is a 2^32-bin
 * count table, so it is counted the way k = 16's dense table is, and only
 * its nonzero bins are written:
 *   k_kpart       the key list in batches of 32 K keys, counting-sorted in LDS
 *                 by r's top 11 bits into 2048 coarse slices (k_part<C32>'s
 *                 row layout: each batch one row of runs of 21-bit codes and a
 *                 row of run words);
 *   k_repart      (as for k = 15, 16) each coarse slice into 64 contiguous
 *                 part streams of 15-bit codes;
 *   k_kp_count    one block per part (2^15 bins, in key order): the part's
 *                 stream into LDS bins, the pads taken off the last bin, the
 *                 nonzero bins' offset from the parts before it (a chained
 *                 scan: each block publishes its distinct count, then looks
 *                 back for the earlier parts' total), then the bins written
 *                 as (key, u32 count) in ascending order with the statistics,
 *                 the rollover check and the adjacent keys' prefix histogram;
 *   k_kp_fold     the blocks' partial statistics into the pass accumulators,
 *                 the prefix histogram of each part's first key against the
 *                 last key of the nonempty part before it, and the pass's
 *                 distinct count.
 */
#define KP_BATCH 32768u      /* keys per k_kpart batch (16 waves x 2048) */
#define KP_SLOTS 64u         /* partial-statistics slots (block % KP_SLOTS) */
#define KP_SLOT_W 36u        /* per slot: 10 statistics, rollover, 24 prefix-histogram entries, spare */
#define KP_EMPTY (~0ull)

/* KT = uint32_t: 32-bit relative keys r (slice r >> 21, code r & (2^21 - 1));
   KT = uint64_t: keys lo + r with r < 2^(cs + 11) (slice r >> cs, code r &
   (2^cs - 1), cs <= 29); keys >= hi (pads past the pass's range) are left out */
/* The top key `tkey` (the pads' value: relative 0xFFFFFFFF, or 4^k - 1 when
   the pass holds it; ~0 for none) is left out of the partition and only
   counted into *tcount: the chunk pads of every emitting wave (tens of
   millions per pass) would otherwise crowd one part, whose k_repart block
   and LDS bin then serialise the whole pass. */
template <typename KT>
__global__ void __launch_bounds__(1024)
k_kpart(const KT *keys, uint64_t n, PartGeo pg, uint64_t lo, uint64_t hi, uint32_t cs, uint64_t tkey,
        unsigned long long *tcount) {
    constexpr bool WIDE = sizeof(KT) == 8;
    __shared__ uint32_t hist[2048], cur[2048], wtot[16];
    __shared__ uint32_t ntop;
    extern __shared__ uint32_t ent[];   /* KP_BATCH codes */
    const uint32_t t = threadIdx.x;
    const uint32_t sh = WIDE ? cs : 21u;
    const KT cmask = (KT)(((uint64_t)1 << sh) - 1);
    for (uint32_t i = t; i < 2048u; i += 1024u) hist[i] = 0;
    if (t == 0) ntop = 0;
    const uint64_t per = (uint64_t)pg.rounds * KP_BATCH;
    const uint64_t k0 = blockIdx.x * per, k1 = min(k0 + per, n);
    uint32_t *codes = reinterpret_cast<uint32_t *>(pg.codes);
    uint32_t mytop = 0;
    for (uint32_t r = 0; r < pg.rounds; r++) {
        const uint32_t row = blockIdx.x * pg.rounds + r;
        const uint64_t b0 = k0 + (uint64_t)r * KP_BATCH;
        const uint32_t nv = b0 < k1 ? (uint32_t)min<uint64_t>(KP_BATCH, k1 - b0) : 0u;
        __syncthreads();
        if (nv == 0) {   /* rows past the block's keys are empty */
            for (uint32_t b = t; b < 2048u; b += 1024u) pg.idx[(size_t)row * 2048u + b] = PART_NO_RUN;
            continue;
        }
        /* each key's slice (two 16-bit slices per word, 0xFFFF: left out --
           past hi, or the top key) and code: 48 registers where 32 64-bit
           keys took 64 and spilled */
        uint32_t cd[32], sp[16];
#pragma unroll
        for (uint32_t j = 0; j < 16u; j++) sp[j] = 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++) {
            cd[j] = 0;
            if (j * 1024u + t < nv) {
                const KT x = keys[b0 + j * 1024u + t];
                uint32_t sl = 0xFFFFu;
                if ((uint64_t)x == tkey) {
                    mytop++;
                } else if (!WIDE) {
                    sl = (uint32_t)x >> 21;
                    cd[j] = (uint32_t)x & 0x1FFFFFu;
                } else if ((uint64_t)x < hi) {
                    const uint64_t r = (uint64_t)x - lo;
                    sl = (uint32_t)(r >> sh);
                    cd[j] = (uint32_t)(r & (uint64_t)cmask);
                }
                sp[j >> 1] = (j & 1) ? (sp[j >> 1] & 0xFFFFu) | (sl << 16) : (sp[j >> 1] & 0xFFFF0000u) | sl;
            }
        }
#define KP_SL(j) ((sp[(j) >> 1] >> (((j) & 1) * 16)) & 0xFFFFu)
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++)
            if (KP_SL(j) != 0xFFFFu) atomicAdd(&hist[KP_SL(j)], 1u);
        __syncthreads();
        {   /* cursors and the row's run words: two slices per thread, a block
               scan (one wave walking 32 slices a lane kept 15 waiting) */
            const uint32_t b = 2u * t, c0 = hist[b], c1 = hist[b + 1u], sum = c0 + c1;
            const uint32_t inc = wscan_incl32(sum);
            if ((t & 63u) == 63u) wtot[t >> 6] = inc;
            __syncthreads();
            uint32_t run = inc - sum;
#pragma unroll
            for (uint32_t w = 0; w < 16u; w++) run += w < (t >> 6) ? wtot[w] : 0u;
            cur[b] = run;
            cur[b + 1u] = run + c0;
            reinterpret_cast<uint2 *>(pg.idx + (size_t)row * 2048u)[t] = make_uint2(run_word(run, c0), run_word(run + c0, c1));
            hist[b] = 0;
            hist[b + 1u] = 0;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++)
            if (KP_SL(j) != 0xFFFFu) ent[atomicAdd(&cur[KP_SL(j)], 1u)] = cd[j];
#undef KP_SL
        __syncthreads();
        /* the row: its runs end at cur[2047] (every entry placed) */
        const uint32_t tot = cur[2047];
        uint4 *dst = reinterpret_cast<uint4 *>(codes + (size_t)row * pg.batch);
        const uint4 *src = reinterpret_cast<const uint4 *>(ent);
        for (uint32_t i = t; i < (tot + 3u) / 4u; i += 1024u) dst[i] = src[i];
    }
    if (mytop) atomicAdd(&ntop, mytop);
    __syncthreads();
    if (t == 0 && ntop) atomicAdd(tcount, (unsigned long long)ntop);
}

/* A chained scan over the blocks in dispatch order (wave 0 of every block
   calls it): this block's `total` published (status A: aggregate), the
   earlier blocks' sum found by looking back 64 flags at a time -- up to the
   nearest one with status P (inclusive prefix) -- and this block's own
   inclusive prefix published.  Returns the exclusive prefix.  Every earlier
   block was dispatched before this one and publishes unconditionally; the
   spin bound only guards a broken invariant (FK_FAULT_PARTS: the pass fails
   with FK_E_INTERNAL instead of hanging the GPU).  The flags are relaxed
   agent-scope atomics: a flag word carries all a reader needs (status and
   value in one 64-bit access), and a release store would write back this
   XCD's whole L2 -- the parts' output just written -- once per part. */
__device__ unsigned long long chain_prefix(unsigned long long *flags, uint32_t blk, uint32_t total,
                                           unsigned long long *err) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long A = 1ull << 62, P = 2ull << 62, M = (1ull << 62) - 1;
    if (blk == 0) {
        if (lane == 0) __hip_atomic_store(&flags[0], P | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&flags[blk], A | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long pre = 0;
    int64_t j = (int64_t)blk - 1;
    uint64_t spin = 0;
    for (;;) {
        const int64_t idx = j - (int64_t)lane;
        unsigned long long f = idx >= 0 ? __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : P;
        /* wait only for the flags up to the nearest inclusive prefix (the
           blocks farther back may still be counting) */
        for (;;) {
            const unsigned long long pm0 = __ballot((f >> 62) == 2);
            const unsigned long long need = pm0 ? (pm0 & (~pm0 + 1)) * 2 - 1 : ~0ull;   /* lanes 0 .. first P */
            if (!(__ballot((f >> 62) == 0) & need)) break;
            if (++spin > (1ull << 22)) {
                if (lane == 0) atomicOr(err, (unsigned long long)FK_FAULT_PARTS);
                return pre;
            }
            __builtin_amdgcn_s_sleep(1);
            if ((f >> 62) == 0) f = __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const unsigned long long pm = __ballot((f >> 62) == 2);
        const unsigned long long val = f & M;
        if (pm) {
            const uint32_t first = (uint32_t)__builtin_ctzll(pm);   /* the nearest prefix */
            pre += wsum64(lane <= first ? val : 0ull);
            break;
        }
        pre += wsum64(val);
        j -= 64;
    }
    if (lane == 0) __hip_atomic_store(&flags[blk], P | (pre + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

/* the bins of a part: thread t takes bins [32 t, 32 t + 32).  The 2^15
   bins are 16-bit halves of 2^14 LDS words (64 KiB instead of 128: half the
   zeroing and reading, 16.9 -> 13.1 ms per k = 17 pass; a second block per
   CU would need <= 64 VGPRs, and forced there the spills made it 21 ms).  A half that wraps (a k-mer 65536 times in
   one part) makes the halves' sum fall short of the codes: the part is then
   counted again as two halves of 2^14 32-bit bins. */
#define KC_WORDS (1u << 14)
__global__ void __launch_bounds__(1024)
k_kp_count(const uint16_t *in, const PartMeta *meta, uint64_t cap_in, uint64_t lo, uint64_t npads,
           const unsigned long long *tcount, uint32_t nparts, int k, unsigned long long *flags, uint64_t *out_k,
           uint32_t *out_c, unsigned long long *slots, uint64_t *fl, unsigned long long *err) {
    extern __shared__ uint32_t bins[];   /* KC_WORDS */
    __shared__ unsigned long long wred[16][10];
    __shared__ uint32_t hpre[24];
    __shared__ uint32_t wnz[16], wmx[16];
    __shared__ unsigned long long bprefix;
    __shared__ uint32_t vblk;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    /* the part: a ticket in the order blocks start (flags[nparts]), not
       blockIdx -- the chained scan may only wait on blocks that are already
       running, and across the 8 XCDs (and other processes' kernels)
       blockIdx order is not start order */
    if (t == 0) vblk = (uint32_t)atomicAdd(&flags[nparts], 1ull);
    for (uint32_t i = t; i < KC_WORDS / 4u; i += 1024u) reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
    if (t < 24) hpre[t] = 0;
    __syncthreads();
    const uint32_t blk = vblk;
    PartMeta m = meta[blk];
    if (m.off + m.n > cap_in) {   /* bound check (k_count_parts's) */
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_META);
        m.n = 0;
        m.off = 0;
    }
    const uint4 *g4 = reinterpret_cast<const uint4 *>(in + m.off);
    const uint32_t nq = (m.n + 7u) >> 3;
    /* each code to its bin, bin b at half b & 1 of word b >> 1 (hsel: the
       32-bit pass of half h, bins [h 2^14, (h + 1) 2^14) only) */
    auto count = [&](int hsel) {
#ifndef KPX_NOCNT
        for (uint32_t q = t; q < nq; q += 1024u) {
            const uint4 v = g4[q];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int h = 0; h < 8; h++) {
                if (q * 8u + (uint32_t)h >= m.n) continue;
                const uint32_t b = (w4[h >> 1] >> (16 * (h & 1))) & 0x7FFFu;
                if (hsel < 0) atomicAdd(&bins[b >> 1], 1u << ((b & 1u) << 4));
                else if ((b >> 14) == (uint32_t)hsel) atomicAdd(&bins[b & (KC_WORDS - 1u)], 1u);
            }
        }
#endif
    };
    count(-1);
    __syncthreads();
    /* thread t's 32 bins: words [16 t, 16 t + 16) */
    uint32_t c[32];
    unsigned long long hs = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4u; j++) {
        const uint4 q = reinterpret_cast<const uint4 *>(bins)[t * 4u + j];
        const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int h = 0; h < 4; h++) {
            c[8 * j + 2 * h] = w4[h] & 0xFFFFu;
            c[8 * j + 2 * h + 1] = w4[h] >> 16;
            hs += (w4[h] & 0xFFFFu) + (w4[h] >> 16);
        }
    }
    {   /* the wrap check (block-wide: the halves' sum against the codes) */
        const unsigned long long a = wsum64(hs);
        if (lane == 0) wred[wv][0] = a;
        __syncthreads();
        unsigned long long sa = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16u; w++) sa += wred[w][0];
#ifndef KPX_NOCNT
        if (sa != (unsigned long long)m.n) {
            for (int h = 0; h < 2; h++) {
                __syncthreads();
                for (uint32_t i = t; i < KC_WORDS / 4u; i += 1024u)
                    reinterpret_cast<uint4 *>(bins)[i] = make_uint4(0, 0, 0, 0);
                __syncthreads();
                count(h);
                __syncthreads();
                if ((t >> 9) == (uint32_t)h) {   /* (thread t's bins lie in half t / 512) */
#pragma unroll
                    for (uint32_t j = 0; j < 8u; j++) {
                        const uint4 q = reinterpret_cast<const uint4 *>(bins)[(t & 511u) * 8u + j];
                        c[4 * j] = q.x; c[4 * j + 1] = q.y; c[4 * j + 2] = q.z; c[4 * j + 3] = q.w;
                    }
                }
            }
        }
#endif
        __syncthreads();   /* (wred is reused below) */
    }
    /* the top key (relative 0xFFFFFFFF, the last bin of the last part) was
       only counted (k_kpart): its real windows, the pads taken off */
    const unsigned long long extra = blk == nparts - 1u ? *tcount - npads : 0ull;
    if (t == 1023u && extra) c[31] += (uint32_t)extra;
    const int fs = 2 * (k - 1);
    const uint64_t kb = lo + ((uint64_t)blk << 15) + t * 32u;   /* key of my first bin (a multiple of 4) */
    /* statistics with constant register indices (a runtime index into a
       register array put it in scratch memory): bin j's last base is j & 3,
       and the first base is the same for all 32 bins */
    uint32_t nz = 0;
    unsigned long long l4[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 32u; j++) {
        nz += c[j] != 0;
        l4[j & 3] += c[j];
    }
    const unsigned long long sum = l4[0] + l4[1] + l4[2] + l4[3];
    const uint32_t fd = (uint32_t)((kb >> fs) & 3);
    unsigned long long st[10] = {nz, sum, l4[0], l4[1], l4[2], l4[3], fd == 0 ? sum : 0ull, fd == 1 ? sum : 0ull,
                                 fd == 2 ? sum : 0ull, fd == 3 ? sum : 0ull};
    /* block scan of the nonzero counts */
    const uint32_t inc = wscan_incl32(nz);
    if (lane == 63) wnz[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16u; w++) {
        const uint32_t x = wnz[w];
        before += w < wv ? x : 0u;
        total += x;
    }
    const uint32_t off = before + inc - nz;
    /* the parts' chained scan */
    if (wv == 0) {
#ifdef KPX_NOLB
        const unsigned long long pre = 0;
#else
        const unsigned long long pre = chain_prefix(flags, blk, total, err);
#endif
        if (lane == 0) {
            bprefix = pre;
            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;
        }
    }
    /* the nearest earlier thread holding a nonzero bin (an exclusive max
       scan of t + 1), for the adjacent pair across threads */
    const uint32_t im = wscan_max32(nz ? t + 1u : 0u);
    if (lane == 63) wmx[wv] = im;
    __syncthreads();   /* (also: every thread has its bins in registers) */
    uint32_t pm = (uint32_t)__shfl_up((int)im, 1, 64);
    if (lane == 0) pm = 0;
    for (uint32_t w = 0; w < wv; w++) pm = max(pm, wmx[w]);
    uint64_t first = 0, prev = 0;
    bool have = false;
    /* adjacent keys inside my 32 bins differ in one of the last three bases
       (depths k, k - 1, k - 2): counted in registers */
    uint32_t h0 = 0, h1 = 0, h2 = 0;
#pragma unroll
    for (uint32_t j = 0; j < 32u; j++) {
        if (c[j]) {
            const uint64_t key = kb + j;
            if (have) {   /* first differing base of adjacent keys (k_sp_wprefix) */
                const uint32_t d = (uint32_t)(key ^ prev);   /* < 32 */
                h0 += d < 4u;
                h1 += d >= 4u && d < 16u;
                h2 += d >= 16u;
            } else {
                first = key;
            }
            prev = key;
            have = true;
        }
    }
    {
        const uint32_t a0 = wsum32(h0), a1 = wsum32(h1), a2 = wsum32(h2);
        if (lane == 0) {
            if (a0) atomicAdd(&hpre[k], a0);
            if (a1) atomicAdd(&hpre[k - 1], a1);
            if (a2) atomicAdd(&hpre[k - 2], a2);
        }
    }
    /* every thread's last key in the (now free) bins' LDS */
    uint64_t *lastk = reinterpret_cast<uint64_t *>(bins);
    lastk[t] = prev;
    __syncthreads();
    if (nz && pm) {
        const uint64_t pk = lastk[pm - 1u];
        const int lz = __clzll((long long)(first ^ pk)) - (64 - 2 * k);
        atomicAdd(&hpre[lz / 2 + 1], 1u);
    }
    if (nz && !pm) fl[2 * (size_t)blk] = first;
    if (nz && off + nz == total) fl[2 * (size_t)blk + 1] = prev;
    /* the nonzero bins out, in rounds of KC_STAGE entries staged in the
       bins' LDS (bin index u16, count u32) and written as contiguous words:
       one thread writing its own bins strided the stores 64 lines per
       instruction, and the output (12 B per distinct k-mer, ~90 GB per
       10 G-base step) cost more than the count */
    constexpr uint32_t KC_STAGE = 8192u;   /* (u16 + u32 each: 48 KiB of the 64) */
    uint16_t *sidx = reinterpret_cast<uint16_t *>(bins);
    uint32_t *scnt = bins + KC_STAGE / 2u;
    const uint64_t kpart = lo + ((uint64_t)blk << 15);
    for (uint32_t r0 = 0; r0 < total; r0 += KC_STAGE) {
        __syncthreads();   /* (the staging area is free: lastk read, or the last round written out) */
        uint32_t o = off;
#pragma unroll
        for (uint32_t j = 0; j < 32u; j++) {
            if (c[j]) {
                if (o >= r0 && o < r0 + KC_STAGE) {
                    sidx[o - r0] = (uint16_t)(t * 32u + j);
                    scnt[o - r0] = c[j];
                }
                o++;
            }
        }
        __syncthreads();
        const uint32_t nr = min(KC_STAGE, total - r0);
#ifndef KPX_NOOUT
        for (uint32_t i = t; i < nr; i += 1024u) {
            __builtin_nontemporal_store((uint64_t)(kpart + sidx[i]), out_k + bprefix + r0 + i);
            __builtin_nontemporal_store(scnt[i], out_c + bprefix + r0 + i);
        }
#endif
    }
    /* the rollover check: a bin past 2^32 codes wrapped, so its sum falls
       short of the codes (less the pads) */
    unsigned long long v10[10];
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(st[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wred[wv][q] = v10[q];
    __syncthreads();
    if (t < 10) {
        unsigned long long a = 0;
        for (uint32_t w = 0; w < 16u; w++) a += wred[w][t];
        if (a) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + t], a);
        if (t == 1 && a != (uint64_t)m.n + extra) atomicOr(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 10], 1ull);
    }
    if (t < 24 && hpre[t]) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 11 + t], (unsigned long long)hpre[t]);
}

/*
 * Wide passes (18 <= k <= 20, a key range of more than 2^32 keys): the same
 * two partition levels (64-bit keys in, the parts' codes 32-bit), then each
 * part -- up to KS_CAP keys of at most 23 bits, ~10 K at k = 20 over 10 G
 * bases -- sorted in LDS instead of counted: bucketed by its top 8 bits
 * (LDS histogram, scan, scatter), each bucket sorted by one wave in
 * registers (a bitonic network over 64 N keys, N = 1..16 per lane), then run-
 * length encoded.  A part or bucket above those sizes (a k-mer repeated
 * tens of thousands of times in one part) flags the pass, which then takes
 * the library sort (fks_sort_runs) instead.
 */
#define KS_CAP 24576u        /* k_kp_sort<KS_CAP>: one block per CU */
#define KS_CAP_S 12288u      /* k_kp_sort<KS_CAP_S>: two (every part of the pass fits) */
#define FK_FAULT_SORTCAP 8u

/* bitonic sort of the 64 N values x[i] (element i * 64 + lane), ascending */
template <int N>
__device__ __forceinline__ void wave_bitonic(uint32_t (&x)[N]) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t s2 = 2; s2 <= 64u * N; s2 <<= 1) {
#pragma unroll
        for (uint32_t d = s2 >> 1; d > 0; d >>= 1) {
            if (d >= 64) {
                const uint32_t dr = d / 64;
#pragma unroll
                for (int i = 0; i < N; i++) {
                    if ((uint32_t)i & dr) continue;
                    const int j = i | (int)dr;
                    const uint32_t e = (uint32_t)i * 64u + lane;
                    const bool up = (e & s2) == 0;
                    const uint32_t a = x[i], b = x[j];
                    x[i] = up ? min(a, b) : max(a, b);
                    x[j] = up ? max(a, b) : min(a, b);
                }
            } else {
#pragma unroll
                for (int i = 0; i < N; i++) {
                    const uint32_t e = (uint32_t)i * 64u + lane;
                    const uint32_t o = (uint32_t)__shfl_xor((int)x[i], (int)d, 64);
                    const bool up = (e & s2) == 0, low = (lane & d) == 0;
                    x[i] = (low == up) ? min(x[i], o) : max(x[i], o);
                }
            }
        }
    }
}

/* Batcher's odd-even merge sort of N (a power of two) registers, ascending
   (63 compare-exchanges at N = 16, every index a constant) */
template <int N>
__device__ __forceinline__ void reg_sort(uint32_t (&x)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; i++)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const uint32_t a = x[i + j], b = x[i + j + k];
                        x[i + j] = min(a, b);
                        x[i + j + k] = max(a, b);
                    }
}

template <int N>
__device__ __forceinline__ void wave_sort_bucket(uint32_t *k, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t e = (uint32_t)i * 64u + lane;
        x[i] = e < n ? k[e] : ~0u;
    }
    wave_bitonic<N>(x);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t e = (uint32_t)i * 64u + lane;
        if (e < n) k[e] = x[i];
    }
}

template <uint32_t CAP>
__global__ void __launch_bounds__(1024)
k_kp_sort(const uint32_t *in, const PartMeta *meta, uint64_t cap_in, uint64_t lo, uint32_t psh, uint64_t npads,
          const unsigned long long *tcount, uint32_t top_part, uint32_t nparts, int k, unsigned long long *flags,
          uint64_t *out_k, uint32_t *out_c, unsigned long long *slots, uint64_t *fl, unsigned long long *err) {
    constexpr uint32_t KSI = CAP / 1024u;
    extern __shared__ uint32_t keys[];   /* CAP keys, then CAP + 1 u16 run starts */
    uint16_t *const rs = reinterpret_cast<uint16_t *>(keys + CAP);
    /* the bucket cursors live where the run starts go later (two blocks of
       the small instance per CU: 80 KB of LDS each at most) */
    uint32_t *const bh = reinterpret_cast<uint32_t *>(rs);
    __shared__ uint32_t bo[1025];
    __shared__ unsigned long long wred[16][10];
    __shared__ uint32_t hpre[24];
    __shared__ uint32_t wnz[16];
    __shared__ unsigned long long bprefix;
    __shared__ uint32_t bad, vblk;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    bh[t] = 0;
    if (t < 24) hpre[t] = 0;
    if (t == 0) {
        bad = 0;
        vblk = (uint32_t)atomicAdd(&flags[nparts], 1ull);   /* (k_kp_count: start order) */
    }
    __syncthreads();
    const uint32_t blk = vblk;
    PartMeta m = meta[blk];
    if (m.off + m.n > cap_in) {
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_META);
        m.n = 0;
        m.off = 0;
    }
    if (m.n > CAP) {   /* too many keys for one block's LDS: the library sort */
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_SORTCAP);
        m.n = 0;
    }
    const uint32_t n = m.n, bsh = psh - 10u;
    /* 1. bucket by the top 10 bits of the part's code (~10 keys a bucket) */
    uint32_t v[KSI];
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++) {
        v[j] = j * 1024u + t < n ? in[m.off + j * 1024u + t] : 0u;
        if (j * 1024u + t < n) atomicAdd(&bh[v[j] >> bsh], 1u);
    }
    __syncthreads();
    {   /* bucket t's start: a block scan */
        const uint32_t c = bh[t], inc = wscan_incl32(c);
        if (lane == 63) wnz[wv] = inc;
        __syncthreads();
        uint32_t before = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16u; w++) before += w < wv ? wnz[w] : 0u;
        bo[t] = bh[t] = before + inc - c;
        if (t == 1023) bo[1024] = before + inc;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++)
        if (j * 1024u + t < n) keys[atomicAdd(&bh[v[j] >> bsh], 1u)] = v[j];
    __syncthreads();
    /* 2. bucket t of up to 16 keys sorted by thread t in registers; the
       larger ones (~2 % at 10 a bucket on average) each by one wave */
#ifndef KPX_NOSORT
    {
        const uint32_t b0 = bo[t], nb = bo[t + 1] - b0;
        if (nb > 1u && nb <= 16u) {
            uint32_t x[16];
#pragma unroll
            for (uint32_t i = 0; i < 16u; i++) x[i] = i < nb ? keys[b0 + i] : ~0u;
            reg_sort<16>(x);
#pragma unroll
            for (uint32_t i = 0; i < 16u; i++)
                if (i < nb) keys[b0 + i] = x[i];
        }
    }
#endif
    for (unsigned long long big = __ballot(bo[wv * 64u + lane + 1] - bo[wv * 64u + lane] > 16u); big; big &= big - 1) {
        const uint32_t b = wv * 64u + (uint32_t)__builtin_ctzll(big);
        const uint32_t b0 = bo[b], nb = bo[b + 1] - b0;
#ifdef KPX_NOSORT
        continue;
#endif
        if (nb <= 64) wave_sort_bucket<1>(keys + b0, nb);
        else if (nb <= 128) wave_sort_bucket<2>(keys + b0, nb);
        else if (nb <= 256) wave_sort_bucket<4>(keys + b0, nb);
        else if (nb <= 512) wave_sort_bucket<8>(keys + b0, nb);
        else if (nb <= 1024) wave_sort_bucket<16>(keys + b0, nb);
        else if (lane == 0) bad = 1;
    }
    __syncthreads();
    if (bad) {
        if (t == 0) atomicOr(err, (unsigned long long)FK_FAULT_SORTCAP);
    }
    const uint32_t nn = bad ? 0u : n;
    /* 3. runs: thread t takes positions [t * KSI, +KSI); a run
       starts where the key changes */
    const uint32_t p0 = t * KSI;
    uint32_t nz = 0;
#pragma unroll
    for (uint32_t j = 0; j < KSI; j++) {
        const uint32_t i = p0 + j;
        if (i < nn && (i == 0 || keys[i] != keys[i - 1])) nz++;
    }
    const uint32_t inc = wscan_incl32(nz);
    if (lane == 63) wnz[wv] = inc;
    __syncthreads();
    uint32_t before = 0, runs = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16u; w++) {
        const uint32_t x = wnz[w];
        before += w < wv ? x : 0u;
        runs += x;
    }
    /* the top key 4^k - 1 (when the pass holds it: the last key of the top
       part) was only counted (k_kpart): its real windows, the pads taken
       off, are one more run after this part's others */
    const unsigned long long extra = blk == top_part ? *tcount - npads : 0ull;
    const uint32_t total = runs + (extra ? 1u : 0u);
    const uint32_t off = before + inc - nz;
    /* every run's start in LDS (rs[runs] = the end), so that run r is
       written by thread r % 1024: contiguous stores */
    {
        uint32_t o = off;
#pragma unroll
        for (uint32_t j = 0; j < KSI; j++) {
            const uint32_t i = p0 + j;
            if (i < nn && (i == 0 || keys[i] != keys[i - 1])) rs[o++] = (uint16_t)i;
        }
        if (t == 0) rs[runs] = (uint16_t)nn;
    }
    if (wv == 0) {
#ifdef KPX_NOLB
        const unsigned long long pre = 0;
#else
        const unsigned long long pre = chain_prefix(flags, blk, total, err);
#endif
        if (lane == 0) {
            bprefix = pre;
            if (!total) fl[2 * (size_t)blk] = KP_EMPTY;
        }
    }
    __syncthreads();
    const int fs = 2 * (k - 1);
    const uint64_t kb = lo + ((uint64_t)blk << psh);
    /* (named accumulators: a runtime index into a register array lives in
       scratch memory; the first base is the part's, psh < 2k - 2) */
    unsigned long long l0 = 0, l1 = 0, l2 = 0, l3 = 0, nd = 0;
    for (uint32_t r = t; r < runs; r += 1024u) {
        const uint32_t i = rs[r];
        const uint64_t key = kb + keys[i];
        const uint32_t c = (uint32_t)rs[r + 1] - i;
#ifndef KPX_NOOUT
        __builtin_nontemporal_store(key, out_k + bprefix + r);
        __builtin_nontemporal_store(c, out_c + bprefix + r);
#endif
        const uint32_t ld = (uint32_t)(key & 3);
        nd += 1;
        l0 += ld == 0 ? c : 0u;
        l1 += ld == 1 ? c : 0u;
        l2 += ld == 2 ? c : 0u;
        l3 += ld == 3 ? c : 0u;
        if (r > 0) {   /* against the run before it, in this part */
            const int lz = __clzll((long long)(key ^ (kb + keys[i - 1]))) - (64 - 2 * k);
            atomicAdd(&hpre[lz / 2 + 1], 1u);
        }
        if (r == 0) fl[2 * (size_t)blk] = key;
        if (r + 1 == total) fl[2 * (size_t)blk + 1] = key;
    }
    if (t == 0 && extra) {   /* the top key's run, last in the part */
        const uint64_t key = (1ull << (2 * k)) - 1;
        const uint32_t c = (uint32_t)extra;
        out_k[bprefix + runs] = key;
        out_c[bprefix + runs] = c;
        nd += 1;
        l3 += c;   /* (the key 4^k - 1 ends in base T = 3) */
        if (runs) {
            const int lz = __clzll((long long)(key ^ (kb + keys[nn - 1]))) - (64 - 2 * k);
            atomicAdd(&hpre[lz / 2 + 1], 1u);
        } else {
            fl[2 * (size_t)blk] = key;
        }
        fl[2 * (size_t)blk + 1] = key;
        if (extra >> 32) atomicOr(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 10], 1ull);   /* a u32 count wrapped */
    }
    const unsigned long long sum = l0 + l1 + l2 + l3;
    const uint32_t fd = (uint32_t)((kb >> fs) & 3);
    const unsigned long long st[10] = {nd, sum, l0, l1, l2, l3, fd == 0 ? sum : 0ull, fd == 1 ? sum : 0ull,
                                       fd == 2 ? sum : 0ull, fd == 3 ? sum : 0ull};
    unsigned long long v10[10];
#pragma unroll
    for (int q = 0; q < 10; q++) v10[q] = wsum64(st[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 10; q++) wred[wv][q] = v10[q];
    __syncthreads();
    if (t < 10) {
        unsigned long long a = 0;
        for (uint32_t w = 0; w < 16u; w++) a += wred[w][t];
        if (a) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + t], a);
    }
    if (t < 24 && hpre[t]) atomicAdd(&slots[(blk % KP_SLOTS) * KP_SLOT_W + 11 + t], (unsigned long long)hpre[t]);
}

/* the partials into the pass accumulators (FKS_ACC layout), the prefix
   histogram of each nonempty part's first key against the last key of the
   nonempty part before it, and the pass's distinct count (res[0]) */
__global__ void __launch_bounds__(256)
k_kp_fold(const unsigned long long *slots, const uint64_t *fl, uint32_t nparts, int k,
          const unsigned long long *flags, unsigned long long *dacc, unsigned long long *res) {
    __shared__ uint32_t h[24];
    if (threadIdx.x < 24) h[threadIdx.x] = 0;
    __syncthreads();
    if (blockIdx.x == 0) {
        if (threadIdx.x < 10) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a += slots[sl * KP_SLOT_W + threadIdx.x];
            if (a) atomicAdd(&dacc[threadIdx.x], a);
        } else if (threadIdx.x == 10) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a |= slots[sl * KP_SLOT_W + 10];
            if (a) atomicAdd(&dacc[FKS_ACC_ROLL], 1ull);   /* (k_sp_stats adds wrapped counts' high words) */
        } else if (threadIdx.x >= 32 && threadIdx.x < 56) {
            unsigned long long a = 0;
            for (uint32_t sl = 0; sl < KP_SLOTS; sl++) a += slots[sl * KP_SLOT_W + 11 + (threadIdx.x - 32)];
            if (a) atomicAdd(&dacc[FKS_ACC_WPREFIX + (threadIdx.x - 32)], a);
        } else if (threadIdx.x == 64) {
            res[0] = flags[nparts - 1] & ((1ull << 62) - 1);
        }
    }
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += gridDim.x * blockDim.x) {
        const uint64_t first = fl[2 * (size_t)p];
        if (first == KP_EMPTY || p == 0) continue;
        uint32_t q = p - 1;
        while (q > 0 && fl[2 * (size_t)q] == KP_EMPTY) q--;
        if (fl[2 * (size_t)q] == KP_EMPTY) continue;
        const uint64_t pk = fl[2 * (size_t)q + 1];
        const int lz = __clzll((long long)(first ^ pk)) - (64 - 2 * k);
        atomicAdd(&h[lz / 2 + 1], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 24 && h[threadIdx.x]) atomicAdd(&dacc[FKS_ACC_WPREFIX + threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

/* The pass (keys lo + r for the n 32-bit r, npads of them the pad
   0xFFFFFFFF) into its runs at out_k / out_c: *nw of them */
static int sp_count_runs32(fk_engine *e, const uint32_t *keys, uint64_t n, uint64_t lo, uint64_t npads,
                           unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw) {
    *nw = 0;
    if (n == 0) return FK_OK;
    const int k = e->k;
    PartGeo pg{};
    pg.nslices = 2048u;
    pg.split = 6u;   /* 2^21-bin coarse slices, 64 parts of 2^15 */
    pg.batch = KP_BATCH;
    const uint32_t grid = (uint32_t)std::max(1, e->cus);
    pg.rounds = (uint32_t)((n + (uint64_t)grid * KP_BATCH - 1) / ((uint64_t)grid * KP_BATCH));
    pg.rows = grid * pg.rounds;
    pg.flag = nullptr;
    const uint64_t ncodes = (uint64_t)pg.rows * KP_BATCH;   /* u32 codes */
    const uint32_t nparts = 2048u << 6;
    int rc = sp_ensure((void **)&e->d_codes, &e->codes_cap, 2 * ncodes, sizeof(uint16_t));
    if (!rc) rc = sp_ensure((void **)&e->d_pidx, &e->pidx_cap, (uint64_t)pg.rows * 2048u, sizeof(uint32_t));
    if (!rc) rc = sp_ensure((void **)&e->d_parts, &e->parts_cap, n + 8ull * nparts + 16, sizeof(uint16_t));
    if (rc) return rc;
    if (!e->d_pmeta && hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
        return FK_E_OOM;
    DevScratch flags, slots, fl, res;
    if (!flags.alloc((size_t)(nparts + 1) * 8) || !slots.alloc((size_t)KP_SLOTS * KP_SLOT_W * 8) ||
        !fl.alloc((size_t)nparts * 16) || !res.alloc(16))
        return FK_E_OOM;
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
    unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
    HIPCHK(hipMemsetAsync(alloc, 0, 2 * sizeof(unsigned long long), e->stream));
    HIPCHK(hipMemsetAsync(flags.p, 0, (size_t)(nparts + 1) * 8, e->stream));   /* (+ the block tickets) */
    HIPCHK(hipMemsetAsync(slots.p, 0, (size_t)KP_SLOTS * KP_SLOT_W * 8, e->stream));
    HIPCHK(hipMemsetAsync(res.p, 0, 16, e->stream));
    unsigned long long *tcount = res.as<unsigned long long>() + 1;
    hipLaunchKernelGGL(k_kpart<uint32_t>, dim3(grid), dim3(1024), (size_t)KP_BATCH * 4, e->stream, keys, n, pg, 0ull,
                       0ull, 21u, 0xFFFFFFFFull, tcount);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_repart<uint16_t>, dim3(2048u / REPART_G), dim3(1024), 0, e->stream, pg, e->d_parts, alloc,
                       meta, (uint64_t)e->parts_cap, alloc + 1, 15u, nullptr);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_kp_count, dim3(nparts), dim3(1024), (size_t)KC_WORDS * 4, e->stream, (const uint16_t *)e->d_parts,
                       (const PartMeta *)meta, (uint64_t)e->parts_cap, lo, npads, (const unsigned long long *)tcount, nparts,
                       k, flags.as<unsigned long long>(), out_k, out_c, slots.as<unsigned long long>(), fl.as<uint64_t>(),
                       alloc + 1);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_kp_fold, dim3(64), dim3(256), 0, e->stream, (const unsigned long long *)slots.p,
                       (const uint64_t *)fl.p, nparts, k, (const unsigned long long *)flags.p, dacc,
                       res.as<unsigned long long>());
    HIPCHK(hipGetLastError());
    unsigned long long r[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&r[0], res.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&r[1], alloc + 1, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (r[1]) return FK_E_INTERNAL;
    *nw = r[0];
    return FK_OK;
}

/* A wide pass (keys[0, n) in [lo, hi), hi - lo > 2^32, npads of them the
   pad 4^k - 1) into its runs at out_k / out_c (*nw).  `fallback` is set
   when a part or bucket is too large for k_kp_sort: nothing was folded into
   dacc and the caller sorts the pass with the library instead. */
static int sp_sort_runs64(fk_engine *e, const uint64_t *keys, uint64_t n, uint64_t lo, uint64_t hi, uint64_t npads,
                          unsigned long long *dacc, uint64_t *out_k, uint32_t *out_c, uint64_t *nw, bool *fallback) {
    *nw = 0;
    *fallback = false;
    if (n == 0) return FK_OK;
    const int k = e->k;
    uint32_t sbits = 33;
    while (sbits < 64 && ((hi - lo - 1) >> sbits)) sbits++;
    /* 2048 coarse slices of 128 parts (k_repart: 4 slices per block): at k
       = 20 a pass of up to 2^32 keys leaves ~16 K per part, within k_kp_sort's
       KS_CAP (64 parts per slice left ~33 K, and every pass took the library
       sort) */
    const uint32_t cs = sbits - 11, psh = cs - 7;
    PartGeo pg{};
    pg.nslices = 2048u;
    pg.split = 7u;
    pg.batch = KP_BATCH;
    const uint32_t grid = (uint32_t)std::max(1, e->cus);
    pg.rounds = (uint32_t)((n + (uint64_t)grid * KP_BATCH - 1) / ((uint64_t)grid * KP_BATCH));
    pg.rows = grid * pg.rounds;
    pg.flag = nullptr;
    const uint64_t ncodes = (uint64_t)pg.rows * KP_BATCH;
    const uint32_t nparts = 2048u << 7;
    int rc = sp_ensure((void **)&e->d_codes, &e->codes_cap, 2 * ncodes, sizeof(uint16_t));
    if (!rc) rc = sp_ensure((void **)&e->d_pidx, &e->pidx_cap, (uint64_t)pg.rows * 2048u, sizeof(uint32_t));
    /* (the part streams as 32-bit codes: twice the u16 capacity) */
    if (!rc) rc = sp_ensure((void **)&e->d_parts, &e->parts_cap, 2 * (n + 8ull * nparts + 16), sizeof(uint16_t));
    if (rc) return rc;
    if (!e->d_pmeta && hipMalloc(&e->d_pmeta, (size_t)2048 * REPART_METAP * sizeof(PartMeta) + 64) != hipSuccess)
        return FK_E_OOM;
    DevScratch flags, slots, fl, res;
    if (!flags.alloc((size_t)(nparts + 1) * 8) || !slots.alloc((size_t)KP_SLOTS * KP_SLOT_W * 8) ||
        !fl.alloc((size_t)nparts * 16) || !res.alloc(16))
        return FK_E_OOM;
    pg.codes = e->d_codes;
    pg.idx = e->d_pidx;
    PartMeta *meta = static_cast<PartMeta *>(e->d_pmeta);
    unsigned long long *alloc = reinterpret_cast<unsigned long long *>(meta + (size_t)2048 * REPART_METAP);
    uint32_t *parts32 = reinterpret_cast<uint32_t *>(e->d_parts);
    const uint64_t cap32 = e->parts_cap / 2;
    HIPCHK(hipMemsetAsync(alloc, 0, 3 * sizeof(unsigned long long), e->stream));
    HIPCHK(hipMemsetAsync(flags.p, 0, (size_t)(nparts + 1) * 8, e->stream));   /* (+ the block tickets) */
    HIPCHK(hipMemsetAsync(slots.p, 0, (size_t)KP_SLOTS * KP_SLOT_W * 8, e->stream));
    HIPCHK(hipMemsetAsync(res.p, 0, 16, e->stream));
    unsigned long long *tcount = res.as<unsigned long long>() + 1;
    /* the top key 4^k - 1 (the pads' value; past hi they are left out as
       out of range) counted apart when the pass holds it */
    const uint64_t top = (1ull << (2 * k)) - 1;
    const bool top_in = top >= lo && top < hi;
    hipLaunchKernelGGL(k_kpart<uint64_t>, dim3(grid), dim3(1024), (size_t)KP_BATCH * 4, e->stream, keys, n, pg, lo, hi,
                       cs, top_in ? top : ~0ull, tcount);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL((k_repart<uint32_t, 4u>), dim3(2048u / 4u), dim3(1024), 0, e->stream, pg, parts32, alloc, meta,
                       cap32, alloc + 1, psh, alloc + 2);
    HIPCHK(hipGetLastError());
    unsigned long long pmax = 0;
    HIPCHK(hipMemcpyAsync(&pmax, alloc + 2, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (pmax > KS_CAP) {   /* a part past one block's LDS: the library sort */
        *fallback = true;
        return FK_OK;
    }
    const bool small = pmax <= KS_CAP_S;
    const uint32_t top_part = top_in ? (uint32_t)((top - lo) >> psh) : ~0u;
    if (small)
        hipLaunchKernelGGL(k_kp_sort<KS_CAP_S>, dim3(nparts), dim3(1024), (size_t)KS_CAP_S * 6 + 16, e->stream,
                           (const uint32_t *)parts32, (const PartMeta *)meta, cap32, lo, psh, top_in ? npads : 0ull,
                           (const unsigned long long *)tcount, top_part, nparts, k, flags.as<unsigned long long>(), out_k,
                           out_c, slots.as<unsigned long long>(), fl.as<uint64_t>(), alloc + 1);
    else
        hipLaunchKernelGGL(k_kp_sort<KS_CAP>, dim3(nparts), dim3(1024), (size_t)KS_CAP * 6 + 16, e->stream,
                           (const uint32_t *)parts32, (const PartMeta *)meta, cap32, lo, psh, top_in ? npads : 0ull,
                           (const unsigned long long *)tcount, top_part, nparts, k, flags.as<unsigned long long>(), out_k,
                           out_c, slots.as<unsigned long long>(), fl.as<uint64_t>(), alloc + 1);
    HIPCHK(hipGetLastError());
    unsigned long long ferr = 0;
    HIPCHK(hipMemcpyAsync(&ferr, alloc + 1, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (ferr & FK_FAULT_SORTCAP) {
        *fallback = true;
        return FK_OK;
    }
    if (ferr) return FK_E_INTERNAL;
    hipLaunchKernelGGL(k_kp_fold, dim3(64), dim3(256), 0, e->stream, (const unsigned long long *)slots.p,
                       (const uint64_t *)fl.p, nparts, k, (const unsigned long long *)flags.p, dacc,
                       res.as<unsigned long long>());
    HIPCHK(hipGetLastError());
    unsigned long long r0 = 0;
    HIPCHK(hipMemcpyAsync(&r0, res.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    *nw = r0;
    return FK_OK;
}

/*
 * The sparse table (17 <= k <= 20) from the retained input, in key-range
 * passes (k_sp_emit):
 *   1. SP_HIST: window count per bucket (the top SP_BUCKET_BITS index bits)
 *      and every short walk;
 *   2. the passes: consecutive buckets merged while their windows fit one
 *      sorted pass (capped by free HBM, or FINDKMER_TUNE sp_pass); a single
 *      bucket above the cap is counted densely (2^(2k - SP_BUCKET_BITS) u64);
 *   3. per pass: emit, sort + run-length encode (or select the nonzero dense
 *      counts), statistics, prefix histogram, short-walk prefix marks, and
 *      the runs kept as one part of the table.
 * `seq`: the final run's length (its short walk if 1 <= seq < k).
 */
static int sparse_finish(fk_engine *e, int32_t seq) {
    const int k = e->k;
    e->sp_distinct = 0;
    memset(e->sp_tstat, 0, sizeof e->sp_tstat);
    e->sp_roll = e->sp_nodes = 0;
    const uint32_t nbk = 1u << SP_BUCKET_BITS;
    const uint32_t shift = 2u * (uint32_t)k - SP_BUCKET_BITS;
    {   /* the HIST launch needs the larger LDS; set it once for every mode */
        const size_t lds = (size_t)SP_WAVES * FK_TILE_BYTES * sizeof(uint64_t) + (size_t)nbk * sizeof(uint32_t);
        HIPCHK(hipFuncSetAttribute((const void *)k_sp_emit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        for (const void *f : {(const void *)k_kpart<uint32_t>, (const void *)k_kpart<uint64_t>})
            HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(KP_BATCH * 4)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_sort<KS_CAP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KS_CAP * 6 + 16)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_sort<KS_CAP_S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KS_CAP_S * 6 + 16)));
        HIPCHK(hipFuncSetAttribute((const void *)k_kp_count, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(KC_WORDS * 4)));
    }
    DevScratch acc, bh, ctr, pctr;
    if (!acc.alloc(FKS_ACC_N * sizeof(unsigned long long)) || !bh.alloc((size_t)nbk * 8) || !ctr.alloc(24) ||
        !pctr.alloc(2 * SP_MAXP * sizeof(unsigned long long)))
        return FK_E_OOM;
    /* a keys pass claims its output in SP_CHUNKs per wave: at most one
       chunk's worth of pads per wave of every emit launch */
    uint64_t pad_max = 0;
    for (const auto &sg : e->spsegs)
        if (sg.nranges)
            pad_max += std::max<uint64_t>(1, std::min<uint64_t>((sg.nranges + SP_WAVES - 1) / SP_WAVES, (uint64_t)e->cus * 8)) *
                       SP_WAVES * SP_CHUNK;
    unsigned long long *dacc = acc.as<unsigned long long>();
    unsigned long long *nctr = ctr.as<unsigned long long>();
    HIPCHK(hipMemsetAsync(dacc, 0, FKS_ACC_N * sizeof(unsigned long long), e->stream));

    /* the pass cap: window keys one sorted pass may hold.  A pass needs
       ~56 B per key (emitted 8, sorted 8, runs 8, run lengths 8, rocPRIM's
       scratch ~8, the part's keys 8 + counts 4, handed over), and the parts
       of all passes together up to 12 B per window (distinct <= windows):
       reserve those first */
    const uint64_t wins = e->last.acc[ACC_WIN];
    uint64_t cap = e->sp_pass;
    uint64_t room = 0;   /* bytes for the passes' key lists and their processing */
    {
        size_t fr = 0, tot = 0;
        HIPCHK(hipMemGetInfo(&fr, &tot));
        /* plus what the engine's sparse buffers already hold (reused, or
           freed and reallocated larger) */
        const uint64_t held = e->spk_cap * 8 + e->spc_cap * 4 + e->emit_cap * 8 + e->spdense_cap * 8 +
                              e->fks.sorted_cap + e->fks.c64_cap + e->fks.tmp_cap + e->codes_cap * 2 +
                              e->parts_cap * 2 + e->pidx_cap * 4;
        const uint64_t avail = (uint64_t)fr + held;
        const uint64_t reserve = (1ull << 30) + 12 * wins;
        room = avail > reserve ? avail - reserve : 0;
    }
    /* a pass takes ~8 B per key for its list and ~9 for its processing
       (k_kpart's row codes 4 + run words, k_repart's part streams 2-4, the
       library sort's ~40 if a pass falls back to it: kept inside the cap) */
    if (!cap) cap = std::max<uint64_t>(1u << 20, std::min<uint64_t>(room / 56, 1ull << 32));
    /* the table's storage: room for every window (distinct <= windows) */
    {
        int rc = sp_ensure((void **)&e->d_spk, &e->spk_cap, wins + 1, 8);
        if (!rc) rc = sp_ensure((void **)&e->d_spc, &e->spc_cap, wins + 1, 4);
        if (rc) return rc;
    }
    /* all windows in one pass (the feed counted them): no histogram launch,
       the keys pass collects the short walks.  Not k = 17: its passes span
       2^32 keys, which sp_count_runs32 counts instead of sorting */
    const bool single = wins <= cap && k != 17;

    const bool tail = !e->state.hdr && seq >= 1 && seq < k;
    const bool nodes = e->opts.want_nodes != 0;
    uint64_t scap = std::max<uint64_t>(1024, e->keep_len / 64);
    DevScratch shorts, found;
    uint64_t ns = 0;
    /* the collected short walks (+ the input's last run, shorter than k:
       :1059-1062 at EOF), distinct, with their found flags */
    auto prep_shorts = [&]() -> int {
        if (tail) {
            const uint64_t v = SP_SHORT | ((uint64_t)seq << 40) | fk_sigma(e->state.code & ((1ull << (2 * seq)) - 1));
            HIPCHK(hipMemcpyAsync(shorts.as<uint64_t>() + ns, &v, sizeof v, hipMemcpyHostToDevice, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            ns++;
        }
        if (!nodes) ns = 0;
        if (ns > 1) {   /* nodeCounter counts distinct prefixes: drop repeated walks */
            uint64_t nu = 0;
            if (fks_unique(&e->fks, shorts.as<uint64_t>(), ns, e->stream, &nu)) return FK_E_HIP;
            ns = nu;
        }
        if (ns) {
            if (!found.alloc(ns * 20)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(found.p, 0, ns * 20, e->stream));
        }
        return FK_OK;
    };

    struct Pass { uint32_t b0, b1; uint64_t n; bool dense; };
    std::vector<Pass> passes;
    if (single) {
        passes.push_back({0, nbk, wins, false});
    } else {
        /* 1. bucket histogram and short walks (a second run if the list overflowed) */
        for (int attempt = 0; attempt < 2; attempt++) {
            if (!shorts.alloc((scap + 1) * 8)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(bh.p, 0, (size_t)nbk * 8, e->stream));
            HIPCHK(hipMemsetAsync(nctr, 0, 16, e->stream));
            SpEmit em{};
            em.mode = SP_HIST;
            em.shift = shift;
            em.bhist = bh.as<unsigned long long>();
            em.nbuckets = nbk;
            em.shorts = shorts.as<uint64_t>();
            em.nshort = nctr + 1;
            em.short_cap = scap;
            int rc = sp_emit_all(e, em);
            if (rc) return rc;
            unsigned long long got = 0;
            HIPCHK(hipMemcpyAsync(&got, nctr + 1, sizeof got, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            ns = got;
            if (ns <= scap) break;
            if (attempt) return FK_E_HIP;
            scap = ns;
        }
        int rc = prep_shorts();
        if (rc) return rc;
        std::vector<unsigned long long> hb(nbk);
        HIPCHK(hipMemcpyAsync(hb.data(), bh.p, (size_t)nbk * 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        /* 2. passes: [b0, b1) buckets; dense when one bucket exceeds the
           cap.  A pass stays inside one aligned block of 2^P keys: k = 17
           (2^34 keys), P = 32, counts 32-bit keys (half the bytes; 4 such
           blocks, as many passes as a 10 G-base input needs anyway); k >= 18
           takes the largest P whose blocks hold at most `cap` windows on
           average, so that a sorted pass spans a power of two and
           sp_sort_runs64's 2^18 parts split it evenly (a pass of 0.28 x 2^40
           keys at k = 20 left half of them empty, and the rest twice as
           large as one block's LDS sorts at full occupancy) */
        uint32_t P = 2u * (uint32_t)k;
        if (k == 17) {
            P = 32;
        } else if (k > 17) {
            P = shift;
            while (P < 2u * (uint32_t)k && (wins >> (2u * (uint32_t)k - P - 1u)) <= cap) P++;
        }
        for (uint32_t b = 0; b < nbk;) {
            if (!hb[b]) { b++; continue; }
            if (hb[b] > cap) { passes.push_back({b, b + 1, hb[b], true}); b++; continue; }
            uint32_t b1 = b;
            uint64_t n = 0;
            while (b1 < nbk && hb[b1] <= cap && n + hb[b1] <= cap && (b1 >> (P - shift)) == (b >> (P - shift)))
                n += hb[b1++];
            passes.push_back({b, b1, n, false});
            b = b1;
        }
    }

    /* 3. the passes.  Consecutive sorted or counted passes share one walk
       (up to SP_MAXP key ranges, their lists side by side in d_emit) as
       far as their lists fit beside one pass's processing */
    uint64_t prev_last = 0;
    bool have_prev = false;
    std::vector<unsigned long long> edges(24, 0);   /* prefix histogram across pass boundaries */
    const uint64_t list_room = room > 9 * cap ? room - 9 * cap : 0;
    bool solo = false;   /* a pass fell back to the library sort: one pass per walk from there on */
    /* after a pass: its runs joined to the table (short-walk marks, the
       prefix pair across the pass boundary) */
    auto join = [&](uint64_t *out_k, uint64_t nw) -> int {
        if (!nw) return FK_OK;
        if (e->sp_distinct + nw > e->spk_cap) return FK_E_HIP;   /* cannot happen: distinct <= windows */
        if (ns && fks_short_mark(out_k, nw, shorts.as<uint64_t>(), ns, k, found.as<uint8_t>(), e->stream))
            return FK_E_HIP;
        uint64_t fl[2];
        HIPCHK(hipMemcpyAsync(&fl[0], out_k, 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipMemcpyAsync(&fl[1], out_k + (nw - 1), 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (have_prev) {   /* the adjacent pair across the boundary: first differing base */
            const uint64_t diff = fl[0] ^ prev_last;
            const int lz = __builtin_clzll(diff) - (64 - 2 * k);
            edges[lz / 2 + 1]++;
        }
        prev_last = fl[1];
        have_prev = true;
        e->sp_distinct += nw;
        return FK_OK;
    };
    for (size_t pi = 0; pi < passes.size();) {
        const Pass &p0 = passes[pi];
        uint64_t *out_k = e->d_spk + e->sp_distinct;   /* this pass's runs follow the earlier ones' */
        uint32_t *out_c = e->d_spc + e->sp_distinct;
        if (p0.dense) {
            SpEmit em{};
            em.shift = shift;
            em.lo = (uint64_t)p0.b0 << shift;
            em.hi = (uint64_t)p0.b1 << shift;
            uint64_t nw = 0;
            const uint64_t nd = 1ull << shift;
            int rc = sp_ensure((void **)&e->d_spdense, &e->spdense_cap, nd, 8);
            if (rc) return rc;
            HIPCHK(hipMemsetAsync(e->d_spdense, 0, nd * 8, e->stream));
            em.mode = SP_DENSE;
            em.dense = e->d_spdense;
            rc = sp_emit_all(e, em);
            if (rc) return rc;
            if (fks_dense_runs(&e->fks, em.dense, nd, em.lo, k, e->stream, dacc, out_k, out_c, &nw)) return FK_E_HIP;
            rc = join(out_k, nw);
            if (rc) return rc;
            pi++;
            continue;
        }
        /* the group: its lists' offsets (16-B aligned) in d_emit */
        size_t pj = pi;
        uint64_t bytes = 0, offs[SP_MAXP];
        while (pj < passes.size() && !passes[pj].dense && pj - pi < (solo ? 1u : SP_MAXP)) {
            const uint64_t span = (uint64_t)(passes[pj].b1 - passes[pj].b0) << shift;
            const uint64_t need = (((passes[pj].n + pad_max) * (span <= (1ull << 32) ? 4u : 8u)) + 15) & ~15ull;
            if (pj > pi && bytes + need > list_room) break;
            offs[pj - pi] = bytes;
            bytes += need;
            pj++;
        }
        {
            int rc = sp_ensure((void **)&e->d_emit, &e->emit_cap, bytes / 8 + 2, 8);
            if (rc) return rc;
        }
        SpEmit em{};
        em.shift = shift;
        em.mode = SP_KEYS;
        em.np = (uint32_t)(pj - pi);
        for (uint32_t q = 0; q < SP_MAXP; q++) em.ps[q].lo = ~0ull;
        em.gend = (uint64_t)passes[pj - 1].b1 << shift;
        unsigned long long *pc = pctr.as<unsigned long long>();
        for (uint32_t q = 0; q < em.np; q++) {
            const Pass &ps = passes[pi + q];
            SpPass &sp = em.ps[q];
            sp.lo = (uint64_t)ps.b0 << shift;
            sp.hi = (uint64_t)ps.b1 << shift;
            uint8_t *base = reinterpret_cast<uint8_t *>(e->d_emit) + offs[q];
            const bool rel32 = sp.hi - sp.lo <= (1ull << 32);
            sp.out = rel32 ? nullptr : reinterpret_cast<uint64_t *>(base);
            sp.out32 = rel32 ? reinterpret_cast<uint32_t *>(base) : nullptr;
            sp.cap = ps.n + pad_max;
            sp.ctr = pc + 2 * q;
        }
        unsigned long long got[2 * SP_MAXP] = {};
        for (int attempt = 0; attempt < 2; attempt++) {
            if (single && !shorts.alloc((scap + 1) * 8)) return FK_E_OOM;
            HIPCHK(hipMemsetAsync(nctr, 0, 24, e->stream));
            HIPCHK(hipMemsetAsync(pc, 0, 2 * SP_MAXP * sizeof(unsigned long long), e->stream));
            em.shorts = single ? shorts.as<uint64_t>() : nullptr;   /* the single pass collects them */
            em.nshort = nctr + 1;
            em.short_cap = scap;
            int rc = sp_emit_all(e, em);
            if (rc) return rc;
            unsigned long long nsh = 0;
            HIPCHK(hipMemcpyAsync(got, pc, 2 * SP_MAXP * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipMemcpyAsync(&nsh, nctr + 1, sizeof nsh, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            if (!single || nsh <= scap) {
                if (single) ns = nsh;
                break;
            }
            if (attempt) return FK_E_HIP;
            scap = nsh;
        }
        if (single) {
            int rc = prep_shorts();
            if (rc) return rc;
        }
#ifdef SPX_NOSTORE
        pi = pj;
        continue;
#endif
        for (uint32_t q = 0; q < em.np; q++) {
            const Pass &ps = passes[pi + q];
            const SpPass &sp = em.ps[q];
            const uint64_t claimed = got[2 * q], real = got[2 * q + 1];
            /* the feed's (or the histogram's) count and the walk agree, and
               the claimed slots (windows + pads) fit */
            if (real != ps.n || claimed > sp.cap) return FK_E_HIP;
            uint64_t *ok = e->d_spk + e->sp_distinct;
            uint32_t *oc = e->d_spc + e->sp_distinct;
            uint64_t nw = 0;
            bool lib = false;
            if (sp.out32) {   /* counted, not sorted (sp_count_runs32) */
                int rc = sp_count_runs32(e, sp.out32, claimed, sp.lo, claimed - real, dacc, ok, oc, &nw);
                if (rc) return rc;
            } else {          /* partitioned and sorted in LDS (sp_sort_runs64) */
                int rc = sp_sort_runs64(e, sp.out, claimed, sp.lo, sp.hi, claimed - real, dacc, ok, oc, &nw, &lib);
                if (rc) return rc;
            }
            /* a part or bucket past k_kp_sort's sizes: the library sort,
               which needs the room the group's other lists hold: walk this
               pass again alone */
            if (lib && em.np > 1) {
                solo = true;
                pj = pi + q;
                break;
            }
            if (lib && fks_sort_runs(&e->fks, sp.out, claimed, k, e->stream, dacc, ok, oc, &nw, claimed - real))
                return FK_E_HIP;
            int rc = join(ok, nw);
            if (rc) return rc;
        }
        pi = pj;
    }

    /* 4. totals: statistics, rollover, nodeCounter */
    unsigned long long r[FKS_ACC_N];
    HIPCHK(hipMemcpyAsync(r, dacc, sizeof r, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int q = 0; q < 10; q++) e->sp_tstat[q] = r[q];
    e->sp_roll = r[FKS_ACC_ROLL];
    if (nodes) {
        unsigned long long left = 0;
        if (ns && fks_short_count(&e->fks, shorts.as<uint64_t>(), ns, found.as<uint8_t>(), e->stream, &left))
            return FK_E_HIP;
        if (e->sp_distinct || ns) {
            unsigned long long nd = 0;
            if (e->sp_distinct) {
                unsigned long long run = 1;
                for (int d = 1; d <= k; d++) {
                    run += r[FKS_ACC_WPREFIX + d] + edges[d];
                    nd += run;
                }
            }
            e->sp_nodes = 1 + nd + left;
        }
    }
    return FK_OK;
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

static int sparse_copy(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n,
                       hipMemcpyKind kind) {
    if (!e || !n) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    *n = e->sp_distinct;
    if (!keys && !counts) return FK_OK;
    if (cap < e->sp_distinct) return FK_E_INVALID;
    int rc = set_dev(e);
    if (rc) return rc;
    if (e->sp_distinct) {
        if (keys) HIPCHK(hipMemcpyAsync(keys, e->d_spk, e->sp_distinct * sizeof(uint64_t), kind, e->stream));
        if (counts) HIPCHK(hipMemcpyAsync(counts, e->d_spc, e->sp_distinct * sizeof(uint32_t), kind, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* The sparse table (17 <= k <= 20) after fk_engine_finish: the distinct
   k-mer indices (reference order, ascending = CSV row order) and their u32
   frequencies.  keys/counts may be NULL to ask for *n only. */
extern "C" int fk_engine_sparse(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n) {
    return sparse_copy(e, keys, counts, cap, n, hipMemcpyDeviceToHost);
}

/* The same into device buffers (the multi-GPU exchange's send buffers). */
extern "C" int fk_engine_sparse_device(fk_engine *e, uint64_t *keys, uint32_t *counts, uint64_t cap, uint64_t *n) {
    return sparse_copy(e, keys, counts, cap, n, hipMemcpyDeviceToDevice);
}

/* first index of the ascending device keys[0, n) with key >= want (binary
   search, one key per probe) */
static int sparse_lower_bound(fk_engine *e, uint64_t want, uint64_t *at) {
    uint64_t lo = 0, hi = e->sp_distinct;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        uint64_t v = 0;
        HIPCHK(hipMemcpyAsync(&v, e->d_spk + mid, 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (v < want) lo = mid + 1;
        else hi = mid;
    }
    *at = lo;
    return FK_OK;
}

/* The runs of the finished sparse table whose keys fall in [key_lo, key_hi)
   (a contiguous piece of it: CSV rows key_lo.. in order), to host memory:
   *n receives their number, min(cap, n) are copied (keys/counts may be
   NULL to ask for *n). */
extern "C" int fk_engine_sparse_range(fk_engine *e, uint64_t key_lo, uint64_t key_hi, uint64_t *keys,
                                      uint32_t *counts, uint64_t cap, uint64_t *n) {
    if (!e || !n || key_hi < key_lo) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    uint64_t a = 0, b = 0;
    if ((rc = sparse_lower_bound(e, key_lo, &a)) || (rc = sparse_lower_bound(e, key_hi, &b))) return rc;
    *n = b - a;
    const uint64_t m = std::min(cap, b - a);
    if (m && keys) HIPCHK(hipMemcpyAsync(keys, e->d_spk + a, m * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    if (m && counts)
        HIPCHK(hipMemcpyAsync(counts, e->d_spc + a, m * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return FK_OK;
}

/* The finished sparse table's runs per owner rank: owner of index x is
   x / S, S = ceil(4^k / world) (fk_merge_layout's slices). */
extern "C" int fk_engine_sparse_split(fk_engine *e, int world, uint64_t *counts) {
    if (!e || !counts || world < 1) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    const uint64_t nb = 1ull << (2 * e->k), S = (nb + (uint64_t)world - 1) / (uint64_t)world;
    for (int r = 0; r < world; r++) counts[r] = 0;
    const uint64_t n = e->sp_distinct;
    if (!n) return FK_OK;
    /* the keys are ascending: owners' runs are contiguous; the boundaries by
       binary search over the device keys, one key per probe */
    const uint64_t *keys = e->d_spk;
    uint64_t first = 0, last = 0;
    HIPCHK(hipMemcpyAsync(&first, keys, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&last, keys + (n - 1), 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    const int r0 = (int)(first / S), r1 = (int)(last / S);
    uint64_t at = 0;
    for (int r = r0; r <= r1; r++) {
        uint64_t lo = at, hi = n;   /* first index with key >= (r + 1) * S */
        if (r == r1) {
            lo = n;
        } else {
            const uint64_t want = (uint64_t)(r + 1) * S;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                uint64_t v = 0;
                HIPCHK(hipMemcpyAsync(&v, keys + mid, 8, hipMemcpyDeviceToHost, e->stream));
                HIPCHK(hipStreamSynchronize(e->stream));
                if (v < want) lo = mid + 1;
                else hi = mid;
            }
        }
        counts[r] = lo - at;
        at = lo;
    }
    return FK_OK;
}

/* Replace the finished sparse table by the runs this rank owns after the
   exchange (keys/counts: device, any order, a key possibly from several
   ranks): counts of a key summed, stats[0] = distinct k-mers, stats[1] = the
   sum of their u32 counts (short of the windows when a sum wrapped: the
   rollover check). */
extern "C" int fk_engine_sparse_adopt(fk_engine *e, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                                      uint64_t *stats) {
    if (!e || !stats || (n && (!keys || !counts))) return FK_E_INVALID;
    if (!e->sparse || !e->sp_done) return FK_E_STATE;
    int rc = set_dev(e);
    if (rc) return rc;
    DevScratch acc;
    if (!acc.alloc(FKS_ACC_N * sizeof(unsigned long long))) return FK_E_OOM;
    HIPCHK(hipMemsetAsync(acc.p, 0, FKS_ACC_N * sizeof(unsigned long long), e->stream));
    rc = sp_ensure((void **)&e->d_spk, &e->spk_cap, n + 1, 8);
    if (!rc) rc = sp_ensure((void **)&e->d_spc, &e->spc_cap, n + 1, 4);
    if (rc) return rc;
    uint64_t nw = 0;
    e->sp_distinct = 0;
    if (fks_merge_runs(&e->fks, keys, counts, n, e->k, e->stream, acc.as<unsigned long long>(), e->d_spk, e->d_spc,
                       &nw))
        return FK_E_HIP;
    unsigned long long r[FKS_ACC_N];
    HIPCHK(hipMemcpyAsync(r, acc.p, sizeof r, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->sp_distinct = nw;
    memcpy(e->sp_tstat, r, sizeof e->sp_tstat);
    e->sp_roll = r[FKS_ACC_ROLL];
    stats[0] = r[0];
    stats[1] = r[1];
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
