/*
 * fk_tiles.h -- the device side every counting kernel shares: 16-B-per-lane
 * tiles, base2int (findKmer.cpp:567-589) and shift_left_and_insert (:947-958)
 * as 2-bit codes, transfer functions, counters and the wave helpers.
 */
#pragma once
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
