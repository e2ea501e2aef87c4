// fmx_device.hpp — the arithmetic of the query hot path, shared by the gfx950
// kernels (fmx_query.hip) and a host-side emulation used by the CPU tests
// (tests/emu): bit-plane rank/popcount, the k-mer seed, the LF loop with the
// single-row text verification, and the sampled-SA walk.  Every function is
// __host__ __device__ so the CPU suite runs exactly the code the GPU runs.
#pragma once

#ifndef FMX_NT_NARROW
#define FMX_NT_NARROW 0  // A/B builds: -DFMX_NT_NARROW=1 (see Occ::hot_fetch)
#endif

#include "fmx_internal.hpp"

#define FMX_HD __host__ __device__ __forceinline__

namespace fmx {

// ------------------------------------------------------------------ vectors

template <int VB> struct VecT;
template <> struct VecT<32> { using W = uint32_t; static constexpr int WPP = 1; };
template <> struct VecT<64> { using W = uint64_t; static constexpr int WPP = 1; };
template <> struct VecT<128> { using W = uint64_t; static constexpr int WPP = 2; };  // lo, hi (little-endian u128)

// The N bit planes of one BlockN<V> (components/bwm/blocks/block{2..6}.rs), held in registers.
template <int N, int VB>
struct Planes {
    using W = typename VecT<VB>::W;
    static constexpr int WPP = VecT<VB>::WPP;
    static constexpr int WORDS = N * WPP;
    W w[WORDS];

    // Block::get_remain_count_of (block3.rs:42-55): occurrences of symbol c among
    // the first `rem` symbols of the block (MSB-first); rem == 0 gives 0.
    FMX_HD uint32_t rank(uint32_t rem, uint32_t c) const {
        if constexpr (VB == 128) {
            uint64_t lo = ~0ull, hi = ~0ull;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const bool b = (c >> j) & 1u;
                lo &= b ? w[2 * j] : ~w[2 * j];
                hi &= b ? w[2 * j + 1] : ~w[2 * j + 1];
            }
            if (rem == 0) return 0;
            if (rem <= 64) return (uint32_t)__builtin_popcountll(hi >> (64 - rem));
            return (uint32_t)__builtin_popcountll(hi) + (uint32_t)__builtin_popcountll(lo >> (128 - rem));
        } else {
            W m = ~W(0);
#pragma unroll
            for (int j = 0; j < N; ++j) m &= ((c >> j) & 1u) ? w[j] : W(~w[j]);
            if (rem == 0) return 0;
            if constexpr (VB == 64) return (uint32_t)__builtin_popcountll(m >> (64 - rem));
            else return (uint32_t)__builtin_popcount(m >> (32 - rem));
        }
    }

    // Block::get_symidx_of (block3.rs:57-63): bit VB-1-rem of plane j is bit j.
    FMX_HD uint32_t sym(uint32_t rem) const {
        const uint32_t b = VB - 1 - rem;
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            uint32_t bit;
            if constexpr (VB == 128) bit = b >= 64 ? (uint32_t)(w[2 * j + 1] >> (b - 64)) & 1u
                                                   : (uint32_t)(w[2 * j] >> b) & 1u;
            else bit = (uint32_t)(w[j] >> b) & 1u;
            s |= bit << j;
        }
        return s;
    }

    FMX_HD void load(const uint8_t *p) {
        const W *src = reinterpret_cast<const W *>(p);
#pragma unroll
        for (int j = 0; j < WORDS; ++j) w[j] = src[j];
    }
};

// Select v[idx] (idx < K) with a tree of v_cndmask on the bits of idx: a
// compare-against-constant chain gets lowered to a scratch-memory table
// lookup by the compiler, this form stays in registers.
template <int K, typename T>
FMX_HD T tree_pick(const T *v, uint32_t idx) {
    if constexpr (K == 1) {
        return v[0];
    } else {
        const T lo = tree_pick<K / 2>(v, idx);
        const T hi = tree_pick<K / 2>(v + K / 2, idx);
        return (idx & (K / 2)) ? hi : lo;
    }
}

constexpr int pow2_ceil(int x) { int p = 1; while (p < x) p <<= 1; return p; }

FMX_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// pos / sr and pos % sr for the SA sampling ratio: a shift for powers of two,
// else a multiply-high by ceil(2^64/sr) and one correction — branch-free, so a
// wavefront whose lanes walk different rows stays converged (the generic
// 64-bit divide expands into divergent branches).
FMX_HD uint64_t sr_div(const QueryArgs &a, uint64_t pos, uint64_t &rem) {
    if (a.sr_pow2) {
        rem = pos & a.sr_pow2_mask;
        return pos >> a.sr_shift;
    }
    uint64_t q = mulhi64(pos, a.sr_magic);
    const uint64_t qd = q * a.sr;
    q = qd > pos ? q - 1 : q;
    rem = pos - q * a.sr;
    return q;
}

// ------------------------------------------------------- occ access (rank)

using V4 = uint32_t __attribute__((ext_vector_type(4)));

// REC == 0 — blob layout: rank_checkpoints [P; blocks*sigma] and blocks
//            [BlockN<V>; blocks] are separate arrays (bwm/mod.rs:145-190).
// REC = 64 or 128 — interleaved layout (FMX_OCC_INTERLEAVED): record q (REC
//            bytes, REC-aligned) holds block q's N bit planes verbatim at
//            [0, PB), then its sigma rank checkpoints as P at PBA + c*P (PBA =
//            PB rounded up to P), zero padding to REC.  A rank query of
//            symbol c reads the planes' 16-B chunks and the one chunk holding
//            checkpoint c — all inside the record's line; when PB is not a
//            multiple of 16 the planes' last chunk already holds the first
//            checkpoints.
// REC = 64|kRecPaired or 128|kRecPaired — paired-chunk records, for planes
//            whose size PB is not a multiple of 16 (tail PT = PB % 16 bytes):
//            the PF = PB / 16 whole plane chunks, then checkpoint chunks that
//            each repeat the planes' PT tail bytes followed by PER = (16 -
//            PTA) / P checkpoints from byte PTA (PT rounded up to P).  Every
//            rank query then reads exactly PF + 1 chunks (C2, Block3<u64>,
//            u32: [p0 p1][p2 ck0 ck1][p2 ck2 ck3][p2 ck4 ck5], 2 chunks for
//            every symbol instead of 2 or 3).
// REC = 64|kRecOneHot or 128|kRecOneHot — symbol-mask records, when sigma
//            units fit: unit c (U = VB/8 + P bytes, at c * U) is symbol c's
//            occurrence mask over the block — the AND of the N planes (or
//            their complements) that Block::get_remain_count_of forms for c
//            (block3.rs:42-55), precomputed once per block — followed by the
//            block's checkpoint c — for VB <= 64 the next block's, i.e. this
//            one's plus the mask's popcount, so that Occ(c, p) = that minus
//            popcount(mask << rem) (no special case for rem = 0).  A rank
//            query of symbol c is one U-byte load (C2: 12 B, one dwordx3, at a
//            32-bit offset from the records' base) and a shift + popcount.
//            When sigma units do not fit one line, the record spans L = RB /
//            128 lines (at most 4) of PL = 128 / U units each (unit c in line
//            c / PL: a unit never straddles two lines), and the block's planes
//            sit verbatim at the record's end (last line's spare bytes) for
//            the walk, which needs the symbol before it can pick a unit
//            (C4: sigma 21, three lines, 384 B per 64 rows).
// REC = (256..512)|kRecOneHot|kRecWalk — multi-line symbol masks with a WALK
//            LINE (round 6): the units fill lines 0 .. L-2 (PL per line, as
//            above), and the last line is the block's plain record — planes
//            verbatim at [0, PB), the block's own sigma checkpoints at PBA +
//            c*P — so that the walk's get_pre_rank_and_symidx reads one line
//            (the symbol from the planes, its checkpoint beside them) instead
//            of the planes and then the symbol's unit: one dependent round
//            trip per walk step instead of two.  Where PBA + sigma*P <= 128
//            (C4: 40 + 84 B; four lines, 512 B per 64 rows).
constexpr int kRecPaired = 1;
constexpr int kRecOneHot = 2;
constexpr int kRecWalk = 4;
static_assert(kRecWalk == (int)kOccRecWalkBit, "fmx_internal.hpp kOccRecWalkBit");

// Whether record encoding rec (0, 64, 128, | kRecPaired, | kRecOneHot) can
// hold a block of N planes of VB bits and at least one checkpoint of pos bytes.
constexpr bool rec_fits(int pos, int N, int VB, int rec) {
    const int pb = N * VB / 8, rb = rec & ~15;
    if (rec == 0) return true;
    if (rec & kRecWalk) {  // units in lines 0 .. L-2, the block's plain record in the last line
        const int u = VB / 8 + pos, pba = (pb + pos - 1) / pos * pos;
        return (rec & kRecOneHot) && u % 4 == 0 && rb % 128 == 0 && rb >= 256 && rb <= 512 && u <= 128 &&
               pba + pos <= 128 && (1 << N) * u > 128;
    }
    if (rec & kRecOneHot) {
        const int u = VB / 8 + pos;
        if (u % 4 != 0) return false;
        if (rb <= 128) return 2 * u <= rb;
        // planes + >= 1 unit in the last line; only where sigma <= 2^N units can overflow one line
        return rb % 128 == 0 && rb <= 512 && u <= 128 - pb && (1 << N) * u > 128;
    }
    const int pta = (pb % 16 + pos - 1) / pos * pos;
    if (rec & kRecPaired) return pb % 16 != 0 && 16 - pta >= pos && (pb / 16 + 1) * 16 <= rb;
    return (pb + pos - 1) / pos * pos + pos <= rb;
}

template <typename P, int N, int VB, int REC>
struct Occ {
    static constexpr bool PAIRED = (REC & kRecPaired) != 0;
    static constexpr bool ONEHOT = (REC & kRecOneHot) != 0;
    static constexpr int U = VB / 8 + (int)sizeof(P);                          // one-hot unit bytes
    static constexpr int RB = REC & ~15;                                        // record bytes
    static constexpr int PB = N * VB / 8;                                      // plane bytes
    static constexpr int PBA = (PB + (int)sizeof(P) - 1) / (int)sizeof(P) * (int)sizeof(P);
    static constexpr int PBC = (PB + 15) / 16;                                 // chunks holding planes
    static constexpr int PF = PB / 16, PT = PB % 16;                           // whole plane chunks, tail bytes
    static constexpr int PTA = (PT + (int)sizeof(P) - 1) / (int)sizeof(P) * (int)sizeof(P);
    static constexpr int PER = PAIRED ? (16 - PTA) / (int)sizeof(P) : 1;       // checkpoints per paired chunk
    static constexpr int NCH = RB / 16;                                        // chunks per record
    static constexpr bool MULTI = ONEHOT && RB > 128;                        // multi-line symbol masks
    static constexpr bool WALK = MULTI && (REC & kRecWalk) != 0;              // ... with a walk line
    static constexpr int PL = RB > 128 ? 128 / U : RB / (U > 0 ? U : 1);       // units per line
    static constexpr int NCKW = (128 - PBA) / (int)sizeof(P);                  // walk line: checkpoint slots
    static constexpr int NCKW2 = pow2_ceil(NCKW);
    static constexpr int NCK = REC == 0 ? (1 << N)
                             : WALK     ? (RB / 128 - 1) * PL
                             : MULTI    ? (RB / 128 - 1) * PL + (128 - PB) / U
                             : ONEHOT   ? RB / U
                             : PAIRED   ? (NCH - PF) * PER
                                        : (RB - PBA) / (int)sizeof(P);         // checkpoint slots
    static constexpr int NCK2 = pow2_ceil(NCK);
    static_assert(rec_fits(sizeof(P), N, VB, REC), "record too small");

    // One block's planes and one checkpoint, as read for a rank query.
    struct Rec {
        Planes<N, VB> pl;
        P ck;
    };

    // dword d of a record's chunk array (d known at compile time after unrolling)
    FMX_HD static uint32_t dw(const V4 *ch, int d) { return ch[d >> 2][d & 3]; }

    FMX_HD static void planes_from(const V4 *ch, Planes<N, VB> &pl) {
        using W = typename VecT<VB>::W;
#pragma unroll
        for (int w = 0; w < Planes<N, VB>::WORDS; ++w) {
            if constexpr (sizeof(W) == 8) pl.w[w] = (uint64_t)dw(ch, 2 * w) | (uint64_t)dw(ch, 2 * w + 1) << 32;
            else pl.w[w] = dw(ch, w);
        }
    }

    // P at dword offset d (runtime, 0..3; P = u64: 0 or 2) of chunk v
    FMX_HD static P pick(const V4 &v, uint32_t d) {
        if constexpr (sizeof(P) == 8) return (P)(d & 2 ? (uint64_t)v[2] | (uint64_t)v[3] << 32
                                                       : (uint64_t)v[0] | (uint64_t)v[1] << 32);
        else return (P)(d & 2 ? (d & 1 ? v[3] : v[2]) : (d & 1 ? v[1] : v[0]));
    }

    // Checkpoint slot i's chunk and dword within it (compile-time i after unrolling).
    FMX_HD static constexpr int ck_dword(int i) {
        return PAIRED ? (PF + i / PER) * 4 + (PTA + (i % PER) * (int)sizeof(P)) / 4 : (PBA + i * (int)sizeof(P)) / 4;
    }

    // One-hot records: symbol c's mask over block q and its checkpoint.
    struct Hot {
        uint64_t m0, m1;  // mask words: VB <= 64 in m0; VB = 128 as lo (m0), hi (m1)
        P ck;
    };
    struct Unit {
        uint32_t d[U / 4];
    };
    FMX_HD static Hot hot_from(const uint32_t *d) {
        Hot h;
        if constexpr (VB == 32) h.m0 = d[0], h.m1 = 0;
        else h.m0 = (uint64_t)d[0] | (uint64_t)d[1] << 32, h.m1 = VB == 128 ? ((uint64_t)d[2] | (uint64_t)d[3] << 32) : 0;
        constexpr int o = VB / 32;
        if constexpr (sizeof(P) == 8) h.ck = (P)((uint64_t)d[o] | (uint64_t)d[o + 1] << 32);
        else h.ck = (P)d[o];
        return h;
    }
    // Records of u32 positions with one record per VB positions (RB == VB,
    // C2: 64-B records of 64 rows) lie below 2^32 bytes for every position
    // (q * RB <= p & ~(VB - 1) < 2^32): a 32-bit offset from the records' base.
    static constexpr bool OFF32 = sizeof(P) == 4 && RB == VB;
    // NT: a record read by one pattern only (a narrow interval's step, a walk
    // step) is loaded non-temporally where FMX_NT_NARROW is built in (A/B),
    // so that it does not displace the records wide intervals share
    template <bool NT = false>
    FMX_HD static Hot hot_fetch(const QueryArgs &a, uint64_t q, uint32_t c) {
        const uint8_t *u;
        if constexpr (OFF32) u = a.occ + ((uint32_t)q * (uint32_t)RB + c * (uint32_t)U);
        else if constexpr (MULTI) u = a.occ + q * RB + (c / (uint32_t)PL) * 128u + (c % (uint32_t)PL) * (uint32_t)U;
        else u = a.occ + q * RB + c * U;
#if defined(__HIP_DEVICE_COMPILE__) && FMX_NT_NARROW
        if constexpr (NT) {
            uint32_t d[U / 4];
#pragma unroll
            for (int j = 0; j < U / 4; ++j) d[j] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(u) + j);
            return hot_from(d);
        }
#endif
        return hot_from(reinterpret_cast<const Unit *>(u)->d);  // one U-byte load
    }
    // Occ(c, block start + rem): the stored checkpoint and the mask's first rem
    // positions (MSB-first, as Planes::rank)
    FMX_HD static P hot_occ(const Hot &h, uint32_t rem) {
        if constexpr (VB == 128) {
            if (rem == 0) return h.ck;
            if (rem <= 64) return h.ck + (P)__builtin_popcountll(h.m1 >> (64 - rem));
            return h.ck + (P)((uint32_t)__builtin_popcountll(h.m1) + (uint32_t)__builtin_popcountll(h.m0 >> (128 - rem)));
        } else if constexpr (VB == 64) {
            return h.ck - (P)__builtin_popcountll(h.m0 << rem);  // ck = next block's checkpoint
        } else {
            return h.ck - (P)__builtin_popcount((uint32_t)h.m0 << rem);
        }
    }
    // whether the mask holds position rem (bit VB - 1 - rem)
    FMX_HD static bool hot_bit(const Hot &h, uint32_t rem) {
        const uint32_t b = VB - 1 - rem;
        if constexpr (VB == 128) return ((b >= 64 ? h.m1 >> (b - 64) : h.m0 >> b) & 1u) != 0;
        else return ((h.m0 >> b) & 1u) != 0;
    }

    // The planes of block q and checkpoint c (rank_checkpoints[q*sigma + c]).
    FMX_HD static Rec fetch(const QueryArgs &a, uint64_t q, uint32_t c) {
        Rec r;
        if constexpr (REC == 0) {
            r.ck = reinterpret_cast<const P *>(a.ckpt)[q * a.sigma + c];
            r.pl.load(a.blocks + q * PB);
        } else if constexpr (PAIRED) {
            const V4 *rp = reinterpret_cast<const V4 *>(a.occ + q * RB);
            V4 ch[PF + 1];
#pragma unroll
            for (int i = 0; i < PF; ++i) ch[i] = rp[i];
            const uint32_t j = c / (uint32_t)PER;
            ch[PF] = rp[PF + j];  // the planes' tail + checkpoints j*PER ..
            planes_from(ch, r.pl);
            r.ck = pick(ch[PF], (uint32_t)(PTA / 4) + (c - j * (uint32_t)PER) * (uint32_t)(sizeof(P) / 4));
        } else {
            const V4 *rp = reinterpret_cast<const V4 *>(a.occ + q * RB);
            V4 ch[PBC];
#pragma unroll
            for (int i = 0; i < PBC; ++i) ch[i] = rp[i];
            planes_from(ch, r.pl);
            const uint32_t o = (uint32_t)PBA + c * (uint32_t)sizeof(P);
            V4 cv;
            if constexpr (PB % 16 != 0) {
                cv = ch[PBC - 1];
                if ((o >> 4) != (uint32_t)(PBC - 1)) cv = rp[o >> 4];
            } else {
                cv = rp[o >> 4];
            }
            r.ck = pick(cv, (o >> 2) & 3u);
        }
        return r;
    }

    // Occ(c, stored position p): BwmView::get_next_rank after the sentinel
    // adjustment (bwm/mod.rs:206-214).  c is known before the loads, so only
    // the planes and the one checkpoint are fetched, all independently.
    FMX_HD static P rank_at(const QueryArgs &a, P p, uint32_t c) {
        if constexpr (ONEHOT) {
            const Hot h = hot_fetch(a, (uint64_t)p / VB, c);
            return hot_occ(h, (uint32_t)((uint64_t)p % VB));
        }
        const Rec r = fetch(a, (uint64_t)p / VB, c);
        return r.ck + (P)r.pl.rank((uint32_t)((uint64_t)p % VB), c);
    }

    // Both rank queries of one LF step, Occ(c, plo) and Occ(c, phi)
    // (next_pos_range, locate/mod.rs:39-45): when the two stored positions
    // fall in the same block — every step once the interval is narrower than
    // a block — that block is read once.
    FMX_HD static void rank_pair(const QueryArgs &a, P plo, P phi, uint32_t c, P &rlo, P &rhi) {
        const uint64_t ql = (uint64_t)plo / VB, qh = (uint64_t)phi / VB;
        if constexpr (ONEHOT) {
#if FMX_NT_NARROW
            Hot hl, hh;
            if (qh == ql) {
                hl = hot_fetch<true>(a, ql, c);
                hh = hl;
            } else {
                hl = hot_fetch(a, ql, c);
                hh = hot_fetch(a, qh, c);
            }
#else
            const Hot hl = hot_fetch(a, ql, c);
            Hot hh = hl;
            if (qh != ql) hh = hot_fetch(a, qh, c);
#endif
            rlo = hot_occ(hl, (uint32_t)((uint64_t)plo % VB));
            rhi = hot_occ(hh, (uint32_t)((uint64_t)phi % VB));
            return;
        }
        const Rec rl = fetch(a, ql, c);
        Rec rh = rl;
        if (qh != ql) rh = fetch(a, qh, c);
        rlo = rl.ck + (P)rl.pl.rank((uint32_t)((uint64_t)plo % VB), c);
        rhi = rh.ck + (P)rh.pl.rank((uint32_t)((uint64_t)phi % VB), c);
    }

    // A one-line symbol-mask record's get_pre_rank_and_symidx from its chunks:
    // the symbol is the unit whose mask holds the position.
    FMX_HD static P pre_rank_sym_from(const V4 (&ch)[NCH > 0 ? NCH : 1], uint32_t rem, uint32_t sigma, uint32_t &c) {
        Hot hs[NCK2];
        c = 0;
#pragma unroll
        for (int i = 0; i < NCK2; ++i) {
            uint32_t d[U / 4 > 0 ? U / 4 : 1];
#pragma unroll
            for (int j = 0; j < U / 4; ++j) d[j] = i < NCK ? dw(ch, i * (U / 4) + j) : 0u;
            hs[i] = hot_from(d);
            if (i < NCK && (uint32_t)i < sigma && hot_bit(hs[i], rem)) c = (uint32_t)i;
        }
        const Hot h = tree_pick<NCK2>(hs, c);
        return hot_occ(h, rem);
    }

    // get_pre_rank_and_symidx body (bwm/mod.rs:223-235) for stored position p:
    // the symbol is only known after the planes arrive, so every checkpoint
    // slot of the block is fetched alongside them (one round trip) and the
    // right one selected in registers.
    FMX_HD static P pre_rank_sym(const QueryArgs &a, P p, uint32_t &c) {
        const uint64_t q = (uint64_t)p / VB;
        const uint32_t rem = (uint32_t)((uint64_t)p % VB);
        Planes<N, VB> pl;
        if constexpr (REC == 0) {
            pl.load(a.blocks + q * PB);
            const P *ckq = reinterpret_cast<const P *>(a.ckpt) + q * a.sigma;
            if constexpr (N <= 3) {
                P all[NCK2];
#pragma unroll
                for (int i = 0; i < NCK2; ++i) all[i] = (uint32_t)i < a.sigma ? ckq[i] : P(0);
                c = pl.sym(rem);
                return tree_pick<NCK2>(all, c) + (P)pl.rank(rem, c);
            } else {
                c = pl.sym(rem);
                return ckq[c] + (P)pl.rank(rem, c);
            }
        } else if constexpr (WALK) {
            // the walk line (the block's plain record): planes and every
            // checkpoint in one round trip, the symbol's picked in registers
            const V4 *rp = reinterpret_cast<const V4 *>(a.occ + q * RB + (RB - 128));
            V4 ch[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) ch[i] = rp[i];
            planes_from(ch, pl);
            c = pl.sym(rem);
            P all[NCKW2];
#pragma unroll
            for (int i = 0; i < NCKW2; ++i) {
                const int d = (PBA + i * (int)sizeof(P)) / 4;
                if (i >= NCKW) all[i] = P(0);
                else if constexpr (sizeof(P) == 8) all[i] = (P)((uint64_t)dw(ch, d) | (uint64_t)dw(ch, d + 1) << 32);
                else all[i] = (P)dw(ch, d);
            }
            return tree_pick<NCKW2>(all, c) + (P)pl.rank(rem, c);
        } else if constexpr (MULTI) {
            // the symbol from the planes kept at the record's end, then its unit
            pl.load(a.occ + q * RB + (RB - PB));
            c = pl.sym(rem);
            return hot_occ(hot_fetch(a, q, c), rem);
        } else if constexpr (ONEHOT) {
            // the whole record in one round trip; the symbol is the unit whose
            // mask holds the position
            const V4 *rp = reinterpret_cast<const V4 *>(a.occ + q * RB);
            V4 ch[NCH];
#pragma unroll
            for (int i = 0; i < NCH; ++i) {
#if defined(__HIP_DEVICE_COMPILE__) && FMX_NT_NARROW
                ch[i] = __builtin_nontemporal_load(rp + i);
#else
                ch[i] = rp[i];
#endif
            }
            return pre_rank_sym_from(ch, rem, a.sigma, c);
        } else {
            const V4 *rp = reinterpret_cast<const V4 *>(a.occ + q * RB);
            V4 ch[NCH];
#pragma unroll
            for (int i = 0; i < NCH; ++i) ch[i] = rp[i];
            planes_from(ch, pl);  // paired: chunk PF (the first checkpoint chunk) holds the tail
            c = pl.sym(rem);
            P all[NCK2];
#pragma unroll
            for (int i = 0; i < NCK2; ++i) {
                const int d = ck_dword(i);
                if (i >= NCK) all[i] = P(0);
                else if constexpr (sizeof(P) == 8) all[i] = (P)((uint64_t)dw(ch, d) | (uint64_t)dw(ch, d + 1) << 32);
                else all[i] = (P)dw(ch, d);
            }
            return tree_pick<NCK2>(all, c) + (P)pl.rank(rem, c);
        }
    }
};

// Interleaved record encoding for a layout (0: too wide, stay on the blob
// layout; multi: whether multi-line symbol masks may be picked — only for the
// faithful index, the derived kernels are not built for them): paired-chunk records when the planes leave a tail and they fit the
// record size the plain layout would take (never larger), else plain 64/128.
FMX_HD uint32_t interleaved_rec_bytes(uint32_t pos_bytes, uint32_t planes, uint32_t vec_bits, uint32_t sigma,
                                      bool paired = true, bool onehot = true, bool multi = true, bool walk = false) {
    const uint32_t pb = planes * vec_bits / 8;
    const uint32_t pba = (pb + pos_bytes - 1) / pos_bytes * pos_bytes;
    const uint32_t need = pba + sigma * pos_bytes;
    const uint32_t plain = need <= 64 ? 64u : need <= 128 ? 128u : 0u;
    const uint32_t u = vec_bits / 8 + pos_bytes, hb = sigma * u;
    const uint32_t hot = hb <= 64 ? 64u : hb <= 128 ? 128u : 0u;
    if (onehot && hot != 0 && u % 4 == 0 && (plain == 0 || hot <= plain)) return hot | (uint32_t)kRecOneHot;
    if (onehot && multi && walk && hot == 0 && u % 4 == 0 && pba + sigma * pos_bytes <= 128) {
        // units in lines 0 .. l-2, the block's plain record (planes + sigma checkpoints) as the last line
        const uint32_t pl = 128 / u;
        for (uint32_t l = 2; l <= 4; ++l)
            if (sigma <= (l - 1) * pl) return 128 * l | (uint32_t)kRecOneHot | (uint32_t)kRecWalk;
    }
    if (onehot && multi && hot == 0 && u % 4 == 0 && u <= 128 - pb) {
        // multi-line: PL units per line, the planes in the last line's spare bytes
        const uint32_t pl = 128 / u, last_cap = (128 - pb) / u;
        for (uint32_t l = 2; l <= 4; ++l)
            if (sigma <= (l - 1) * pl + last_cap) return 128 * l | (uint32_t)kRecOneHot;
    }
    const uint32_t pt = pb % 16, pta = (pt + pos_bytes - 1) / pos_bytes * pos_bytes;
    if (paired && plain != 0 && pt != 0 && 16 - pta >= pos_bytes) {
        const uint32_t per = (16 - pta) / pos_bytes;
        const uint32_t bytes = 16 * (pb / 16 + (sigma + per - 1) / per);
        if (bytes <= plain) return plain | (uint32_t)kRecPaired;
    }
    return plain;
}

// Record q of the interleaved layout from the blob's block q (PB bytes of
// planes) and its checkpoint row (sigma P's): k_relayout, and the CPU
// emulation's copy (tests/emu).
template <typename P, int N, int VB, int REC>
FMX_HD void write_record(uint8_t *dst, const uint8_t *planes, const uint8_t *ckrow, uint32_t sigma) {
    using O = Occ<P, N, VB, REC>;
    constexpr int RB = O::RB;
    uint32_t w[RB / 4];
#pragma unroll
    for (int i = 0; i < RB / 4; ++i) w[i] = 0;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(planes);
    const uint32_t *cw = reinterpret_cast<const uint32_t *>(ckrow);
    constexpr int CW = (int)sizeof(P) / 4;  // dwords per checkpoint
    if constexpr (O::ONEHOT) {
        // unit c: the AND over planes j of plane j (bit j of c set) or its
        // complement — Block::get_remain_count_of's mask — then checkpoint c
        constexpr int MW = VB / 32;  // mask dwords
        if constexpr (O::WALK) {
            // the walk line: planes, then this block's checkpoints (rank_checkpoints[q*sigma + c])
            constexpr int WL = (RB - 128) / 4;
            for (int i = 0; i < O::PB / 4; ++i) w[WL + i] = pw[i];
            for (uint32_t i = 0; i < sigma * (uint32_t)CW && i < (uint32_t)(128 - O::PBA) / 4; ++i)
                w[WL + O::PBA / 4 + i] = cw[i];
        } else if constexpr (O::MULTI) {
            for (int i = 0; i < O::PB / 4; ++i) w[(RB - O::PB) / 4 + i] = pw[i];
        }
        for (int c = 0; c < O::NCK; ++c) {  // (load time only; not unrolled)
            if ((uint32_t)c >= sigma) break;
            const int ub = O::MULTI ? (c / O::PL) * 32 + (c % O::PL) * (O::U / 4) : c * (O::U / 4);  // unit dword
#pragma unroll
            for (int i = 0; i < MW; ++i) {
                uint32_t m = ~0u;
#pragma unroll
                for (int j = 0; j < N; ++j) m &= ((c >> j) & 1) ? pw[j * MW + i] : ~pw[j * MW + i];
                w[ub + i] = m;
            }
            uint64_t ck = cw[c * CW];
            if constexpr (CW == 2) ck |= (uint64_t)cw[c * CW + 1] << 32;
            if constexpr (VB <= 64) {  // the next block's checkpoint: + the mask's popcount
                uint32_t pc = 0;
#pragma unroll
                for (int i = 0; i < MW; ++i) pc += (uint32_t)__builtin_popcount(w[ub + i]);
                ck += pc;
            }
            w[ub + MW] = (uint32_t)ck;
            if constexpr (CW == 2) w[ub + MW + 1] = (uint32_t)(ck >> 32);
        }
    } else if constexpr (O::PAIRED) {
#pragma unroll
        for (int i = 0; i < O::PF * 4; ++i) w[i] = pw[i];
#pragma unroll
        for (int j = O::PF; j < O::NCH; ++j) {
#pragma unroll
            for (int i = 0; i < O::PT / 4; ++i) w[4 * j + i] = pw[4 * O::PF + i];
        }
#pragma unroll
        for (int s = 0; s < O::NCK; ++s)
#pragma unroll
            for (int i = 0; i < CW; ++i)
                if ((uint32_t)s < sigma) w[O::ck_dword(s) + i] = cw[s * CW + i];
    } else {
#pragma unroll
        for (int i = 0; i < O::PB / 4; ++i) w[i] = pw[i];
        const uint32_t ncw = sigma * (uint32_t)CW;
#pragma unroll
        for (int i = 0; i < (RB - O::PBA) / 4; ++i)
            if ((uint32_t)i < ncw) w[O::PBA / 4 + i] = cw[i];
    }
    V4 *d = reinterpret_cast<V4 *>(dst);
#pragma unroll
    for (int i = 0; i < RB / 16; ++i) d[i] = V4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
}

// ----------------------------------------------------- shared kernel parts

template <typename P>
struct Tables {
    uint8_t enc[256];
    uint8_t dig[kMaxSigma];  // symbol -> deep-table digit (QueryArgs::dlut_dig)
    P C[kMaxSigma + 1];
    uint64_t mult[kMaxK];
    const P *kt;  // the blob's k-mer count table: a workgroup's LDS copy, or the blob itself
};

// One pattern, position j = 0..m-1 in pattern order.  Either staged: the
// encoded symbols in LDS (the workgroup copies its patterns' bytes once,
// through the encoding table, reversed for *_rev_iter input), or raw: the
// input bytes in HBM, encoded on each access.
struct PatView {
    const uint8_t *sym;  // staged symbols (pattern order), or null
    const uint8_t *raw;  // raw bytes (input order)
    const uint8_t *enc;  // encoding table
    uint64_t m;
    bool rev;
    FMX_HD uint32_t at(uint64_t j) const { return sym ? sym[j] : enc[raw[rev ? m - 1 - j : j]]; }
};

// Four text symbols t[a..a+4) from two aligned words (the text buffer is
// padded by 16 bytes past n).
FMX_HD uint32_t load4(const uint8_t *t, uint64_t a) {
    const uint64_t al = a & ~3ull;
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t w0 = *reinterpret_cast<const uint32_t *>(t + al);
    const uint32_t w1 = *reinterpret_cast<const uint32_t *>(t + al + 4);
    return sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
}

// Single-row tail, short form (kernels for batches of short patterns): the
// same contract as tail_mismatch_long below, four positions per step, inline
// and register-light (most such tails are a few symbols long, or none).
FMX_HD int64_t tail_mismatch_short(const uint8_t *text, const PatView &pv, uint64_t idx, uint64_t x, uint64_t top) {
    const uint64_t lowest = idx > x ? idx - x : 0;  // positions below have no text before them
    const uint64_t tb = x - idx;                     // text position of P[0] (mod 2^64)
    uint64_t hj = top;
    while (hj > lowest) {
        const uint64_t lj = hj - lowest >= 4 ? hj - 4 : lowest;
        const uint32_t tw = load4(text, tb + lj);
        uint32_t mism = 0;
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
            if (lj + u < hj && ((tw >> (8 * u)) & 0xffu) != pv.at(lj + u)) mism |= 1u << u;
        if (mism) return (int64_t)(lj + (31 - __builtin_clz(mism)));
        hj = lj;
    }
    return lowest > 0 ? (int64_t)(lowest - 1) : -1;
}

// Single-row tail (FMX_OPT_TEXT): the interval of P[idx..m) is the one row
// whose suffix starts at text position x, so P occurs at most once, at
// x - idx.  The LF loop would consume P[idx-1], P[idx-2], ... and stop at the
// first symbol that does not precede the suffix (or at the text start); here
// the same positions are compared with T[x-1], T[x-2], ..., 64 per round: the
// round's text bytes are five aligned 16-B vectors, all in flight at once
// (the text buffer is padded by 16 bytes past n), compared word by word
// against the staged pattern symbols.  Only positions below `top` are
// compared (top = idx: all of them).  Returns the highest position jm that
// fails (-1: P occurs at x - idx).
// One out-of-line copy (not one per kernel instantiation): it only touches
// the text and the pattern.  Its call costs the calling kernel registers, so
// only the long-pattern kernel variants (LT) use it.
__host__ __device__ __noinline__ inline int64_t tail_mismatch_long(const uint8_t *text, PatView pv, uint64_t idx,
                                                                   uint64_t x, uint64_t top) {
    using V4 = uint32_t __attribute__((ext_vector_type(4)));
    const uint64_t lowest = idx > x ? idx - x : 0;  // positions below have no text before them
    const uint64_t tb = x - idx;                     // text position of P[0] (mod 2^64)
    uint64_t hj = top;
    while (hj > lowest) {
        const uint64_t lj = hj - lowest > 64 ? hj - 64 : lowest;
        const uint64_t t0 = tb + lj, t1 = tb + hj;  // text range [t0, t1), at most 64 bytes
        const uint64_t a0 = t0 & ~15ull;
        const V4 *src = reinterpret_cast<const V4 *>(text + a0);
        V4 v[5];
#pragma unroll
        for (uint32_t u = 0; u < 5; ++u) {
            if (a0 + 16ull * u < t1) v[u] = src[u];
            else v[u] = V4{0u, 0u, 0u, 0u};
        }
        int64_t best = -1;  // positions rise with (u, w): the last mismatching word holds the highest
#pragma unroll
        for (uint32_t u = 0; u < 5; ++u) {
#pragma unroll
            for (uint32_t w = 0; w < 4; ++w) {
                const uint64_t base = a0 + 16ull * u + 4ull * w;
                if (base + 4 <= t0 || base >= t1) continue;
                uint32_t pw = 0, valid = 0;
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) {
                    const uint64_t tp = base + b;
                    const bool in = tp >= t0 && tp < t1;
                    pw |= (in ? pv.at(tp - tb) : 0u) << (8 * b);
                    valid |= in ? 0xffu << (8 * b) : 0u;
                }
                const uint32_t d = (v[u][w] ^ pw) & valid;
                if (d) best = (int64_t)(base + (uint64_t)((31 - __builtin_clz(d)) >> 3) - tb);
            }
        }
        if (best >= 0) return best;
        hj = lj;
    }
    return lowest > 0 ? (int64_t)(lowest - 1) : -1;
}

template <bool LT>
FMX_HD int64_t tail_mismatch(const uint8_t *text, const PatView &pv, uint64_t idx, uint64_t x, uint64_t top) {
    if constexpr (LT) return tail_mismatch_long(text, pv, idx, x, top);
    else return tail_mismatch_short(text, pv, idx, x, top);
}

// How a search ended (what the locate phase does with an occurrence):
constexpr uint32_t kHitRows = 0;  // rows lo..hi of the final interval: walk (or read the full SA)
constexpr uint32_t kHitOne = 1;   // resolved: the count is hi - lo <= 1 and rloc is the location
constexpr uint32_t kHitMask = 2;  // set bits b of `mask`: location SA[lo + b] - rloc

// Row-context scan (FMX_OPT_ROW_CONTEXT).  Every row r of the interval
// [lo, hi) of P[idx..m) starts with P[idx..m); P occurs at SA[r] - idx iff the
// idx symbols before that suffix are P[0..idx).  The nearest ctx_len of them
// are ctx[r] (digits sigma+1-ary, T[SA-1] most significant, 0 = before the
// text start), so one comparison of ctx[r] against a range settles up to
// ctx_len positions, and the rest (idx > ctx_len) is compared with the text.
// The matching rows keep the interval's row order, which is the final
// interval's order: all occurrences share the prefix P[0..idx), so their
// suffixes at SA - idx sort as the suffixes at SA do.  This is the LF loop's
// result over the same rows (with_slice.rs:27-31); callers only scan when no
// symbol of P is >= sigma (which the LF loop would have to reject in place).
template <typename P, bool LT>
FMX_HD void scan_rows(const QueryArgs &a, const PatView &pv, uint64_t idx, P &lo, P &hi, P &rloc, uint64_t &mask,
                      uint32_t &mode) {
    const uint32_t W = a.sigma + 1, Cl = a.ctx_len;
    const uint64_t L = idx < Cl ? idx : Cl;
    uint64_t code = 0;
    for (uint64_t j = 0; j < L; ++j) code = code * W + (pv.at(idx - 1 - j) + 1);
    const uint64_t span = a.wpow[Cl - L];
    const uint64_t clo = code * span, chi = clo + span;  // ctx in [clo, chi)
    // Records are read as 16-B vectors, NV of them issued before any is used
    // (one round covers 16 u32 / 8 u64 rows; the row-record buffer is padded so
    // the last vector never leaves it).  Bits of msk are rows relative to lo.
    using V4 = uint32_t __attribute__((ext_vector_type(4)));
    constexpr uint32_t RPV = 16 / (2 * sizeof(P));
    constexpr uint32_t NV = 8;
    const V4 *vec = reinterpret_cast<const V4 *>(a.safull);
    const uint64_t v0 = (uint64_t)lo / RPV, v1 = ((uint64_t)hi + RPV - 1) / RPV;
    uint64_t msk = 0;
    P first = 0;
    for (uint64_t vb = v0; vb < v1; vb += NV) {
        V4 x[NV];
#pragma unroll
        for (uint32_t u = 0; u < NV; ++u) {
            if (vb + u < v1) x[u] = vec[vb + u];  // (no duplicate requests past the interval)
            else x[u] = V4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (uint32_t u = 0; u < NV; ++u) {
#pragma unroll
            for (uint32_t w = 0; w < RPV; ++w) {
                const uint64_t row = (vb + u) * RPV + w;
                P sa, ctx;
                if constexpr (sizeof(P) == 4) {
                    sa = (P)x[u][2 * w];
                    ctx = (P)x[u][2 * w + 1];
                } else {
                    sa = (P)((uint64_t)x[u][0] | (uint64_t)x[u][1] << 32);
                    ctx = (P)((uint64_t)x[u][2] | (uint64_t)x[u][3] << 32);
                }
                if (row >= (uint64_t)lo && row < (uint64_t)hi && (uint64_t)ctx >= clo && (uint64_t)ctx < chi) {
                    if (!msk) first = sa;
                    msk |= 1ull << (row - (uint64_t)lo);
                }
            }
        }
    }
    if (idx > Cl && msk) {
        // the symbols beyond the context: compare with the text, row by row
        const P *sa = reinterpret_cast<const P *>(a.safull);
        uint64_t keep = 0;
        for (uint64_t m2 = msk; m2; m2 &= m2 - 1) {
            const uint64_t b = (uint64_t)__builtin_ctzll(m2);
            const P x = sa[2 * ((uint64_t)lo + b)];
            if (tail_mismatch<LT>(a.text, pv, idx, (uint64_t)x, idx - Cl) < 0) {
                if (!keep) first = x;
                keep |= 1ull << b;
            }
        }
        msk = keep;
    }
    const uint32_t cnt = (uint32_t)__builtin_popcountll(msk);
    if (cnt <= 1) {
        mode = kHitOne;
        hi = lo + (P)cnt;
        rloc = cnt ? (P)(first - (P)idx) : P(0);
    } else {
        mode = kHitMask;
        hi = lo + (P)cnt;
        rloc = (P)idx;
        mask = msk;
    }
}

// Marks a single-row entry of the deep k-mer table (FMX_OPT_LUT_ROWS): the top
// bit of the first word, which no row number has (n < 2^(8P-1) is required).
template <typename P>
FMX_HD constexpr P row_flag() { return P(1) << (8 * sizeof(P) - 1); }

// Single-row deep-table entry {row_flag | ctx, x}: the last K symbols of the
// pattern occur once in the text, as the suffix at x = SA of that row, and ctx
// packs T[x-1], T[x-2], ..., T[x-dlut_ctx] (symbol + 1, 0 before the text
// start), dlut_bps bits each, the nearest in the low bits.  The LF loop over
// P[0..idx) (with_slice.rs:27-31) keeps that one row while every symbol equals
// the text symbol before the suffix and empties at the first (highest)
// position that does not — where it reads, and for PassThrough rejects, that
// pattern symbol.  Here the nearest dlut_ctx positions are compared in one
// XOR and the rest against the text.
template <typename P, bool LT>
FMX_HD uint32_t one_row(const QueryArgs &a, const PatView &pv, uint64_t idx, P w0, P w1, P &lo, P &hi, P &rloc,
                        uint32_t &mode) {
    const uint32_t bps = a.dlut_bps, Ld = a.dlut_ctx;
    const uint64_t x = (uint64_t)w1;
    const uint64_t L = idx < Ld ? idx : Ld;
    uint64_t pc = 0;
    if (pv.sym != nullptr) {  // staged: no per-symbol source test
        const uint8_t *q = pv.sym + idx - 1;
        for (uint32_t j = 0; j < (uint32_t)L; ++j) {
            const uint32_t c = q[-(int32_t)j];
            const uint64_t d = c < a.sigma ? c + 1 : a.sigma + 1;  // sigma + 1: never a stored digit
            pc |= d << (bps * j);
        }
    } else {
        for (uint64_t j = 0; j < L; ++j) {
            const uint32_t c = pv.at(idx - 1 - j);
            const uint64_t d = c < a.sigma ? c + 1 : a.sigma + 1;
            pc |= d << (bps * j);
        }
    }
    const uint64_t keep = L * bps >= 64 ? ~0ull : (1ull << (L * bps)) - 1;
    const uint64_t diff = (pc ^ (uint64_t)(w0 & (P)~row_flag<P>())) & keep;
    int64_t jm;
    if (diff) jm = (int64_t)(idx - 1 - (uint64_t)__builtin_ctzll(diff) / bps);
    else jm = idx > Ld ? tail_mismatch<LT>(a.text, pv, idx, x, idx - Ld) : -1;
    mode = kHitOne;
    lo = 0;
    hi = 0;
    if (jm >= 0) return pv.at((uint64_t)jm) >= a.sigma ? kStatusSymbol : 0;
    hi = 1;
    rloc = (P)(x - idx);
    return 0;
}

// The deep k-mer table's index for the last K symbols of the pattern, or
// false when the table does not apply (no table, m < K, a symbol that does
// not occur in the text or is >= sigma: the blob's seed and the LF loop then
// empty the interval — or reject the symbol — exactly there).
template <typename P>
FMX_HD bool dlut_code(const QueryArgs &a, const Tables<P> &s, const PatView &pv, uint64_t &code) {
    code = 0;
    if (a.dlut == nullptr || pv.m == 0 || pv.m < a.dlut_k) return false;
    const uint32_t K = a.dlut_k, S = a.dlut_sigma, sigma = a.sigma;
    const uint64_t m = pv.m;
    uint32_t miss = 0;
    if (pv.sym != nullptr) {  // staged (the common case): no per-symbol source test
        const uint8_t *q = pv.sym + (m - K);
#pragma unroll 4
        for (uint32_t j = 0; j < K; ++j) {
            const uint32_t c = q[j];
            const uint32_t d = c < sigma ? s.dig[c] : kNoDigit;
            miss |= d == kNoDigit;
            code = code * S + d;
        }
        return !miss;
    }
#pragma unroll 4
    for (uint32_t j = 0; j < K; ++j) {
        const uint32_t c = pv.at(m - K + j);
        const uint32_t d = c < sigma ? s.dig[c] : kNoDigit;
        miss |= d == kNoDigit;
        code = code * S + d;
    }
    return !miss;
}

// The latest SAMPLED row of a search's single-row phase (round 6).  Once the
// interval is one row r_j, every LF step maps it to the row of the suffix
// one text position earlier, so the final row's location (what the locate
// walk finds, locate/mod.rs:19-35) is SA[r_j] - (the steps taken since r_j).
// If some r_j of that phase is a sampled row (r_j % sr == 0: its SA is
// SAs[r_j / sr], suffix_array/mod.rs:100-105), the location is one sampled-SA
// read — no walk step (E[walk] = sr - 1 steps of one record each, C2: ~1);
// with sr = 2 and ~5 single-row steps at 1 Gbp, nearly every pattern has one.
// valid = 0: none seen (walk the final row as before).
template <typename P>
struct SampledRow {
    uint64_t slot;  // its SAs index
    P off;          // LF steps since it
    uint32_t valid;
};

// Kernel variants of the search (template parameter VAR):
constexpr int kVarFaithful = 0;  // the blob's structures only (+ FMX_OCC_INTERLEAVED): no derived-index code
constexpr int kVarDerived = 1;   // derived structures, short single-row tail compares
constexpr int kVarDerivedLong = 2;  // derived structures, vectorised long tail compares

template <typename P, int N, int VB, int REC, int VAR = kVarDerived>
FMX_HD uint32_t search_seeded(const QueryArgs &a, const Tables<P> &s, const PatView &pv, bool have, P w0, P w1,
                              P &lo, P &hi, P &rloc, uint64_t &mask, uint32_t &mode, SampledRow<P> *smp);

// k-mer seed + LF loop: FmIndex::get_pos_range (with_slice.rs:21-33).
// Returns status bits (0 = ok).  The result is the interval [lo, hi) with
// mode kHitRows, or (derived structures) an interval finished early: a
// single row checked against the text (kHitOne), or a row-context scan
// (kHitOne / kHitMask, see scan_rows).  The count is always hi - lo.
template <typename P, int N, int VB, int REC, int VAR = kVarDerived>
FMX_HD uint32_t search(const QueryArgs &a, const Tables<P> &s, const PatView &pv, P &lo, P &hi, P &rloc,
                       uint64_t &mask, uint32_t &mode, SampledRow<P> *smp = nullptr) {
    if constexpr (VAR == kVarFaithful) {
        return search_seeded<P, N, VB, REC, VAR>(a, s, pv, false, P(0), P(0), lo, hi, rloc, mask, mode, smp);
    } else {
        uint64_t code;
        const bool have = dlut_code<P>(a, s, pv, code);
        P w0 = 0, w1 = 0;
        if (have) {
            const P *dl = reinterpret_cast<const P *>(a.dlut) + 2 * code;
            w0 = dl[0];
            w1 = dl[1];
        }
        return search_seeded<P, N, VB, REC, VAR>(a, s, pv, have, w0, w1, lo, hi, rloc, mask, mode, smp);
    }
}

// search() after the deep-table read: `have` = the entry {w0, w1} of the
// pattern's last K symbols (the interval K-k more LF steps from the blob's
// seed reach, or a single-row entry) was read.
template <typename P, int N, int VB, int REC, int VAR>
FMX_HD uint32_t search_seeded(const QueryArgs &a, const Tables<P> &s, const PatView &pv, bool have, P w0, P w1,
                              P &lo, P &hi, P &rloc, uint64_t &mask, uint32_t &mode, SampledRow<P> *smp) {
    using O = Occ<P, N, VB, REC>;
    if (smp) smp->valid = 0;
    constexpr bool LT = VAR == kVarDerivedLong, DER = VAR != kVarFaithful;
    const uint32_t sigma = a.sigma, k = a.k;
    const uint64_t m = pv.m;
    const P sent = (P)a.sentinel;
    lo = hi = 0;
    rloc = 0;
    mask = 0;
    mode = kHitRows;
    if (m == 0) return kStatusEmpty;  // count_array.rs:211 panics on an empty pattern
    uint64_t idx = 0;
    uint32_t bad = 0;
    bool seeded = false;
    if (DER && have) {
        idx = m - a.dlut_k;
        if (a.dlut_rows && (w0 & row_flag<P>())) return one_row<P, LT>(a, pv, idx, w0, w1, lo, hi, rloc, mode);
        lo = w0;
        hi = w1;
        seeded = true;
    }
    if (!seeded) {
        // seed: count_array.rs:203-233
        uint64_t code = 0, e;
        const uint64_t take = m < k ? m : k, first = m < k ? 0 : m - k;
        for (uint64_t j = 0; j < take; ++j) {
            const uint32_t c = pv.at(first + j);
            bad |= c >= sigma;
            code += (uint64_t)(c + 1) * s.mult[j];
        }
        if (bad) return kStatusSymbol;
        if (m < k) { e = code + s.mult[m - 1] - 1; idx = 0; }
        else { e = code; idx = m - k; }
        lo = s.kt[code - 1];
        hi = s.kt[e];
    }
    // a PassThrough pattern with a byte >= sigma must reach it in the LF loop
    bool scan = DER && a.ctx_len != 0;
    if (scan && a.strict)
        for (uint64_t j = 0; j < idx; ++j) scan &= pv.at(j) < sigma;
    // the single-row phase's latest sampled row (SampledRow; only when the
    // caller locates, and FMX_SAMPLED_ROW=0 builds keep the walk for A/B)
    const bool track = FMX_SAMPLED_ROW && smp != nullptr && a.safull == nullptr;
    uint64_t sslot = 0;
    P soff = 0;
    bool shave = false;
    auto note = [&]() {
        if (shave) soff += P(1);
        if (hi - lo == P(1)) {
            uint64_t rem;
            const uint64_t sl = sr_div(a, (uint64_t)lo, rem);
            if (rem == 0) {
                sslot = sl;
                soff = 0;
                shave = true;
            }
        }
    };
    if (track) note();
    // LF loop: with_slice.rs:27-31, next_pos_range (locate/mod.rs:39-45)
    uint32_t c = idx > 0 ? pv.at(idx - 1) : 0;  // next symbol, fetched one step ahead
    while (lo < hi && idx > 0) {
        if constexpr (DER) {
            if (scan && hi - lo <= (P)a.scan_rows) {
                scan_rows<P, LT>(a, pv, idx, lo, hi, rloc, mask, mode);
                return 0;
            }
            if (a.text != nullptr && hi - lo == P(1)) {
                const uint64_t x = (uint64_t)reinterpret_cast<const P *>(a.safull)[(uint64_t)lo * a.sa_stride];
                const int64_t jm = tail_mismatch<LT>(a.text, pv, idx, x, idx);
                mode = kHitOne;
                if (jm >= 0) {
                    // the LF loop reads (and would reject) the symbol at jm before
                    // the interval empties there
                    if (pv.at((uint64_t)jm) >= sigma) { lo = hi = 0; return kStatusSymbol; }
                    hi = lo;
                } else {
                    rloc = (P)(x - idx);
                }
                return 0;
            }
        }
        idx -= 1;
        if (c >= sigma) { lo = hi = 0; return kStatusSymbol; }
        const P plo = lo + (lo < sent ? P(1) : P(0));  // bwm/mod.rs:202-204
        const P phi = hi + (hi < sent ? P(1) : P(0));
        P rlo, rhi;
        O::rank_pair(a, plo, phi, c, rlo, rhi);
        const P pre = s.C[c];
        c = idx > 0 ? pv.at(idx - 1) : 0;
        lo = pre + rlo;
        hi = pre + rhi;
        if (track) note();
    }
    if (track && shave && hi - lo == P(1)) {
        smp->slot = sslot;
        smp->off = soff;
        smp->valid = 1;
    }
    return 0;
}

// A value read once by one lane (the sampled-SA entry of a walk): a
// non-temporal load on the device, so that its line does not displace the
// occ records that other patterns read again.
template <typename T>
FMX_HD T load_once(const T *p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// The location of a one-row result: from the search's latest sampled row
// (SampledRow: one sampled-SA read), else by the walk below.
template <typename P, int N, int VB, int REC>
FMX_HD P locate_one(const QueryArgs &a, const P *C, P row, const SampledRow<P> &smp);

// Walk one suffix-array row to a sampled row or to the text start
// (locate/mod.rs:19-35; suffix_array/mod.rs:100-105).
template <typename P, int N, int VB, int REC>
FMX_HD P walk_row(const QueryArgs &a, const P *C, P pos) {
    using O = Occ<P, N, VB, REC>;
    if (a.safull != nullptr) return reinterpret_cast<const P *>(a.safull)[(uint64_t)pos * a.sa_stride];
    const P sent = (P)a.sentinel;
    P off = 0;
    uint64_t rem;
    uint64_t slot = sr_div(a, (uint64_t)pos, rem);
    while (rem != 0) {
        if (pos == (P)(sent - P(1))) return off;  // get_pre_rank_and_symidx -> None
        const P p = pos + (pos < sent ? P(1) : P(0));
        uint32_t c;
        const P rank = O::pre_rank_sym(a, p, c);
        pos = C[c] + rank;
        off += 1;
        slot = sr_div(a, (uint64_t)pos, rem);
    }
    return load_once(reinterpret_cast<const P *>(a.sa) + slot) + off;
}

template <typename P, int N, int VB, int REC>
FMX_HD P locate_one(const QueryArgs &a, const P *C, P row, const SampledRow<P> &smp) {
    if (smp.valid) return load_once(reinterpret_cast<const P *>(a.sa) + smp.slot) - smp.off;
    return walk_row<P, N, VB, REC>(a, C, row);
}


// ------------------------------------------- two patterns per lane (grouped)

// The faithful search (search_seeded, VAR 0: seed count_array.rs:203-233,
// LF loop with_slice.rs:27-31, next_pos_range locate/mod.rs:39-45) of two
// patterns advanced in lockstep by one lane, so that every LF step has both
// chains' record loads in flight at once (symbol-mask records: both fetched,
// then both ranked).  live[q] = false: no pattern (lo = hi = 0).
template <typename P, int N, int VB, int REC>
FMX_HD void search_pair(const QueryArgs &a, const Tables<P> &s, const PatView (&pv)[2], const bool (&live)[2],
                        P (&lo)[2], P (&hi)[2], uint32_t (&bad)[2]) {
    using O = Occ<P, N, VB, REC>;
    const uint32_t sigma = a.sigma, k = a.k;
    const P sent = (P)a.sentinel;
    uint64_t idx[2];
    uint32_t c[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        lo[q] = hi[q] = 0;
        bad[q] = 0;
        idx[q] = 0;
        c[q] = 0;
        if (!live[q]) continue;
        const uint64_t m = pv[q].m;
        if (m == 0) {
            bad[q] = kStatusEmpty;  // count_array.rs:211 panics on an empty pattern
            continue;
        }
        uint64_t code = 0, e;
        const uint64_t take = m < k ? m : k, first = m < k ? 0 : m - k;
        uint32_t b = 0;
        for (uint64_t j = 0; j < take; ++j) {
            const uint32_t cj = pv[q].at(first + j);
            b |= cj >= sigma;
            code += (uint64_t)(cj + 1) * s.mult[j];
        }
        if (b) {
            bad[q] = kStatusSymbol;
            continue;
        }
        if (m < k) { e = code + s.mult[m - 1] - 1; idx[q] = 0; }
        else { e = code; idx[q] = m - k; }
        lo[q] = s.kt[code - 1];
        hi[q] = s.kt[e];
        c[q] = idx[q] > 0 ? pv[q].at(idx[q] - 1) : 0;
    }
    for (;;) {
        bool act[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            act[q] = lo[q] < hi[q] && idx[q] > 0;
            if (act[q] && c[q] >= sigma) {
                lo[q] = hi[q] = 0;
                bad[q] = kStatusSymbol;
                act[q] = false;
            }
        }
        if (!act[0] && !act[1]) break;
        P plo[2], phi[2], rlo[2], rhi[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            plo[q] = lo[q] + (lo[q] < sent ? P(1) : P(0));  // bwm/mod.rs:202-204
            phi[q] = hi[q] + (hi[q] < sent ? P(1) : P(0));
        }
        if constexpr (O::ONEHOT) {
            typename O::Hot hl[2], hh[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!act[q]) continue;
                const uint64_t ql = (uint64_t)plo[q] / VB, qh = (uint64_t)phi[q] / VB;
                hl[q] = O::hot_fetch(a, ql, c[q]);
                hh[q] = hl[q];
                if (qh != ql) hh[q] = O::hot_fetch(a, qh, c[q]);
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!act[q]) continue;
                rlo[q] = O::hot_occ(hl[q], (uint32_t)((uint64_t)plo[q] % VB));
                rhi[q] = O::hot_occ(hh[q], (uint32_t)((uint64_t)phi[q] % VB));
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (act[q]) O::rank_pair(a, plo[q], phi[q], c[q], rlo[q], rhi[q]);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (!act[q]) continue;
            idx[q] -= 1;
            const P pre = s.C[c[q]];
            c[q] = idx[q] > 0 ? pv[q].at(idx[q] - 1) : 0;
            lo[q] = pre + rlo[q];
            hi[q] = pre + rhi[q];
        }
    }
}

// walk_row for two rows of one lane in lockstep (locate/mod.rs:19-35,
// suffix_array/mod.rs:100-105); live[q] = false: no row.
template <typename P, int N, int VB, int REC>
FMX_HD void walk_pair(const QueryArgs &a, const P *C, P (&pos)[2], const bool (&live)[2], P (&loc)[2]) {
    using O = Occ<P, N, VB, REC>;
    const P sent = (P)a.sentinel;
    P off[2] = {P(0), P(0)};
    uint64_t rem[2], slot[2];
    bool w[2], top[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        slot[q] = sr_div(a, (uint64_t)pos[q], rem[q]);
        w[q] = live[q] && rem[q] != 0;
        top[q] = false;
        loc[q] = 0;
    }
    while (w[0] || w[1]) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (w[q] && pos[q] == (P)(sent - P(1))) {  // get_pre_rank_and_symidx -> None
                loc[q] = off[q];
                w[q] = false;
                top[q] = true;
            }
        P rank[2];
        uint32_t cc[2];
        if constexpr (O::ONEHOT && !O::MULTI) {
            V4 ch[2][O::NCH];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!w[q]) continue;
                const P p = pos[q] + (pos[q] < sent ? P(1) : P(0));
                const V4 *rp = reinterpret_cast<const V4 *>(a.occ + ((uint64_t)p / VB) * O::RB);
#pragma unroll
                for (int i = 0; i < O::NCH; ++i) ch[q][i] = rp[i];
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!w[q]) continue;
                const P p = pos[q] + (pos[q] < sent ? P(1) : P(0));
                rank[q] = O::pre_rank_sym_from(ch[q], (uint32_t)((uint64_t)p % VB), a.sigma, cc[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (!w[q]) continue;
                const P p = pos[q] + (pos[q] < sent ? P(1) : P(0));
                rank[q] = O::pre_rank_sym(a, p, cc[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (!w[q]) continue;
            pos[q] = C[cc[q]] + rank[q];
            off[q] += 1;
            slot[q] = sr_div(a, (uint64_t)pos[q], rem[q]);
            w[q] = rem[q] != 0;
        }
    }
    P v[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) v[q] = live[q] && !top[q] ? load_once(reinterpret_cast<const P *>(a.sa) + slot[q]) : P(0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (live[q] && !top[q]) loc[q] = v[q] + off[q];
}

}  // namespace fmx
