// TEST INFRASTRUCTURE — host emulation of the query kernels.
//
// Runs the engine's own __host__ __device__ arithmetic
// (sview-fmindex_amd/csrc/fmx_device.hpp: rank/popcount, seed, LF loop,
// single-row text verification, walk) on the CPU, one pattern at a time, over
// the same derived structures the loader builds on the GPU (interleaved occ
// records, deep k-mer table, full SA, text), so the CPU test suite checks the
// device code paths against the oracle without a GPU.  Blob offsets come from
// the oracle's parser (oracle/fmx_oracle.c).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../sview-fmindex_amd/csrc/fmx_device.hpp"
#include "../../oracle/fmx_oracle.h"

using namespace fmx;

namespace {

template <typename P, int N, int VB, int REC>
int run(const orc_index &ox, uint32_t options, const uint8_t *bytes, const uint64_t *offs, uint64_t npat,
        uint32_t flags, uint64_t *counts, uint64_t *locs, uint64_t cap, uint64_t *needed) {
    const uint32_t scan_rows = options >> 8 ? options >> 8 : 32;  // options bits 8..: FMX_SCAN_ROWS
    const bool long_tails = (options & 128u) != 0;
    options &= 0x7fu;
    QueryArgs a{};
    const uint8_t *blob = ox.blob;
    a.ckpt = blob + ox.off_ckpt;
    a.blocks = blob + ox.off_blocks;
    a.sa = blob + ox.off_sa;
    a.kmer = blob + ox.off_kmer;
    a.n = ox.n;
    a.sentinel = ox.sentinel;
    a.sigma = ox.sigma;
    a.k = ox.k;
    a.sr = ox.sr;
    a.sr_pow2 = (ox.sr & (ox.sr - 1)) == 0;
    a.sr_pow2_mask = a.sr_pow2 ? ox.sr - 1 : 0;
    a.sr_shift = a.sr_pow2 ? (uint32_t)__builtin_ctz(ox.sr) : 0;
    a.sr_magic = a.sr_pow2 ? 0 : (uint64_t)((((unsigned __int128)1 << 64) + ox.sr - 1) / ox.sr);
    a.strict = ox.L.encoder == 1;
    for (uint32_t c = 0; c <= ox.sigma; ++c) a.C[c] = ox.count_array[c];
    for (uint32_t i = 0; i < ox.k && i < (uint32_t)kMaxK; ++i) a.mult[i] = ox.mult[i];
    memcpy(a.enc, ox.enc, 256);
    Tables<P> t{};
    memcpy(t.enc, ox.enc, 256);
    for (uint32_t c = 0; c <= ox.sigma; ++c) t.C[c] = (P)ox.count_array[c];
    for (uint32_t i = 0; i < ox.k && i < (uint32_t)kMaxK; ++i) t.mult[i] = ox.mult[i];
    t.kt = reinterpret_cast<const P *>(a.kmer);  // (the kernels' LDS copy holds the same entries)

    // interleaved records (k_relayout)
    std::vector<uint8_t> occ;
    if constexpr (REC != 0) {
        constexpr int PB = N * VB / 8, RB = REC & ~15;
        occ.assign(ox.blocks_len * RB + 16, 0);
        for (uint64_t q = 0; q < ox.blocks_len; ++q)
            write_record<P, N, VB, REC>(&occ[q * RB], a.blocks + q * PB, a.ckpt + q * ox.sigma * sizeof(P),
                                        ox.sigma);
        a.occ = occ.data();
    }
    using O = Occ<P, N, VB, REC>;
    // deep k-mer table over the symbols that occur in the text (k_dlut_root / k_dlut_level)
    uint32_t S = 0;
    for (uint32_t c = 0; c < (uint32_t)kMaxSigma; ++c) a.dlut_dig[c] = kNoDigit;
    for (uint32_t c = 0; c < ox.sigma; ++c)
        if (a.C[c + 1] > a.C[c]) {
            a.dlut_dig[c] = (uint8_t)S;
            a.dlut_sym[S++] = (uint8_t)c;
        }
    memcpy(t.dig, a.dlut_dig, sizeof(t.dig));
    std::vector<P> lut, lev;
    if ((options & 2u) && S >= 2 && ox.n > 0) {
        uint64_t budget = 1ull << 20;  // what tests/test_gpu.py sets (FMX_DEEP_LUT_MB=1)
        uint32_t K = 0;
        uint64_t cnt = 1;
        while (K < 32 && cnt <= budget / (2 * sizeof(P)) / S) { cnt *= S; ++K; }
        if (K > ox.k) {
            lev.assign(2 * S, 0);
            for (uint32_t d = 0; d < S; ++d) {
                lev[2 * d] = (P)a.C[a.dlut_sym[d]];
                lev[2 * d + 1] = (P)a.C[a.dlut_sym[d] + 1];
            }
            uint64_t np = S;
            for (uint32_t j = 1; j < K; ++j) {
                std::vector<P> nxt(2 * np * S, 0);
                for (uint64_t x = 0; x < np; ++x) {
                    const P lo = lev[2 * x], hi = lev[2 * x + 1];
                    if (!(lo < hi)) continue;
                    for (uint32_t d = 0; d < S; ++d) {
                        const uint32_t c = a.dlut_sym[d];
                        const P pre = (P)a.C[c];
                        nxt[2 * (d * np + x)] = pre + O::rank_at(a, lo + (lo < (P)a.sentinel ? P(1) : P(0)), c);
                        nxt[2 * (d * np + x) + 1] = pre + O::rank_at(a, hi + (hi < (P)a.sentinel ? P(1) : P(0)), c);
                    }
                }
                lev.swap(nxt);
                np *= S;
            }
            lut.swap(lev);
            a.dlut = reinterpret_cast<const uint8_t *>(lut.data());
            a.dlut_k = K;
            a.dlut_sigma = S;
        }
    }
    // full SA (k_full_sa), text (k_text), row contexts (k_row_ctx)
    std::vector<unsigned __int128> safull_store;  // 16-B aligned, padded like the device buffer
    P *safull = nullptr;
    std::vector<uint8_t> text;
    if (options & 16u) options |= 4u | 8u;
    if ((options & (4u | 8u)) && ox.n > 0) {
        uint32_t ctx_len = 0;
        if (options & 16u) {
            const unsigned __int128 lim = (unsigned __int128)1 << (8 * sizeof(P));
            unsigned __int128 w = 1;
            while (ctx_len < 64 && w * (ox.sigma + 1) < lim) { w *= ox.sigma + 1; ++ctx_len; }
        }
        const uint32_t stride = ctx_len ? 2 : 1;
        a.sa_stride = stride;
        safull_store.assign((ox.n * stride * sizeof(P) + 64) / 16 + 1, 0);
        safull = reinterpret_cast<P *>(safull_store.data());
        for (uint64_t r = 0; r < ox.n; ++r) safull[r * stride] = walk_row<P, N, VB, REC>(a, t.C, (P)r);
        a.safull = reinterpret_cast<const uint8_t *>(safull);
        if (options & 8u) {
            text.assign(ox.n + 16, 0);  // padded like the device copy
            for (uint64_t r = 0; r < ox.n; ++r) {
                uint32_t c = 0;
                while (c + 1 < ox.sigma && (uint64_t)t.C[c + 1] <= r) ++c;
                text[(uint64_t)safull[r * stride]] = (uint8_t)c;
            }
            a.text = text.data();
        }
        if (ctx_len) {
            a.ctx_len = ctx_len;
            a.scan_rows = scan_rows;
            a.wpow[0] = 1;
            for (uint32_t i = 1; i <= ctx_len; ++i) a.wpow[i] = a.wpow[i - 1] * (ox.sigma + 1);
            for (uint64_t r = 0; r < ox.n; ++r) {
                const uint64_t x = (uint64_t)safull[2 * r];
                uint64_t v = 0;
                for (uint32_t j = 1; j <= ctx_len; ++j) v = v * (ox.sigma + 1) + (j <= x ? text[x - j] + 1ull : 0);
                safull[2 * r + 1] = (P)v;
            }
        }
    }
    // single-row deep-table entries (k_dlut_rows)
    if ((options & 32u) && a.dlut && a.text && safull && (sizeof(P) == 8 || ox.n < (1ull << 31))) {
        uint32_t bps = 1;
        while ((1u << bps) < ox.sigma + 2) ++bps;
        a.dlut_bps = bps;
        a.dlut_ctx = (8 * sizeof(P) - 1) / bps;
        for (uint64_t e = 0; e < lut.size() / 2; ++e) {
            const P lo = lut[2 * e], hi = lut[2 * e + 1];
            if (!(lo < hi && hi - lo == P(1))) continue;
            const uint64_t x = (uint64_t)safull[(uint64_t)lo * a.sa_stride];
            uint64_t v = 0;
            for (uint32_t j = 1; j <= a.dlut_ctx; ++j) v |= (j <= x ? (uint64_t)text[x - j] + 1 : 0ull) << (bps * (j - 1));
            lut[2 * e] = row_flag<P>() | (P)v;
            lut[2 * e + 1] = (P)x;
        }
        a.dlut_rows = 1;
    }
    // queries (k_locate without the scan: outputs are in pattern order anyway)
    uint64_t out = 0;
    std::vector<uint8_t> staged;
    for (uint64_t i = 0; i < npat; ++i) {
        P lo, hi, rloc;
        uint64_t mask;
        uint32_t mode;
        PatView pv;
        pv.m = offs[i + 1] - offs[i];
        pv.rev = (flags & 1u) != 0;
        pv.raw = bytes + offs[i];
        pv.enc = t.enc;
        pv.sym = nullptr;
        if (i % 2 == 0) {  // odd patterns read raw bytes, even ones a staged copy (both kernel paths)
            staged.resize(pv.m + 1);
            for (uint64_t j = 0; j < pv.m; ++j) staged[j] = pv.at(j);
            pv.sym = staged.data();
        }
        // option bit 128: the long-pattern kernels' tail compare (LT)
        // the variant the engine launches (fmx_query.hip search_var)
        const bool derived = a.dlut || a.safull || a.text || a.ctx_len;
        SampledRow<P> smp;
        const uint32_t bad =
            !derived     ? search<P, N, VB, REC, kVarFaithful>(a, t, pv, lo, hi, rloc, mask, mode, &smp)
            : long_tails ? search<P, N, VB, REC, kVarDerivedLong>(a, t, pv, lo, hi, rloc, mask, mode, &smp)
                         : search<P, N, VB, REC, kVarDerived>(a, t, pv, lo, hi, rloc, mask, mode, &smp);
        if (bad) return bad == kStatusEmpty ? ORC_E_EMPTY_PATTERN : ORC_E_SYMBOL;
        const uint64_t cnt = (uint64_t)(hi - lo);
        if (mode == kHitRows && cnt == 1) {  // k_search settles a single row (its sampled row, else its walk)
            rloc = locate_one<P, N, VB, REC>(a, t.C, lo, smp);
            mode = kHitOne;
        }
        counts[i] = cnt;
        for (uint64_t j = 0; j < cnt; ++j, ++out) {
            P loc;
            if (mode == kHitOne) {
                loc = rloc;
            } else if (mode == kHitMask) {  // the k_locate locate phase
                uint64_t mk = mask;
                for (uint64_t u = 0; u < j; ++u) mk &= mk - 1;
                const P row = lo + (P)__builtin_ctzll(mk);
                loc = safull[(uint64_t)row * a.sa_stride] - rloc;
            } else {
                loc = walk_row<P, N, VB, REC>(a, t.C, lo + (P)j);
            }
            if (out < cap) locs[out] = (uint64_t)loc;
        }
    }
    *needed = out;
    return out > cap ? ORC_E_CAPACITY : ORC_OK;
}

template <typename P, int N, int VB, int R>
int run_if(const orc_index &ox, uint32_t options, const uint8_t *b, const uint64_t *o, uint64_t n, uint32_t f,
           uint64_t *c, uint64_t *l, uint64_t cap, uint64_t *need) {
    if constexpr (rec_fits(sizeof(P), N, VB, R)) return run<P, N, VB, R>(ox, options, b, o, n, f, c, l, cap, need);
    return -1;
}

template <typename P, int N, int VB>
int by_rec(uint32_t rec, const orc_index &ox, uint32_t options, const uint8_t *b, const uint64_t *o, uint64_t n,
           uint32_t f, uint64_t *c, uint64_t *l, uint64_t cap, uint64_t *need) {
    switch (rec) {
        case 64: return run_if<P, N, VB, 64>(ox, options, b, o, n, f, c, l, cap, need);
        case 128: return run_if<P, N, VB, 128>(ox, options, b, o, n, f, c, l, cap, need);
        case 64 | kRecPaired: return run_if<P, N, VB, 64 | kRecPaired>(ox, options, b, o, n, f, c, l, cap, need);
        case 128 | kRecPaired: return run_if<P, N, VB, 128 | kRecPaired>(ox, options, b, o, n, f, c, l, cap, need);
        case 64 | kRecOneHot: return run_if<P, N, VB, 64 | kRecOneHot>(ox, options, b, o, n, f, c, l, cap, need);
        case 128 | kRecOneHot: return run_if<P, N, VB, 128 | kRecOneHot>(ox, options, b, o, n, f, c, l, cap, need);
        case 256 | kRecOneHot: return run_if<P, N, VB, 256 | kRecOneHot>(ox, options, b, o, n, f, c, l, cap, need);
        case 384 | kRecOneHot: return run_if<P, N, VB, 384 | kRecOneHot>(ox, options, b, o, n, f, c, l, cap, need);
        case 512 | kRecOneHot: return run_if<P, N, VB, 512 | kRecOneHot>(ox, options, b, o, n, f, c, l, cap, need);
        case 256 | kRecOneHot | kRecWalk:
            return run_if<P, N, VB, 256 | kRecOneHot | kRecWalk>(ox, options, b, o, n, f, c, l, cap, need);
        case 384 | kRecOneHot | kRecWalk:
            return run_if<P, N, VB, 384 | kRecOneHot | kRecWalk>(ox, options, b, o, n, f, c, l, cap, need);
        case 512 | kRecOneHot | kRecWalk:
            return run_if<P, N, VB, 512 | kRecOneHot | kRecWalk>(ox, options, b, o, n, f, c, l, cap, need);
        default: return run<P, N, VB, 0>(ox, options, b, o, n, f, c, l, cap, need);
    }
}

template <typename P, int N>
int by_vb(uint32_t vb, uint32_t rec, const orc_index &ox, uint32_t options, const uint8_t *b, const uint64_t *o,
          uint64_t n, uint32_t f, uint64_t *c, uint64_t *l, uint64_t cap, uint64_t *need) {
    if (vb == 32) return by_rec<P, N, 32>(rec, ox, options, b, o, n, f, c, l, cap, need);
    if (vb == 64) return by_rec<P, N, 64>(rec, ox, options, b, o, n, f, c, l, cap, need);
    return by_rec<P, N, 128>(rec, ox, options, b, o, n, f, c, l, cap, need);
}

}  // namespace

// Built once per (P, N) pair (-DEMU_P=4|8 -DEMU_N=2..6, tests/emu/Makefile:
// ten objects compiled in parallel) plus the dispatching object (no EMU_P).
#define EMU_NAME2(p, n) emu_run_##p##_##n
#define EMU_NAME(p, n) EMU_NAME2(p, n)
#define EMU_ARGS                                                                                                   \
    uint32_t vb, uint32_t rec, const orc_index &ox, uint32_t options, const uint8_t *b, const uint64_t *o,        \
        uint64_t n, uint32_t f, uint64_t *c, uint64_t *l, uint64_t cap, uint64_t *need

#if defined(EMU_P)
int EMU_NAME(EMU_P, EMU_N)(EMU_ARGS) {
    using PT = std::conditional_t<EMU_P == 4, uint32_t, uint64_t>;
    return by_vb<PT, EMU_N>(vb, rec, ox, options, b, o, n, f, c, l, cap, need);
}
#else
int emu_run_4_2(EMU_ARGS); int emu_run_4_3(EMU_ARGS); int emu_run_4_4(EMU_ARGS); int emu_run_4_5(EMU_ARGS);
int emu_run_4_6(EMU_ARGS); int emu_run_8_2(EMU_ARGS); int emu_run_8_3(EMU_ARGS); int emu_run_8_4(EMU_ARGS);
int emu_run_8_5(EMU_ARGS); int emu_run_8_6(EMU_ARGS);

extern "C" {

// options: the fmx_load bit field (1 interleaved, 2 deep LUT, 4 full SA, 8 text,
// 16 row contexts, 32 single-row deep-table entries; 64 here: plain records,
// neither paired-chunk nor symbol-mask; bit 30 here: multi-line symbol masks
// with a walk line where they fit); bits 8.. = the scan limit
// (FMX_SCAN_ROWS, 0 = default 32).
// Outputs are u64: counts[npat] and the concatenated locations.
int emu_locate(const uint8_t *blob, uint64_t len, uint32_t pos_bytes, uint32_t planes, uint32_t vec_bits,
               uint32_t encoder, uint32_t options, const uint8_t *bytes, const uint64_t *offs, uint64_t npat,
               uint32_t flags, uint64_t *counts, uint64_t *locs, uint64_t cap, uint64_t *needed) {
    orc_layout L{pos_bytes, planes, vec_bits, encoder};
    orc_index ox;
    int st = orc_load(blob, len, L, &ox, nullptr, nullptr);
    if (st) return st;
    // the loader's record choice (fmx_load / k_relayout): option bit 64 keeps
    // plain records; multi-line symbol masks only without derived structures
    const bool fancy = (options & 64u) == 0, multi = fancy && (options & 62u) == 0, walk = (options & (1u << 30)) != 0;
    const uint32_t rec =
        (options & 1u) ? interleaved_rec_bytes(pos_bytes, planes, vec_bits, ox.sigma, fancy, fancy, multi, walk) : 0u;
    using Run = int (*)(EMU_ARGS);
    static const Run tab[2][5] = {{emu_run_4_2, emu_run_4_3, emu_run_4_4, emu_run_4_5, emu_run_4_6},
                                  {emu_run_8_2, emu_run_8_3, emu_run_8_4, emu_run_8_5, emu_run_8_6}};
    if (planes < 2 || planes > 6) return -1;
    return tab[pos_bytes == 4 ? 0 : 1][planes - 2](vec_bits, rec, ox, options, bytes, offs, npat, flags, counts, locs,
                                                   cap, needed);
}

}  // extern "C"
#endif
