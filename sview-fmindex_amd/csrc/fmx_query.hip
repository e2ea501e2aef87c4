// fmx_query.hip — gfx950 kernels for the FM-index query hot path.
//
//   k_count    : k-mer seed + backward-search LF loop, one lane per pattern
//                (FmIndex::get_pos_range, src/locate/with_slice.rs:21-33;
//                 next_pos_range, src/locate/mod.rs:38-45;
//                 BwmView::get_next_rank, components/bwm/mod.rs:197-215;
//                 CountArrayView seed, components/count_array.rs:203-233)
//   k_locate   : sampled-SA locate walk, one lane per occurrence row, rows
//                balanced across the 64 lanes of a wavefront
//                (write_locations_to_buffer, src/locate/mod.rs:14-37;
//                 get_pre_rank_and_symidx, components/bwm/mod.rs:217-236;
//                 SuffixArrayView::get_location_of, suffix_array/mod.rs:100-105)
//   k_relayout : optional one-time re-layout of (rank checkpoint, bit planes)
//                into one HBM record per block (FMX_OCC_INTERLEAVED).
//
// All integer work: no MFMA.  The hot loop is a chain of dependent random
// gathers, so the kernels keep many independent chains (lanes) in flight and
// make each LF step cost one HBM round trip: the checkpoint and bit-plane loads
// of a step are independent of each other, and in the interleaved layout they
// are the same line.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "fmx_internal.hpp"

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
    W w[N * WPP];

    // Block::get_remain_count_of (block3.rs:42-55): occurrences of symbol c among
    // the first `rem` symbols of the block (MSB-first); rem == 0 gives 0.
    __device__ __forceinline__ uint32_t rank(uint32_t rem, uint32_t c) const {
        if constexpr (VB == 128) {
            uint64_t lo = ~0ull, hi = ~0ull;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const bool b = (c >> j) & 1u;
                lo &= b ? w[2 * j] : ~w[2 * j];
                hi &= b ? w[2 * j + 1] : ~w[2 * j + 1];
            }
            if (rem == 0) return 0;
            if (rem <= 64) return __popcll(hi >> (64 - rem));
            return __popcll(hi) + __popcll(lo >> (128 - rem));
        } else {
            W m = ~W(0);
#pragma unroll
            for (int j = 0; j < N; ++j) m &= ((c >> j) & 1u) ? w[j] : W(~w[j]);
            if (rem == 0) return 0;
            if constexpr (VB == 64) return __popcll(m >> (64 - rem));
            else return __popc(m >> (32 - rem));
        }
    }

    // Block::get_symidx_of (block3.rs:57-63): bit VB-1-rem of plane j is bit j.
    __device__ __forceinline__ uint32_t sym(uint32_t rem) const {
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
};

// ------------------------------------------------------- occ access (rank)

// Blob layout: rank_checkpoints and blocks are separate arrays
// (bwm/mod.rs:145-190).  REC == 0.
// Interleaved layout: record q = [planes (N*VB/8 B)][ckpt[0..sigma) (P each)][pad]
// of REC bytes (64 or 128), one HBM line per LF step.
template <typename P, int N, int VB, int REC>
struct Occ {
    static constexpr int PLANE_BYTES = N * VB / 8;
    static constexpr int MAXC = REC == 0 ? 1 : (REC - PLANE_BYTES) / (int)sizeof(P);

    // A fetched block: planes + (blob mode) the one checkpoint asked for, or
    // (interleaved) every checkpoint of the record.
    struct Rec {
        Planes<N, VB> pl;
        P ck[MAXC];
    };

    __device__ __forceinline__ static void fetch_planes(const QueryArgs &a, uint64_t q, Planes<N, VB> &pl) {
        using W = typename VecT<VB>::W;
        const W *bp = reinterpret_cast<const W *>(a.blocks) + q * (uint64_t)(N * VecT<VB>::WPP);
#pragma unroll
        for (int j = 0; j < N * VecT<VB>::WPP; ++j) pl.w[j] = bp[j];
    }

    // Interleaved: load the whole record with 16-byte loads.
    __device__ __forceinline__ static void fetch_record(const QueryArgs &a, uint64_t q, Rec &r) {
        static_assert(REC == 64 || REC == 128, "record size");
        const uint4 *rp = reinterpret_cast<const uint4 *>(a.occ + q * (uint64_t)REC);
        uint32_t words[REC / 4];
#pragma unroll
        for (int i = 0; i < REC / 16; ++i) {
            const uint4 v = rp[i];
            words[4 * i + 0] = v.x; words[4 * i + 1] = v.y; words[4 * i + 2] = v.z; words[4 * i + 3] = v.w;
        }
        using W = typename VecT<VB>::W;
#pragma unroll
        for (int j = 0; j < N * VecT<VB>::WPP; ++j) {
            if constexpr (sizeof(W) == 8) r.pl.w[j] = (uint64_t)words[2 * j] | ((uint64_t)words[2 * j + 1] << 32);
            else r.pl.w[j] = words[j];
        }
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            constexpr int base = PLANE_BYTES / 4;
            if constexpr (sizeof(P) == 8) r.ck[i] = (P)((uint64_t)words[base + 2 * i] | ((uint64_t)words[base + 2 * i + 1] << 32));
            else r.ck[i] = (P)words[base + i];
        }
    }

    __device__ __forceinline__ static P pick(const Rec &r, uint32_t c) {
        P v = r.ck[0];
#pragma unroll
        for (int i = 1; i < MAXC; ++i) v = (c == (uint32_t)i) ? r.ck[i] : v;
        return v;
    }

    // Occ(c, stored position p): BwmView::get_next_rank after the sentinel
    // adjustment (bwm/mod.rs:206-214).
    __device__ __forceinline__ static P rank_at(const QueryArgs &a, P p, uint32_t c) {
        const uint64_t q = (uint64_t)p / VB;
        const uint32_t rem = (uint32_t)((uint64_t)p % VB);
        if constexpr (REC == 0) {
            const P ck = reinterpret_cast<const P *>(a.ckpt)[q * a.sigma + c];
            Planes<N, VB> pl;
            fetch_planes(a, q, pl);
            return ck + (P)pl.rank(rem, c);
        } else {
            Rec r;
            fetch_record(a, q, r);
            return pick(r, c) + (P)r.pl.rank(rem, c);
        }
    }

    // get_pre_rank_and_symidx body (bwm/mod.rs:223-235) for stored position p.
    __device__ __forceinline__ static P pre_rank_sym(const QueryArgs &a, P p, uint32_t &c) {
        const uint64_t q = (uint64_t)p / VB;
        const uint32_t rem = (uint32_t)((uint64_t)p % VB);
        if constexpr (REC == 0) {
            Planes<N, VB> pl;
            fetch_planes(a, q, pl);
            const P *ckq = reinterpret_cast<const P *>(a.ckpt) + q * a.sigma;
            if constexpr (N <= 3) {
                // sigma <= 8: fetch every checkpoint of the block alongside the
                // planes so the step costs one round trip, not two.
                P all[1 << N];
#pragma unroll
                for (int i = 0; i < (1 << N); ++i) all[i] = (uint32_t)i < a.sigma ? ckq[i] : P(0);
                c = pl.sym(rem);
                P ck = all[0];
#pragma unroll
                for (int i = 1; i < (1 << N); ++i) ck = (c == (uint32_t)i) ? all[i] : ck;
                return ck + (P)pl.rank(rem, c);
            } else {
                c = pl.sym(rem);
                return ckq[c] + (P)pl.rank(rem, c);
            }
        } else {
            Rec r;
            fetch_record(a, q, r);
            c = r.pl.sym(rem);
            return pick(r, c) + (P)r.pl.rank(rem, c);
        }
    }
};

// ----------------------------------------------------------------- k_count

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_count(const QueryArgs a, const uint8_t *__restrict__ bytes,
                                               const uint64_t *__restrict__ offs, uint64_t npat,
                                               uint32_t flags, P *__restrict__ out_cnt,
                                               uint64_t *__restrict__ cnt64, P *__restrict__ out_lo) {
    using O = Occ<P, N, VB, REC>;
    __shared__ uint8_t s_enc[256];
    __shared__ P s_C[kMaxSigma + 1];
    __shared__ uint64_t s_mult[kMaxK];
    const int t = threadIdx.x;
    s_enc[t] = a.enc[t];
    if ((uint32_t)t <= a.sigma) s_C[t] = (P)a.C[t];
    if ((uint32_t)t < a.k) s_mult[t] = a.mult[t];
    __syncthreads();

    const uint64_t i = (uint64_t)blockIdx.x * 256u + t;
    if (i >= npat) return;
    const uint64_t beg = offs[i];
    const uint64_t m = offs[i + 1] - beg;
    const uint8_t *p = bytes + beg;
    const bool rev = flags & FMX_PATTERN_REVERSED;
    const uint32_t sigma = a.sigma, k = a.k;
    const P sent = (P)a.sentinel;
    uint32_t bad = 0;
    P lo = 0, hi = 0;

    if (m == 0) {
        bad = kStatusEmpty;  // count_array.rs:211 panics on an empty pattern
    } else {
        // k-mer seed: count_array.rs:203-233.  Pattern position j is p[j]
        // (forward) or p[m-1-j] (bytes given reversed, with_rev_iter.rs).
        uint64_t s = 0, e, idx;
        const uint64_t take = m < k ? m : k, first = m < k ? 0 : m - k;
        for (uint64_t j = 0; j < take; ++j) {
            const uint64_t pj = first + j;
            const uint8_t b = p[rev ? m - 1 - pj : pj];
            const uint32_t c = s_enc[b];
            if (c >= sigma) bad = kStatusSymbol;
            s += (uint64_t)(c + 1) * s_mult[j];
        }
        if (m < k) { e = s + s_mult[m - 1] - 1; idx = 0; }
        else { e = s; idx = m - k; }
        const P *kt = reinterpret_cast<const P *>(a.kmer);
        if (!bad) { lo = kt[s - 1]; hi = kt[e]; }
        // LF loop: with_slice.rs:27-31 / next_pos_range (locate/mod.rs:39-45)
        while (!bad && lo < hi && idx > 0) {
            idx -= 1;
            const uint8_t b = p[rev ? m - 1 - idx : idx];
            const uint32_t c = s_enc[b];
            if (c >= sigma) { bad = kStatusSymbol; break; }
            const P pre = s_C[c];
            const P plo = lo + (lo < sent ? P(1) : P(0));  // bwm/mod.rs:202-204
            const P phi = hi + (hi < sent ? P(1) : P(0));
            const P rlo = O::rank_at(a, plo, c);
            const P rhi = O::rank_at(a, phi, c);
            lo = pre + rlo;
            hi = pre + rhi;
        }
    }
    if (bad) {
        atomicOr(a.status, bad);
        lo = hi = 0;
    }
    const P cnt = hi - lo;
    if (out_cnt) out_cnt[i] = cnt;
    if (cnt64) cnt64[i] = (uint64_t)cnt;
    if (out_lo) out_lo[i] = lo;
}

// ---------------------------------------------------------------- k_locate

// Walk one suffix-array row to a sampled row or to the text start
// (locate/mod.rs:19-35; suffix_array/mod.rs:100-105).
template <typename P, int N, int VB, int REC>
__device__ __forceinline__ P walk_row(const QueryArgs &a, const P *s_C, P pos) {
    using O = Occ<P, N, VB, REC>;
    const P sent = (P)a.sentinel;
    const P sr = (P)a.sr;
    const P mask = (P)a.sr_pow2_mask;
    P off = 0;
    while (mask ? (pos & mask) != 0 : (pos % sr) != 0) {
        if (pos == (P)(sent - P(1))) return off;  // get_pre_rank_and_symidx -> None
        const P p = pos + (pos < sent ? P(1) : P(0));
        uint32_t c;
        const P rank = O::pre_rank_sym(a, p, c);
        pos = s_C[c] + rank;
        off += 1;
    }
    const P *sa = reinterpret_cast<const P *>(a.sa);
    return sa[mask ? (uint64_t)pos >> (__builtin_popcount(a.sr_pow2_mask)) : (uint64_t)(pos / sr)] + off;
}

// Rows of the wave's 64 patterns are dealt to its 64 lanes in turns of 64
// consecutive output slots: a pattern with many occurrences is spread over
// all lanes instead of serialising one lane.
template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_locate(const QueryArgs a, const uint64_t *__restrict__ loc_off,
                                                const P *__restrict__ lo_arr, uint64_t npat,
                                                P *__restrict__ out, uint64_t cap) {
    __shared__ P s_C[kMaxSigma + 1];
    if ((uint32_t)threadIdx.x <= a.sigma) s_C[threadIdx.x] = (P)a.C[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t base = ((uint64_t)blockIdx.x * 256u + threadIdx.x - lane);
    if (base >= npat) return;  // wave-uniform
    const uint64_t idx = base + lane;
    const uint64_t my_off = loc_off[idx < npat ? idx : npat];
    const P my_lo = idx < npat ? lo_arr[idx] : P(0);
    const uint64_t start = __shfl(my_off, 0);
    const uint64_t end = loc_off[base + 64 < npat ? base + 64 : npat];
    for (uint64_t t0 = start; t0 < end; t0 += 64) {
        const uint64_t t = t0 + lane;
        // largest j with off[j] <= t (off[0] = start <= t)
        int j = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint64_t o = __shfl(my_off, j + step);
            if (o <= t) j += step;
        }
        const P lo_j = __shfl(my_lo, j);
        const uint64_t off_j = __shfl(my_off, j);
        if (t < end) {
            const P row = lo_j + (P)(t - off_j);
            const P loc = walk_row<P, N, VB, REC>(a, s_C, row);
            if (t < cap) out[t] = loc;
        }
    }
}

// -------------------------------------------------------------- k_relayout

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_relayout(const QueryArgs a, uint64_t blocks_len, uint8_t *__restrict__ occ) {
    constexpr int PB = N * VB / 8;
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= blocks_len) return;
    uint32_t words[REC / 4];
#pragma unroll
    for (int i = 0; i < REC / 4; ++i) words[i] = 0;
    const uint32_t *bp = reinterpret_cast<const uint32_t *>(a.blocks + q * PB);
#pragma unroll
    for (int i = 0; i < PB / 4; ++i) words[i] = bp[i];
    const uint32_t *cp = reinterpret_cast<const uint32_t *>(a.ckpt + q * a.sigma * sizeof(P));
    const uint32_t cw = a.sigma * (uint32_t)(sizeof(P) / 4);
#pragma unroll
    for (int i = 0; i < (REC - PB) / 4; ++i)
        if ((uint32_t)i < cw) words[PB / 4 + i] = cp[i];
    uint4 *rp = reinterpret_cast<uint4 *>(occ + q * REC);
#pragma unroll
    for (int i = 0; i < REC / 16; ++i)
        rp[i] = make_uint4(words[4 * i], words[4 * i + 1], words[4 * i + 2], words[4 * i + 3]);
}

// ------------------------------------------------------------- dispatch

uint32_t interleaved_record_bytes(const BlobView &bv) {
    const uint32_t need = bv.L.planes * bv.L.vec_bits / 8 + bv.sigma * bv.L.pos_bytes;
    if (need <= 64) return 64;
    if (need <= 128) return 128;
    return 0;  // too wide: stay on the blob layout
}

// Compile-time dispatch over the layout: F is a generic lambda called as
// f.template operator()<P, N, VB, REC>().
template <typename P, int N, int VB, class F>
static hipError_t disp_rec(uint32_t rec, F &&f) {
    switch (rec) {
        case 0: return f.template operator()<P, N, VB, 0>();
        case 64:
            if constexpr (N * VB / 8 + (int)sizeof(P) <= 64) return f.template operator()<P, N, VB, 64>();
            else return hipErrorInvalidValue;
        case 128:
            if constexpr (N * VB / 8 + (int)sizeof(P) <= 128) return f.template operator()<P, N, VB, 128>();
            else return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}
template <typename P, int N, class F>
static hipError_t disp_vb(uint32_t vb, uint32_t rec, F &&f) {
    switch (vb) {
        case 32: return disp_rec<P, N, 32>(rec, f);
        case 64: return disp_rec<P, N, 64>(rec, f);
        case 128: return disp_rec<P, N, 128>(rec, f);
        default: return hipErrorInvalidValue;
    }
}
template <typename P, class F>
static hipError_t disp_n(const fmx_layout &L, uint32_t rec, F &&f) {
    switch (L.planes) {
        case 2: return disp_vb<P, 2>(L.vec_bits, rec, f);
        case 3: return disp_vb<P, 3>(L.vec_bits, rec, f);
        case 4: return disp_vb<P, 4>(L.vec_bits, rec, f);
        case 5: return disp_vb<P, 5>(L.vec_bits, rec, f);
        case 6: return disp_vb<P, 6>(L.vec_bits, rec, f);
        default: return hipErrorInvalidValue;
    }
}
template <class F>
static hipError_t dispatch(const fmx_index *ix, F &&f) {
    const uint32_t rec = ix->occ_mode == FMX_OCC_INTERLEAVED ? ix->rec_bytes : 0;
    if (ix->bv.L.pos_bytes == 4) return disp_n<uint32_t>(ix->bv.L, rec, f);
    return disp_n<uint64_t>(ix->bv.L, rec, f);
}

static inline unsigned grid_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }

hipError_t launch_count(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets,
                        uint64_t n, uint32_t flags, void *d_counts_p, uint64_t *d_counts_u64,
                        void *d_lo_p, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        hipLaunchKernelGGL((k_count<P, N, VB, R>), dim3(grid_for(n)), dim3(256), 0, stream, ix->qa, d_bytes,
                           d_offsets, n, flags, (P *)d_counts_p, d_counts_u64, (P *)d_lo_p);
        return hipGetLastError();
    });
}

hipError_t launch_locate(const fmx_index *ix, const uint64_t *d_loc_offsets, const void *d_lo_p,
                         uint64_t n, void *d_locs, uint64_t cap, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        hipLaunchKernelGGL((k_locate<P, N, VB, R>), dim3(grid_for(n)), dim3(256), 0, stream, ix->qa, d_loc_offsets,
                           (const P *)d_lo_p, n, (P *)d_locs, cap);
        return hipGetLastError();
    });
}

hipError_t launch_relayout(fmx_index *ix, hipStream_t stream) {
    const uint64_t nb = ix->bv.blocks_len;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        if constexpr (R != 0) {
            hipLaunchKernelGGL((k_relayout<P, N, VB, R>), dim3(grid_for(nb)), dim3(256), 0, stream, ix->qa, nb,
                               ix->d_occ);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    });
}

hipError_t scan_workspace_bytes(uint64_t n, size_t *bytes) {
    size_t b = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                           (uint64_t)0, (size_t)(n + 1), rocprim::plus<uint64_t>());
    *bytes = b;
    return e;
}

hipError_t launch_scan(const uint64_t *d_in, uint64_t *d_out, uint64_t n_plus_1, void *tmp, size_t tmp_bytes,
                       hipStream_t stream) {
    size_t b = tmp_bytes;
    return rocprim::exclusive_scan(tmp, b, d_in, d_out, (uint64_t)0, (size_t)n_plus_1, rocprim::plus<uint64_t>(),
                                   stream);
}

}  // namespace fmx
