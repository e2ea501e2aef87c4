// fmx_query.hip — gfx950 kernels for the FM-index query hot path.
//
//   k_count   : k-mer seed + backward-search LF loop, one lane per pattern
//               (FmIndex::get_pos_range, src/locate/with_slice.rs:21-33;
//                next_pos_range, src/locate/mod.rs:38-45;
//                BwmView::get_next_rank, components/bwm/mod.rs:197-215;
//                CountArrayView seed, components/count_array.rs:203-233)
//   k_search  : the same search for a locate batch; a pattern whose interval
//               is one row walks that row to its sampled SA entry right away
//               (write_locations_to_buffer, src/locate/mod.rs:14-37;
//                get_pre_rank_and_symidx, components/bwm/mod.rs:217-236;
//                SuffixArrayView::get_location_of, suffix_array/mod.rs:100-105)
//               and leaves a search record per pattern plus its tile's count
//   k_scan    : tile offsets of batches too large for k_emit's own sum
//   k_emit    : output offsets, then every location: settled ones copied,
//               the rows of multi-row intervals walked, dealt across the 64
//               lanes of a wavefront
//   k_relayout: optional one-time re-layout of (rank checkpoints, bit planes)
//               into one HBM record per block (FMX_OCC_INTERLEAVED).
//
// All integer work: no MFMA.  The hot loop is a chain of dependent random
// gathers, so the kernels keep many independent chains (lanes) in flight and
// make each LF step cost one record read per rank query — one for both when
// lo and hi share a block.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "fmx_device.hpp"
#include "fmx_internal.hpp"

namespace fmx {

// The per-workgroup tables: encoding table, C array, k-mer multipliers, and
// — when it is small (QueryArgs::kt_lds_bytes) — the blob's k-mer count
// table, copied into LDS at `kt_lds` so that the seed's two reads are LDS
// reads.  Visible after the caller's next barrier.
template <typename P>
__device__ __forceinline__ void stage_tables(const QueryArgs &a, Tables<P> &s, uint8_t *kt_lds) {
    const int t = threadIdx.x;
    s.enc[t] = a.enc[t];
    if (t < kMaxSigma) s.dig[t] = a.dlut_dig[t];
    if ((uint32_t)t <= a.sigma) s.C[t] = (P)a.C[t];
    if ((uint32_t)t < a.k) s.mult[t] = a.mult[t];
    if (a.kt_lds_bytes && kt_lds) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(a.kmer);
        uint32_t *dst = reinterpret_cast<uint32_t *>(kt_lds);
        for (uint32_t i = t; i < a.kt_lds_bytes / 4; i += 256) dst[i] = src[i];
        if (t == 0) s.kt = reinterpret_cast<const P *>(kt_lds);
    } else if (t == 0) {
        s.kt = reinterpret_cast<const P *>(a.kmer);
    }
}

// 256-thread workgroup exclusive scan of one u64 per thread.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total, uint64_t *sh /*[4]*/) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < w) before += sh[i];
        all += sh[i];
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

// ----------------------------------------------------------------- k_count

// Stage the workgroup's patterns [first, first+256) as encoded symbols in
// LDS (pattern order; a reversed input range is stored reversed, which puts
// every pattern back in pattern order).  One round trip for the offsets (each
// thread its own pattern's bounds, plus the tile's), one for the bytes: 16-B
// aligned vectors, up to four per thread in flight (an aligned vector holding
// at least one byte of the batch never leaves the batch's page).  Returns
// false if the tile does not fit; the patterns are then read from HBM.
// NP patterns per thread (a pair of tiles: NP = 2): thread t stages and
// later searches patterns first + t, first + 256 + t, ... of one span.
template <typename P, int NP>
__device__ __forceinline__ bool stage_span(const Tables<P> &s, uint8_t *s_pat, const uint8_t *bytes,
                                           const uint64_t *offs, uint64_t npat, uint64_t first, bool rev,
                                           uint32_t stage_bytes, uint32_t stride, uint32_t *status,
                                           uint64_t *beg, uint64_t *end, uint64_t &b0, uint64_t &b1) {
    const uint64_t last = first + 256 * NP < npat ? first + 256 * NP : npat;
    uint64_t chk[NP];
    if (stride) {
        // FMX_HINT_FIXED_LEN: offs[i] == i * stride, so the byte loads need
        // not wait for the offsets; each thread's own end offsets are loaded
        // alongside them and checked once they have arrived.
        b0 = first * stride;
        b1 = last * stride;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const uint64_t i = first + 256 * q + threadIdx.x;
            beg[q] = i < npat ? i * stride : 0;
            end[q] = i < npat ? beg[q] + stride : 0;
            chk[q] = i < npat ? offs[i + 1] : 0;
        }
        if (first == 0 && threadIdx.x == 0 && offs[0] != 0) atomicOr(status, kStatusStride);
    } else {
        b0 = offs[first];
        b1 = offs[last];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const uint64_t i = first + 256 * q + threadIdx.x;
            beg[q] = i < npat ? offs[i] : 0;
            end[q] = i < npat ? offs[i + 1] : 0;
            chk[q] = end[q];
        }
    }
    const uint64_t len = b1 - b0;
    uint32_t bad_stride = 0;
#pragma unroll
    for (int q = 0; q < NP; ++q) bad_stride |= chk[q] != end[q];
    // the encoding table (stage_tables, written by every thread) is read below
    __syncthreads();
    if (len > stage_bytes) {
        if (bad_stride) atomicOr(status, kStatusStride);
        return false;
    }
    using V4 = uint32_t __attribute__((ext_vector_type(4)));
    const uint64_t a0 = b0 & ~15ull;
    const uint32_t nv = (uint32_t)((b1 - a0 + 15) >> 4);
    const V4 *src = reinterpret_cast<const V4 *>(bytes + a0);
    // 32-bit positions within the span (len <= stage_bytes): byte w of
    // vector v is span byte 16 v + w - lead, kept if below len (unsigned)
    const uint32_t lead = (uint32_t)(b0 - a0), len32 = (uint32_t)len;
    for (uint32_t v0 = 0; v0 < nv; v0 += 4 * 256) {
        V4 x[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t v = v0 + u * 256 + threadIdx.x;
            if (v < nv) x[u] = src[v];
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t v = v0 + u * 256 + threadIdx.x;
            if (v >= nv) continue;
            const uint32_t base = 16u * v - lead;
#pragma unroll
            for (uint32_t w = 0; w < 16; ++w) {
                const uint32_t x0 = base + w;
                if (x0 < len32)
                    s_pat[rev ? len32 - 1u - x0 : x0] = s.enc[(x[u][w >> 2] >> (8 * (w & 3))) & 0xffu];
            }
        }
    }
    if (bad_stride) atomicOr(status, kStatusStride);
    return true;
}

template <typename P>
__device__ __forceinline__ bool stage_patterns(const Tables<P> &s, uint8_t *s_pat, const uint8_t *bytes,
                                               const uint64_t *offs, uint64_t npat, uint64_t first, bool rev,
                                               uint32_t stage_bytes, uint32_t stride, uint32_t *status,
                                               uint64_t &beg, uint64_t &end, uint64_t &b0, uint64_t &b1) {
    return stage_span<P, 1>(s, s_pat, bytes, offs, npat, first, rev, stage_bytes, stride, status, &beg, &end, b0,
                            b1);
}

template <typename P>
__device__ __forceinline__ PatView pattern_view(const Tables<P> &s, const uint8_t *s_pat, bool staged,
                                                const uint8_t *bytes, uint64_t beg, uint64_t end, uint64_t b0,
                                                uint64_t b1, bool rev) {
    PatView pv;
    pv.m = end - beg;
    pv.rev = rev;
    pv.raw = bytes + beg;
    pv.enc = s.enc;
    pv.sym = staged ? s_pat + (rev ? b1 - end : beg - b0) : nullptr;
    return pv;
}

template <typename P, int N, int VB, int REC, int VAR>
__global__ __launch_bounds__(256) void k_count(const QueryArgs a, const uint8_t *__restrict__ bytes,
                                               const uint64_t *__restrict__ offs, uint64_t npat,
                                               uint32_t flags, P *__restrict__ out_cnt, uint32_t stage_bytes) {
    __shared__ Tables<P> s;
    extern __shared__ uint8_t s_pat[];  // stage_bytes, then the k-mer table (dynamic)
    stage_tables(a, s, s_pat + stage_bytes);
    __syncthreads();
    const bool rev = (flags & FMX_PATTERN_REVERSED) != 0;
    const uint64_t first = (uint64_t)blockIdx.x * 256u;
    uint64_t beg, end, b0, b1;
    const bool staged = stage_patterns(s, s_pat, bytes, offs, npat, first, rev, stage_bytes, flags >> 16, a.status, beg,
                                       end, b0, b1);
    __syncthreads();
    const uint64_t i = first + threadIdx.x;
    if (i >= npat) return;
    const PatView pv = pattern_view(s, s_pat, staged, bytes, beg, end, b0, b1, rev);
    P lo, hi, rloc;
    uint64_t mask;
    uint32_t mode;
    const uint32_t bad = search<P, N, VB, REC, VAR>(a, s, pv, lo, hi, rloc, mask, mode);
    if (bad) atomicOr(a.status, bad);
    out_cnt[i] = hi - lo;
}

// ------------------------------------------------------------ locations

// The locations of a wave's 64 patterns (lane j: pattern with output slots
// [my_off, my_off + cnt) and its search result), every occurrence row dealt
// to the next free lane so that skewed counts keep the wave busy
// (write_locations_to_buffer, src/locate/mod.rs:14-37): lane t of a round
// finds its pattern by a binary search over the lanes' first slots.
template <typename P, int N, int VB, int REC>
__device__ __forceinline__ void emit_locations(const QueryArgs &a, const P *C, uint64_t my_off, uint64_t cnt, P lo,
                                               P rloc, uint64_t mask, uint32_t mode, uint64_t cap,
                                               P *__restrict__ out_locs) {
    const int lane = threadIdx.x & 63;
    const uint64_t w_start = __shfl(my_off, 0);
    const uint64_t w_end = __shfl(my_off + cnt, 63);
    for (uint64_t t0 = w_start; t0 < w_end; t0 += 64) {
        const uint64_t t = t0 + lane;
        int jl = 0;  // largest lane whose first slot is <= t
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint64_t o = __shfl(my_off, jl + step);
            if (o <= t) jl += step;
        }
        const P lo_j = __shfl(lo, jl);
        const uint64_t off_j = __shfl(my_off, jl);
        const P rloc_j = __shfl(rloc, jl);
        const uint32_t mode_j = (uint32_t)__shfl((int)mode, jl);
        const uint64_t mask_j = __shfl(mask, jl);
        if (t < w_end) {
            const uint64_t q = t - off_j;  // occurrence q of pattern jl
            P loc;
            if (mode_j == kHitOne) {
                loc = rloc_j;  // resolved against the text: its one location
            } else if (mode_j == kHitMask) {
                uint64_t mk = mask_j;  // the q-th matching row of a scanned interval
                for (uint64_t u = 0; u < q; ++u) mk &= mk - 1;
                const P row = lo_j + (P)__builtin_ctzll(mk);
                loc = reinterpret_cast<const P *>(a.safull)[(uint64_t)row * a.sa_stride] - rloc_j;
            } else {
                loc = walk_row<P, N, VB, REC>(a, C, lo_j + (P)q);
            }
            if (t < cap) out_locs[t] = loc;
        }
    }
}


// ------------------------------------------------- k_search + k_emit (split)

// A pattern's search result, handed from k_search to k_emit (P-typed words):
//   rows (kHitRows): a = lo,   b = count, x = 0
//   one  (kHitOne):  a = rloc, b = count, x = 1
//   mask (kHitMask): a = lo,   b = rloc,  x = mask (>= 2 bits set, count = popcount)
template <typename P>
struct SearchRec {
    P a, b;
    uint64_t x;
};

template <typename P>
__device__ __forceinline__ SearchRec<P> pack_rec(P lo, P hi, P rloc, uint64_t mask, uint32_t mode) {
    if (mode == kHitOne) return {rloc, (P)(hi - lo), 1ull};
    if (mode == kHitMask) return {lo, rloc, mask};
    return {lo, (P)(hi - lo), 0ull};
}

template <typename P>
__device__ __forceinline__ uint64_t unpack_rec(const SearchRec<P> &r, P &lo, P &rloc, uint64_t &mask,
                                               uint32_t &mode) {
    // Selects, not branches: the if-chain form of this decode was miscompiled
    // (hipcc 7.2, gfx950: lo/rloc left undefined on the x > 1 path).
    const uint64_t x = r.x;
    const bool is_one = x == 1, is_mask = x > 1;
    mode = is_mask ? kHitMask : (is_one ? kHitOne : kHitRows);
    lo = is_one ? P(0) : r.a;
    rloc = is_mask ? r.b : (is_one ? r.a : P(0));
    mask = is_mask ? x : 0ull;
    return is_mask ? (uint64_t)__builtin_popcountll(x) : (uint64_t)r.b;
}

// The locate launch: k_search, (k_scan,) k_emit.
// No workgroup ever waits on another, so nothing depends on the order or
// placement in which workgroups are dispatched (MI355X_MICROARCH.md: HIP
// promises neither; a look-back that assumes in-order dispatch can deadlock
// when launches on several streams share the CUs).  Per batch of a group:
// workspace = [256 B][tile counts: G][tile offsets: G][search records: n].

// This workgroup's batch of a grouped launch (workgroup-uniform).
__device__ __forceinline__ uint32_t group_batch(const LocateGroup &grp, uint32_t vt) {
    uint32_t jb = 0;
#pragma unroll
    for (uint32_t t = 1; t < kMaxGroup; ++t)
        if (t < grp.n && vt >= grp.tile_begin[t]) jb = t;
    return jb;
}

// 1. Search every pattern; its result record, its count; the tile's count.
template <typename P, int N, int VB, int REC, int VAR>
__device__ __forceinline__ void search_tile(const QueryArgs &a, const LocateGroup &grp, const Tables<P> &s,
                                            uint8_t *s_pat, uint64_t *s_scan, uint32_t stage_bytes, uint32_t vt) {
    const uint32_t jb = group_batch(grp, vt);
    const LocateBatch &B = grp.b[jb];
    const uint8_t *__restrict__ bytes = B.bytes;
    const uint64_t *__restrict__ offs = B.offs;
    const uint64_t npat = B.npat;
    const bool rev = B.rev != 0;
    const uint32_t g = vt - grp.tile_begin[jb];
    const uint64_t G = (npat + 255) / 256;
    SearchRec<P> *__restrict__ recs = reinterpret_cast<SearchRec<P> *>(B.tiles + 2 * G);
    uint64_t beg, end, b0, b1;
    const bool staged =
        stage_patterns(s, s_pat, bytes, offs, npat, (uint64_t)g * 256u, rev, stage_bytes, B.stride, a.status,
                       beg, end, b0, b1);
    __syncthreads();
    const uint64_t i = (uint64_t)g * 256u + threadIdx.x;
    uint64_t cnt = 0;
    if (i < npat) {
        const PatView pv = pattern_view(s, s_pat, staged, bytes, beg, end, b0, b1, rev);
        P lo, hi, rloc;
        uint64_t mask;
        uint32_t mode;
        const uint32_t bad = search<P, N, VB, REC, VAR>(a, s, pv, lo, hi, rloc, mask, mode);
        if (bad) atomicOr(a.status, bad);
        cnt = (uint64_t)(hi - lo);
        if (B.out_cnt) reinterpret_cast<P *>(B.out_cnt)[i] = hi - lo;
        // one row (most patterns of a large text): its location now, while
        // this lane's chain is live (locate/mod.rs:19-35); k_emit then only
        // copies it
        if (mode == kHitRows && cnt == 1) {
            rloc = walk_row<P, N, VB, REC>(a, s.C, lo);
            mode = kHitOne;
        }
        recs[i] = pack_rec<P>(lo, hi, rloc, mask, mode);
    }
    uint64_t agg;
    block_excl_scan(cnt, &agg, s_scan);  // (its barriers end every read of s_pat)
    if (threadIdx.x == 0) B.tiles[g] = agg;
}

template <typename P, int N, int VB, int REC, int VAR>
__global__ __launch_bounds__(256, VAR == kVarDerivedLong ? 4 : 8) void k_search(const QueryArgs a, const LocateGroup grp,
                                                             uint32_t stage_bytes) {
    __shared__ Tables<P> s;
    extern __shared__ uint8_t s_pat[];  // stage_bytes, then the k-mer table (dynamic)
    __shared__ uint64_t s_scan[4];
    stage_tables(a, s, s_pat + stage_bytes);
    search_tile<P, N, VB, REC, VAR>(a, grp, s, s_pat, s_scan, stage_bytes, blockIdx.x);
}

// 2. One workgroup per batch: exclusive scan of its tile counts into tile
// offsets, and the batch total (16 tiles per thread per pass, every load of
// a pass in flight at once).
__global__ __launch_bounds__(256) void k_scan(const LocateGroup grp) {
    __shared__ uint64_t s_scan[4];
    const LocateBatch &B = grp.b[blockIdx.x];
    const uint64_t G = (B.npat + 255) / 256;
    const uint64_t *cnt = B.tiles;
    uint64_t *off = B.tiles + G;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < G; base += 256 * 16) {
        uint64_t v[16], sum = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint64_t t = base + threadIdx.x * 16ull + u;
            v[u] = t < G ? cnt[t] : 0;
            sum += v[u];
        }
        uint64_t tot;
        uint64_t run = carry + block_excl_scan(sum, &tot, s_scan);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint64_t t = base + threadIdx.x * 16ull + u;
            if (t < G) off[t] = run;
            run += v[u];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        B.loc_off[B.npat] = carry;
        *B.needed = carry;
    }
}

// 3. Output offsets (tile offset + in-tile scan) and every location, rows
// dealt across each wave's lanes (emit_locations).
// fold: batches of at most kFoldTiles tiles need no k_scan: each workgroup
// sums the counts of the tiles before its own (all final: k_search is done),
// and the last tile writes the batch total.
constexpr uint64_t kFoldTiles = 2048;

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_emit(const QueryArgs a, const LocateGroup grp, uint32_t fold) {
    __shared__ P sC[kMaxSigma + 1];
    __shared__ uint64_t s_scan[4];
    if (threadIdx.x <= a.sigma) sC[threadIdx.x] = (P)a.C[threadIdx.x];
    const uint32_t jb = group_batch(grp, blockIdx.x);
    const LocateBatch &B = grp.b[jb];
    const uint64_t npat = B.npat, G = (npat + 255) / 256;
    const uint64_t g = blockIdx.x - grp.tile_begin[jb], i = g * 256u + threadIdx.x;
    const SearchRec<P> *__restrict__ recs = reinterpret_cast<const SearchRec<P> *>(B.tiles + 2 * G);
    P lo = 0, rloc = 0;
    uint64_t mask = 0, cnt = 0;
    uint32_t mode = kHitOne;
    if (i < npat) cnt = unpack_rec<P>(recs[i], lo, rloc, mask, mode);
    uint64_t base;
    if (fold) {
        uint64_t part = 0;
        for (uint64_t t = threadIdx.x; t < g; t += 256) part += B.tiles[t];
        uint64_t tot;
        block_excl_scan(part, &tot, s_scan);
        base = tot;
    } else {
        base = B.tiles[G + g];
    }
    uint64_t agg;
    const uint64_t my_off = base + block_excl_scan(cnt, &agg, s_scan);  // (its barriers publish sC)
    if (fold && g == G - 1 && threadIdx.x == 0) {
        B.loc_off[npat] = base + agg;
        *B.needed = base + agg;
    }
    if (i < npat) B.loc_off[i] = my_off;
    emit_locations<P, N, VB, REC>(a, sC, my_off, cnt, lo, rloc, mask, mode, B.cap,
                                  reinterpret_cast<P *>(B.out_locs));
}

// ------------------------------------------------------------ deep k-mer table

// The table's digits are the S symbols that occur in the text (dlut_sym).
// Level 1: the interval of each single symbol c is [C[c], C[c+1]) (the root,
// the empty string, is full row 0..n which the reduced row numbering cannot
// represent, so level 1 is written directly; count_array.rs:139-145).
template <typename P>
__global__ void k_dlut_root(const QueryArgs a, P *__restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d < a.dlut_sigma) {
        const uint32_t c = a.dlut_sym[d];
        out[2 * d] = (P)a.C[c];
        out[2 * d + 1] = (P)a.C[c + 1];
    }
}

// Level j -> j+1: child string cS has code digit(c)*S^j + code(S); its
// interval is one LF step (next_pos_range, locate/mod.rs:39-45) from S's.
template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_dlut_level(const QueryArgs a, const P *__restrict__ parent, uint64_t np,
                                                    P *__restrict__ child) {
    using O = Occ<P, N, VB, REC>;
    const P sent = (P)a.sentinel;
    // grid-stride: a launch covers at most 2^32 - 1 work-items (S^16 parents
    // for a K = 17 table would not fit one thread each)
    for (uint64_t x = (uint64_t)blockIdx.x * 256u + threadIdx.x; x < np; x += (uint64_t)gridDim.x * 256u) {
    const P lo = parent[2 * x], hi = parent[2 * x + 1];
    for (uint32_t d = 0; d < a.dlut_sigma; ++d) {
        const uint32_t c = a.dlut_sym[d];
        P clo = 0, chi = 0;
        if (lo < hi) {
            const P pre = (P)a.C[c];
            clo = pre + O::rank_at(a, lo + (lo < sent ? P(1) : P(0)), c);
            chi = pre + O::rank_at(a, hi + (hi < sent ? P(1) : P(0)), c);
        }
        P *dst = child + 2 * ((uint64_t)d * np + x);
        dst[0] = clo;
        dst[1] = chi;
    }
    }
}

// Single-row entries (FMX_OPT_LUT_ROWS): an interval of exactly one row r
// becomes {row_flag | T[x-1], T[x-2], ..., T[x-dlut_ctx] packed, x = SA[r]}
// (see one_row in fmx_device.hpp).
template <typename P>
__global__ __launch_bounds__(256) void k_dlut_rows(const QueryArgs a, uint64_t entries, P *__restrict__ dl) {
    const P *sa = reinterpret_cast<const P *>(a.safull);
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < entries; e += (uint64_t)gridDim.x * 256) {
        const P lo = dl[2 * e], hi = dl[2 * e + 1];
        if (!(lo < hi && hi - lo == P(1))) continue;
        const uint64_t x = (uint64_t)sa[(uint64_t)lo * a.sa_stride];
        uint64_t v = 0;
        for (uint32_t j = 1; j <= a.dlut_ctx; ++j)
            v |= (j <= x ? (uint64_t)a.text[x - j] + 1 : 0ull) << (a.dlut_bps * (j - 1));
        dl[2 * e] = row_flag<P>() | (P)v;
        dl[2 * e + 1] = (P)x;
    }
}

// ------------------------------------------------ full SA and text recovery

// SA[r] for every reduced row r: the locate walk of every row
// (locate/mod.rs:19-35), done once at load.
template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_full_sa(const QueryArgs a, uint64_t n, P *__restrict__ sa_out,
                                                 uint32_t stride) {
    __shared__ Tables<P> s;
    stage_tables(a, s, nullptr);
    __syncthreads();
    QueryArgs b = a;
    b.safull = nullptr;
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (uint64_t)gridDim.x * 256)
        sa_out[r * stride] = walk_row<P, N, VB, REC>(b, s.C, (P)r);
}

// T[SA[r]] = first symbol of row r's suffix = the c with C[c] <= r < C[c+1].
template <typename P>
__global__ __launch_bounds__(256) void k_text(const QueryArgs a, uint64_t n, const P *__restrict__ sa,
                                              uint32_t stride, uint8_t *__restrict__ text) {
    __shared__ P sC[kMaxSigma + 1];
    if (threadIdx.x <= a.sigma) sC[threadIdx.x] = (P)a.C[threadIdx.x];
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (uint64_t)gridDim.x * 256) {
        uint32_t c = 0;
        while (c + 1 < a.sigma && (uint64_t)sC[c + 1] <= r) ++c;
        text[(uint64_t)sa[r * stride]] = (uint8_t)c;
    }
}

// Row contexts (FMX_OPT_ROW_CONTEXT): rec[2r+1] = T[x-1], T[x-2], ..., T[x-ctx_len]
// (x = SA[r] = rec[2r]) as sigma+1-ary digits, symbol + 1, 0 before the text
// start, the nearest symbol most significant.
template <typename P>
__global__ __launch_bounds__(256) void k_row_ctx(const QueryArgs a, uint64_t n, const uint8_t *__restrict__ text,
                                                 P *__restrict__ rec) {
    const uint32_t W = a.sigma + 1, Cl = a.ctx_len;
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (uint64_t)gridDim.x * 256) {
        const uint64_t x = (uint64_t)rec[2 * r];
        uint64_t v = 0;
        for (uint32_t j = 1; j <= Cl; ++j) v = v * W + (j <= x ? (uint64_t)text[x - j] + 1 : 0);
        rec[2 * r + 1] = (P)v;
    }
}

// -------------------------------------------------------------- k_relayout

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_relayout(const QueryArgs a, uint64_t blocks_len, uint8_t *__restrict__ occ) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= blocks_len) return;
    write_record<P, N, VB, REC>(occ + q * REC, a.blocks + q * (N * VB / 8), a.ckpt + q * a.sigma * sizeof(P),
                                a.sigma);
}

// ------------------------------------------------------------- dispatch

uint32_t interleaved_record_bytes(const BlobView &bv) {
    return interleaved_rec_bytes(bv.L.pos_bytes, bv.L.planes, bv.L.vec_bits, bv.sigma);
}

// Compile-time dispatch over the layout: F is a generic lambda called as
// f.template operator()<P, N, VB, REC>().
template <typename P, int N, int VB, class F>
static hipError_t disp_rec(uint32_t rec, F &&f) {
    switch (rec) {
        case 0: return f.template operator()<P, N, VB, 0>();
        case 64:
            if constexpr (Occ<P, N, VB, 0>::PBA + (int)sizeof(P) <= 64) return f.template operator()<P, N, VB, 64>();
            else return hipErrorInvalidValue;
        case 128:
            if constexpr (Occ<P, N, VB, 0>::PBA + (int)sizeof(P) <= 128) return f.template operator()<P, N, VB, 128>();
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
// k_dlut_level: one thread per parent up to 2^24 workgroups, then grid-stride
static inline unsigned grid_dlut(uint64_t np) {
    const uint64_t g = (np + 255) / 256;
    return (unsigned)(g < (1ull << 24) ? (g ? g : 1) : (1ull << 24) - 1);
}

// look-back tiles needed for n patterns (one per 256-pattern workgroup)
uint64_t locate_tiles_cap(uint64_t n) { return (n + 255) / 256 > 0 ? (n + 255) / 256 : 1; }

static inline uint32_t stage_bytes_for(uint32_t flags) {
    const uint32_t kb = (flags >> 8) & 0xffu;  // FMX_HINT_STAGE_KB
    if (kb) return std::min<uint32_t>(kb, kStageBytesLong / 1024) * 1024u;
    return (flags & FMX_HINT_LONG_PATTERNS) ? (uint32_t)kStageBytesLong : (uint32_t)kStageBytes;
}

// The search variant for an index and a launch's staging size: the faithful
// kernels when no derived structure is loaded; else the derived ones, with
// the vectorised tail compare for long patterns (56 KB staging).
static inline int search_var(const QueryArgs &qa, uint32_t sb) {
    const bool derived = qa.dlut != nullptr || qa.safull != nullptr || qa.text != nullptr || qa.ctx_len != 0;
    if (!derived) return kVarFaithful;
    return sb > (uint32_t)kStageBytes ? kVarDerivedLong : kVarDerived;
}

hipError_t launch_count(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                        uint32_t flags, void *d_counts, uint32_t *status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    QueryArgs qa = ix->qa;
    qa.status = status;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        const uint32_t sb = stage_bytes_for(flags), lds = sb + qa.kt_lds_bytes;
        switch (search_var(qa, sb)) {
            case kVarFaithful:
                hipLaunchKernelGGL((k_count<P, N, VB, R, kVarFaithful>), dim3(grid_for(n)), dim3(256), lds, stream,
                                   qa, d_bytes, d_offsets, n, flags, (P *)d_counts, sb);
                break;
            case kVarDerived:
                hipLaunchKernelGGL((k_count<P, N, VB, R, kVarDerived>), dim3(grid_for(n)), dim3(256), lds, stream,
                                   qa, d_bytes, d_offsets, n, flags, (P *)d_counts, sb);
                break;
            default:
                hipLaunchKernelGGL((k_count<P, N, VB, R, kVarDerivedLong>), dim3(grid_for(n)), dim3(256), lds,
                                   stream, qa, d_bytes, d_offsets, n, flags, (P *)d_counts, sb);
        }
        return hipGetLastError();
    });
}

// The kernels of a (grouped) locate, one after another on `stream`.
template <typename P, int N, int VB, int R>
static hipError_t launch_split(const QueryArgs &qa, const LocateGroup &grp, uint32_t tiles, uint32_t sb,
                               hipStream_t stream) {
    const uint32_t lds = sb + qa.kt_lds_bytes;
    switch (search_var(qa, sb)) {
        case kVarFaithful:
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarFaithful>), dim3(tiles), dim3(256), lds, stream, qa, grp,
                               sb);
            break;
        case kVarDerived:
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarDerived>), dim3(tiles), dim3(256), lds, stream, qa, grp,
                               sb);
            break;
        default:
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarDerivedLong>), dim3(tiles), dim3(256), lds, stream, qa,
                               grp, sb);
    }
    uint32_t fold = 1;
    for (uint32_t j = 0; j < grp.n; ++j) fold &= (grp.b[j].npat + 255) / 256 <= kFoldTiles ? 1u : 0u;
    if (!fold) hipLaunchKernelGGL(k_scan, dim3(grp.n), dim3(256), 0, stream, grp);
    hipLaunchKernelGGL((k_emit<P, N, VB, R>), dim3(tiles), dim3(256), 0, stream, qa, grp, fold);
    return hipGetLastError();
}

hipError_t launch_locate(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                         uint32_t flags, void *d_counts, uint64_t *d_loc_offsets, void *d_locs, uint64_t cap,
                         uint64_t *d_needed, uint64_t *d_tiles, uint64_t tiles_cap, uint32_t *status,
                         hipStream_t stream) {
    if (n == 0) return hipSuccess;
    QueryArgs qa = ix->qa;
    qa.status = status;
    if ((n + 255) / 256 > tiles_cap || tiles_cap > 0xFFFFFFFFull) return hipErrorInvalidValue;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        LocateGroup grp{};
        grp.b[0] = LocateBatch{d_bytes, d_offsets, n, d_counts, d_loc_offsets, d_locs, cap, d_needed, d_tiles,
                               (flags & FMX_PATTERN_REVERSED) ? 1u : 0u, flags >> 16};
        grp.n = 1;
        return launch_split<P, N, VB, R>(qa, grp, (uint32_t)((n + 255) / 256), stage_bytes_for(flags), stream);
    });
}

hipError_t launch_locate_group(const fmx_index *ix, const LocateGroup &grp, uint32_t stage_flags,
                               uint32_t *status, hipStream_t stream) {
    QueryArgs qa = ix->qa;
    qa.status = status;
    if (grp.n == 0 || grp.n > kMaxGroup || grp.tile_begin[0] != 0) return hipErrorInvalidValue;
    uint64_t tiles = 0;
    for (uint32_t j = 0; j < grp.n; ++j) {
        if (grp.b[j].npat == 0 || grp.tile_begin[j] != tiles) return hipErrorInvalidValue;
        tiles += (grp.b[j].npat + 255) / 256;
    }
    if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
    return dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        return launch_split<P, N, VB, R>(qa, grp, (uint32_t)tiles, stage_bytes_for(stage_flags), stream);
    });
}

uint64_t locate_rec_bytes(uint32_t pos_bytes) {
    return pos_bytes == 4 ? sizeof(SearchRec<uint32_t>) : sizeof(SearchRec<uint64_t>);
}

hipError_t build_deep_lut(fmx_index *ix, uint32_t K, hipStream_t stream) {
    const uint64_t sigma = ix->qa.dlut_sigma, pb = ix->bv.L.pos_bytes;
    uint64_t total = 1;
    for (uint32_t j = 0; j < K; ++j) total *= sigma;
    uint8_t *tmp = nullptr;
    const uint64_t tmp_entries = total / sigma;
    hipError_t e = hipMalloc(&ix->d_dlut, total * 2 * pb);
    if (e != hipSuccess) return e;
    ix->dlut_bytes = total * 2 * pb;
    if (K > 1) {
        e = hipMalloc(&tmp, std::max<uint64_t>(tmp_entries, 1) * 2 * pb);
        if (e != hipSuccess) return e;
    }
    // level j lives in the final buffer when (K - j) is even, else in tmp
    auto buf = [&](uint32_t j) { return ((K - j) % 2 == 0) ? ix->d_dlut : tmp; };
    QueryArgs qa = ix->qa;
    qa.dlut = nullptr;
    e = dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        hipLaunchKernelGGL((k_dlut_root<P>), dim3(1), dim3(64), 0, stream, qa, (P *)buf(1));
        uint64_t np = sigma;
        for (uint32_t j = 1; j < K; ++j) {
            hipLaunchKernelGGL((k_dlut_level<P, N, VB, R>), dim3(grid_dlut(np)), dim3(256), 0, stream, qa,
                               (const P *)buf(j), np, (P *)buf(j + 1));
            np *= sigma;
        }
        return hipGetLastError();
    });
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (tmp) hipFree(tmp);
    return e;
}

static inline unsigned grid_stride_for(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 65536 ? (g ? g : 1) : 65536);
}

hipError_t build_dlut_rows(fmx_index *ix, hipStream_t stream) {
    const uint64_t entries = ix->dlut_bytes / (2ull * ix->bv.L.pos_bytes);
    if (ix->bv.L.pos_bytes == 4)
        hipLaunchKernelGGL((k_dlut_rows<uint32_t>), dim3(grid_stride_for(entries)), dim3(256), 0, stream, ix->qa,
                           entries, (uint32_t *)ix->d_dlut);
    else
        hipLaunchKernelGGL((k_dlut_rows<uint64_t>), dim3(grid_stride_for(entries)), dim3(256), 0, stream, ix->qa,
                           entries, (uint64_t *)ix->d_dlut);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e;
}

hipError_t build_full_sa(fmx_index *ix, uint32_t stride, hipStream_t stream) {
    const uint64_t n = ix->bv.n;
    // padded: scan_rows reads whole 16-B vectors of row records
    ix->safull_bytes = std::max<uint64_t>(n, 1) * ix->bv.L.pos_bytes * stride + 64;
    hipError_t e = hipMalloc(&ix->d_safull, ix->safull_bytes);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(ix->d_safull, 0, ix->safull_bytes, stream);
    if (e != hipSuccess) return e;
    e = dispatch(ix, [&]<typename P, int N, int VB, int R>() {
        hipLaunchKernelGGL((k_full_sa<P, N, VB, R>), dim3(grid_stride_for(n)), dim3(256), 0, stream, ix->qa, n,
                           (P *)ix->d_safull, stride);
        return hipGetLastError();
    });
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e;
}

hipError_t build_text(fmx_index *ix, hipStream_t stream) {
    const uint64_t n = ix->bv.n;
    // padded by 16 zero bytes: tail_mismatch reads aligned words past the end
    hipError_t e = hipMalloc(&ix->d_text, n + 16);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(ix->d_text, 0, n + 16, stream);
    if (e != hipSuccess) return e;
    const uint32_t stride = ix->qa.sa_stride;
    if (ix->bv.L.pos_bytes == 4)
        hipLaunchKernelGGL((k_text<uint32_t>), dim3(grid_stride_for(n)), dim3(256), 0, stream, ix->qa, n,
                           (const uint32_t *)ix->d_safull, stride, ix->d_text);
    else
        hipLaunchKernelGGL((k_text<uint64_t>), dim3(grid_stride_for(n)), dim3(256), 0, stream, ix->qa, n,
                           (const uint64_t *)ix->d_safull, stride, ix->d_text);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e;
}

hipError_t build_row_context(fmx_index *ix, hipStream_t stream) {
    const uint64_t n = ix->bv.n;
    if (ix->bv.L.pos_bytes == 4)
        hipLaunchKernelGGL((k_row_ctx<uint32_t>), dim3(grid_stride_for(n)), dim3(256), 0, stream, ix->qa, n,
                           ix->d_text, (uint32_t *)ix->d_safull);
    else
        hipLaunchKernelGGL((k_row_ctx<uint64_t>), dim3(grid_stride_for(n)), dim3(256), 0, stream, ix->qa, n,
                           ix->d_text, (uint64_t *)ix->d_safull);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e;
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

}  // namespace fmx

