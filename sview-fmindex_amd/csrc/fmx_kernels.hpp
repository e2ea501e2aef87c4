// fmx_kernels.hpp — the query kernels that depend on the occ layout (P, N,
// V, record size): k_count, k_search, k_emit, the deep-table level step, the
// full-SA walk and the record re-layout.  Instantiated per (P, N) in its own
// translation unit (fmx_layout.hip, one object per layout, built in
// parallel); launched through the LayoutOps table (fmx_internal.hpp).
// Search/walk arithmetic: fmx_device.hpp.
#pragma once

#include <hip/hip_runtime.h>

#include "fmx_device.hpp"
#include "fmx_internal.hpp"

namespace fmx {

static inline unsigned grid_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }
// k_dlut_level: one thread per parent up to 2^24 workgroups, then grid-stride
static inline unsigned grid_dlut(uint64_t np) {
    const uint64_t g = (np + 255) / 256;
    return (unsigned)(g < (1ull << 24) ? (g ? g : 1) : (1ull << 24) - 1);
}
static inline unsigned grid_stride_for(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 65536 ? (g ? g : 1) : 65536);
}

// The per-workgroup tables: encoding table, C array, k-mer multipliers, and
// — when it is small (QueryArgs::kt_lds_bytes) — the blob's k-mer count
// table, copied into LDS at `kt_lds` so that the seed's two reads are LDS
// reads.  Visible after the caller's next barrier.
template <typename P>
__device__ __forceinline__ void stage_tables(const QueryArgs &a, Tables<P> &s, uint8_t *kt_lds) {
    const int t = threadIdx.x;
    const QueryTables &g = *a.tab;
    s.enc[t] = g.enc[t];
    if (t < kMaxSigma) s.dig[t] = g.dig[t];
    if ((uint32_t)t <= a.sigma) s.C[t] = (P)g.C[t];
    if ((uint32_t)t < a.k) s.mult[t] = g.mult[t];
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
    FMX_DYN_LDS(s_pat);  // stage_bytes, then the k-mer table (dynamic)
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
    // settled wave (every pattern of a large text, k_search walked its row):
    // each lane writes its own location, no dealing
    if (__all(mode == kHitOne)) {
        if (cnt == 1 && my_off < cap) out_locs[my_off] = rloc;
        return;
    }
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

// A grouped launch's record (the faithful search, which walks every
// single-row interval: a count of 1 is always kHitOne): a = rloc when b = 1,
// else lo; b = count.  Half of SearchRec<u32> for k_group_tiles and k_emit to
// read; it sits at the start of the batch's SearchRec slot array.
template <typename P>
struct NarrowRec {
    P a, b;
};

template <typename P>
__device__ __forceinline__ uint64_t unpack_narrow(const NarrowRec<P> &r, P &lo, P &rloc, uint64_t &mask,
                                                  uint32_t &mode) {
    const bool one = r.b == P(1);
    mode = one ? kHitOne : kHitRows;
    lo = one ? P(0) : r.a;
    rloc = one ? r.a : P(0);
    mask = 0ull;
    return (uint64_t)r.b;
}

// The locate launch: k_search, (k_scan,) k_emit.
// No workgroup ever waits on another, so nothing depends on the order or
// placement in which workgroups are dispatched (MI355X_MICROARCH.md: HIP
// promises neither; a look-back that assumes in-order dispatch can deadlock
// when launches on several streams share the CUs).  Per batch of a group:
// workspace = [256 B][tile counts: G][tile offsets: G][search records: n].

// This workgroup's batch of a grouped launch (workgroup-uniform): the last
// batch whose first workgroup is at most vt, by binary search.
__device__ __forceinline__ uint32_t group_batch(const LocateGroup &grp, uint32_t vt) {
    uint32_t lo = 0, hi = grp.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (grp.tile_begin[mid] <= vt) lo = mid;
        else hi = mid;
    }
    return lo;
}

// 1. Search this lane's pattern of tile g (staged with the tile's others):
// its count (the optional counts output written), its interval or located
// row (lo, rloc, mask, mode as SearchRec holds them; a lane past the batch:
// count 0, kHitOne).  The caller's next barrier ends every read of s_pat.
template <typename P, int N, int VB, int REC, int VAR>
__device__ __forceinline__ uint64_t search_lane(const QueryArgs &a, const LocateBatch &B, uint32_t g,
                                                const Tables<P> &s, uint8_t *s_pat, uint32_t stage_bytes, P &lo,
                                                P &rloc, uint64_t &mask, uint32_t &mode) {
    const uint8_t *__restrict__ bytes = B.bytes;
    const uint64_t npat = B.npat;
    const bool rev = B.rev != 0;
    uint64_t beg, end, b0, b1;
    const bool staged =
        stage_patterns(s, s_pat, bytes, B.offs, npat, (uint64_t)g * 256u, rev, stage_bytes, B.stride, a.status,
                       beg, end, b0, b1);
    __syncthreads();
    const uint64_t i = (uint64_t)g * 256u + threadIdx.x;
    uint64_t cnt = 0;
    lo = rloc = 0;
    mask = 0;
    mode = kHitOne;
    if (i < npat) {
        const PatView pv = pattern_view(s, s_pat, staged, bytes, beg, end, b0, b1, rev);
        P hi;
        SampledRow<P> smp;
        const uint32_t bad = search<P, N, VB, REC, VAR>(a, s, pv, lo, hi, rloc, mask, mode, &smp);
        if (bad) atomicOr(a.status, bad);
        cnt = (uint64_t)(hi - lo);
        if (B.out_cnt) reinterpret_cast<P *>(B.out_cnt)[i] = hi - lo;
        // one row (most patterns of a large text): its location now, while
        // this lane's chain is live (locate/mod.rs:19-35: from the search's
        // latest sampled row, else by the walk); k_emit then only copies it
        if (mode == kHitRows && cnt == 1) {
            rloc = locate_one<P, N, VB, REC>(a, s.C, lo, smp);
            mode = kHitOne;
        }
        if (mode == kHitOne) lo = 0;
    }
    return cnt;
}

// 1. Search every pattern; its result record, its count; the tile's count.
template <typename P, int N, int VB, int REC, int VAR>
__device__ __forceinline__ void search_tile(const QueryArgs &a, const LocateGroup &grp, const Tables<P> &s,
                                            uint8_t *s_pat, uint64_t *s_scan, uint32_t stage_bytes, uint32_t vt) {
    const uint32_t jb = group_batch(grp, vt);
    const LocateBatch &B = grp.b[jb];
    const uint32_t g = vt - grp.tile_begin[jb];
    const uint64_t G = (B.npat + 255) / 256, i = (uint64_t)g * 256u + threadIdx.x;
    SearchRec<P> *__restrict__ recs = reinterpret_cast<SearchRec<P> *>(B.tiles + 2 * G);
    P lo, rloc;
    uint64_t mask;
    uint32_t mode;
    const uint64_t cnt = search_lane<P, N, VB, REC, VAR>(a, B, g, s, s_pat, stage_bytes, lo, rloc, mask, mode);
    if (i < B.npat) recs[i] = pack_rec<P>(lo, lo + (P)cnt, rloc, mask, mode);
    uint64_t agg;
    block_excl_scan(cnt, &agg, s_scan);  // (its barriers end every read of s_pat)
    if (threadIdx.x == 0) B.tiles[g] = agg;
}

template <typename P, int N, int VB, int REC, int VAR>
__global__ __launch_bounds__(256, VAR == kVarDerivedLong ? 4 : 8) void k_search(const QueryArgs a, const LocateGroup grp,
                                                             uint32_t stage_bytes) {
    __shared__ Tables<P> s;
    FMX_DYN_LDS(s_pat);  // stage_bytes, then the k-mer table (dynamic)
    __shared__ uint64_t s_scan[4];
    stage_tables(a, s, s_pat + stage_bytes);
    search_tile<P, N, VB, REC, VAR>(a, grp, s, s_pat, s_scan, stage_bytes, blockIdx.x);
}

// The same on a resident-sized grid (FMX_SEARCH_PERSISTENT=1, A/B): each
// workgroup stages the tables once, then takes 256-pattern tiles from an
// atomic counter until none is left; no workgroup waits on another.
template <typename P, int N, int VB, int REC, int VAR>
__global__ __launch_bounds__(256, VAR == kVarDerivedLong ? 4 : 8) void k_search_tiles(const QueryArgs a,
                                                                                      const LocateGroup grp,
                                                                                      uint32_t stage_bytes,
                                                                                      uint32_t tiles) {
    __shared__ Tables<P> s;
    FMX_DYN_LDS(s_pat);  // stage_bytes, then the k-mer table (dynamic)
    __shared__ uint64_t s_scan[4];
    __shared__ uint32_t s_tile;
    stage_tables(a, s, s_pat + stage_bytes);
    // Bounded, with a wave-uniform (scalar) exit: an unbounded for (;;) whose
    // only exit was a branch on the LDS value hung on the GPU (the compiler
    // cannot prove that branch uniform around the barriers).
    for (uint32_t it = 0; it < tiles; ++it) {
        if (threadIdx.x == 0) s_tile = atomicAdd(grp.tile_ctr, 1u);
        __syncthreads();  // (also publishes the tables on the first pass)
        const uint32_t vt = __builtin_amdgcn_readfirstlane(s_tile);
        if (vt >= tiles) break;
        // (search_tile's closing barriers order every read of s_tile before the next write)
        search_tile<P, N, VB, REC, VAR>(a, grp, s, s_pat, s_scan, stage_bytes, vt);
    }
}

// ------------------------------------------- k_locate (search + emit, fused)
// A launch in launch order as ONE kernel: each workgroup searches its tile
// (search_lane, as k_search), publishes the tile's count, sums the counts of
// its batch's earlier tiles as they are published, and writes its patterns'
// output offsets and locations (emit_locations, as k_emit) — no search
// records, no second kernel (a lone 100k batch: k_search 55.6 + k_emit
// 13.3 us, profiles/r5/r5i_*).  Unlike every other kernel here, a workgroup
// waits on others: on the earlier tiles of its own batch.  Which tile a
// workgroup answers is its TICKET (take_ticket: the number of the batch's
// workgroups that started before it, as rocPRIM's ordered block id), not its
// index: the XCDs dispatch a launch's workgroups independently, and beside
// another stream's launch a lower-index workgroup could wait for a slot held
// by waiters.  A ticket-ordered workgroup waits only on
// workgroups that are already running and publish before they wait, so every
// wait ends; it is bounded all the same (late_ticks of the 100 MHz wall
// clock, then kStatusLate: FMX_E_DEVICE, never a hang), and only launches
// whose patterns are short enough that a tile's search is bounded take this
// path (fmx_query.hip, launch_split).
// The hand-off (MI355X_MICROARCH.md § visibility, the first row of the
// sc1 table; cdna_hip_programming.md Guideline 16): one lane stores the
// tile's count (an 8-B agent-scope relaxed store: sc1, write-through), waits
// for it to leave (vmcnt(0)), then stores the tag word; a reader polls the
// tag with agent-scope relaxed loads (sc1: past its CU's L1) and loads the
// count the same way once it matched.  The tag is the launch's own 64-bit
// value (a process-wide launch counter through a bijective mix with a random
// nonce), so no word needs zeroing before the launch and no stale word of an
// earlier launch on the workspace can match; launches under stream capture
// (a replayed graph would reuse the tag) take the split path.
// Per batch workspace: [header][tile counts: G][tags: G] (the split path's
// tile counts / offsets).
#ifndef FMX_HANDOFF
#define FMX_GLOBAL_AS __attribute__((address_space(1)))
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load((const FMX_GLOBAL_AS uint64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store((FMX_GLOBAL_AS uint64_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent32(uint32_t *p, uint32_t v) {
    __hip_atomic_store((FMX_GLOBAL_AS uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every store of this wave has left it (inline asm: the compiler cannot drop it, Guideline 16 / the
// compiler hazard of MI355X_MICROARCH.md § visibility)
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void poll_pause() { __builtin_amdgcn_s_sleep(2); }
// no load moves above the poll that matched (no instruction)
__device__ __forceinline__ void after_poll() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); }
__device__ __forceinline__ uint64_t wall_ticks() { return wall_clock64(); }
#endif

// This workgroup's tile in batch jb: with grp.tickets (one 32-bit counter per
// batch of the launch, zero before it: fmx_index::d_tickets, per status slot)
// thread 0 takes the batch's next ticket; without, the tile is the
// workgroup's index.  Read after the caller's next barrier (claim_tile).
__device__ __forceinline__ void take_ticket(const LocateGroup &grp, uint32_t jb, uint32_t *s_tk) {
    if (threadIdx.x == 0) *s_tk = grp.tickets ? atomicAdd(grp.tickets + jb, 1u) : blockIdx.x - grp.tile_begin[jb];
}
// After that barrier: the tile (workgroup-uniform), or G when the ticket is
// out of range (a counter not zero at the launch: never expected; the
// workgroup then answers nothing and the batch's waits end late, FMX_E_DEVICE,
// and the host zeroes the slot's counters, read_status).  The workgroup that
// took the batch's last ticket puts the counter back to zero: every other
// ticket of the launch was taken before it.
__device__ __forceinline__ uint32_t claim_tile(const LocateGroup &grp, uint32_t jb, uint64_t G, const uint32_t *s_tk,
                                               uint32_t *status) {
    const uint32_t g = __builtin_amdgcn_readfirstlane(*s_tk);
    if (g >= G) {
        if (threadIdx.x == 0) atomicOr(status, kStatusLate);
        return (uint32_t)G;
    }
    if (grp.tickets && g + 1 == G && threadIdx.x == 0) st_agent32(grp.tickets + jb, 0u);
    return g;
}

// Tile g's base offset in its batch (of G tiles) from the hand-off: publish
// this tile's count agg (the last tile's is read by no one), then sum the
// earlier tiles' counts as they are published, lane t taking tiles t, t + 256,
// ... below g.  Ends with a barrier (s_part).
__device__ __forceinline__ uint64_t chain_base(const LocateBatch &B, uint64_t G, uint32_t g, uint64_t agg,
                                               uint64_t tag, uint64_t late_ticks, uint32_t *status,
                                               uint64_t *s_part /*[4]*/) {
    uint64_t *cnts = B.tiles, *tags = B.tiles + G;
    if (threadIdx.x == 0 && g + 1 < G) {
        st_agent(cnts + g, agg);
        drain_stores();
        st_agent(tags + g, tag);
    }
    uint64_t part = 0;
    uint32_t late = 0;
    if (g) {
        const uint64_t t_end = wall_ticks() + late_ticks;
        for (uint64_t t = threadIdx.x; t < g; t += 256) {
            while (ld_agent(tags + t) != tag) {
                if (wall_ticks() > t_end) {
                    late = 1;
                    break;
                }
                poll_pause();
            }
            after_poll();
            part += ld_agent(cnts + t);
        }
    }
    if (late) atomicOr(status, kStatusLate);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) part += __shfl_xor(part, d);
    if (lane == 0) s_part[wv] = part;
    __syncthreads();
    return s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

template <typename P, int N, int VB, int REC, int VAR>
__global__ __launch_bounds__(256, VAR == kVarDerivedLong ? 4 : 8) void k_locate(const QueryArgs a, const LocateGroup grp,
                                                                               uint32_t stage_bytes, uint64_t tag,
                                                                               uint64_t late_ticks) {
    __shared__ Tables<P> s;
    FMX_DYN_LDS(s_pat);  // stage_bytes, then the k-mer table (dynamic)
    __shared__ uint64_t s_scan[4], s_part[4];
    __shared__ uint32_t s_tk;
    const uint32_t jb = group_batch(grp, blockIdx.x);
    take_ticket(grp, jb, &s_tk);
    stage_tables(a, s, s_pat + stage_bytes);
    __syncthreads();
    const LocateBatch &B = grp.b[jb];
    const uint64_t npat = B.npat, G = (npat + 255) / 256;
    const uint32_t g = claim_tile(grp, jb, G, &s_tk, a.status);
    if (g >= G) return;  // (workgroup-uniform)
    P lo, rloc;
    uint64_t mask;
    uint32_t mode;
    const uint64_t cnt = search_lane<P, N, VB, REC, VAR>(a, B, g, s, s_pat, stage_bytes, lo, rloc, mask, mode);
    uint64_t agg;
    const uint64_t excl = block_excl_scan(cnt, &agg, s_scan);  // (its barriers end every read of s_pat)
    const uint64_t base = chain_base(B, G, g, agg, tag, late_ticks, a.status, s_part);
    const uint64_t my_off = base + excl, i = (uint64_t)g * 256u + threadIdx.x;
    if (g + 1 == G && threadIdx.x == 0) {
        B.loc_off[npat] = base + agg;
        *B.needed = base + agg;
    }
    if (i < npat) B.loc_off[i] = my_off;
    emit_locations<P, N, VB, REC>(a, s.C, my_off, cnt, lo, rloc, mask, mode, B.cap, reinterpret_cast<P *>(B.out_locs));
}

// ---------------------------------------------------------- grouped launches
// (fmx_internal.hpp, kWsHeader) k_group_key<count> (one workgroup per chunk
// of kGroupChunkTiles tiles), k_group_scan and k_group_key<place> deal the
// launch's patterns out in the order of their keys, each carrying its packed
// symbols; k_search_grouped searches them in that order and writes each
// result at the pattern's own index; k_group_tiles sums each tile's counts
// for k_emit.  No workgroup waits on another.

using U4 = uint32_t __attribute__((ext_vector_type(4)));

// A batch's share of the launch's sorted order ({symbols: 96 bits, pattern
// id} per position), after its search records, 16-B aligned (24-B records
// of u64 positions leave an odd count 8-B aligned).
__device__ __forceinline__ U4 *group_sorted(const LocateBatch &B, uint32_t rec_bytes) {
    const uint64_t n = B.npat, G = (n + 255) / 256;
    return reinterpret_cast<U4 *>(reinterpret_cast<uint8_t *>(B.tiles + 2 * G) + ((n * rec_bytes + 15) & ~15ull));
}

// This workgroup's batch of a key launch (workgroup-uniform, binary search).
__device__ __forceinline__ uint32_t group_chunk_batch(const LocateGroup &grp, uint32_t c) {
    uint32_t lo = 0, hi = grp.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (grp.chunk_begin[mid] <= c) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The last index j < n with key[j] <= x (key ascending, key[0] <= x): a
// per-lane binary search over an LDS table.
template <typename T, typename K>
__device__ __forceinline__ uint32_t lds_upper(const T *tab, uint32_t n, K x) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tab[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Per chunk of kGroupChunkTiles tiles (1,024 threads, four patterns each,
// fixed length m <= 4 W - 3 bytes), each pattern's bytes as W aligned words
// straight into registers (consecutive patterns lie back to back, so a wave's
// loads are contiguous), decoded byte by byte at compile-time register
// indices into its key — its last gkey_len symbols as digits over the
// symbols that occur in the text, the last symbol most significant (the
// order in which the backward search reads them) — and, when placing, its
// symbols packed gbits each (a symbol >= sigma kept as sigma: the search
// rejects it the same way).  An LDS histogram gives the chunk's count per
// key and each pattern's rank among them.
//   PLACE = false (1. count): the chunk's counts are added to the launch's
//     (gcount); the offsets are checked against the length hint here (the
//     grouped search never reads them).
//   PLACE = true (3. place, after k_group_scan turned the counts into each
//     key's first position): one returning add per key reserves the chunk's
//     positions, and each pattern's packed record, tagged with its pattern id
//     (tile_begin * 256 + index), is written at its sorted position (chunk
//     base + rank) — the sorted order is held by the batches one after
//     another.
//   RAW (grp.graw: patterns too long to pack, e.g. C5's 150 bp): only the W
//     words holding the key's symbols are read (the pattern's last gkey_len
//     symbols: its last bytes, or its first for reversed input), and the
//     record carries the pattern id alone — k_search_grouped reads the
//     pattern's bytes itself.  The count pass of every grouped launch runs
//     this way (it needs the key alone).
template <int W, bool PLACE, bool RAW = false>
__global__ __launch_bounds__(1024, W <= 8 ? 2 : 1) void k_group_key(const QueryArgs a, const LocateGroup grp, uint32_t rec_bytes) {
    constexpr uint32_t T = 1024, PPT = kGroupChunkTiles * 256 / T;  // patterns per thread
    __shared__ uint8_t s_enc[256];
    __shared__ uint8_t s_dig[kMaxSigma];
    __shared__ uint32_t s_pw[32];
    __shared__ uint32_t hist[kGroupBins];
    // (place) the launch's batches (GroupTab): sorted positions before each (32-bit: a launch's pattern ids
    // are), and where each holds its share of the sorted order
    __shared__ uint32_t s_first[PLACE ? kMaxMega : 1];
    __shared__ U4 *s_sorted[PLACE ? kMaxMega : 1];
    const uint32_t t = threadIdx.x;
    if constexpr (PLACE)
        for (uint32_t j = t; j < grp.gn; j += T) {  // (the compact copies: 96 lines per workgroup, not 320)
            s_first[j] = grp.gtab->first32[j];
            s_sorted[j] = reinterpret_cast<U4 *>(grp.gtab->sorted[j]);
        }
    if (t < 256) s_enc[t] = a.tab->enc[t];
    if (t < (uint32_t)kMaxSigma) s_dig[t] = a.tab->dig[t] == kNoDigit ? 0 : a.tab->dig[t];  // (absent: occurs nowhere)
    if (t == 0) {
        uint32_t w = 1;
        for (uint32_t e = 0; e < 32; ++e) {
            s_pw[e] = w;  // base^e while it fits the key
            w = e + 1 < grp.gkey_len ? w * grp.gkey_base : w;
        }
    }
    for (uint32_t x = t; x < kGroupBins; x += T) hist[x] = 0;
    __syncthreads();
    // the count pass takes kCountChunks chunks per workgroup (one set of
    // global adds for all of them; measured no faster than one, r4w: the
    // atomics do not bound it), the place pass one
    constexpr uint32_t CPW = PLACE ? 1u : kCountChunks;
    // the chunks' slot (kGroupSlots): the place pass's chunk is its workgroup; the count pass's
    // workgroup w takes chunks of one slot, w mod S + S (CPW (w div S) + r), r < CPW
    constexpr uint32_t S = kGroupSlots;
    const uint32_t slot = blockIdx.x % S;
    uint32_t key_r[PPT], rank_r[PPT];
    U4 rec_r[PLACE ? PPT : 1];
    uint64_t pfirst = 0, pn = 0;  // (the place pass's one chunk, after the loop)
#pragma unroll
    for (uint32_t r = 0; r < CPW; ++r) {
    const uint32_t c = PLACE ? blockIdx.x : (blockIdx.x / S) * (S * CPW) + r * S + slot;
    if constexpr (!PLACE) {
        const uint32_t nchunks = grp.chunk_begin[grp.n - 1] +
                                 (uint32_t)(((grp.b[grp.n - 1].npat + 255) / 256 + kGroupChunkTiles - 1) /
                                            kGroupChunkTiles);
        if (c >= nchunks) break;  // (workgroup-uniform)
    }
    const uint32_t jb = group_chunk_batch(grp, c);
    const LocateBatch &B = grp.b[jb];
    const uint64_t n = B.npat, first = (uint64_t)(c - grp.chunk_begin[jb]) * kGroupChunkTiles * 256u;
    const uint32_t m = B.stride, bits = grp.gbits, sym_max = a.sigma, L = grp.gkey_len;
    const bool rev = B.rev != 0;
    if constexpr (PLACE) {
        pfirst = first;
        pn = n;
    }
    if (!PLACE && first == 0 && t == 0 && B.offs[0] != 0) atomicOr(a.status, kStatusStride);
    // G patterns' words in flight at once (all of a thread's when they are short)
    constexpr uint32_t G = W <= 8 ? PPT : 1;
#pragma unroll
    for (uint32_t p0 = 0; p0 < PPT; p0 += G) {
    uint32_t x[G][W], lead[G];
    uint64_t chk[G];
    // the bytes read: the whole pattern, or (RAW) its key's: the last kl
    // input bytes, or the first kl of a reversed one
    const uint32_t kl = L < m ? L : m, span = RAW ? kl : m;
    const uint32_t skip = RAW && !rev ? m - kl : 0u;  // input bytes before the span
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) {
        const uint64_t i = first + (p0 + g) * T + t;
        const uint64_t beg = i * m + skip, a0 = beg & ~3ull;
        lead[g] = (uint32_t)(beg - a0);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(B.bytes + a0);
        const bool ok = i < n;
#pragma unroll
        for (uint32_t q = 0; q < W; ++q) x[g][q] = ok && 4 * q < lead[g] + span ? src[q] : 0u;
        chk[g] = ok && !PLACE ? B.offs[i + 1] : 0;
    }
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t p = p0 + g;
        const uint64_t i = first + p * T + t;
        key_r[p] = rank_r[p] = 0;
        if (i >= n) continue;
        if (!PLACE && chk[g] != (i + 1) * m) atomicOr(a.status, kStatusStride);
        uint64_t lo = 0, hi = 0;
        uint32_t key = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4 * W; ++b) {
            const uint32_t sp = b - lead[g];  // byte of the span (wraps below 0: skipped)
            if (sp >= span) continue;
            const uint32_t pos = sp + skip;  // input byte index
            const uint32_t j = rev ? m - 1 - pos : pos;  // pattern position
            uint32_t cj = s_enc[(x[g][b >> 2] >> (8 * (b & 3))) & 0xffu];
            const uint32_t back = m - 1 - j;  // 0 = the last symbol
            if (back < L) key += (cj < (uint32_t)kMaxSigma ? s_dig[cj] : 0u) * s_pw[L - 1 - back];
            if constexpr (PLACE && !RAW) {
                cj = cj < sym_max ? cj : sym_max;
                const uint32_t at = j * bits;
                if (at < 64) {
                    lo |= (uint64_t)cj << at;
                    if (at + bits > 64) hi |= (uint64_t)cj >> (64 - at);
                } else {
                    hi |= (uint64_t)cj << (at - 64);
                }
            }
        }
        key_r[p] = key;
        if constexpr (PLACE) {
            rank_r[p] = atomicAdd(&hist[key], 1u);
            rec_r[p].x = (uint32_t)lo;
            rec_r[p].y = (uint32_t)(lo >> 32);
            rec_r[p].z = (uint32_t)hi;
            rec_r[p].w = (uint32_t)((grp.vbase + (uint64_t)grp.tile_begin[jb]) * 256ull + i);
        } else {
            atomicAdd(&hist[key], 1u);
        }
    }
    }
    }
    __syncthreads();
    constexpr uint32_t per = kGroupBins / T;
    if constexpr (!PLACE) {
        // the chunk's counts into the launch's
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) {
            const uint32_t h = hist[u * T + t];
            if (h) atomicAdd(grp.gcount + (u * T + t) * S + slot, h);
        }
        return;
    } else {
        // every returning add of a thread in flight at once
        uint32_t h[per], base[per];
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) h[u] = hist[u * T + t];
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) base[u] = h[u] ? atomicAdd(grp.gcount + (u * T + t) * S + slot, h[u]) : 0u;
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) hist[u * T + t] = base[u];  // the chunk's first position per key
        __syncthreads();
#pragma unroll
        for (uint32_t p = 0; p < PPT; ++p) {
            const uint64_t i = pfirst + p * T + t;
            if (i >= pn) continue;
            const uint64_t sp = (uint64_t)hist[key_r[p]] + rank_r[p];
            if (sp >= grp.gtotal) {  // (counters not zero at entry: never write outside the sorted order)
                atomicOr(a.status, kStatusGroup);
                continue;
            }
            const uint32_t js = lds_upper(s_first, grp.gn, (uint32_t)sp);  // (the batch holding position sp)
            s_sorted[js][sp - s_first[js]] = rec_r[p];
        }
    }
}

// 3b. Refine (packed records): the run of each key in the sorted order —
// the patterns sharing their last gkey_len symbols — re-sorted by their next
// gkey_len symbols, the nearest one most significant (one workgroup per key;
// a run longer than kRefineSeg records is sorted in independent segments).
// Patterns sharing up to 2 gkey_len last symbols (C2: 12) are then searched
// side by side, so their LF steps below the key read the same records in
// the same wave instructions or from L2.  Opt-in (FMX_GROUP_REFINE_MIN): on
// C2 at 25.6 M patterns per launch it takes 462 us and saves 352 us of
// k_search_grouped (the bench's --presorted +31 % comes mostly
// from result writes in pattern order, which no internal order can give).  An LDS counting sort; in place: every record of a
// segment is in registers before any is written back.  After k_group_key
// <place> the key counters hold each run's end (run k = [cnt[k-1], cnt[k])).
// Workgroup b takes keys b, b + grid, ... (a smaller launch, fewer workgroups).
constexpr uint32_t kRefinePer = 4;  // records per thread and segment
constexpr uint32_t kRefineSeg = 1024 * kRefinePer;

// symbol j of a packed record (bits each)
__device__ __forceinline__ uint32_t packed_sym(const U4 &e, uint32_t j, uint32_t bits) {
    const uint64_t lo = (uint64_t)e.x | ((uint64_t)e.y << 32), hi = e.z;
    const uint32_t at = j * bits;
    uint64_t x;
    if (at < 64) {
        x = lo >> at;
        if (at + bits > 64) x |= hi << (64 - at);
    } else {
        x = hi >> (at - 64);
    }
    return (uint32_t)(x & ((1u << bits) - 1u));
}

template <int UNUSED = 0>
__global__ __launch_bounds__(1024) void k_group_refine(const QueryArgs a, const LocateGroup grp, uint32_t rec_bytes) {
    constexpr uint32_t T = 1024, per = kGroupBins / T, NW = T / 64;
    __shared__ uint32_t hist[kGroupBins];
    __shared__ uint8_t s_dig[kMaxSigma + 1];
    __shared__ uint32_t s_pw[32];
    __shared__ uint32_t s_wsum[NW];
    const uint32_t t = threadIdx.x;
    const uint64_t total = grp.gtotal;
    const GroupTab &gt = *grp.gtab;  // (the launch's batches: a sorted position's or a pattern id's batch)
    const uint32_t sym_max = a.sigma, L = grp.gkey_len, bits = grp.gbits;
    if (t <= (uint32_t)kMaxSigma) s_dig[t] = t < sym_max && a.tab->dig[t] != kNoDigit ? a.tab->dig[t] : 0;
    if (t == 0) {
        uint32_t w = 1;
        for (uint32_t e = 0; e < 32; ++e) {
            s_pw[e] = w;
            w = e + 1 < L ? w * grp.gkey_base : w;
        }
    }
    __syncthreads();
    for (uint32_t k = blockIdx.x; k < kGroupBins; k += gridDim.x) {
    // (key k's run: its slots' sub-runs, one after another)
    uint64_t end = grp.gcount[k * kGroupSlots + kGroupSlots - 1], beg = k ? grp.gcount[k * kGroupSlots - 1] : 0;
    end = end < total ? end : total;
    beg = beg < end ? beg : end;
    if (end - beg < 2) continue;  // (workgroup-uniform)
    for (uint64_t s0 = beg; s0 < end; s0 += kRefineSeg) {
        const uint64_t sn = end - s0 < kRefineSeg ? end - s0 : kRefineSeg;
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) hist[u * T + t] = 0;
        __syncthreads();
        U4 rec[kRefinePer];
        uint32_t key[kRefinePer], rank[kRefinePer];
#pragma unroll
        for (uint32_t u = 0; u < kRefinePer; ++u) {
            const uint64_t p = s0 + u * T + t;
            key[u] = rank[u] = 0;
            if (p >= s0 + sn) continue;
            const uint32_t js = lds_upper(gt.first, grp.gn, p);
            rec[u] = reinterpret_cast<const U4 *>(gt.desc[js].sorted)[p - gt.first[js]];
        }
#pragma unroll
        for (uint32_t u = 0; u < kRefinePer; ++u) {
            const uint64_t p = s0 + u * T + t;
            if (p >= s0 + sn) continue;
            const uint32_t m = gt.desc[lds_upper(gt.vfirst, grp.gn, rec[u].w)].stride;
            uint32_t k2 = 0;
            for (uint32_t d = 0; d < L; ++d) {
                const uint32_t back = L + d;  // 0 = the pattern's last symbol
                const uint32_t c = back < m ? packed_sym(rec[u], m - 1 - back, bits) : sym_max;
                k2 += (uint32_t)s_dig[c] * s_pw[L - 1 - d];
            }
            key[u] = k2;
            rank[u] = atomicAdd(&hist[k2], 1u);
        }
        __syncthreads();
        // exclusive scan of the histogram: thread t owns entries [per t, per t + per)
        uint32_t v[per], sum = 0;
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) {
            v[u] = hist[per * t + u];
            sum += v[u];
        }
        const uint32_t lane = t & 63, wv = t >> 6;
        uint32_t x = sum;
#pragma unroll
        for (uint32_t dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(x, dd);
            if (lane >= dd) x += y;
        }
        if (lane == 63) s_wsum[wv] = x;
        __syncthreads();
        uint32_t run = x - sum;
        for (uint32_t w = 0; w < wv; ++w) run += s_wsum[w];
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) {
            hist[per * t + u] = run;
            run += v[u];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < kRefinePer; ++u) {
            const uint64_t p = s0 + u * T + t;
            if (p >= s0 + sn) continue;
            const uint64_t np = s0 + hist[key[u]] + rank[u];
            const uint32_t js = lds_upper(gt.first, grp.gn, np);
            reinterpret_cast<U4 *>(gt.desc[js].sorted)[np - gt.first[js]] = rec[u];
        }
        __syncthreads();  // (the next segment's histogram)
    }
    }
}


// 3. Search the launch's patterns in key order: workgroup b takes sorted
// positions [256 K b, 256 K (b + 1)), K = 1 or 2 patterns per lane (lane t:
// positions 256 K b + t + 256 j) — their records are read in order, the
// symbols unpacked into cap bytes of LDS per pattern — searches (K = 2: both
// chains in lockstep, search_pair), walks a single row, and leaves each
// record at its pattern's own index.
template <typename P>
__device__ __forceinline__ void grouped_unpack(const U4 &e, uint32_t m, uint32_t bits, uint8_t *dst) {
    const uint32_t msk = (1u << bits) - 1u;
    const uint64_t lo = (uint64_t)e.x | ((uint64_t)e.y << 32), hi = e.z;
    for (uint32_t j = 0; j < m; ++j) {
        const uint32_t at = j * bits;
        uint64_t x;
        if (at < 64) {
            x = lo >> at;
            if (at + bits > 64) x |= hi << (64 - at);
        } else {
            x = hi >> (at - 64);
        }
        dst[j] = (uint8_t)(x & msk);
    }
}

// The LDS before the k-mer table: each lane's cap bytes of symbols, or the
// in-workgroup sort's room when that is larger (it is done with before the
// symbols are unpacked).
__host__ __device__ constexpr uint32_t grouped_pat_bytes(uint32_t k, uint32_t cap, uint32_t wsort) {
    return 256u * k * cap > kWsortBytes || !wsort ? 256u * k * cap : kWsortBytes;
}

// opts bit 0 (kGroupedXcd): the XCD deal below; bits 8-15 = wsort: a full
// workgroup of packed records (K = 1) first sorts its 256 patterns by their
// next wsort symbols after the first opts >> 16 last symbols — those the
// sorted order is already ordered by: the key's, or with the refine pass
// twice as many (digits over the key's base, the nearest
// symbol most significant; base^wsort <= 256) — an LDS counting sort — so
// that a wave's lanes share up to gkey_len + 1 or 2 last symbols and the LF
// steps just below the key read the same lines in the same wave instruction
// (one request each) instead of up to 64 different ones.  Which lane answers
// which pattern changes nothing in the results (each is written at its own
// index).
template <typename P, int N, int VB, int REC, int K>
__global__ __launch_bounds__(256, K == 2 ? 6 : 8) void k_search_grouped(const QueryArgs a, const LocateGroup grp,
                                                           uint64_t total, uint32_t cap, uint32_t opts) {
    static_assert(K == 1 || K == 2, "one or two patterns per lane");
    __shared__ Tables<P> s;
    __shared__ uint8_t s_dig[kMaxSigma + 1];  // (wsort) symbol -> digit; sigma (past the pattern's start) -> 0
    __shared__ uint64_t s_wscan[4];
    // the launch's batches (GroupTab), for the lanes' binary searches: sorted positions and pattern ids
    // before each (32-bit: a launch's are), and each one's pattern length
    __shared__ uint32_t s_first[kMaxMega], s_vfirst[kMaxMega];
    __shared__ uint16_t s_stride[kMaxMega];
    const uint32_t wsort = K == 1 && !grp.graw ? (opts >> 8) & 0xffu : 0u, xcd = opts & kGroupedXcd;
    const uint32_t wskip = opts >> 16;
    FMX_DYN_LDS(s_pat);  // 256 K x cap B of symbols (cap >= every batch's length), then the k-mer table
    stage_tables(a, s, s_pat + grouped_pat_bytes(K, cap, wsort));
    if (threadIdx.x <= (uint32_t)kMaxSigma)
        s_dig[threadIdx.x] =
            threadIdx.x < a.sigma && a.tab->dig[threadIdx.x] != kNoDigit ? a.tab->dig[threadIdx.x] : 0;
    const GroupTab &gt = *grp.gtab;
    for (uint32_t j = threadIdx.x; j < grp.gn; j += 256) {  // (the compact copies: 10 B per batch)
        s_first[j] = gt.first32[j];
        s_vfirst[j] = gt.vfirst[j];
        s_stride[j] = gt.stride16[j];
    }
    __syncthreads();
    // xcd: workgroup b takes chunk start(b % 8) + b / 8, so that (under the
    // round-robin placement of workgroups over the 8 XCDs, which only speed
    // depends on) each XCD's L2 serves one eighth of the key order
    uint32_t chunk = blockIdx.x;
    if (xcd) {
        const uint32_t q = gridDim.x / 8, rem = gridDim.x % 8, x = blockIdx.x % 8;
        chunk = x * q + (x < rem ? x : rem) + blockIdx.x / 8;
    }
    PatView pv[K];
    bool live[K];
    uint64_t pi[K];
    uint8_t *recp[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const uint64_t sp = (uint64_t)chunk * (256u * K) + (uint32_t)q * 256u + threadIdx.x;
        live[q] = sp < total;
        pi[q] = 0;
        recp[q] = nullptr;
        uint8_t *dst = s_pat + ((uint32_t)q * 256u + threadIdx.x) * cap;
        pv[q].m = 0;
        pv[q].rev = false;
        pv[q].raw = nullptr;
        pv[q].enc = s.enc;
        pv[q].sym = dst;
        if (!live[q]) continue;
        const uint32_t js = lds_upper(s_first, grp.gn, (uint32_t)sp);
        U4 e = reinterpret_cast<const U4 *>(gt.desc[js].sorted)[sp - s_first[js]];
        if (K == 1 && wsort && (uint64_t)chunk * 256u + 256u <= total) {  // (workgroup-uniform: all lanes live)
            uint32_t *hist = reinterpret_cast<uint32_t *>(s_pat);
            U4 *stage = reinterpret_cast<U4 *>(s_pat + 1024);
            const uint32_t t = threadIdx.x, base = grp.gkey_base;
            const uint32_t m = s_stride[lds_upper(s_vfirst, grp.gn, e.w)];
            uint32_t k2 = 0;
            for (uint32_t d = 0; d < wsort; ++d) {
                const uint32_t back = wskip + d;  // 0 = the pattern's last symbol
                k2 = k2 * base + s_dig[back < m ? packed_sym(e, m - 1 - back, grp.gbits) : a.sigma];
            }
            hist[t] = 0;
            __syncthreads();
            const uint32_t rank = atomicAdd(&hist[k2], 1u);
            __syncthreads();
            uint64_t agg;
            const uint32_t before = (uint32_t)block_excl_scan(hist[t], &agg, s_wscan);
            hist[t] = before;  // (each thread its own counter; read after the next barrier)
            __syncthreads();
            stage[hist[k2] + rank] = e;
            __syncthreads();
            e = stage[t];
            __syncthreads();  // (the stage is s_pat: every lane has its record before any unpacks)
        }
        const uint32_t v = e.w;
        const uint32_t jb = lds_upper(s_vfirst, grp.gn, v);
        const GroupDesc &dj = gt.desc[jb];  // (recs: written at the end; bytes, rev: id-only records)
        recp[q] = dj.recs;
        pi[q] = (uint64_t)(v - s_vfirst[jb]);
        pv[q].m = s_stride[jb];
        if (grp.graw) {
            const uint32_t m = s_stride[jb];
            const uint8_t *src = dj.bytes + pi[q] * m;
            if (cap >= m) {
                // the pattern's bytes (input order) into its cap bytes of LDS,
                // encoded, in pattern order: aligned 16-B vectors, four in
                // flight per round trip (grp.graw with m <= kGroupRawStage)
                const uint64_t a = reinterpret_cast<uint64_t>(src), a0 = a & ~15ull;
                const uint32_t lead = (uint32_t)(a - a0), nv = (lead + m + 15) >> 4;
                const bool rv = dj.rev != 0;
                const U4 *vp = reinterpret_cast<const U4 *>(a0);
                for (uint32_t v0 = 0; v0 < nv; v0 += 4) {
                    U4 x[4];
#pragma unroll
                    for (uint32_t u = 0; u < 4; ++u)
                        if (v0 + u < nv) x[u] = vp[v0 + u];
#pragma unroll
                    for (uint32_t u = 0; u < 4; ++u) {
                        if (v0 + u >= nv) continue;
#pragma unroll
                        for (uint32_t w = 0; w < 16; ++w) {
                            const uint32_t pos = 16u * (v0 + u) + w - lead;  // (wraps below 0: skipped)
                            if (pos < m) dst[rv ? m - 1 - pos : pos] = s.enc[(x[u][w >> 2] >> (8 * (w & 3))) & 0xffu];
                        }
                    }
                }
            } else {  // longer than the LDS room: the bytes from HBM, encoded on each access
                pv[q].raw = src;
                pv[q].rev = dj.rev != 0;
                pv[q].sym = nullptr;
            }
        } else {
            grouped_unpack<P>(e, s_stride[jb], grp.gbits, dst);
        }
    }
    P lo_r[K], hi_r[K], rloc[K];
    uint64_t mask[K];
    uint32_t mode[K];
    if constexpr (K == 1) {
        if (!live[0]) return;
        SampledRow<P> smp;
        const uint32_t bad = search<P, N, VB, REC, kVarFaithful>(a, s, pv[0], lo_r[0], hi_r[0], rloc[0], mask[0],
                                                                  mode[0], &smp);
        if (bad) atomicOr(a.status, bad);
        if (mode[0] == kHitRows && hi_r[0] - lo_r[0] == P(1)) {
            rloc[0] = locate_one<P, N, VB, REC>(a, s.C, lo_r[0], smp);
            mode[0] = kHitOne;
        }
    } else {
        uint32_t bad[2];
        search_pair<P, N, VB, REC>(a, s, pv, live, lo_r, hi_r, bad);
        if (bad[0] | bad[1]) atomicOr(a.status, bad[0] | bad[1]);
        bool one[2];
        P row[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            mode[q] = kHitRows;
            mask[q] = 0;
            rloc[q] = 0;
            one[q] = live[q] && hi_r[q] - lo_r[q] == P(1);
            row[q] = lo_r[q];
        }
        if (one[0] || one[1]) {
            P loc[2];
            walk_pair<P, N, VB, REC>(a, s.C, row, one, loc);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (one[q]) {
                    rloc[q] = loc[q];
                    mode[q] = kHitOne;
                }
        }
    }
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (live[q])
            reinterpret_cast<NarrowRec<P> *>(recp[q])[pi[q]] =
                NarrowRec<P>{mode[q] == kHitOne ? rloc[q] : lo_r[q], (P)(hi_r[q] - lo_r[q])};
}

// This workgroup's batch of a k_group_tiles launch (workgroup-uniform).
__device__ __forceinline__ uint32_t emit_batch(const LocateGroup &grp, uint32_t w) {
    uint32_t lo = 0, hi = grp.n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (grp.emit_begin[mid] <= w) lo = mid;
        else hi = mid;
    }
    return lo;
}

// 3. Output offsets (tile offset + in-tile scan) and every location, rows
// dealt across each wave's lanes (emit_locations).  Workgroup w takes tile
// w - tile_begin of its batch (E = 1 tile per workgroup; the code handles E
// tiles, lane t loading its pattern of each first).
// fold bit 0: batches of at most kFoldTiles tiles need no k_scan: each
// workgroup sums the counts of the tiles before its first (all final:
// k_search is done), then carries the base across its own, and the last tile
// writes the batch total.  Bit 1: the records are NarrowRec (a grouped
// launch).

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_emit(const QueryArgs a, const LocateGroup grp, uint32_t flags) {
    constexpr uint32_t E = 1;
    const uint32_t fold = flags & 1u, narrow = flags & 2u;
    __shared__ P sC[kMaxSigma + 1];
    __shared__ uint64_t s_scan[E][4], s_part[4];
    if (threadIdx.x <= a.sigma) sC[threadIdx.x] = (P)a.tab->C[threadIdx.x];
    const uint32_t jb = group_batch(grp, blockIdx.x);
    const LocateBatch &B = grp.b[jb];
    const uint64_t npat = B.npat, G = (npat + 255) / 256;
    const uint64_t g0 = (uint64_t)(blockIdx.x - grp.tile_begin[jb]) * E;
    const SearchRec<P> *__restrict__ recs = reinterpret_cast<const SearchRec<P> *>(B.tiles + 2 * G);
    P lo[E], rloc[E];
    uint64_t mask[E], cnt[E];
    uint32_t mode[E];
#pragma unroll
    for (uint32_t k = 0; k < E; ++k) {
        const uint64_t i = (g0 + k) * 256u + threadIdx.x;
        lo[k] = rloc[k] = 0;
        mask[k] = cnt[k] = 0;
        mode[k] = kHitOne;
        if (i < npat)
            cnt[k] = narrow ? unpack_narrow<P>(reinterpret_cast<const NarrowRec<P> *>(recs)[i], lo[k], rloc[k],
                                               mask[k], mode[k])
                            : unpack_rec<P>(recs[i], lo[k], rloc[k], mask[k], mode[k]);
    }
    // the first tile's base offset (fold: the earlier tiles' counts, summed
    // here) and the exclusive scans of the counts, one barrier for all
    uint64_t part = 0;
    if (fold)
        for (uint64_t t = threadIdx.x; t < g0; t += 256) part += B.tiles[t];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t x[E];
#pragma unroll
    for (uint32_t k = 0; k < E; ++k) x[k] = cnt[k];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (uint32_t k = 0; k < E; ++k) {
            const uint64_t y = __shfl_up(x[k], d);
            if (lane >= d) x[k] += y;
        }
        part += __shfl_xor(part, d);
    }
    if (lane == 63) {
#pragma unroll
        for (uint32_t k = 0; k < E; ++k) s_scan[k][wv] = x[k];
        s_part[wv] = part;
    }
    __syncthreads();  // (also publishes sC)
    uint64_t base = fold ? s_part[0] + s_part[1] + s_part[2] + s_part[3] : 0;
    if (grp.tile_ctr && blockIdx.x == 0 && threadIdx.x == 0) *grp.tile_ctr = 0u;  // (k_search is done with it)
#pragma unroll
    for (uint32_t k = 0; k < E; ++k) {
        const uint64_t g = g0 + k;
        if (g >= G) break;  // (workgroup-uniform)
        uint64_t before = 0, agg = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (w < wv) before += s_scan[k][w];
            agg += s_scan[k][w];
        }
        const uint64_t tb = fold ? base : B.tiles[G + g];
        const uint64_t my_off = tb + before + x[k] - cnt[k], i = g * 256u + threadIdx.x;
        if (fold && g == G - 1 && threadIdx.x == 0) {
            B.loc_off[npat] = tb + agg;
            *B.needed = tb + agg;
        }
        if (i < npat) B.loc_off[i] = my_off;
        emit_locations<P, N, VB, REC>(a, sC, my_off, cnt[k], lo[k], rloc[k], mask[k], mode[k], B.cap,
                                      reinterpret_cast<P *>(B.out_locs));
        base = tb + agg;
    }
}

// A grouped launch's last kernel (replaces k_group_tiles + k_emit): one tile
// per workgroup reads its patterns' NarrowRec results (written at each
// pattern's index by k_search_grouped), writes the optional counts, hands its
// tile's count to the batch's later tiles as k_locate does (chain_base) and
// writes the offsets and locations.  Its workgroups are short and alike, so
// the waits are, too.
template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_emit_chain(const QueryArgs a, const LocateGroup grp, uint64_t tag,
                                                    uint64_t late_ticks) {
    __shared__ P sC[kMaxSigma + 1];
    __shared__ uint64_t s_scan[4], s_part[4];
    __shared__ uint32_t s_tk;
    const uint32_t jb = group_batch(grp, blockIdx.x);
    take_ticket(grp, jb, &s_tk);
    if (threadIdx.x <= a.sigma) sC[threadIdx.x] = (P)a.tab->C[threadIdx.x];
    __syncthreads();
    const LocateBatch &B = grp.b[jb];
    const uint64_t npat = B.npat, G = (npat + 255) / 256;
    const uint32_t g = claim_tile(grp, jb, G, &s_tk, a.status);
    if (g >= G) return;  // (workgroup-uniform)
    const uint64_t i = (uint64_t)g * 256u + threadIdx.x;
    P lo = 0, rloc = 0;
    uint64_t mask = 0, cnt = 0;
    uint32_t mode = kHitOne;
    if (i < npat) {
        cnt = unpack_narrow<P>(reinterpret_cast<const NarrowRec<P> *>(B.tiles + 2 * G)[i], lo, rloc, mask, mode);
        if (B.out_cnt) reinterpret_cast<P *>(B.out_cnt)[i] = (P)cnt;
    }
    uint64_t agg;
    const uint64_t excl = block_excl_scan(cnt, &agg, s_scan);  // (its barriers publish sC)
    const uint64_t base = chain_base(B, G, g, agg, tag, late_ticks, a.status, s_part);
    const uint64_t my_off = base + excl;
    if (g + 1 == G && threadIdx.x == 0) {
        B.loc_off[npat] = base + agg;
        *B.needed = base + agg;
    }
    if (i < npat) B.loc_off[i] = my_off;
    emit_locations<P, N, VB, REC>(a, sC, my_off, cnt, lo, rloc, mask, mode, B.cap, reinterpret_cast<P *>(B.out_locs));
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

// -------------------------------------------------------------- k_relayout

template <typename P, int N, int VB, int REC>
__global__ __launch_bounds__(256) void k_relayout(const QueryArgs a, uint64_t blocks_len, uint8_t *__restrict__ occ) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= blocks_len) return;
    write_record<P, N, VB, REC>(occ + q * (REC & ~15), a.blocks + q * (N * VB / 8), a.ckpt + q * a.sigma * sizeof(P),
                                a.sigma);
}

}  // namespace fmx
