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
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstring>
#include <memory>
#include <random>

#include "fmx_kernels.hpp"

namespace fmx {

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

// ---------------------------------------------------------- grouped launches
// (k_group_key<count / place> and k_search_grouped: fmx_kernels.hpp)

// 2. The launch's key counts (per key and slot, key-major) -> each sub-run's
// first sorted position (exclusive scan in place; 16 counters per thread per
// pass, every load of a pass in flight at once).
__global__ __launch_bounds__(256) void k_group_scan(uint32_t *cnt) {
    __shared__ uint64_t s_scan[4];
    constexpr uint32_t per = 16;
    // whole passes only: a partial last pass would read and write past the
    // counters into the batch table that follows them
    static_assert(kGroupCounterRoom % (256 * per) == 0, "kGroupCounterRoom must be a multiple of 4,096");
    uint32_t carry = 0;
    for (uint32_t base = 0; base < kGroupCounterRoom; base += 256 * per) {
        uint32_t v[per], sum = 0;
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) {
            v[u] = cnt[base + threadIdx.x * per + u];
            sum += v[u];
        }
        uint64_t tot;
        uint32_t run = carry + (uint32_t)block_excl_scan(sum, &tot, s_scan);
#pragma unroll
        for (uint32_t u = 0; u < per; ++u) {
            cnt[base + threadIdx.x * per + u] = run;
            run += v[u];
        }
        carry += (uint32_t)tot;
    }
}

// 4. Each tile's count (k_emit's tile offsets) and each pattern's count (the
// optional counts output, in order here); kEmitTiles tiles per workgroup, as
// k_emit (every record load of a lane in flight at once).
template <typename P>
__global__ __launch_bounds__(256) void k_group_tiles(const LocateGroup grp) {
    constexpr uint32_t E = kEmitTiles;
    __shared__ uint64_t s_w[E][4];
    const uint32_t jb = emit_batch(grp, blockIdx.x);
    const LocateBatch &B = grp.b[jb];
    const uint64_t G = (B.npat + 255) / 256, g0 = (uint64_t)(blockIdx.x - grp.emit_begin[jb]) * E;
    const NarrowRec<P> *__restrict__ recs = reinterpret_cast<const NarrowRec<P> *>(B.tiles + 2 * G);
    uint64_t cnt[E];
#pragma unroll
    for (uint32_t k = 0; k < E; ++k) {
        const uint64_t i = (g0 + k) * 256u + threadIdx.x;
        cnt[k] = i < B.npat ? (uint64_t)recs[i].b : 0ull;
    }
#pragma unroll
    for (uint32_t k = 0; k < E; ++k) {
        const uint64_t i = (g0 + k) * 256u + threadIdx.x;
        if (B.out_cnt && i < B.npat) reinterpret_cast<P *>(B.out_cnt)[i] = (P)cnt[k];
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) cnt[k] += __shfl_xor(cnt[k], d);
        if ((threadIdx.x & 63) == 0) s_w[k][threadIdx.x >> 6] = cnt[k];
    }
    __syncthreads();
    if (threadIdx.x < E && g0 + threadIdx.x < G)
        B.tiles[g0 + threadIdx.x] = s_w[threadIdx.x][0] + s_w[threadIdx.x][1] + s_w[threadIdx.x][2] +
                                    s_w[threadIdx.x][3];
}

// ------------------------------------------- grouped launches: debug check
// FMX_GROUP_CHECK=1 (fmx_index::group_check): after the place (and refine)
// pass and before the search, the launch's sorted order is checked against
// the patterns themselves — every sorted position holds a pattern id of the
// launch, each id exactly once (a per-pattern tally in the batch's search
// records, which the search overwrites afterwards), under the key of the run
// it sits in (gcount, which after the place pass holds each run's end), and
// (packed records) with the pattern's own symbols.  A failure latches
// kStatusCheck (FMX_E_DEVICE; FMX_DEBUG names it).  Three launches; no
// workgroup waits on another.

__device__ __forceinline__ uint32_t *group_tally(const LocateBatch &B) {
    return reinterpret_cast<uint32_t *>(B.tiles + 2 * ((B.npat + 255) / 256));
}

// 1. and 3.: every pattern's tally zeroed / checked to be 1 (one workgroup per tile)
template <bool ZERO>
__global__ __launch_bounds__(256) void k_group_check_tally(const QueryArgs a, const LocateGroup grp) {
    const uint32_t vt = blockIdx.x, jb = group_batch(grp, vt);
    const LocateBatch &B = grp.b[jb];
    const uint64_t i = (uint64_t)(vt - grp.tile_begin[jb]) * 256u + threadIdx.x;
    if (i >= B.npat) return;
    uint32_t *tally = group_tally(B);
    if (ZERO) tally[i] = 0;
    else if (tally[i] != 1u) atomicOr(a.status, kStatusCheck);
}

// 2. each sorted position (one per thread)
__global__ __launch_bounds__(256) void k_group_check_order(const QueryArgs a, const LocateGroup grp,
                                                           uint32_t rec_bytes) {
    __shared__ uint8_t s_enc[256];
    __shared__ uint8_t s_dig[kMaxSigma];
    __shared__ uint32_t s_pw[32];
    const uint32_t t = threadIdx.x, L = grp.gkey_len;
    const GroupTab &gt = *grp.gtab;  // (the launch's batches)
    s_enc[t] = a.tab->enc[t];
    if (t < (uint32_t)kMaxSigma) s_dig[t] = a.tab->dig[t] == kNoDigit ? 0 : a.tab->dig[t];
    if (t == 0) {
        uint32_t w = 1;
        for (uint32_t e = 0; e < 32; ++e) {
            s_pw[e] = w;
            w = e + 1 < L ? w * grp.gkey_base : w;
        }
    }
    __syncthreads();
    const uint64_t sp = (uint64_t)blockIdx.x * 256u + t, total = grp.gtotal;
    if (sp >= total) return;
    bool bad = grp.gcount[kGroupCounterRoom - 1] != total;  // (the last run ends at the launch's end)
    const uint32_t js = lds_upper(gt.first, grp.gn, sp);
    const U4 e = reinterpret_cast<const U4 *>(gt.desc[js].sorted)[sp - gt.first[js]];
    const uint32_t jb = lds_upper(gt.vfirst, grp.gn, e.w);
    const GroupDesc B = gt.desc[jb];
    const uint64_t i = (uint64_t)(e.w - gt.vfirst[jb]);
    const uint64_t npat = (jb + 1 < grp.gn ? gt.first[jb + 1] : total) - gt.first[jb];
    if (e.w < gt.vfirst[jb] || i >= npat) {
        atomicOr(a.status, kStatusCheck);
        return;
    }
    atomicAdd(reinterpret_cast<uint32_t *>(B.recs) + i, 1u);  // (the batch's tallies: group_tally)
    // the run holding sp: the first key whose end is past it
    uint32_t lo = 0, hi = kGroupBins - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)grp.gcount[mid * kGroupSlots + kGroupSlots - 1] > sp) hi = mid;
        else lo = mid + 1;
    }
    const uint32_t m = B.stride;
    const bool rev = B.rev != 0;
    const uint8_t *pat = B.bytes + i * m;
    uint32_t key = 0;
    for (uint32_t back = 0; back < L && back < m; ++back) {
        const uint32_t j = m - 1 - back, c = s_enc[pat[rev ? m - 1 - j : j]];
        key += (c < (uint32_t)kMaxSigma ? s_dig[c] : 0u) * s_pw[L - 1 - back];
    }
    bad |= key != lo;
    if (!grp.graw) {
        for (uint32_t j = 0; j < m; ++j) {
            uint32_t c = s_enc[pat[rev ? m - 1 - j : j]];
            c = c < a.sigma ? c : a.sigma;
            bad |= packed_sym(e, j, grp.gbits) != c;
        }
    }
    if (bad) atomicOr(a.status, kStatusCheck);
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

// T[SA[r]] = first symbol of row r's suffix = the c with C[c] <= r < C[c+1].
template <typename P>
__global__ __launch_bounds__(256) void k_text(const QueryArgs a, uint64_t n, const P *__restrict__ sa,
                                              uint32_t stride, uint8_t *__restrict__ text) {
    __shared__ P sC[kMaxSigma + 1];
    if (threadIdx.x <= a.sigma) sC[threadIdx.x] = (P)a.tab->C[threadIdx.x];
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

// ------------------------------------------------------------- dispatch

// FMX_OCC_ONEHOT=0 / FMX_OCC_PAIRED=0 keep the next simpler record encoding
// (A/B runs; results are identical); FMX_OCC_WALK=1 / 0: multi-line symbol
// masks with / without a walk line (fmx_device.hpp kRecWalk; kOccWalkDefault)
uint32_t interleaved_record_bytes(const BlobView &bv, bool multi, bool walk_ok) {
    const char *ep = getenv("FMX_OCC_PAIRED"), *eh = getenv("FMX_OCC_ONEHOT"), *ew = getenv("FMX_OCC_WALK");
    const bool paired = !(ep && ep[0] == '0'), onehot = !(eh && eh[0] == '0');
    const bool walk = walk_ok && (ew ? ew[0] != '0' : kOccWalkDefault);
    return interleaved_rec_bytes(bv.L.pos_bytes, bv.L.planes, bv.L.vec_bits, bv.sigma, paired, onehot, multi, walk);
}

// one kernel table per (P, N, V) object of fmx_layout.hip
extern const LayoutOps layout_ops_4_2_32, layout_ops_4_2_64, layout_ops_4_2_128, layout_ops_4_3_32, layout_ops_4_3_64,
    layout_ops_4_3_128, layout_ops_4_4_32, layout_ops_4_4_64, layout_ops_4_4_128, layout_ops_4_5_32,
    layout_ops_4_5_64, layout_ops_4_5_128, layout_ops_4_6_32, layout_ops_4_6_64, layout_ops_4_6_128,
    layout_ops_8_2_32, layout_ops_8_2_64, layout_ops_8_2_128, layout_ops_8_3_32, layout_ops_8_3_64,
    layout_ops_8_3_128, layout_ops_8_4_32, layout_ops_8_4_64, layout_ops_8_4_128, layout_ops_8_5_32,
    layout_ops_8_5_64, layout_ops_8_5_128, layout_ops_8_6_32, layout_ops_8_6_64, layout_ops_8_6_128;

// The layout's kernel table and the run-time part of its layout (V, record).
struct Disp {
    const LayoutOps *ops;
    uint32_t vb, rec;
};
static Disp dispatch(const fmx_index *ix) {
    static const LayoutOps *const tab[2][5][3] = {
        {{&layout_ops_4_2_32, &layout_ops_4_2_64, &layout_ops_4_2_128},
         {&layout_ops_4_3_32, &layout_ops_4_3_64, &layout_ops_4_3_128},
         {&layout_ops_4_4_32, &layout_ops_4_4_64, &layout_ops_4_4_128},
         {&layout_ops_4_5_32, &layout_ops_4_5_64, &layout_ops_4_5_128},
         {&layout_ops_4_6_32, &layout_ops_4_6_64, &layout_ops_4_6_128}},
        {{&layout_ops_8_2_32, &layout_ops_8_2_64, &layout_ops_8_2_128},
         {&layout_ops_8_3_32, &layout_ops_8_3_64, &layout_ops_8_3_128},
         {&layout_ops_8_4_32, &layout_ops_8_4_64, &layout_ops_8_4_128},
         {&layout_ops_8_5_32, &layout_ops_8_5_64, &layout_ops_8_5_128},
         {&layout_ops_8_6_32, &layout_ops_8_6_64, &layout_ops_8_6_128}}};
    const fmx_layout &L = ix->bv.L;
    const uint32_t rec = ix->occ_mode == FMX_OCC_INTERLEAVED ? ix->rec_bytes : 0;
    const uint32_t vi = L.vec_bits == 32 ? 0 : L.vec_bits == 64 ? 1 : 2;
    return Disp{tab[L.pos_bytes == 4 ? 0 : 1][L.planes - 2][vi], L.vec_bits, rec};
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
    const Disp d = dispatch(ix);
    const uint32_t sb = stage_bytes_for(flags);
    return d.ops->count(qa, d.vb, d.rec, search_var(qa, sb), d_bytes, d_offsets, n, flags, d_counts, sb, stream);
}

// k_locate's hand-off tag for one launch: a process-wide launch counter
// through a bijective mix (odd multiplier, splitmix64 finaliser) with a random
// nonce — distinct for every launch of this process, and unrelated to the
// words another process (or nothing) left in a workspace.
static uint64_t launch_tag() {
    static const uint64_t nonce = [] {
        std::random_device rd;
        return ((uint64_t)rd() << 32) ^ (uint64_t)rd() ^
               (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    }();
    static std::atomic<uint64_t> seq{0};
    uint64_t z = nonce + 0x9E3779B97F4A7C15ull * (seq.fetch_add(1, std::memory_order_relaxed) + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z ? z : 1;  // (0: what zeroed memory holds)
}

// The ticket counters of the launch's status slot (take_ticket), or null:
// workgroup index order (FMX_FUSED_TICKETS=0, A/B).
static uint32_t *slot_tickets(const fmx_index *ix, const QueryArgs &qa) {
    if (!ix->fused_tickets || !ix->d_tickets || qa.status < ix->d_status || qa.status >= ix->d_status + kStatusSlots)
        return nullptr;
    return ix->d_tickets + (uint64_t)(qa.status - ix->d_status) * kMaxGroup;
}

// Bits per packed symbol for a grouped launch of the ng groups, or 0 when it
// cannot be grouped (a batch without the fixed-length hint); *raw: some
// batch's patterns do not pack into kGroupPackBits, so the sorted records
// carry pattern ids alone (FMX_GROUPED_RAW=1 forces that for every launch).
static uint32_t group_pack_bits(const fmx_index *ix, const LocateGroup *grps, uint32_t ng, bool *raw) {
    uint32_t bits = 1;
    while ((1u << bits) < ix->bv.sigma + 1) ++bits;
    *raw = ix->grouped_raw;
    for (uint32_t g = 0; g < ng; ++g)
        for (uint32_t j = 0; j < grps[g].n; ++j) {
            if (grps[g].b[j].stride == 0) return 0;
            if (grps[g].b[j].stride * bits > kGroupPackBits) *raw = true;
        }
    return bits;
}

static uint32_t group_tiles(const LocateGroup &grp) {
    return grp.tile_begin[grp.n - 1] + (uint32_t)((grp.b[grp.n - 1].npat + 255) / 256);
}

// k_group_tiles' workgroups of each batch (kEmitTiles tiles of one batch each); their count
static uint32_t set_emit_begin(LocateGroup &grp) {
    uint32_t ewg = 0;
    for (uint32_t j = 0; j < grp.n; ++j) {
        grp.emit_begin[j] = ewg;
        ewg += (uint32_t)(((grp.b[j].npat + 255) / 256 + kEmitTiles - 1) / kEmitTiles);
    }
    return ewg;
}

static bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

// The tile offsets of batches too large for k_emit's own sum (k_scan), then
// k_emit: a group's last kernels.  flags bit 1: NarrowRec records (grouped).
static hipError_t launch_emit(const fmx_index *ix, const QueryArgs &qa, const LocateGroup &grp, uint32_t tiles,
                              uint32_t narrow, hipStream_t stream) {
    const Disp d = dispatch(ix);
    // (a grouped launch's batches get k_scan: 885-895 vs 923-939 us per 102.4 M-pattern launch with
    // k_emit's own sums, profiles/r5/r5fold_*; FMX_EMIT_FOLD=1 / 0 forces either)
    uint32_t fold = (ix->emit_fold == 1 || (ix->emit_fold < 0 && !narrow)) ? 1u : 0u;
    for (uint32_t j = 0; j < grp.n; ++j) fold &= (grp.b[j].npat + 255) / 256 <= kFoldTiles ? 1u : 0u;
    if (!fold) {
        hipLaunchKernelGGL(k_scan, dim3(grp.n), dim3(256), 0, stream, grp);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return d.ops->emit(qa, d.vb, d.rec, grp, tiles, fold | (narrow ? 2u : 0u), stream);
}

// Host bytes into HBM in stream order through kernel arguments (a grouped
// launch's batch table): no DMA from host memory and no host wait on the
// GPU in an asynchronous launch — the pinned stage's buffers, shared by every
// stream, would make one stream's launch wait for another's earlier copy (and
// rocprofv3's counter passes hung at that wait, profiles/r5/r5z*).  A few
// one-workgroup kernels of kPutChunk bytes each (per-lane reads of the
// kernel argument: ~10 us each, r5g_kernarg_cost).
constexpr uint32_t kPutChunk = 24576;
struct PutChunk {
    uint64_t n;
    uint8_t b[kPutChunk];
};
__global__ __launch_bounds__(256) void k_put_bytes(uint8_t *__restrict__ dst, const PutChunk c) {
    for (uint64_t i = threadIdx.x; i < c.n; i += 256) dst[i] = c.b[i];
}
static hipError_t put_bytes(void *dst, const void *src, uint64_t n, hipStream_t s) {
    std::unique_ptr<PutChunk> c(new (std::nothrow) PutChunk);
    if (!c) return hipErrorOutOfMemory;
    for (uint64_t o = 0; o < n; o += kPutChunk) {
        c->n = std::min<uint64_t>(kPutChunk, n - o);
        memcpy(c->b, static_cast<const uint8_t *>(src) + o, c->n);
        hipLaunchKernelGGL(k_put_bytes, dim3(1), dim3(256), 0, s, static_cast<uint8_t *>(dst) + o, *c);
    }
    return hipGetLastError();
}

// One grouped launch over the ng groups' batches (kWsHeader): key counts
// (per group), their scan, the sorted order (per group: every position of the
// launch's order, GroupTab), the optional refine and check passes, the search
// in key order (once), then per group the tile counts and k_emit.  The key
// counters and the batch table sit in the first batch's workspace.
static hipError_t launch_grouped(const fmx_index *ix, const QueryArgs &qa, LocateGroup *grps, uint32_t ng,
                                 uint64_t total, uint32_t bits, bool raw, bool chain, hipStream_t stream,
                                 hipEvent_t mid) {
    const Disp d = dispatch(ix);
    const bool p4 = ix->bv.L.pos_bytes == 4;
    const uint32_t rb = (uint32_t)locate_rec_bytes(ix->bv.L.pos_bytes);
    uint8_t *ws0 = reinterpret_cast<uint8_t *>(grps[0].b[0].tiles) - kWsHeader;
    uint32_t *gcount = reinterpret_cast<uint32_t *>(ws0 + 256);
    GroupTab *d_tab = reinterpret_cast<GroupTab *>(ws0 + kWsGroupTab);
    // the batch table (what the kernels that see the whole launch read per lane)
    std::unique_ptr<GroupTab> tab(new (std::nothrow) GroupTab);
    if (!tab) return hipErrorOutOfMemory;
    uint32_t gn = 0, vt = 0, maxm = 1, cap = 4;
    uint64_t first = 0;
    for (uint32_t g = 0; g < ng; ++g) {
        LocateGroup &grp = grps[g];
        grp.vbase = vt;
        uint32_t chunks = 0;
        for (uint32_t j = 0; j < grp.n; ++j) {
            LocateBatch &B = grp.b[j];
            const uint64_t G = (B.npat + 255) / 256;
            B.first = first;
            tab->first[gn] = first;
            tab->vfirst[gn] = (vt + grp.tile_begin[j]) * 256u;
            tab->first32[gn] = (uint32_t)first;
            tab->stride16[gn] = (uint16_t)B.stride;
            tab->sorted[gn] = reinterpret_cast<uint8_t *>(B.tiles + 2 * G) + ((B.npat * rb + 15) & ~15ull);
            tab->desc[gn] = GroupDesc{reinterpret_cast<uint8_t *>(B.tiles + 2 * G),
                                      reinterpret_cast<uint8_t *>(B.tiles + 2 * G) + ((B.npat * rb + 15) & ~15ull),
                                      B.bytes, B.stride, B.rev};
            ++gn;
            first += B.npat;
            grp.chunk_begin[j] = chunks;
            chunks += (uint32_t)group_chunks(B.npat);
            maxm = std::max<uint32_t>(maxm, B.stride);
            cap = std::max<uint32_t>(cap, (B.stride + 3) & ~3u);
        }
        vt += group_tiles(grp);
    }
    for (uint32_t g = 0; g < ng; ++g) {
        LocateGroup &grp = grps[g];
        grp.gcount = gcount;
        grp.gkey_len = ix->gkey_len;
        grp.gkey_base = ix->gkey_base;
        grp.gbits = bits;
        grp.graw = raw ? 1u : 0u;
        grp.gtotal = total;
        grp.gtab = d_tab;
        grp.gn = gn;
    }
    // the key counters start at zero whatever an earlier launch on this
    // workspace did, and the table is in place: both ordered
    // before the count pass on the stream
    hipError_t e = hipMemsetAsync(gcount, 0, 4ull * kGroupCounterRoom, stream);
    if (e != hipSuccess) return e;
    // (vfirst, first32 and stride16 are contiguous: one upload of the three)
    static_assert(offsetof(GroupTab, first32) == offsetof(GroupTab, vfirst) + 4 * kMaxMega &&
                      offsetof(GroupTab, stride16) == offsetof(GroupTab, first32) + 4 * kMaxMega,
                  "GroupTab: vfirst, first32, stride16 contiguous");
    if ((e = put_bytes(d_tab->first, tab->first, 8ull * gn, stream)) != hipSuccess ||
        (e = put_bytes(d_tab->vfirst, tab->vfirst, offsetof(GroupTab, stride16) - offsetof(GroupTab, vfirst) +
                       2ull * gn, stream)) != hipSuccess ||
        (e = put_bytes(d_tab->sorted, tab->sorted, sizeof(void *) * gn, stream)) != hipSuccess ||
        (e = put_bytes(d_tab->desc, tab->desc, sizeof(GroupDesc) * gn, stream)) != hipSuccess)
        return e;
    // the count pass needs each pattern's key alone: it reads and decodes only the key's bytes (the
    // id-only variant's count pass, for packed records too: the decode, one LDS lookup per byte, bounds
    // these passes, not their loads — profiles/r4/r4q_*, r4r_*)
    for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t chunks = grps[g].chunk_begin[grps[g].n - 1] +
                                (uint32_t)group_chunks(grps[g].b[grps[g].n - 1].npat);
        // (workgroups of kCountChunks chunks of one slot each: kGroupSlots per kGroupSlots x kCountChunks chunks)
        const uint32_t span = kGroupSlots * kCountChunks;
        hipLaunchKernelGGL((k_group_key<5, false, true>), dim3((chunks + span - 1) / span * kGroupSlots),
                           dim3(1024), 0, stream, qa, grps[g], rb);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_group_scan, dim3(1), dim3(256), 0, stream, gcount);
    // the place pass holds each pattern in W registers (W = 6 words hold patterns up to 21 bytes at any
    // alignment, 8 up to 29, 25 up to 97; raw: the key's gkey_len <= 16 bytes in 5)
    for (uint32_t g = 0; g < ng; ++g) {
        const LocateGroup &grp = grps[g];
        const uint32_t chunks = grp.chunk_begin[grp.n - 1] + (uint32_t)group_chunks(grp.b[grp.n - 1].npat);
        if (raw)
            hipLaunchKernelGGL((k_group_key<5, true, true>), dim3(chunks), dim3(1024), 0, stream, qa, grp, rb);
        else if (maxm <= 21)
            hipLaunchKernelGGL((k_group_key<6, true>), dim3(chunks), dim3(1024), 0, stream, qa, grp, rb);
        else if (maxm <= 29)
            hipLaunchKernelGGL((k_group_key<8, true>), dim3(chunks), dim3(1024), 0, stream, qa, grp, rb);
        else
            hipLaunchKernelGGL((k_group_key<25, true>), dim3(chunks), dim3(1024), 0, stream, qa, grp, rb);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const bool refined = !raw && total >= ix->group_refine_min;
    if (refined) {
        // one workgroup per key from 4,096 patterns per key on average (C2's 25.6 M: every key its own)
        const uint32_t rg = (uint32_t)std::min<uint64_t>(kGroupBins, std::max<uint64_t>(1, total / 4096));
        hipLaunchKernelGGL(k_group_refine<0>, dim3(rg), dim3(1024), 0, stream, qa, grps[0], rb);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (ix->group_check) {
        const uint32_t ord = (uint32_t)((total + 255) / 256);
        for (uint32_t g = 0; g < ng; ++g)
            hipLaunchKernelGGL(k_group_check_tally<true>, dim3(group_tiles(grps[g])), dim3(256), 0, stream, qa,
                               grps[g]);
        hipLaunchKernelGGL(k_group_check_order, dim3(ord), dim3(256), 0, stream, qa, grps[0], rb);
        for (uint32_t g = 0; g < ng; ++g)
            hipLaunchKernelGGL(k_group_check_tally<false>, dim3(group_tiles(grps[g])), dim3(256), 0, stream, qa,
                               grps[g]);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // each lane unpacks (or, raw, stages) its pattern into `cap` bytes of LDS: the longest batch's length,
    // 4-byte aligned (raw records longer than kGroupRawStage: the search reads the bytes from HBM, cap 4)
    if (raw && cap > kGroupRawStage) cap = 4;
    // (two patterns per lane: packed records only — 512 lanes' staging would not fit LDS)
    // the in-workgroup sort's symbols: as many after those already in order (the key's, and the refine
    // pass's as many again) as base^w <= 256 allows (none when every pattern ends within them)
    const uint32_t sorted_len = ix->gkey_len * (refined ? 2u : 1u);
    uint32_t wsort = 0;
    if (ix->grouped_wsort && !raw && !(ix->grouped_pair) && maxm > sorted_len)
        for (uint32_t w = 1, p = ix->gkey_base; p <= 256 && w <= 8 && w <= maxm - sorted_len; ++w, p *= ix->gkey_base)
            wsort = w;
    const uint32_t opts = (ix->grouped_xcd ? kGroupedXcd : 0u) | wsort << 8 | sorted_len << 16;
    if ((e = d.ops->search_grouped(qa, d.vb, d.rec, grps[0], total, cap, ix->grouped_pair && !raw, opts,
                                   stream)) != hipSuccess)
        return e;
    if (!chain)
        for (uint32_t g = 0; g < ng; ++g) {
            const uint32_t ewg = set_emit_begin(grps[g]);
            if (p4)
                hipLaunchKernelGGL(k_group_tiles<uint32_t>, dim3(ewg), dim3(256), 0, stream, grps[g]);
            else
                hipLaunchKernelGGL(k_group_tiles<uint64_t>, dim3(ewg), dim3(256), 0, stream, grps[g]);
        }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    (raw ? ix->launches_grouped_raw : ix->launches_grouped).fetch_add(1, std::memory_order_relaxed);
    if (mid && (e = hipEventRecord(mid, stream)) != hipSuccess) return e;
    for (uint32_t g = 0; g < ng; ++g) {
        if (chain) {
            grps[g].tickets = slot_tickets(ix, qa);
            e = d.ops->emit_chain(qa, d.vb, d.rec, grps[g], group_tiles(grps[g]), launch_tag(), ix->fused_late_ticks,
                                  stream);
        } else {
            e = launch_emit(ix, qa, grps[g], group_tiles(grps[g]), 1u, stream);
        }
        if (e != hipSuccess) return e;
    }
    if (chain) ix->launches_chained.fetch_add(1, std::memory_order_relaxed);
    return hipSuccess;
}

// Whether the ng groups (every batch with its fields filled, tile_begin[0] =
// 0 in each) run as one grouped launch: the index has a key, every batch the
// fixed-length hint, the launch at least grouped_min patterns (grouped_raw_min
// when the records must be id-only), the faithful search, and 32-bit pattern
// ids.
static bool is_grouped(const fmx_index *ix, const QueryArgs &qa, const LocateGroup *grps, uint32_t ng, uint32_t sb,
                       uint64_t *total, uint32_t *bits, bool *raw) {
    uint64_t n = 0, tiles = 0;
    for (uint32_t g = 0; g < ng; ++g) {
        if (grps[g].tile_ctr) return false;
        for (uint32_t j = 0; j < grps[g].n; ++j) n += grps[g].b[j].npat;
        tiles += group_tiles(grps[g]);
    }
    *total = n;
    *bits = group_pack_bits(ix, grps, ng, raw);
    return ix->gkey_len != 0 && *bits != 0 && n >= (*raw ? ix->grouped_raw_min : ix->grouped_min) &&
           search_var(qa, sb) == kVarFaithful && tiles * 256u <= 0xFFFFFFFFull;
}

// The kernels of a locate of one group, one after another on `stream`.
static hipError_t launch_split(const fmx_index *ix, const QueryArgs &qa, LocateGroup &grp, uint32_t tiles,
                               uint32_t sb, hipStream_t stream, hipEvent_t mid = nullptr) {
    const Disp d = dispatch(ix);
    uint64_t total = 0;
    uint32_t bits = 0;
    bool raw = false;
    bool small = true;
    for (uint32_t j = 0; small && j < grp.n; ++j) small = (grp.b[j].npat + 255) / 256 <= kFoldTiles;
    if (is_grouped(ix, qa, &grp, 1, sb, &total, &bits, &raw)) {
        // grouped, batches of at most kFoldTiles tiles: k_emit_chain may end the launch (FMX_EMIT_CHAIN=1)
        const bool chain = small && ix->emit_chain && !stream_capturing(stream);
        return launch_grouped(ix, qa, &grp, 1, total, bits, raw, chain, stream, mid);
    }
    uint64_t first = 0;
    for (uint32_t j = 0; j < grp.n; ++j) {
        grp.b[j].first = first;
        first += grp.b[j].npat;
    }
    // in launch order, batches of at most kFoldTiles tiles of short fixed-length patterns: one kernel
    // (k_locate), unless the stream is being captured (a replayed graph would reuse the launch's tag)
    bool fused = small && ix->fused && !grp.tile_ctr && tiles <= ix->fused_max_tiles;
    for (uint32_t j = 0; fused && j < grp.n; ++j) fused = grp.b[j].stride != 0 && grp.b[j].stride <= kFusedMaxLen;
    if (fused && stream_capturing(stream)) fused = false;
    hipError_t e;
    if (fused) {
        grp.tickets = slot_tickets(ix, qa);
        if ((e = d.ops->locate(qa, d.vb, d.rec, search_var(qa, sb), grp, tiles, sb, launch_tag(),
                               ix->fused_late_ticks, stream)) != hipSuccess)
            return e;
        ix->launches_ordered.fetch_add(1, std::memory_order_relaxed);
        ix->launches_fused.fetch_add(1, std::memory_order_relaxed);
        // (timing: the whole launch is the first phase)
        return mid ? hipEventRecord(mid, stream) : hipSuccess;
    }
    if ((e = d.ops->search(qa, d.vb, d.rec, search_var(qa, sb), grp, tiles, sb, stream)) != hipSuccess) return e;
    ix->launches_ordered.fetch_add(1, std::memory_order_relaxed);
    if (mid && (e = hipEventRecord(mid, stream)) != hipSuccess) return e;
    return launch_emit(ix, qa, grp, tiles, 0u, stream);
}

hipError_t launch_locate(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                         uint32_t flags, void *d_counts, uint64_t *d_loc_offsets, void *d_locs, uint64_t cap,
                         uint64_t *d_needed, uint64_t *d_tiles, uint64_t tiles_cap, uint32_t *status,
                         hipStream_t stream) {
    if (n == 0) return hipSuccess;
    QueryArgs qa = ix->qa;
    qa.status = status;
    if ((n + 255) / 256 > tiles_cap || tiles_cap > 0xFFFFFFFFull) return hipErrorInvalidValue;
    LocateGroup grp;
    group_reset(grp);
    grp.tile_begin[0] = 0;
    grp.b[0] = LocateBatch{d_bytes, d_offsets, n, d_counts, d_loc_offsets, d_locs, cap, d_needed, d_tiles,
                           (flags & FMX_PATTERN_REVERSED) ? 1u : 0u, flags >> 16};
    grp.n = 1;
    return launch_split(ix, qa, grp, (uint32_t)((n + 255) / 256), stage_bytes_for(flags), stream);
}

static hipError_t check_group(const LocateGroup &grp, uint64_t *tiles) {
    if (grp.n == 0 || grp.n > kMaxGroup || grp.tile_begin[0] != 0) return hipErrorInvalidValue;
    uint64_t t = 0;
    for (uint32_t j = 0; j < grp.n; ++j) {
        if (grp.b[j].npat == 0 || grp.tile_begin[j] != t) return hipErrorInvalidValue;
        t += (grp.b[j].npat + 255) / 256;
    }
    if (t > 0x7FFFFFFFull) return hipErrorInvalidValue;
    *tiles = t;
    return hipSuccess;
}

hipError_t launch_locate_group(const fmx_index *ix, LocateGroup &grp, uint32_t stage_flags,
                               uint32_t *status, hipStream_t stream, hipEvent_t mid) {
    QueryArgs qa = ix->qa;
    qa.status = status;
    uint64_t tiles = 0;
    hipError_t e = check_group(grp, &tiles);
    if (e != hipSuccess) return e;
    return launch_split(ix, qa, grp, (uint32_t)tiles, stage_bytes_for(stage_flags), stream, mid);
}

hipError_t launch_locate_groups(const fmx_index *ix, LocateGroup *grps, uint32_t ng, uint32_t stage_flags,
                                uint32_t *status, hipStream_t stream, hipEvent_t mid) {
    if (ng == 0 || (uint64_t)ng * kMaxGroup > kMaxMega) return hipErrorInvalidValue;
    if (ng == 1) return launch_locate_group(ix, grps[0], stage_flags, status, stream, mid);
    QueryArgs qa = ix->qa;
    qa.status = status;
    const uint32_t sb = stage_bytes_for(stage_flags);
    uint64_t tiles[kMaxMega / kMaxGroup];
    hipError_t e;
    for (uint32_t g = 0; g < ng; ++g)
        if ((e = check_group(grps[g], &tiles[g])) != hipSuccess) return e;
    uint64_t total = 0;
    uint32_t bits = 0;
    bool raw = false;
    if (is_grouped(ix, qa, grps, ng, sb, &total, &bits, &raw)) {
        bool small = true;
        for (uint32_t g = 0; g < ng; ++g)
            for (uint32_t j = 0; small && j < grps[g].n; ++j) small = (grps[g].b[j].npat + 255) / 256 <= kFoldTiles;
        const bool chain = small && ix->emit_chain && !stream_capturing(stream);
        return launch_grouped(ix, qa, grps, ng, total, bits, raw, chain, stream, mid);
    }
    // in launch order: one launch per group (timing: the last group's search ends the first phase)
    for (uint32_t g = 0; g < ng; ++g)
        if ((e = launch_split(ix, qa, grps[g], (uint32_t)tiles[g], sb, stream, g + 1 == ng ? mid : nullptr)) !=
            hipSuccess)
            return e;
    return hipSuccess;
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
    if (pb == 4)
        hipLaunchKernelGGL((k_dlut_root<uint32_t>), dim3(1), dim3(64), 0, stream, qa, (uint32_t *)buf(1));
    else
        hipLaunchKernelGGL((k_dlut_root<uint64_t>), dim3(1), dim3(64), 0, stream, qa, (uint64_t *)buf(1));
    e = hipGetLastError();
    const Disp d = dispatch(ix);
    uint64_t np = sigma;
    for (uint32_t j = 1; j < K && e == hipSuccess; ++j) {
        e = d.ops->dlut_level(qa, d.vb, d.rec, buf(j), np, buf(j + 1), stream);
        np *= sigma;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (tmp) hipFree(tmp);
    return e;
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
    {
        const Disp d = dispatch(ix);
        e = d.ops->full_sa(ix->qa, d.vb, d.rec, n, ix->d_safull, stride, stream);
    }
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
    const Disp d = dispatch(ix);
    return d.ops->relayout(ix->qa, d.vb, d.rec, ix->bv.blocks_len, ix->d_occ, stream);
}

}  // namespace fmx

