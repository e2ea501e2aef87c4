// Internal declarations shared by the C-ABI (fmx_api.cpp), the query kernels
// (fmx_query.hip) and the GPU blob builder (fmx_build.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/fmx.h"

// A kernel's dynamic LDS (a macro: the host emulation under tests/simt
// supplies its own buffer per workgroup).
#ifndef FMX_DYN_LDS
#define FMX_DYN_LDS(name) extern __shared__ uint8_t name[]
#endif

namespace fmx {

constexpr int kMaxSigma = 64;  // Block6 indexes at most 2^6 symbols (blocks/block6.rs:15)
constexpr int kMaxK = 40;      // W^k must fit the u32 header field anyway (count_array.rs:68)
constexpr int kStageBytes = 16384;      // LDS bytes for a workgroup's 256 patterns (else read from HBM)
constexpr int kStageBytesLong = 57344;  // the same with FMX_HINT_LONG_PATTERNS

// Parsed blob headers.  Field-for-field what FmIndex::load derives
// (src/load_from_blob.rs:28-85); offsets are byte offsets into the blob.
struct BlobView {
    fmx_layout L{};
    uint32_t align = 8, bl = 64, block_bytes = 0;
    uint32_t sigma = 0, k = 0, sr = 0;
    uint64_t n = 0, sentinel = 0;
    uint64_t C[kMaxSigma + 1] = {};
    uint64_t mult[kMaxK] = {};
    uint8_t enc[256] = {};
    uint64_t kmer_len = 0, sa_len = 0, ckpt_len = 0, blocks_len = 0;
    uint64_t off_ca = 0, off_mult = 0, off_kmer = 0, off_sa = 0, off_sent = 0, off_ckpt = 0,
             off_blocks = 0;
    uint64_t header_size = 0, total = 0;
};

// Reads `len` bytes at blob offset `off` into dst (host or device source).
using BlobReader = std::function<bool(uint64_t off, uint64_t len, void *dst)>;

fmx_status parse_blob(const BlobReader &rd, uint64_t blob_len, fmx_layout L, BlobView *out,
                      uint64_t *expected_total, uint64_t *actual_total);

// Blob section sizes for the builder (FmIndexBuilder::blob_size, builder/mod.rs:165-181).
struct BlobSizes {
    uint64_t magic, enc, cah, sah, bwh, header;
    uint64_t ca, mult, kt, kt_len, sa_len, sa, sent, ckpt_len, ckpt, blocks_len, blocks, total;
};
fmx_status blob_sizes(uint64_t n, uint32_t sigma, fmx_layout L, uint32_t k, uint32_t sr, BlobSizes *S);

// The per-symbol tables of QueryArgs that kernels read one entry per lane
// (staging them into LDS), in HBM: a kernel argument lives in the kernarg
// segment, where a per-lane (vector) load costs ~12 us per kernel while a
// scalar load costs nothing measurable (scripts/micro/kernarg_cost.hip,
// profiles/r5/r5g_*: 14.4 vs 2.6 us for a 98-workgroup kernel) — the same
// tables read from HBM cost no more than the scalar path.  Filled at load.
struct QueryTables {
    uint8_t enc[256];
    uint8_t dig[kMaxSigma];  // = QueryArgs::dlut_dig
    uint64_t C[kMaxSigma + 1];
    uint64_t mult[kMaxK];
};

// Kernel arguments for the query kernels (passed by value; < 2 KB).  Arrays
// indexed per lane are read from `tab` (QueryTables), not from here.
struct QueryArgs {
    const uint8_t *ckpt;      // rank_checkpoints [P; blocks_len * sigma]
    const uint8_t *blocks;    // blocks [BlockN<V>; blocks_len]
    const uint8_t *sa;        // sampled suffix array [P; sa_len]
    const uint8_t *kmer;      // kmer_count_table [P; W^k]
    const uint8_t *occ;       // interleaved occ records (FMX_OCC_INTERLEAVED), else null
    uint32_t *status;         // latched device status bits
    const QueryTables *tab;   // enc, dlut_dig, C, mult in HBM (per-lane reads)
    uint64_t n, sentinel;
    uint32_t sigma, k, sr, sr_pow2_mask;  // sr_pow2_mask = sr-1 if sr is a power of two, else 0
    uint32_t sr_pow2, sr_shift;          // sr is a power of two (1 included), log2(sr)
    uint64_t sr_magic;                   // ceil(2^64 / sr) for sr not a power of two
    uint32_t strict;          // PassThrough: bytes >= sigma are an error
    uint32_t rec_bytes;       // interleaved record encoding (bytes | kRecPaired)
    const uint8_t *dlut;      // deep k-mer table: (lo, hi) as P for every dlut_sigma^dlut_k string, or null
    uint32_t dlut_k;
    uint32_t dlut_sigma;      // digits of the table: the symbols that occur in the text (C[c] < C[c+1])
    uint32_t dlut_rows;       // single-row entries are {row_flag | preceding symbols, SA} (FMX_OPT_LUT_ROWS)
    uint32_t dlut_bps;        // bits per packed preceding symbol in a single-row entry
    uint32_t dlut_ctx;        // packed preceding symbols per single-row entry
    uint32_t pad_;
    const uint8_t *safull;    // full suffix array: SA[r] = P at safull[r * sa_stride] (FMX_OPT_FULL_SA), or null
    const uint8_t *text;      // text as symbol indices [u8; n] (FMX_OPT_TEXT), or null
    uint32_t sa_stride;       // 1: plain full SA; 2: row records {SA[r], ctx[r]} (FMX_OPT_ROW_CONTEXT)
    uint32_t ctx_len;         // symbols per row context (0: no contexts)
    uint32_t scan_rows;       // intervals of at most this many rows are finished by a record scan
    uint32_t kt_lds_bytes;    // k-mer count table bytes when a workgroup copies it into LDS (else 0)
    uint64_t wpow[65];        // (sigma+1)^i, i <= ctx_len
    uint64_t C[kMaxSigma + 1];
    uint64_t mult[kMaxK];
    uint8_t enc[256];
    uint8_t dlut_dig[kMaxSigma];  // symbol -> digit of the deep table (kNoDigit: absent from the text)
    uint8_t dlut_sym[kMaxSigma];  // digit -> symbol
};

constexpr uint8_t kNoDigit = 0xFF;
// Multi-line symbol-mask records with a walk line (fmx_device.hpp kRecWalk)
// by default: C4 3.858 / 3.866 vs 3.661 / 3.657 x 10^9 without (same box,
// alternating, profiles/r6/r6b_c4_{walk,nowalk}_*); FMX_OCC_WALK=0 / 1 at
// load overrides; build option for A/B
#ifndef FMX_OCC_WALK_DEFAULT
#define FMX_OCC_WALK_DEFAULT 1
#endif
constexpr bool kOccWalkDefault = FMX_OCC_WALK_DEFAULT != 0;
constexpr uint32_t kOccRecWalkBit = 4;
// A one-row search result is located from the search's latest sampled row
// when it has one (fmx_device.hpp SampledRow; build option for A/B: 0 walks
// the final row as the reference does)
#ifndef FMX_SAMPLED_ROW
#define FMX_SAMPLED_ROW 1
#endif  // = kRecWalk (fmx_device.hpp), for the host code that does not include it
constexpr uint32_t kStatusSlots = 1024;   // status words per index (one per stream)
constexpr uint64_t kKmerLdsMax = 4096;    // k-mer count tables up to this size are staged in LDS

// Device status bits
constexpr uint32_t kStatusEmpty = 1u;
constexpr uint32_t kStatusSymbol = 2u;
constexpr uint32_t kStatusStride = 8u;  // FMX_HINT_FIXED_LEN given, offsets disagree
constexpr uint32_t kStatusGroup = 16u;  // a grouped launch's sorted position out of range (never expected)
constexpr uint32_t kStatusCheck = 32u;  // FMX_GROUP_CHECK=1: a grouped launch's sorted order failed its check
constexpr uint32_t kStatusLate = 64u;   // k_locate: an earlier tile's count not published in time (never expected)

// One bracketed launch: events a -> b on its stream, and for a split locate
// launch m between its two phases; timers[0] gets a -> b, timers[1] a -> m
// and timers[2] m -> b (-1: none).  Spans are folded into their timers as
// they complete (the oldest first, whenever more than kTimedKeep are
// pending, so a long timed region does not hold thousands of events) and
// all of them by fmx_timing_read.
struct TimedSpan {
    hipEvent_t a, m, b;
    int timers[3];
    uint64_t units;
};
constexpr size_t kTimedKeep = 64;

struct Timer {
    std::string name;
    uint64_t launches = 0;
    double ms = 0.0;
    uint64_t units = 0;
};

// Pinned staging for every copy between host memory the engine does not own
// (the caller's buffers, its own locals and vectors) and HBM: the CPU copies
// between those pages and two pinned buffers, the DMA engine only ever reads
// or writes the pinned buffers.  No DMA touches pageable memory, so no copy
// depends on how the runtime pins or stages it, and none can outlive the
// host buffer it came from (round 4).  Double-buffered: the
// CPU copy of one chunk overlaps the DMA of the previous one, and a buffer
// is refilled only after the event recorded behind its last copy.
//   h2d: returns once the source has been copied into the stage; the DMA is
//        ordered on `s` (later work on `s` sees the bytes).
//   d2h: synchronous — returns once the bytes are in the caller's buffer.
// One mutex per stage: calls from several threads take turns.
struct Stage {
    explicit Stage(uint64_t max_chunk = 8ull << 20) : max_chunk_(max_chunk) {}
    Stage(const Stage &) = delete;
    Stage &operator=(const Stage &) = delete;
    ~Stage();
    hipError_t h2d(void *d, const void *h, uint64_t n, hipStream_t s);
    hipError_t d2h(void *h, const void *d, uint64_t n, hipStream_t s);
    hipError_t drain();  // every copy from or into the stage has completed
    uint64_t chunk_bytes() const { return chunk_; }

  private:
    hipError_t reserve(uint64_t n);
    hipError_t wait(int b);
    uint8_t *buf_[2] = {nullptr, nullptr};
    hipEvent_t ev_[2] = {nullptr, nullptr};
    bool pending_[2] = {false, false};
    int next_ = 0;
    uint64_t chunk_ = 0;
    const uint64_t max_chunk_;
    std::mutex mu_;
};

// A status word's owner: the stream it is assigned to, its recency (for
// least-recently-used recycling) and what is known about its launches: a
// slot is recycled only when its stream is known to be idle.  Completion
// events are recorded only once the words run short (pressure mode): one per
// launch costs ~1 % of throughput (profiles/r3/r3b_status_events.txt).
struct StatusSlot {
    const void *key = nullptr;
    hipEvent_t done = nullptr;
    uint64_t last = 0;
    uint32_t inflight = 0;   // held by a launch call in progress
    bool launched = false;   // `done` follows the stream's latest launch
    bool maybe_busy = false; // launched without an event: idle only after a device sync
    bool pinned = false;     // the index's own stream: never recycled
};

}  // namespace fmx

struct fmx_index {
    fmx::BlobView bv;
    int device = 0;
    hipStream_t stream = nullptr;
    const uint8_t *host_blob = nullptr;
    uint64_t blob_len = 0;
    uint8_t *d_blob_owned = nullptr;
    const uint8_t *d_blob = nullptr;
    uint8_t *d_occ = nullptr;
    uint64_t occ_bytes = 0;
    uint32_t occ_mode = FMX_OCC_BLOB;
    uint32_t rec_bytes = 0;
    uint32_t *d_status = nullptr;  // kStatusSlots words: one per stream launched on
    // per status slot, kMaxGroup ticket counters for the fused launches on its stream (take_ticket:
    // zero between launches); FMX_FUSED_TICKETS=0 (A/B): workgroup index order instead
    uint32_t *d_tickets = nullptr;
    bool fused_tickets = true;
    uint32_t *h_status = nullptr;               // pinned: kStatusSlots words (read_status)
    std::unique_ptr<std::mutex[]> slot_mu;      // one per status slot (read_status)
    std::vector<fmx::StatusSlot> slots;                   // kStatusSlots
    std::unordered_map<const void *, uint32_t> status_of;  // stream -> slot
    std::vector<uint32_t> free_slots;
    uint64_t status_clock = 0;
    bool status_pressure = false;  // most words assigned: launches record completion events
    bool search_persistent = false;  // FMX_SEARCH_PERSISTENT=1: k_search on a resident-sized grid (A/B)
    // grouped launches (fmx::kWsHeader): launches of at least grouped_min
    // patterns on the faithful index — by default 2^20 when the key spans
    // at least 5 symbols (finish_load), FMX_GROUPED_MIN sets it, FMX_GROUPED=1
    // groups every launch that can be, FMX_GROUPED=0 none; the key = the last
    // gkey_len symbols, digits over the gkey_base symbols that occur in the text
    uint64_t grouped_min = 0;
    // launches of this index by path (fmx_index_info): grouped (packed / id-only records) and in
    // launch order — the tests assert which path a launch took
    mutable std::atomic<uint64_t> launches_grouped{0}, launches_grouped_raw{0}, launches_ordered{0};
    uint32_t gkey_len = 0, gkey_base = 0;
    uint32_t grouped_xcd = 0;  // each XCD searches one eighth of the key order (default; FMX_GROUPED_XCD=0 off)
    uint32_t grouped_pair = 0; // FMX_GROUPED_PAIR=1: two patterns per lane in the grouped search
    // the grouped search sorts each workgroup's 256 patterns by their next symbols after the key
    // (k_search_grouped; default on, FMX_GROUPED_WSORT=0 off)
    bool grouped_wsort = true;
    bool grouped_raw = false;  // FMX_GROUPED_RAW=1: id-only sorted records even for patterns that pack (A/B)
    uint64_t grouped_raw_min = ~0ull;  // launches needing id-only records: grouped from this many (default never)
    // grouped launches of at least this many patterns re-sort each key's run by the next gkey_len
    // symbols (k_group_refine; default never — measured even on C2 —, FMX_GROUP_REFINE_MIN sets it,
    // FMX_GROUP_REFINE=0: never)
    uint64_t group_refine_min = ~0ull;
    // FMX_GROUP_CHECK=1 (debug): every grouped launch checks its sorted order before the search —
    // each pattern placed exactly once, under its own key, with its own symbols (k_group_check_*)
    bool group_check = false;
    // launches in launch order run as one kernel (k_locate: search, then offsets and locations) when
    // every batch has at most kFoldTiles tiles, the fixed-length hint and patterns of at most
    // kFusedMaxLen symbols, and the launch has at most fused_max_tiles tiles (FMX_FUSED=0: never;
    // FMX_FUSED_MAX_TILES); fused_late_ticks bounds its waits (FMX_FUSED_TIMEOUT_MS, 100 MHz ticks)
    bool fused = true;
    uint64_t fused_max_tiles = ~0ull;
    uint64_t fused_late_ticks = 0;
    mutable std::atomic<uint64_t> launches_fused{0};  // (a subset of launches_ordered)
    // FMX_EMIT_CHAIN=1 (A/B): grouped launches end with k_emit_chain (tile counts handed from tile to tile,
    // as k_locate) instead of k_group_tiles + k_emit, when every batch has at most kFoldTiles tiles
    // (680 vs 235 us per C2 launch: the polls of ~2,000 short resident workgroups, profiles/r5/r5w_chain_*)
    bool emit_chain = false;
    // k_emit sums the earlier tiles' counts itself for batches of at most kFoldTiles tiles in launch order;
    // grouped launches run k_scan first (-1: that policy; FMX_EMIT_FOLD=1 / 0: fold / k_scan everywhere)
    int emit_fold = -1;
    mutable std::atomic<uint64_t> launches_chained{0};  // (a subset of the grouped launches)
    std::mutex status_mu;
    uint8_t *d_dlut = nullptr;
    uint64_t dlut_bytes = 0;
    uint8_t *d_safull = nullptr;
    uint64_t safull_bytes = 0;
    uint8_t *d_text = nullptr;
    fmx::QueryTables *d_tab = nullptr;
    uint32_t options = 0;
    fmx::QueryArgs qa{};
    // host-API scratch (grown on demand) and its private locate workspace
    uint8_t *d_scratch = nullptr;
    uint64_t scratch_bytes = 0;
    // pinned host staging of every host-memory copy of the index (the host-API batches, status
    // words, totals): the caller's pageable buffers are only ever memcpy'd by the CPU
    fmx::Stage stage;
    uint8_t *d_ws = nullptr;
    uint64_t ws_bytes = 0;
    // timing
    bool timing = false;
    uint32_t timing_every = 1;   // bracket every k-th launch
    uint64_t timing_seq = 0;
    std::vector<fmx::Timer> timers;
    std::deque<fmx::TimedSpan> spans;  // bracketed launches not folded into their timers yet
    std::vector<hipEvent_t> event_pool;
    std::mutex timing_mu;  // timers, event_pool, timing_seq
    std::mutex mu;         // the host-buffer calls' scratch and workspace
};

namespace fmx {

// Query launchers (fmx_query.hip).  All asynchronous on `stream`.
hipError_t launch_count(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                        uint32_t flags, void *d_counts, uint32_t *status, hipStream_t stream);
// Count + offsets scan + locate: k_search, (k_scan,) k_emit.  d_tiles =
// [tile counts: G][tile offsets: G][n search records] (G = ceil(n / 256)).
hipError_t launch_locate(const fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                         uint32_t flags, void *d_counts, uint64_t *d_loc_offsets, void *d_locs, uint64_t cap,
                         uint64_t *d_needed, uint64_t *d_tiles, uint64_t tiles_cap, uint32_t *status,
                         hipStream_t stream);
// One batch of a locate launch; a launch runs up to kMaxGroup of them, each
// with its own patterns, outputs and workspace (fmx_locate_group_async).
#ifndef FMX_MAX_GROUP
#define FMX_MAX_GROUP 256  // (build option: 128 was the round-3 default until the A/B in profiles/r3/narrow)
#endif
constexpr uint32_t kMaxGroup = FMX_MAX_GROUP;  // (the kernel argument then holds ~25 KB: gfx950 / ROCm 7 take up to
                                               // 32 KB, scripts/micro/kernarg.hip)
struct LocateBatch {
    const uint8_t *bytes;
    const uint64_t *offs;
    uint64_t npat;
    void *out_cnt;  // optional P-wide counts
    uint64_t *loc_off;
    void *out_locs;
    uint64_t cap;
    uint64_t *needed;
    uint64_t *tiles;
    uint32_t rev;
    uint32_t stride;  // FMX_HINT_FIXED_LEN: offs[i] == i * stride (0: read the offsets)
    uint64_t first;   // the launch's patterns in the batches before this one (set by launch_split)
};
struct LocateGroup {
    LocateBatch b[kMaxGroup];
    uint32_t tile_begin[kMaxGroup];  // first workgroup of batch j (tile_begin[0] = 0)
    uint32_t emit_begin[kMaxGroup];  // first k_group_tiles workgroup of batch j (kEmitTiles tiles each)
    uint32_t n;
    // Grouped launch (kWsHeader below): the group's key counters (batch 0's
    // workspace, zeroed on the launch's stream before its first kernel), the
    // key's symbol count and digit base, the bits per packed symbol, the
    // launch's pattern count, and the first key/place workgroup of each
    // batch; gcount null = launch order
    uint32_t *gcount;
    uint32_t gkey_len, gkey_base, gbits;
    uint32_t graw;  // 1: the sorted records hold pattern ids alone (patterns too long to pack)
    uint64_t gtotal;
    uint32_t chunk_begin[kMaxGroup];
    // A grouped launch may span several LocateGroups (kernel arguments of at
    // most kMaxGroup batches): gn batches in all, this group's tiles are the
    // launch's tiles vbase + tile_begin[j] (pattern ids (vbase + tile_begin[j])
    // x 256 + i), and gtab (the launch's first batch's workspace) maps a
    // sorted position or a pattern id of the whole launch to its batch
    const struct GroupTab *gtab;
    uint32_t gn, vbase;
    // FMX_SEARCH_PERSISTENT=1 (A/B): k_search runs a resident-sized grid whose
    // workgroups take tiles from this counter (batch 0's workspace header,
    // zero between launches: k_emit resets it); null = one workgroup per tile
    uint32_t *tile_ctr;
    // k_locate / k_emit_chain: one ticket counter per batch (fmx_index::d_tickets, the launch's status
    // slot's kMaxGroup words; take_ticket); null = each workgroup answers the tile of its own index
    uint32_t *tickets;
};
// A LocateGroup ready to be filled: no batches, launch-order fields clear.
// (Not zeroed as a whole: 25 KB per launch of host memset, and the kernels
// read only the first n entries of each array.)
inline void group_reset(LocateGroup &g) {
    g.n = 0;
    g.gcount = nullptr;
    g.gkey_len = g.gkey_base = g.gbits = g.graw = 0;
    g.gtotal = 0;
    g.gtab = nullptr;
    g.gn = g.vbase = 0;
    g.tile_ctr = nullptr;
    g.tickets = nullptr;
}
// `mid` (optional): an event recorded between k_search and k_emit (timing).
// Fills grp's per-launch fields (first, emit_begin, the grouped fields) in place.
hipError_t launch_locate_group(const fmx_index *ix, LocateGroup &grp, uint32_t stage_flags,
                               uint32_t *status, hipStream_t stream, hipEvent_t mid = nullptr);
// Up to kMaxMega batches as ng LocateGroups (each filled as for
// launch_locate_group, tile_begin[0] = 0 in each): one grouped launch over all
// of them when the launch is grouped, else each group in launch order.
hipError_t launch_locate_groups(const fmx_index *ix, LocateGroup *grps, uint32_t ng, uint32_t stage_flags,
                                uint32_t *status, hipStream_t stream, hipEvent_t mid = nullptr);
// k_emit sums the earlier tiles' counts itself for batches of at most this
// many tiles; larger ones get their tile offsets from k_scan first.
constexpr uint64_t kFoldTiles = 2048;
// k_locate (the fused launch) only for patterns up to this long: it gains
// where a tile's search is short (20 bp: one 100k batch 64.0 vs 66.7 us, C1
// +12 %, profiles/r5/r5t_*) and loses where it is long (C5's 150 bp: 3.25
// vs 3.33 x 10^9 — workgroups that finish early hold their slots while they
// wait for their batch's slower tiles, r5c5f_*); it also keeps every wait far
// below its bound (fmx_index::fused_late_ticks).
constexpr uint32_t kFusedMaxLen = 64;
// k_group_tiles takes this many tiles of one batch per workgroup: each of its
// waves has that many record loads in flight instead of one (a workgroup's
// life is mostly one HBM round trip; 121 -> 64 us per C2 launch at 4,
// profiles/r4/r4k_*).  Build option for A/B.  k_emit takes one tile per
// workgroup (its workgroups are the search's tiles: tile_begin): 4 did not
// change it on the headline (227 us either way, r4k) and cost a lone 100k
// batch 3.6 us (66.8 vs 70.4 us per call, profiles/r5/r5n_*).
#ifndef FMX_EMIT_TILES
#define FMX_EMIT_TILES 4
#endif
constexpr uint32_t kEmitTiles = FMX_EMIT_TILES;

// Grouped launches.  A launch's patterns are searched in the order of their
// last gkey_len symbols (a counting sort on one key per pattern) instead of
// the order they were given in, so that patterns whose backward searches
// share their first LF steps' intervals run in the same wavefronts at the
// same time and read those occ records once (one request per wave
// instruction, or an L2 hit) instead of once each.  Results are written at
// each pattern's own index: identical to a launch in the given order.
// Fixed-length batches whose patterns pack into 96 bits (gbits per symbol)
// only: the sorted order carries each pattern's symbols, so that the search
// reads its patterns in order.
// Locate workspace of a batch of n patterns (G = ceil(n / 256), R =
// locate_rec_bytes):
//   [256 B header][kGroupCounterRoom u32 key counters][tile counts: G][tile
//   offsets: G][search records: n x R][its share of the sorted order: n x 16 B]
// The counters sit at a fixed offset in batch 0's workspace; every grouped
// launch zeroes them on its stream first (32 KB, a few microseconds), so no
// launch depends on how an earlier one on the workspace ended.
#ifndef FMX_GROUP_KEY_BITS
// 8,192 bins: DNA keys on its last 6 symbols (4,096 bins), a 20-residue
// alphabet on its last 3 (8,000) — the k-mer seed's, after which the refine
// pass orders each run by the next 3 (round 5).  (Build option, A/B: 12 was
// the round-4 width; 14 = 16,384 bins, C2 keys on 7 symbols: slower, round 3.)
#define FMX_GROUP_KEY_BITS 13
#endif
constexpr uint32_t kGroupKeyBits = FMX_GROUP_KEY_BITS;
constexpr uint32_t kGroupBins = 1u << kGroupKeyBits;
constexpr uint32_t kGroupChunkTiles = 16;   // tiles (of 256 patterns) per key / place workgroup
constexpr uint32_t kCountChunks = 4;        // chunks per count-pass workgroup
constexpr uint32_t kGroupPackBits = 96;
constexpr uint32_t kGroupedXcd = 1;  // k_search_grouped opts: deal the key order out XCD by XCD
constexpr uint32_t kWsortBytes = 1024 + 256 * 16;  // its in-workgroup sort's LDS (256 counters, 256 records)
constexpr uint32_t kGroupRawStage = 216;  // raw records: patterns up to this long are staged in LDS by the search
// Build option (A/B): each key's run of the sorted order split into
// kGroupSlots sub-runs, one per slot = chunk mod kGroupSlots (8: the XCD that
// places the chunk, under the round-robin placement of workgroups), so that
// an XCD's scattered 16-B record writes would fill whole lines in its L2.
// Measured slower at 8 (C2: place 894 vs 566 us, count 229 vs 157 us per
// group, 3.85 vs 4.01e9; profiles/r5/r5sab_*): the place pass is not bound
// by partial-line writes.  Counters key-major: key k, slot s at
// k * kGroupSlots + s.
#ifndef FMX_GROUP_SLOTS
#define FMX_GROUP_SLOTS 1
#endif
constexpr uint32_t kGroupSlots = FMX_GROUP_SLOTS;
constexpr uint32_t kGroupCounterRoom = kGroupBins * kGroupSlots;
// Batches per grouped launch: up to kMaxMega, as several LocateGroups of at
// most kMaxGroup (kernel arguments) whose key, place, tile and emit kernels run
// per group and whose count scan, refine and search run once over the whole
// launch (fmx_query.hip, launch_locate_groups).  Each doubling of a grouped
// launch read fewer lines per pattern: C2's search 271 / 248 / 236 ns per
// pattern at 25.6 / 51.2 / 102.4 M patterns per launch (profiles/r5/r5w_*).
#ifndef FMX_MAX_MEGA
#define FMX_MAX_MEGA 1024
#endif
constexpr uint32_t kMaxMega = FMX_MAX_MEGA;
// A grouped launch's batch table, what its kernels read per lane to find the
// batch of a sorted position or a pattern id (binary searches; the arrays stay
// in L1).  In the launch's first batch's workspace, after the key counters;
// uploaded (pinned stage) before the launch's first kernel.
struct GroupDesc {
    uint8_t *recs;          // the batch's search records (a grouped launch: NarrowRec<P>)
    void *sorted;           // its share of the sorted order (U4 records)
    const uint8_t *bytes;   // its patterns (id-only records: read by the search)
    uint32_t stride, rev;
};
struct GroupTab {
    uint64_t first[kMaxMega];   // the launch's sorted positions (= patterns) before batch j
    // the compact copies the search's workgroups stage into LDS (one contiguous
    // upload): vfirst[j] = batch j's first pattern id, first32 = first (a
    // launch's positions fit 32 bits: is_grouped), stride16 = its pattern
    // length — 80 lines per workgroup prologue at 1,024 batches, where
    // first (u64) and desc[].stride (one line per 4 entries) took 352 (round 6)
    uint32_t vfirst[kMaxMega];
    uint32_t first32[kMaxMega];
    uint16_t stride16[kMaxMega];
    void *sorted[kMaxMega];  // = desc[j].sorted, compact for the place pass's staging (64 lines, not 256)
    GroupDesc desc[kMaxMega];
};
constexpr uint64_t kWsGroupTab = 256 + 4ull * kGroupCounterRoom;  // (16-B aligned)
constexpr uint64_t kWsHeader = kWsGroupTab + ((sizeof(GroupTab) + 15) & ~15ull);
inline uint64_t group_chunks(uint64_t n) { return ((n + 255) / 256 + kGroupChunkTiles - 1) / kGroupChunkTiles; }

// The kernels that depend on the occ layout, one table per (P, N) pair
// (fmx_layout.hip, one translation unit per pair); vb = V bits, rec = 0
// (blob layout) or the interleaved record bytes, var = search variant
// (kVarFaithful / kVarDerived / kVarDerivedLong, fmx_device.hpp).
struct LayoutOps {
    hipError_t (*count)(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const uint8_t *bytes,
                        const uint64_t *offs, uint64_t n, uint32_t flags, void *counts, uint32_t sb, hipStream_t s);
    hipError_t (*search)(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const LocateGroup &grp,
                         uint32_t tiles, uint32_t sb, hipStream_t s);
    hipError_t (*emit)(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp, uint32_t tiles,
                       uint32_t fold, hipStream_t s);
    // grouped launch (faithful variant): k_search_grouped over `total` patterns in key order;
    // opts = kGroupedXcd | wsort << 8 (k_search_grouped)
    hipError_t (*search_grouped)(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp,
                                 uint64_t total, uint32_t cap, uint32_t pair, uint32_t opts, hipStream_t s);
    hipError_t (*dlut_level)(const QueryArgs &qa, uint32_t vb, uint32_t rec, const void *parent, uint64_t np,
                             void *child, hipStream_t s);
    hipError_t (*full_sa)(const QueryArgs &qa, uint32_t vb, uint32_t rec, uint64_t n, void *sa_out,
                          uint32_t stride, hipStream_t s);
    hipError_t (*relayout)(const QueryArgs &qa, uint32_t vb, uint32_t rec, uint64_t blocks_len, uint8_t *occ,
                           hipStream_t s);
    // launch order as one kernel (k_locate): tag = the launch's hand-off tag, late_ticks its wait bound
    hipError_t (*locate)(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const LocateGroup &grp,
                         uint32_t tiles, uint32_t sb, uint64_t tag, uint64_t late_ticks, hipStream_t s);
    // a grouped launch's last kernel with the tile counts handed from tile to tile (k_emit_chain)
    hipError_t (*emit_chain)(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp, uint32_t tiles,
                             uint64_t tag, uint64_t late_ticks, hipStream_t s);
};
uint64_t locate_tiles_cap(uint64_t n);
// Bytes per pattern of the search-result records in the locate workspace.
uint64_t locate_rec_bytes(uint32_t pos_bytes);
hipError_t launch_relayout(fmx_index *ix, hipStream_t stream);
// Build the deep k-mer table (FMX_OPT_DEEP_LUT) for K into ix->d_dlut.
hipError_t build_deep_lut(fmx_index *ix, uint32_t K, hipStream_t stream);
// Turn its single-row intervals into {row_flag | preceding symbols, SA} entries
// (FMX_OPT_LUT_ROWS; needs the full SA and the text).
hipError_t build_dlut_rows(fmx_index *ix, hipStream_t stream);
// Recover the full suffix array into ix->d_safull (FMX_OPT_FULL_SA).
hipError_t build_full_sa(fmx_index *ix, uint32_t stride, hipStream_t stream);
// Recover the text (symbol indices) into ix->d_text from d_safull (FMX_OPT_TEXT).
hipError_t build_text(fmx_index *ix, hipStream_t stream);
// Fill the context half of the row records (FMX_OPT_ROW_CONTEXT) from d_text.
hipError_t build_row_context(fmx_index *ix, hipStream_t stream);
uint32_t interleaved_record_bytes(const BlobView &bv, bool multi, bool walk_ok = true);

// GPU builder (fmx_build.hip).
fmx_status build_device(const uint8_t *d_text, uint64_t n, const uint8_t *table, uint32_t sigma,
                        fmx_layout L, uint32_t k, uint32_t sr, uint8_t *d_blob, uint64_t blob_len,
                        hipStream_t stream);

}  // namespace fmx
