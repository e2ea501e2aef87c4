// fmx_api.cpp — the C ABI (include/fmx.h): blob validation, HBM residency,
// batch orchestration, timing.  Host side of the MI355X engine.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "fmx_internal.hpp"

namespace fmx {

static uint64_t align_up(uint64_t raw, uint64_t a) {
    const uint64_t r = raw % a;
    return r == 0 ? raw : raw + (a - r);
}

static bool layout_valid(const fmx_layout &L) {
    return (L.pos_bytes == 4 || L.pos_bytes == 8) && L.planes >= 2 && L.planes <= 6 &&
           (L.vec_bits == 32 || L.vec_bits == 64 || L.vec_bits == 128) &&
           (L.encoder == FMX_ENC_TABLE || L.encoder == FMX_ENC_PASS);
}

// Vector::ALIGN_SIZE (blocks/vector.rs:16,31,46): 8 for u32/u64, 16 for u128.
static uint64_t align_of(const fmx_layout &L) { return L.vec_bits == 128 ? 16 : 8; }

static uint64_t read_p(const uint8_t *p, uint32_t pb) {
    if (pb == 4) { uint32_t v; memcpy(&v, p, 4); return v; }
    uint64_t v; memcpy(&v, p, 8); return v;
}

// FmIndex::load's header walk and exact body-size check
// (src/load_from_blob.rs:28-58; Header::read_from_blob, components/mod.rs:18-22;
// MagicNumber::is_valid/is_supported_version, magic_number.rs:38-47), plus the
// consistency checks that the reference gets from its type parameters.
fmx_status parse_blob(const BlobReader &rd, uint64_t len, fmx_layout L, BlobView *bv,
                      uint64_t *expected_total, uint64_t *actual_total) {
    if (!layout_valid(L)) return FMX_E_LAYOUT;
    const uint64_t A = align_of(L), pb = L.pos_bytes;
    BlobView &v = *bv;
    v = BlobView{};
    v.L = L;
    v.align = (uint32_t)A;
    v.bl = L.vec_bits;
    v.block_bytes = L.planes * L.vec_bits / 8;

    uint8_t hdr[8 + 256 + 32 + 16 + 32];
    const uint64_t want = std::min<uint64_t>(len, sizeof(hdr));
    if (want < 8 || !rd(0, want, hdr)) return FMX_E_FORMAT;
    if (!(hdr[0] == 'F' && hdr[1] == 'I' && hdr[2] == '0' && hdr[3] == '0')) return FMX_E_FORMAT;
    uint64_t off = align_up(8, A);
    if (L.encoder == FMX_ENC_TABLE) {
        if (off + 256 > want) return FMX_E_FORMAT;
        memcpy(v.enc, hdr + off, 256);
        off += align_up(256, A);
    } else {
        for (int i = 0; i < 256; ++i) v.enc[i] = (uint8_t)i;  // PassThrough::idx_of
    }
    auto u32at = [&](uint64_t o) { uint32_t x; memcpy(&x, hdr + o, 4); return x; };
    auto u64at = [&](uint64_t o) { uint64_t x; memcpy(&x, hdr + o, 8); return x; };
    if (off + 24 > want) return FMX_E_FORMAT;
    const uint32_t ca_sigma = u32at(off), ca_k = u32at(off + 4), ca_len = u32at(off + 8),
                   mult_len = u32at(off + 12);
    const uint64_t kt_len = u64at(off + 16);
    off += align_up(24, A);
    if (off + 16 > want) return FMX_E_FORMAT;
    const uint32_t sr = u32at(off);
    const uint64_t sa_len = u64at(off + 8);
    off += align_up(16, A);
    if (off + 24 > want) return FMX_E_FORMAT;
    const uint32_t bw_sigma = u32at(off);
    const uint64_t ckpt_len = u64at(off + 8), blocks_len = u64at(off + 16);
    off += align_up(24, A);
    v.header_size = off;

    if (ca_len > (1u << 20) || mult_len > 64 || kt_len > (1ull << 40) || sa_len > (1ull << 40) ||
        ckpt_len > (1ull << 46) || blocks_len > (1ull << 40))
        return FMX_E_LAYOUT;
    const uint64_t body_ca = align_up((uint64_t)ca_len * pb, A) + align_up((uint64_t)mult_len * 8, A) +
                             align_up(kt_len * pb, A);
    const uint64_t body_sa = align_up(sa_len * pb, A);
    const uint64_t body_bwm = align_up(pb, A) + align_up(ckpt_len * pb, A) + align_up(blocks_len * v.block_bytes, A);
    v.total = v.header_size + body_ca + body_sa + body_bwm;
    if (expected_total) *expected_total = v.total;
    if (actual_total) *actual_total = len;
    if (len != v.total) return FMX_E_SIZE;  // LoadError::MismatchedBlobSize

    v.off_ca = v.header_size;
    v.off_mult = v.off_ca + align_up((uint64_t)ca_len * pb, A);
    v.off_kmer = v.off_mult + align_up((uint64_t)mult_len * 8, A);
    v.off_sa = v.off_kmer + align_up(kt_len * pb, A);
    v.off_sent = v.off_sa + body_sa;
    v.off_ckpt = v.off_sent + align_up(pb, A);
    v.off_blocks = v.off_ckpt + align_up(ckpt_len * pb, A);

    if (ca_sigma == 0 || ca_sigma > (uint32_t)kMaxSigma || ca_sigma > (1u << L.planes)) return FMX_E_LAYOUT;
    if (ca_sigma != bw_sigma || ca_len != ca_sigma + 1 || mult_len != ca_k || ca_k == 0 ||
        ca_k > (uint32_t)kMaxK || sr == 0)
        return FMX_E_LAYOUT;
    v.sigma = ca_sigma; v.k = ca_k; v.sr = sr;
    uint8_t small[(kMaxSigma + 1) * 8];
    if (!rd(v.off_ca, (uint64_t)ca_len * pb, small)) return FMX_E_FORMAT;
    for (uint32_t c = 0; c <= ca_sigma; ++c) v.C[c] = read_p(small + c * pb, (uint32_t)pb);
    v.n = v.C[ca_sigma];
    const uint64_t W = ca_sigma + 1;
    uint64_t wk = 1;
    for (uint32_t i = 0; i < ca_k; ++i) {
        if (wk > (1ull << 40) / W) return FMX_E_LAYOUT;
        wk *= W;
    }
    if (kt_len != wk) return FMX_E_LAYOUT;
    uint64_t mult[kMaxK];
    if (!rd(v.off_mult, (uint64_t)ca_k * 8, mult)) return FMX_E_FORMAT;
    uint64_t pw = 1;
    for (uint32_t i = 0; i < ca_k; ++i) {  // [W^(k-1), .., W^0] (count_array.rs:89-93)
        if (mult[ca_k - 1 - i] != pw) return FMX_E_LAYOUT;
        v.mult[ca_k - 1 - i] = pw;
        pw *= W;
    }
    if (blocks_len != v.n / v.bl + 1 || ckpt_len != blocks_len * ca_sigma) return FMX_E_LAYOUT;
    if (sa_len != (v.n + sr - 1) / sr) return FMX_E_LAYOUT;
    uint8_t sent[8];
    if (!rd(v.off_sent, pb, sent)) return FMX_E_FORMAT;
    v.sentinel = read_p(sent, (uint32_t)pb);
    if (v.n > 0 && (v.sentinel == 0 || v.sentinel > v.n)) return FMX_E_LAYOUT;
    if (pb == 4 && v.n >= 0xFFFFFFFFull) return FMX_E_LAYOUT;
    v.kmer_len = kt_len; v.sa_len = sa_len; v.ckpt_len = ckpt_len; v.blocks_len = blocks_len;
    return FMX_OK;
}

// FmIndexBuilder::blob_size (builder/mod.rs:165-181) with the headers of
// CountArrayHeader::new (count_array.rs:57-77), SuffixArrayHeader::new
// (suffix_array/mod.rs:43-56), BwmHeader::new (bwm/mod.rs:69-90).
fmx_status blob_sizes(uint64_t n, uint32_t sigma, fmx_layout L, uint32_t k, uint32_t sr, BlobSizes *S) {
    if (!layout_valid(L)) return FMX_E_LAYOUT;
    if (sigma == 0 || sigma > (1u << L.planes)) return FMX_E_SYMBOL;  // BuildError::SymbolCountOver
    if (k == 0 || sr == 0 || k > (uint32_t)kMaxK) return FMX_E_CONFIG;
    const uint64_t A = align_of(L), pb = L.pos_bytes, W = sigma + 1;
    uint64_t wk = 1;
    for (uint32_t i = 0; i < k; ++i) {
        wk *= W;
        if (wk > 0xFFFFFFFFull) return FMX_E_CONFIG;  // u32 pow overflow (count_array.rs:68)
    }
    if (pb == 4 && n >= 0xFFFFFFFFull) return FMX_E_CONFIG;
    S->magic = align_up(8, A);
    S->enc = L.encoder == FMX_ENC_TABLE ? align_up(256, A) : 0;
    S->cah = align_up(24, A);
    S->sah = align_up(16, A);
    S->bwh = align_up(24, A);
    S->header = S->magic + S->enc + S->cah + S->sah + S->bwh;
    S->ca = align_up(W * pb, A);
    S->mult = align_up((uint64_t)k * 8, A);
    S->kt_len = wk;
    S->kt = align_up(wk * pb, A);
    S->sa_len = (n + sr - 1) / sr;
    S->sa = align_up(S->sa_len * pb, A);
    S->sent = align_up(pb, A);
    S->blocks_len = n / L.vec_bits + 1;
    S->ckpt_len = S->blocks_len * sigma;
    S->ckpt = align_up(S->ckpt_len * pb, A);
    S->blocks = align_up(S->blocks_len * L.planes * (L.vec_bits / 8), A);
    S->total = S->header + S->ca + S->mult + S->kt + S->sa + S->sent + S->ckpt + S->blocks;
    return FMX_OK;
}

// --------------------------------------------------------------- helpers

static hipEvent_t take_event(fmx_index *ix) {
    if (!ix->event_pool.empty()) {
        hipEvent_t e = ix->event_pool.back();
        ix->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

static int timer(fmx_index *ix, const char *name) {
    for (size_t i = 0; i < ix->timers.size(); ++i)
        if (ix->timers[i].name == name) return (int)i;
    ix->timers.push_back(Timer{});
    ix->timers.back().name = name;
    return (int)ix->timers.size() - 1;
}

// Fold span sp into its timers (its events have completed) and recycle its events.
static void fold_span(fmx_index *ix, const TimedSpan &sp) {
    const hipEvent_t from[3] = {sp.a, sp.a, sp.m}, to[3] = {sp.b, sp.m, sp.b};
    for (int k = 0; k < 3; ++k) {
        if (sp.timers[k] < 0) continue;
        float ms = 0.f;
        hipEventElapsedTime(&ms, from[k], to[k]);
        Timer &t = ix->timers[sp.timers[k]];
        t.ms += ms;
        t.launches += 1;
        t.units += sp.units;
    }
    ix->event_pool.push_back(sp.a);
    ix->event_pool.push_back(sp.b);
    if (sp.m) ix->event_pool.push_back(sp.m);
}

// While more than kTimedKeep spans are pending, fold every completed one
// among the oldest 2 kTimedKeep — whatever stream it was on: a slow stream's
// span at the front does not hold back the finished spans of the others
// (caller holds timing_mu).
static void harvest_spans(fmx_index *ix) {
    if (ix->spans.size() <= kTimedKeep) return;
    const size_t look = std::min(ix->spans.size(), 2 * kTimedKeep);
    size_t keep = 0;
    for (size_t i = 0; i < look; ++i) {
        const TimedSpan sp = ix->spans[i];
        if (hipEventQuery(sp.b) == hipSuccess) fold_span(ix, sp);
        else ix->spans[keep++] = sp;
    }
    ix->spans.erase(ix->spans.begin() + keep, ix->spans.begin() + look);
}

// Bracket one launch with events on its stream when timing is on.
template <class F>
static hipError_t timed(fmx_index *ix, const char *name, hipStream_t s, uint64_t units, F &&launch) {
    std::unique_lock<std::mutex> g(ix->timing_mu);
    if (!ix->timing || (ix->timing_seq++ % ix->timing_every) != 0) {
        g.unlock();
        return launch();
    }
    harvest_spans(ix);
    hipEvent_t a = take_event(ix), b = take_event(ix);
    if (!a || !b) return hipErrorOutOfMemory;
    hipEventRecord(a, s);
    hipError_t e = launch();
    hipEventRecord(b, s);
    ix->spans.push_back(TimedSpan{a, nullptr, b, {timer(ix, name), -1, -1}, units});
    return e;
}

// The same for a locate launch, with a third event between its two kernels:
// timers `name` (the launch), `first` (k_search) and `second` (k_emit).
template <class F>
static hipError_t timed_split(fmx_index *ix, const char *name, const char *first, const char *second, hipStream_t s,
                              uint64_t units, F &&launch) {
    std::unique_lock<std::mutex> g(ix->timing_mu);
    if (!ix->timing || (ix->timing_seq++ % ix->timing_every) != 0) {
        g.unlock();
        return launch(nullptr);
    }
    harvest_spans(ix);
    hipEvent_t a = take_event(ix), m = take_event(ix), b = take_event(ix);
    if (!a || !m || !b) return hipErrorOutOfMemory;
    hipEventRecord(a, s);
    hipError_t e = launch(m);
    hipEventRecord(b, s);
    ix->spans.push_back(TimedSpan{a, m, b, {timer(ix, name), timer(ix, first), timer(ix, second)}, units});
    return e;
}

// FMX_DEBUG=1: name the HIP error behind an FMX_E_DEVICE on stderr
static fmx_status dev_err(hipError_t e) {
    if (e == hipSuccess) return FMX_OK;
    static const bool debug = getenv("FMX_DEBUG") != nullptr;
    if (debug) fprintf(stderr, "fmx: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
    return FMX_E_DEVICE;
}

// Makes the index's device current for one entry point and restores the
// caller's current device on every return path.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

// FMX_LOAD_TRACE=1: each load stage's wall time on stderr.
struct LoadTrace {
    bool on = getenv("FMX_LOAD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[fmx load] %-22s %9.3f ms\n", what,
                std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// The status word of `s`: every stream an index launches on gets a device
// word of its own, so fmx_sync(s) reads and clears only what that stream's
// launches latched (stream-ordered), never another stream's.  A stream seen
// for the first time takes a free word, or else recycles the least recently
// used word whose stream is known to be idle: the word changes owner and is
// zeroed on the new stream before that stream's first launch, so bits an
// earlier owner latched and never read are dropped (fmx_sync or
// fmx_stream_release collect them).  Idle is known from a completion event
// recorded after each launch — only once 3/4 of the words are assigned
// (pressure mode), since an event per launch costs ~1 % — or, for words
// assigned before that, from one device-wide synchronisation when no word is
// otherwise free (a process cycling through more than ~1,000 streams).
// `launch`: the word is held until status_launched().  Caller holds status_mu.
static int pick_recyclable(fmx_index *ix) {
    int idx = -1;
    uint64_t best = ~0ull;
    for (uint32_t i = 0; i < ix->slots.size(); ++i) {
        const StatusSlot &sl = ix->slots[i];
        if (sl.pinned || sl.inflight || sl.maybe_busy || sl.last >= best) continue;
        if (sl.launched && hipEventQuery(sl.done) != hipSuccess) continue;
        best = sl.last;
        idx = (int)i;
    }
    return idx;
}

static int status_slot_locked(fmx_index *ix, hipStream_t s, bool launch) {
    auto it = ix->status_of.find((const void *)s);
    if (it != ix->status_of.end()) {
        StatusSlot &sl = ix->slots[it->second];
        sl.last = ++ix->status_clock;
        sl.inflight += launch ? 1u : 0u;
        return (int)it->second;
    }
    if (!launch) return -1;  // (a stream that never launched has nothing latched)
    int idx = -1;
    if (!ix->free_slots.empty()) {
        idx = (int)ix->free_slots.back();
        ix->free_slots.pop_back();
    } else {
        idx = pick_recyclable(ix);
        if (idx < 0) {
            // words assigned before pressure mode have no events: one device
            // sync makes every word not held by a launch call idle
            if (hipDeviceSynchronize() != hipSuccess) return -1;
            for (auto &sl : ix->slots)
                if (!sl.inflight) { sl.maybe_busy = false; sl.launched = false; }
            // (every word is known idle now: completion events are needed again
            // only once the words run short anew)
            ix->status_pressure = false;
            idx = pick_recyclable(ix);
        }
        if (idx < 0) return -1;
        ix->status_of.erase(ix->slots[idx].key);
    }
    StatusSlot &sl = ix->slots[idx];
    if (hipMemsetAsync(ix->d_status + idx, 0, 4, s) != hipSuccess ||
        hipMemsetAsync(ix->d_tickets + (uint64_t)idx * kMaxGroup, 0, 4ull * kMaxGroup, s) != hipSuccess) {
        sl.key = nullptr;
        ix->free_slots.push_back((uint32_t)idx);
        return -1;
    }
    sl.key = (const void *)s;
    sl.last = ++ix->status_clock;
    sl.inflight = 1;
    sl.launched = false;
    sl.maybe_busy = false;
    ix->status_of.emplace((const void *)s, (uint32_t)idx);
    if (ix->free_slots.size() < ix->slots.size() / 4) ix->status_pressure = true;
    return idx;
}

static uint32_t *status_slot(fmx_index *ix, hipStream_t s, int *idx) {
    std::lock_guard<std::mutex> g(ix->status_mu);
    *idx = status_slot_locked(ix, s, true);
    return *idx < 0 ? nullptr : ix->d_status + *idx;
}

// After the launch(es) of a status_slot() call were queued on s: release the
// hold and note how the word's idleness will be known (pressure mode: an event).
static void status_launched(fmx_index *ix, int idx, hipStream_t s) {
    std::lock_guard<std::mutex> g(ix->status_mu);
    StatusSlot &sl = ix->slots[idx];
    if (sl.inflight) --sl.inflight;
    if (sl.pinned) return;
    if (ix->status_pressure) {
        if (!sl.done && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) sl.done = nullptr;
        if (sl.done && hipEventRecord(sl.done, s) == hipSuccess) {
            sl.launched = true;
            sl.maybe_busy = false;
            return;
        }
    }
    sl.launched = false;
    sl.maybe_busy = true;
}

// status_slot + status_launched around one launch function.
template <class F>
static fmx_status with_status(fmx_index *ix, hipStream_t s, F &&launch) {
    int idx = -1;
    uint32_t *status = status_slot(ix, s, &idx);
    if (!status) return FMX_E_DEVICE;
    const fmx_status st = launch(status);
    status_launched(ix, idx, s);
    return st;
}

static fmx_status ensure_scratch(fmx_index *ix, uint64_t bytes) {
    if (ix->scratch_bytes >= bytes) return FMX_OK;
    if (ix->d_scratch) hipFree(ix->d_scratch);
    ix->d_scratch = nullptr;
    ix->scratch_bytes = 0;
    const uint64_t want = std::max<uint64_t>(bytes, 1 << 20);
    if (hipMalloc(&ix->d_scratch, want) != hipSuccess) return FMX_E_DEVICE;
    ix->scratch_bytes = want;
    return FMX_OK;
}

// ----------------------------------------------------------------- Stage
// (fmx_internal.hpp).  Chunks of up to max_chunk_ bytes alternate between the
// two pinned buffers; the CPU copy of a large chunk is split over a few
// threads (one thread copies ~10 GB/s: a 2.7 GB blob would otherwise be
// bound by it).

static void host_copy(void *dst, const void *src, uint64_t n) {
    constexpr uint64_t kPar = 8ull << 20;  // below this, one thread
    if (n < kPar) {
        memcpy(dst, src, n);
        return;
    }
    // up to 8 threads of >= 4 MiB each (a 2.7 GB blob: 88 ms host -> HBM with 4, r5p)
    const unsigned nt = (unsigned)std::min<uint64_t>(8, n / (4ull << 20));
    const uint64_t part = (n / nt + 4095) & ~4095ull;
    std::vector<std::thread> th;
    uint64_t o = part;
    try {  // (no exception may leave the C ABI)
        for (; o < n; o += part)
            th.emplace_back([=] { memcpy((uint8_t *)dst + o, (const uint8_t *)src + o, std::min(part, n - o)); });
    } catch (...) {
        for (; o < n; o += part) memcpy((uint8_t *)dst + o, (const uint8_t *)src + o, std::min(part, n - o));
    }
    memcpy(dst, src, std::min(part, n));
    for (auto &t : th) t.join();
}

Stage::~Stage() {
    drain();
    for (int b = 0; b < 2; ++b) {
        if (ev_[b]) hipEventDestroy(ev_[b]);
        if (buf_[b]) hipHostFree(buf_[b]);
    }
}

hipError_t Stage::wait(int b) {
    if (!pending_[b]) return hipSuccess;
    const hipError_t e = hipEventSynchronize(ev_[b]);
    if (e == hipSuccess) pending_[b] = false;
    return e;
}

hipError_t Stage::drain() {
    hipError_t e = wait(0);
    const hipError_t e1 = wait(1);
    return e != hipSuccess ? e : e1;
}

// Buffers of min(max(n, 64 KiB), max_chunk_) bytes (regrown only once both
// are idle).
hipError_t Stage::reserve(uint64_t n) {
    uint64_t cap = max_chunk_;
    if (const char *e = getenv("FMX_STAGE_CHUNK")) {  // (tests: small chunks exercise the double buffering)
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v >= 64) cap = std::min(cap, v);
    }
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>(n, 64 << 10), cap);
    if (!ev_[0] || !ev_[1]) {
        for (int b = 0; b < 2; ++b)
            if (!ev_[b]) {
                const hipError_t e = hipEventCreateWithFlags(&ev_[b], hipEventDisableTiming);
                if (e != hipSuccess) { ev_[b] = nullptr; return e; }
            }
    }
    if (chunk_ >= want) return hipSuccess;
    hipError_t e = drain();
    if (e != hipSuccess) return e;
    for (int b = 0; b < 2; ++b) {
        if (buf_[b]) hipHostFree(buf_[b]);
        buf_[b] = nullptr;
    }
    chunk_ = 0;
    for (int b = 0; b < 2; ++b)
        if ((e = hipHostMalloc(&buf_[b], want, hipHostMallocDefault)) != hipSuccess) {
            buf_[b] = nullptr;
            return e;
        }
    chunk_ = want;
    return hipSuccess;
}

hipError_t Stage::h2d(void *d, const void *h, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    std::lock_guard<std::mutex> g(mu_);
    hipError_t e = reserve(n);
    for (uint64_t o = 0; e == hipSuccess && o < n; o += chunk_) {
        const uint64_t c = std::min(n - o, chunk_);
        const int b = next_;
        next_ ^= 1;
        if ((e = wait(b)) != hipSuccess) break;  // (the buffer's previous copy has read it)
        host_copy(buf_[b], static_cast<const uint8_t *>(h) + o, c);
        e = hipMemcpyAsync(static_cast<uint8_t *>(d) + o, buf_[b], c, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(ev_[b], s);
        if (e == hipSuccess) pending_[b] = true;
    }
    return e;
}

hipError_t Stage::d2h(void *h, const void *d, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    std::lock_guard<std::mutex> g(mu_);
    hipError_t e = reserve(n);
    if (e == hipSuccess) e = drain();  // (both buffers free: an earlier h2d may still be reading them)
    const uint64_t chunks = e == hipSuccess ? (n + chunk_ - 1) / chunk_ : 0;
    // chunk i goes to buffer i & 1: the DMA of chunk i + 1 is queued before
    // the CPU copies chunk i out
    auto issue = [&](uint64_t i) {
        const uint64_t o = i * chunk_, c = std::min(n - o, chunk_);
        const int b = (int)(i & 1);
        hipError_t x = hipMemcpyAsync(buf_[b], static_cast<const uint8_t *>(d) + o, c, hipMemcpyDeviceToHost, s);
        if (x == hipSuccess) x = hipEventRecord(ev_[b], s);
        if (x == hipSuccess) pending_[b] = true;
        return x;
    };
    if (chunks) e = issue(0);
    for (uint64_t i = 0; e == hipSuccess && i < chunks; ++i) {
        if (i + 1 < chunks && (e = issue(i + 1)) != hipSuccess) break;
        const int b = (int)(i & 1);
        if ((e = wait(b)) != hipSuccess) break;
        const uint64_t o = i * chunk_;
        host_copy(static_cast<uint8_t *>(h) + o, buf_[b], std::min(n - o, chunk_));
    }
    next_ = 0;
    return e;
}

static fmx_status finish_load(fmx_index *ix, uint32_t options) {
    QueryArgs &q = ix->qa;
    const BlobView &v = ix->bv;
    q = QueryArgs{};
    q.ckpt = ix->d_blob + v.off_ckpt;
    q.blocks = ix->d_blob + v.off_blocks;
    q.sa = ix->d_blob + v.off_sa;
    q.kmer = ix->d_blob + v.off_kmer;
    q.n = v.n;
    q.sentinel = v.sentinel;
    q.sigma = v.sigma;
    q.k = v.k;
    q.sr = v.sr;
    q.sr_pow2 = (v.sr & (v.sr - 1)) == 0;
    q.sr_pow2_mask = q.sr_pow2 ? v.sr - 1 : 0;
    q.sr_shift = q.sr_pow2 ? (uint32_t)__builtin_ctz(v.sr) : 0;
    q.sr_magic = q.sr_pow2 ? 0 : (uint64_t)((((unsigned __int128)1 << 64) + v.sr - 1) / v.sr);
    q.strict = v.L.encoder == FMX_ENC_PASS;
    memcpy(q.C, v.C, sizeof(q.C));
    memcpy(q.mult, v.mult, sizeof(q.mult));
    memcpy(q.enc, v.enc, 256);
    if (!ix->stream && hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking) != hipSuccess) return FMX_E_DEVICE;
    if (hipMalloc(&ix->d_status, kStatusSlots * 4) != hipSuccess) return FMX_E_DEVICE;
    if (hipMemsetAsync(ix->d_status, 0, kStatusSlots * 4, ix->stream) != hipSuccess) return FMX_E_DEVICE;
    if (hipMalloc(&ix->d_tickets, 4ull * kStatusSlots * kMaxGroup) != hipSuccess) return FMX_E_DEVICE;
    if (hipMemsetAsync(ix->d_tickets, 0, 4ull * kStatusSlots * kMaxGroup, ix->stream) != hipSuccess)
        return FMX_E_DEVICE;
    // each slot's status word is read back into a pinned word of its own (read_status)
    if (hipHostMalloc(&ix->h_status, kStatusSlots * 4, hipHostMallocDefault) != hipSuccess) {
        ix->h_status = nullptr;
        return FMX_E_DEVICE;
    }
    ix->slot_mu.reset(new (std::nothrow) std::mutex[kStatusSlots]);
    if (!ix->slot_mu) return FMX_E_DEVICE;
    if (const char *e = getenv("FMX_FUSED_TICKETS")) ix->fused_tickets = e[0] != '0';
    if (hipStreamSynchronize(ix->stream) != hipSuccess) return FMX_E_DEVICE;
    ix->slots.assign(kStatusSlots, StatusSlot{});
    if (const char *e = getenv("FMX_SEARCH_PERSISTENT")) ix->search_persistent = e[0] == '1';
    // the fused launch (k_locate) and the bound on its waits: 4 s of the wall clock by default
    if (const char *e = getenv("FMX_FUSED")) ix->fused = e[0] != '0';
    if (const char *e = getenv("FMX_EMIT_CHAIN")) ix->emit_chain = e[0] != '0';
    if (const char *e = getenv("FMX_EMIT_FOLD")) ix->emit_fold = e[0] != '0' ? 1 : 0;
    if (const char *e = getenv("FMX_FUSED_MAX_TILES")) ix->fused_max_tiles = strtoull(e, nullptr, 0);
    {
        uint64_t ms = 4000;
        if (const char *e = getenv("FMX_FUSED_TIMEOUT_MS")) ms = std::max<uint64_t>(1, strtoull(e, nullptr, 0));
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ix->device) != hipSuccess || khz <= 0)
            khz = 100000;
        ix->fused_late_ticks = ms * (uint64_t)khz;
    }
    for (uint32_t i = kStatusSlots; i-- > 0;) ix->free_slots.push_back(i);
    {
        int idx = -1;
        q.status = status_slot(ix, ix->stream, &idx);
        if (!q.status) return FMX_E_DEVICE;
        ix->slots[idx].pinned = true;
        ix->slots[idx].inflight = 0;
    }
    // the tables kernels read one entry per lane, in HBM (QueryTables; uploaded
    // below, once dlut_dig is known — the record re-layout does not read them)
    if (hipMalloc(&ix->d_tab, sizeof(QueryTables)) != hipSuccess) return FMX_E_DEVICE;
    q.tab = ix->d_tab;
    // the k-mer count table (W^k entries of P) goes to LDS when it is small
    {
        const uint64_t ktb = v.kmer_len * v.L.pos_bytes;
        q.kt_lds_bytes = ktb <= kKmerLdsMax && ktb % 4 == 0 ? (uint32_t)ktb : 0u;
    }
    ix->occ_mode = FMX_OCC_BLOB;
    if (options & FMX_OCC_INTERLEAVED) {
        // multi-line symbol masks only for the faithful index (no derived
        // structures); if their records do not fit in HBM, the one-line
        // encodings, and if those do not fit either, the blob layout
        uint32_t rec = interleaved_record_bytes(v, (options & ~FMX_OCC_INTERLEAVED) == 0);
        // (FMX_OCC_MAX_MB caps the records' HBM: the same fallback, testable)
        const char *cap_env = getenv("FMX_OCC_MAX_MB");
        const uint64_t cap = cap_env ? strtoull(cap_env, nullptr, 10) << 20 : ~0ull;
        auto alloc = [&](uint32_t r) {
            if (r == 0 || v.blocks_len * (r & ~15u) > cap) return false;
            if (hipMalloc(&ix->d_occ, v.blocks_len * (r & ~15u)) == hipSuccess) return true;
            (void)hipGetLastError();  // (clear the out-of-memory error)
            ix->d_occ = nullptr;
            return false;
        };
        if (!alloc(rec)) {
            // the multi-line records without their walk line, then the one-line encodings
            const uint32_t nowalk = (rec & kOccRecWalkBit) ? interleaved_record_bytes(v, true, false) : 0u;
            const uint32_t one = interleaved_record_bytes(v, false);
            if (nowalk != 0 && nowalk != rec && alloc(nowalk)) rec = nowalk;
            else rec = one != rec && alloc(one) ? one : 0u;
        }
        if (rec != 0) {
            ix->rec_bytes = rec;
            ix->occ_bytes = v.blocks_len * (rec & ~15u);
            q.occ = ix->d_occ;
            q.rec_bytes = rec;
            ix->occ_mode = FMX_OCC_INTERLEAVED;
            if (launch_relayout(ix, ix->stream) != hipSuccess) return FMX_E_DEVICE;
            if (hipStreamSynchronize(ix->stream) != hipSuccess) return FMX_E_DEVICE;
        }
    }
    ix->options = ix->occ_mode;
    // deep-table digits: the symbols that occur in the text (a pattern holding
    // any other symbol is left to the blob's seed and the LF loop)
    uint32_t S = 0;
    for (uint32_t c = 0; c < (uint32_t)kMaxSigma; ++c) q.dlut_dig[c] = kNoDigit;
    for (uint32_t c = 0; c < v.sigma; ++c)
        if (v.C[c + 1] > v.C[c]) {
            q.dlut_dig[c] = (uint8_t)S;
            q.dlut_sym[S++] = (uint8_t)c;
        }
    // grouped launches: the key's digits are these S symbols; as many of the
    // last symbols as fit kGroupBins bins (C2: 6 of ACGT; C4: 2 residues)
    {
        QueryTables t{};
        memcpy(t.enc, q.enc, 256);
        memcpy(t.dig, q.dlut_dig, sizeof(t.dig));
        memcpy(t.C, q.C, sizeof(t.C));
        memcpy(t.mult, q.mult, sizeof(t.mult));
        if (ix->stage.h2d(ix->d_tab, &t, sizeof(t), ix->stream) != hipSuccess ||
            hipStreamSynchronize(ix->stream) != hipSuccess)
            return FMX_E_DEVICE;
    }
    ix->gkey_base = S;
    ix->gkey_len = 0;
    if (S >= 2)
        for (uint64_t bins = S; bins <= kGroupBins && ix->gkey_len < 16; bins *= S) ++ix->gkey_len;
    // on by default for launches of at least 3 x 2^20 patterns whose key spans
    // at least 5 symbols (DNA: 6), and of at least 2^26 whose key is shorter (a
    // 20-residue alphabet keys on 3, no more than its k-mer seed: at 25.6 M
    // patterns per launch grouping lost, 3.29 vs 3.59 x 10^9, profiles/r5/
    // r5f_*; at 102.4 M it won, 3.68 vs 3.42-3.45, r5c4m_*).  Below ~1 M
    // patterns the dealing out's fixed cost eats the sharing: at 256 batches
    // of 1,000 (C1) launch order runs 8.0 vs 4.2 x 10^9 grouped (r5p_*,
    // r5q_*), at 0.8 M patterns on 1 Gbp the two were equal and at 1.6 M
    // grouping gained 6 % (round 3); at 25.6 M patterns it gains 4 % on a
    // 4 Mbp text and 50 % from 16 Mbp up (r5q_size_*, r5r_size_*).  Round 6,
    // C3's per-rank slabs on 1 Gbp (256 batches per launch, same box,
    // profiles/r6/r6d_c3{g,o}_*): grouped vs launch order 2.97 vs 2.65 x 10^9
    // at 5 M, 2.62 vs 2.61 at 2.5 M, 2.42 vs 2.54 at 1.6 M, 2.25 vs 2.48 at
    // 1.25 M (C3's slab at 8 ranks) — the crossover is ~2.5 M, so 3 x 2^20.
    ix->grouped_min = ix->gkey_len >= 5 ? (3ull << 20) : (1ull << 26);
    if (const char *e = getenv("FMX_GROUPED")) {
        if (e[0] == '0') ix->grouped_min = ~0ull;
        else if (e[0] == '1') ix->grouped_min = 1;
    }
    if (const char *e = getenv("FMX_GROUPED_MIN")) ix->grouped_min = strtoull(e, nullptr, 10);
    ix->grouped_xcd = 1;
    if (const char *e = getenv("FMX_GROUPED_XCD")) ix->grouped_xcd = e[0] == '1';
    ix->grouped_pair = 0;
    if (const char *e = getenv("FMX_GROUPED_PAIR")) ix->grouped_pair = e[0] == '1';
    ix->grouped_wsort = true;
    if (const char *e = getenv("FMX_GROUPED_WSORT")) ix->grouped_wsort = e[0] != '0';
    ix->grouped_raw = false;
    if (const char *e = getenv("FMX_GROUPED_RAW")) ix->grouped_raw = e[0] == '1';
    // patterns too long to pack (id-only records) are grouped only on request:
    // C5 (1 M x 150 bp) measured slower grouped (3.1 vs 3.5 x 10^8)
    ix->grouped_raw_min = ~0ull;
    if (const char *e = getenv("FMX_GROUPED"))
        if (e[0] == '1') ix->grouped_raw_min = 1;
    if (ix->grouped_raw) ix->grouped_raw_min = ix->grouped_min;
    // (opt-in: on C2 at 25.6 M patterns per launch the refine pass costs 462 us and
    // saves 352 us of k_search_grouped)
    ix->group_refine_min = ~0ull;
    if (const char *e = getenv("FMX_GROUP_REFINE_MIN")) ix->group_refine_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("FMX_GROUP_REFINE")) if (e[0] == '0') ix->group_refine_min = ~0ull;
    if (const char *e = getenv("FMX_GROUP_CHECK")) ix->group_check = e[0] == '1';
    if ((options & FMX_OPT_DEEP_LUT) && S >= 2 && v.n > 0) {
        // the largest K with S^K * 2P <= budget, deeper than the blob's k;
        // budget: FMX_DEEP_LUT_MB, else 160 GiB capped at half the free HBM
        // (C2: K = 17, 128 GiB, 5 % above K = 16; C5: K = 16, 64 GiB, 9 % above
        // K = 15; profiles/r1_ab/r1lk*).  The build briefly needs 1/S more.
        uint64_t budget = 163840ull << 20;
        size_t hfree = 0, htotal = 0;
        if (hipMemGetInfo(&hfree, &htotal) == hipSuccess) budget = std::min<uint64_t>(budget, hfree / 2);
        if (const char *env = getenv("FMX_DEEP_LUT_MB")) budget = strtoull(env, nullptr, 10) << 20;
        const uint64_t per = 2ull * v.L.pos_bytes;
        uint32_t K = 0;
        uint64_t cnt = 1;
        // ... and no deeper than the first K with S^K >= 16 n (at most one
        // text position per 16 entries: deeper buys next to nothing)
        while (K < 32 && cnt <= budget / per / S && cnt < 16 * v.n) { cnt *= S; ++K; }
        if (K > v.k) {
            q.dlut_sigma = S;
            if (build_deep_lut(ix, K, ix->stream) != hipSuccess) return FMX_E_DEVICE;
            q.dlut = ix->d_dlut;
            q.dlut_k = K;
            ix->options |= FMX_OPT_DEEP_LUT;
        }
    }
    if (options & FMX_OPT_ROW_CONTEXT) options |= FMX_OPT_FULL_SA | FMX_OPT_TEXT;
    if ((options & (FMX_OPT_FULL_SA | FMX_OPT_TEXT)) && v.n > 0) {
        // row records {SA, ctx}: ctx_len = the most sigma+1-ary digits below 2^(8P)
        uint32_t ctx_len = 0;
        if (options & FMX_OPT_ROW_CONTEXT) {
            const unsigned __int128 lim = (unsigned __int128)1 << (8 * v.L.pos_bytes);
            unsigned __int128 w = 1;
            while (ctx_len < 64 && w * (v.sigma + 1) < lim) { w *= v.sigma + 1; ++ctx_len; }
        }
        q.sa_stride = ctx_len ? 2 : 1;
        if (build_full_sa(ix, q.sa_stride, ix->stream) != hipSuccess) return FMX_E_DEVICE;
        q.safull = ix->d_safull;
        ix->options |= FMX_OPT_FULL_SA;
        if (options & FMX_OPT_TEXT) {
            if (build_text(ix, ix->stream) != hipSuccess) return FMX_E_DEVICE;
            q.text = ix->d_text;
            ix->options |= FMX_OPT_TEXT;
        }
        if (ctx_len) {
            uint32_t scan = 32;
            if (const char *env = getenv("FMX_SCAN_ROWS")) scan = (uint32_t)strtoul(env, nullptr, 10);
            if (scan < 1 || scan > 64) return FMX_E_CONFIG;
            q.ctx_len = ctx_len;
            q.scan_rows = scan;
            q.wpow[0] = 1;
            for (uint32_t i = 1; i <= ctx_len; ++i) q.wpow[i] = q.wpow[i - 1] * (v.sigma + 1);
            if (build_row_context(ix, ix->stream) != hipSuccess) return FMX_E_DEVICE;
            ix->options |= FMX_OPT_ROW_CONTEXT;
        }
    }
    // single-row deep-table entries: the row flag needs n < 2^(8P-1)
    if ((options & FMX_OPT_LUT_ROWS) && q.dlut && q.text && q.safull &&
        (v.L.pos_bytes == 8 || v.n < (1ull << 31))) {
        uint32_t bps = 1;
        while ((1u << bps) < v.sigma + 2) ++bps;  // digits 0..sigma stored, sigma+1 = "no match"
        q.dlut_bps = bps;
        q.dlut_ctx = (8 * v.L.pos_bytes - 1) / bps;
        if (build_dlut_rows(ix, ix->stream) != hipSuccess) return FMX_E_DEVICE;
        q.dlut_rows = 1;
        ix->options |= FMX_OPT_LUT_ROWS;
    }
    return FMX_OK;
}

static fmx_status read_status(fmx_index *ix, hipStream_t s) {
    int idx;
    {
        std::lock_guard<std::mutex> g(ix->status_mu);
        idx = status_slot_locked(ix, s, false);
    }
    if (idx < 0) return dev_err(hipStreamSynchronize(s));  // never launched on: nothing latched
    uint32_t *w = ix->d_status + idx;
    uint32_t st = 0;
    {
        // into the slot's own pinned word (no DMA into pageable memory), waiting on s alone: no lock
        // that another stream's call needs is held across the wait (ADVICE r5 — the shared Stage was);
        // the word is readable once s has drained, so every launch queued on s before has finished
        std::lock_guard<std::mutex> g(ix->slot_mu[idx]);
        volatile uint32_t *h = ix->h_status + idx;
        *h = 0;
        if (hipMemcpyAsync((void *)h, w, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return FMX_E_DEVICE;
        st = *h;
    }
    if (st) {
        // ordered on s after every launch that could have set it: nothing is lost; a late fused
        // launch may have left its ticket counters off zero (claim_tile): they are zeroed too
        if (hipMemsetAsync(w, 0, 4, s) != hipSuccess ||
            ((st & kStatusLate) &&
             hipMemsetAsync(ix->d_tickets + (uint64_t)idx * kMaxGroup, 0, 4ull * kMaxGroup, s) != hipSuccess) ||
            hipStreamSynchronize(s) != hipSuccess)
            return FMX_E_DEVICE;
    }
    if (st & kStatusEmpty) return FMX_E_EMPTY_PATTERN;
    if (st & kStatusSymbol) return FMX_E_SYMBOL;
    if (st & kStatusStride) return FMX_E_ARG;
    if (st & (kStatusGroup | kStatusCheck | kStatusLate)) {
        static const bool debug = getenv("FMX_DEBUG") != nullptr;
        if (debug)
            fprintf(stderr, "fmx: %s\n",
                    (st & kStatusLate)    ? "fused launch: an earlier tile's count was not published in time"
                    : (st & kStatusCheck) ? "grouped launch: sorted order failed FMX_GROUP_CHECK"
                                          : "grouped launch: sorted position out of range");
        return FMX_E_DEVICE;
    }
    return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

// =================================================================== C ABI

extern "C" {

uint32_t fmx_abi_version(void) { return FMX_ABI_VERSION; }

const char *fmx_status_str(fmx_status s) {
    switch (s) {
        case FMX_OK: return "ok";
        case FMX_E_FORMAT: return "invalid FM-index format";
        case FMX_E_SIZE: return "mismatched blob size";
        case FMX_E_ALIGN: return "misaligned blob";
        case FMX_E_LAYOUT: return "layout does not match blob";
        case FMX_E_EMPTY_PATTERN: return "empty pattern";
        case FMX_E_SYMBOL: return "symbol out of range";
        case FMX_E_CAPACITY: return "output capacity too small";
        case FMX_E_DEVICE: return "device error";
        case FMX_E_ARG: return "invalid argument";
        case FMX_E_CONFIG: return "invalid build configuration";
    }
    return "unknown";
}

int fmx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

fmx_status fmx_load(const uint8_t *blob, uint64_t blob_len, fmx_layout layout, int device, uint32_t options,
                    fmx_index **out, uint64_t *expected_total, uint64_t *actual_total) {
    if (!out || (!blob && blob_len)) return FMX_E_ARG;
    *out = nullptr;
    if (!layout_valid(layout)) return FMX_E_LAYOUT;
    if (((uintptr_t)blob) % align_of(layout) != 0) return FMX_E_ALIGN;  // zerocopy alignment panic
    BlobView bv;
    BlobReader rd = [&](uint64_t off, uint64_t len, void *dst) {
        if (off + len > blob_len) return false;
        memcpy(dst, blob + off, len);
        return true;
    };
    LoadTrace tr;
    fmx_status st = parse_blob(rd, blob_len, layout, &bv, expected_total, actual_total);
    if (st) return st;
    tr.mark("parse headers");
    DeviceGuard dg(device);
    if (!dg.ok) return FMX_E_DEVICE;
    tr.mark("device (first HIP call)");
    fmx_index *ix = new (std::nothrow) fmx_index();
    if (!ix) return FMX_E_DEVICE;
    ix->bv = bv;
    ix->device = device;
    ix->host_blob = blob;
    ix->blob_len = blob_len;
    if (hipMalloc(&ix->d_blob_owned, blob_len) != hipSuccess) {
        fmx_free(ix);
        return FMX_E_DEVICE;
    }
    tr.mark("hipMalloc blob");
    // On the index's own stream, waited for: a plain hipMemcpy from pageable
    // memory may return before its DMA lands, and the load's kernels (the
    // record re-layout reads the blob) run on this non-blocking stream, which
    // is not ordered after the null stream — they could read the allocation's
    // previous contents (intermittent wrong counts with
    // interleaved records only; reproduced by tests/test_simt.py).  Through a
    // pinned stage of its own (32 MiB chunks, freed after the load): no DMA
    // reads the caller's pageable blob (round 4).
    if (hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking) != hipSuccess) {
        fmx_free(ix);
        return FMX_E_DEVICE;
    }
    {
        Stage up(32ull << 20);
        if (up.h2d(ix->d_blob_owned, blob, blob_len, ix->stream) != hipSuccess ||
            hipStreamSynchronize(ix->stream) != hipSuccess) {
            fmx_free(ix);
            return FMX_E_DEVICE;
        }
    }
    tr.mark("host -> HBM");
    ix->d_blob = ix->d_blob_owned;
    st = finish_load(ix, options);
    if (st) { fmx_free(ix); return st; }
    tr.mark("finish_load");
    *out = ix;
    return FMX_OK;
}

fmx_status fmx_load_device(const uint8_t *d_blob, uint64_t blob_len, fmx_layout layout, int device,
                           uint32_t options, fmx_index **out, uint64_t *expected_total, uint64_t *actual_total) {
    if (!out || !d_blob) return FMX_E_ARG;
    *out = nullptr;
    if (!layout_valid(layout)) return FMX_E_LAYOUT;
    if (((uintptr_t)d_blob) % align_of(layout) != 0) return FMX_E_ALIGN;
    DeviceGuard dg(device);
    if (!dg.ok) return FMX_E_DEVICE;
    if (hipDeviceSynchronize() != hipSuccess) return FMX_E_DEVICE;  // the blob's writers, on any stream
    BlobView bv;
    Stage hdr(64 << 10);  // the header reads land in pinned memory, then in the parser's locals
    BlobReader rd = [&](uint64_t off, uint64_t len, void *dst) {
        if (off + len > blob_len) return false;
        return hdr.d2h(dst, d_blob + off, len, nullptr) == hipSuccess;
    };
    fmx_status st = parse_blob(rd, blob_len, layout, &bv, expected_total, actual_total);
    if (st) return st;
    fmx_index *ix = new (std::nothrow) fmx_index();
    if (!ix) return FMX_E_DEVICE;
    ix->bv = bv;
    ix->device = device;
    ix->blob_len = blob_len;
    ix->d_blob = d_blob;
    st = finish_load(ix, options);
    if (st) { fmx_free(ix); return st; }
    *out = ix;
    return FMX_OK;
}

// Streamed file ingest: pread into two pinned chunks, each handed to the DMA
// engine as soon as it is full; the read of chunk i+1 overlaps the copy of
// chunk i (the event of a chunk's previous copy gates its reuse).
static bool read_full(int fd, uint64_t off, uint64_t len, void *dst) {
    uint8_t *d = (uint8_t *)dst;
    while (len) {
        const ssize_t r = pread(fd, d, len > (1ull << 30) ? (1ull << 30) : len, (off_t)off);
        if (r <= 0) return false;
        d += r;
        off += (uint64_t)r;
        len -= (uint64_t)r;
    }
    return true;
}

// O_DIRECT read of [off, off + len): off and dst are 4 KiB aligned; the
// request is rounded up to whole 4 KiB blocks (the file's end makes the last
// one short), so dst must have room for the rounded length.
static bool read_direct(int fd, uint64_t off, uint64_t len, void *dst) {
    uint8_t *d = (uint8_t *)dst;
    uint64_t want = align_up(len, 4096), got = 0;
    while (got < len) {
        const uint64_t ask = std::min<uint64_t>(want - got, 1ull << 30);
        const ssize_t r = pread(fd, d + got, ask, (off_t)(off + got));
        if (r <= 0) return false;
        got += (uint64_t)r;
        if ((uint64_t)r < ask && got < len && (got & 4095)) return false;  // short, unaligned: cannot go on
    }
    return true;
}

// File -> HBM through a ring of pinned chunks: each chunk is read by
// kReadThreads threads (page-cache copies run ~5-10 GB/s per thread) while
// earlier chunks are in flight to the device on one stream.  direct: fd was
// opened with O_DIRECT (reads bypass the page cache: a cold load).
static fmx_status stream_file(int fd, uint64_t len, uint8_t *d_dst, uint64_t chunk, bool direct) {
    constexpr int kBufs = 4, kReadThreads = 8;
    hipStream_t s = nullptr;
    void *buf[kBufs] = {};
    hipEvent_t ev[kBufs] = {};
    bool used[kBufs] = {};
    fmx_status st = FMX_OK;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return FMX_E_DEVICE;
    const int nb = (int)std::min<uint64_t>(kBufs, (len + chunk - 1) / std::max<uint64_t>(chunk, 1));
    for (int b = 0; b < nb && st == FMX_OK; ++b)
        if (hipHostMalloc(&buf[b], chunk, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) != hipSuccess)
            st = FMX_E_DEVICE;
    for (uint64_t off = 0, i = 0; st == FMX_OK && off < len; off += chunk, ++i) {
        const int b = (int)(i % (uint64_t)nb);
        const uint64_t n = std::min<uint64_t>(chunk, len - off);
        if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) { st = FMX_E_DEVICE; break; }
        // slices of >= 4 MB, page aligned
        const uint64_t slice = std::max<uint64_t>(align_up((n + kReadThreads - 1) / kReadThreads, 4096), 4ull << 20);
        std::vector<std::thread> th;
        std::atomic<bool> ok{true};
        auto rd = [&](uint64_t o) {
            const uint64_t l = std::min(slice, n - o);
            return direct ? read_direct(fd, off + o, l, (uint8_t *)buf[b] + o)
                          : read_full(fd, off + o, l, (uint8_t *)buf[b] + o);
        };
        uint64_t o = slice;
        try {  // (no exception may leave the C ABI)
            for (; o < n; o += slice)
                th.emplace_back([&, o] {
                    if (!rd(o)) ok = false;
                });
        } catch (...) {  // no more threads: this one reads the rest
            for (; o < n; o += slice)
                if (!rd(o)) ok = false;
        }
        if (!rd(0)) ok = false;
        for (auto &t : th) t.join();
        if (!ok) { st = FMX_E_ARG; break; }
        if (hipMemcpyAsync(d_dst + off, buf[b], n, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipEventRecord(ev[b], s) != hipSuccess) { st = FMX_E_DEVICE; break; }
        used[b] = true;
    }
    if (hipStreamSynchronize(s) != hipSuccess && st == FMX_OK) st = FMX_E_DEVICE;
    for (int b = 0; b < kBufs; ++b) {
        if (ev[b]) hipEventDestroy(ev[b]);
        if (buf[b]) hipHostFree(buf[b]);
    }
    hipStreamDestroy(s);
    return st;
}

fmx_status fmx_load_file(const char *path, fmx_layout layout, int device, uint32_t options, uint64_t chunk_bytes,
                         fmx_index **out, uint64_t *expected_total, uint64_t *actual_total) {
    if (!out || !path) return FMX_E_ARG;
    *out = nullptr;
    if (!layout_valid(layout)) return FMX_E_LAYOUT;
    const bool direct = (options & FMX_LOAD_DIRECT) != 0;
    options &= ~FMX_LOAD_DIRECT;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return FMX_E_ARG;
    int dfd = -1;  // the body's reads bypass the page cache (the header's go through it)
    if (direct && (dfd = open(path, O_RDONLY | O_CLOEXEC | O_DIRECT)) < 0) { close(fd); return FMX_E_ARG; }
    auto close_all = [&] {
        close(fd);
        if (dfd >= 0) close(dfd);
    };
    struct stat sb;
    if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) { close_all(); return FMX_E_ARG; }
    const uint64_t blob_len = (uint64_t)sb.st_size;
    LoadTrace tr;
    BlobView bv;
    BlobReader rd = [&](uint64_t off, uint64_t len, void *dst) {
        return off + len <= blob_len && read_full(fd, off, len, dst);
    };
    fmx_status st = parse_blob(rd, blob_len, layout, &bv, expected_total, actual_total);
    if (st) { close_all(); return st; }
    tr.mark("parse headers");
    DeviceGuard dg(device);
    if (!dg.ok) { close_all(); return FMX_E_DEVICE; }
    tr.mark("device (first HIP call)");
    fmx_index *ix = new (std::nothrow) fmx_index();
    if (!ix) { close_all(); return FMX_E_DEVICE; }
    ix->bv = bv;
    ix->device = device;
    ix->blob_len = blob_len;
    if (hipMalloc(&ix->d_blob_owned, std::max<uint64_t>(blob_len, 1)) != hipSuccess) {
        close_all();
        fmx_free(ix);
        return FMX_E_DEVICE;
    }
    tr.mark("hipMalloc blob");
    const uint64_t chunk = chunk_bytes ? align_up(chunk_bytes, 4096) : (16ull << 20);
    st = stream_file(direct ? dfd : fd, blob_len, ix->d_blob_owned, chunk, direct);
    close_all();
    if (st) { fmx_free(ix); return st; }
    tr.mark(direct ? "file -> HBM (O_DIRECT)" : "file -> HBM");
    ix->d_blob = ix->d_blob_owned;
    st = finish_load(ix, options);
    if (st) { fmx_free(ix); return st; }
    tr.mark("finish_load");
    *out = ix;
    return FMX_OK;
}

void fmx_free(fmx_index *ix) {
    if (!ix) return;
    DeviceGuard dg(ix->device);
    if (ix->stream) hipStreamSynchronize(ix->stream);
    for (const TimedSpan &sp : ix->spans) {
        hipEventDestroy(sp.a);
        hipEventDestroy(sp.b);
        if (sp.m) hipEventDestroy(sp.m);
    }
    for (auto e : ix->event_pool) hipEventDestroy(e);
    for (auto &sl : ix->slots)
        if (sl.done) hipEventDestroy(sl.done);
    if (ix->d_scratch) hipFree(ix->d_scratch);
    if (ix->d_ws) hipFree(ix->d_ws);
    if (ix->d_occ) hipFree(ix->d_occ);
    if (ix->d_dlut) hipFree(ix->d_dlut);
    if (ix->d_safull) hipFree(ix->d_safull);
    if (ix->d_text) hipFree(ix->d_text);
    if (ix->d_tab) hipFree(ix->d_tab);
    if (ix->d_status) hipFree(ix->d_status);
    if (ix->d_tickets) hipFree(ix->d_tickets);
    if (ix->h_status) hipHostFree(ix->h_status);
    if (ix->d_blob_owned) hipFree(ix->d_blob_owned);
    if (ix->stream) hipStreamDestroy(ix->stream);
    delete ix;
}

const uint8_t *fmx_blob(const fmx_index *ix, uint64_t *len) {
    if (!ix) return nullptr;
    if (len) *len = ix->host_blob ? ix->blob_len : 0;
    return ix->host_blob;
}

fmx_status fmx_info(const fmx_index *ix, fmx_index_info *o) {
    if (!ix || !o) return FMX_E_ARG;
    memset(o, 0, sizeof(*o));
    o->text_len = ix->bv.n;
    o->sentinel_index = ix->bv.sentinel;
    o->blob_len = ix->blob_len;
    o->device_bytes = (ix->d_blob_owned ? ix->blob_len : 0) + ix->occ_bytes + ix->dlut_bytes +
                      ix->safull_bytes + (ix->d_text ? ix->bv.n + 16 : 0);
    o->symbol_count = ix->bv.sigma;
    o->kmer_size = ix->bv.k;
    o->sampling_ratio = ix->bv.sr;
    o->block_len = ix->bv.bl;
    o->options = ix->options;
    o->deep_lut_k = ix->qa.dlut_k;
    o->context_len = ix->qa.ctx_len;
    o->scan_rows = ix->qa.scan_rows;
    o->occ_record = ix->occ_mode == FMX_OCC_INTERLEAVED ? ix->rec_bytes : 0;
    const bool faithful = !ix->qa.dlut && !ix->qa.safull && !ix->qa.text && ix->qa.ctx_len == 0;
    o->group_key_len = faithful ? ix->gkey_len : 0;
    o->group_key_base = faithful ? ix->gkey_base : 0;
    o->grouped_min = faithful && ix->gkey_len ? ix->grouped_min : ~0ull;
    o->launches_grouped = ix->launches_grouped.load();
    o->launches_grouped_raw = ix->launches_grouped_raw.load();
    o->launches_ordered = ix->launches_ordered.load();
    o->launches_fused = ix->launches_fused.load();
    o->launches_chained = ix->launches_chained.load();
    o->device = ix->device;
    return FMX_OK;
}

// ---------------------------------------------------------------- async

fmx_status fmx_count_batch_async(fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                 uint32_t flags, void *d_counts, void *stream) {
    if (!ix || (n && (!d_bytes || !d_offsets || !d_counts))) return FMX_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : ix->stream;
    DeviceGuard dg(ix->device);
    return with_status(ix, s, [&](uint32_t *status) {
        return dev_err(timed(ix, "count", s, n, [&] {
            return launch_count(ix, d_bytes, d_offsets, n, flags, d_counts, status, s);
        }));
    });
}

// Locate workspace (fmx_internal.hpp, kWsHeader): [256 B reserved][group
// key counters][tile counts: G][tile offsets: G][search records: n x
// locate_rec_bytes(P)][to 16 B][sorted order: n x 16 B], G = ceil(n / 256).
static uint64_t ws_bytes_of(uint64_t n, uint32_t pos_bytes) {
    return kWsHeader + 2 * locate_tiles_cap(n) * 8 + n * locate_rec_bytes(pos_bytes) + 16 + 16 * n;
}
static uint64_t ws_bytes_for(const fmx_index *ix, uint64_t n) { return ws_bytes_of(n, ix->bv.L.pos_bytes); }

fmx_status fmx_locate_workspace_size(fmx_index *ix, uint64_t n, uint64_t *bytes) {
    if (!ix || !bytes) return FMX_E_ARG;
    *bytes = ws_bytes_for(ix, n);
    return FMX_OK;
}

fmx_status fmx_workspace_bytes(uint64_t n, uint32_t pos_bytes, uint64_t *bytes) {
    if (!bytes || (pos_bytes != 4 && pos_bytes != 8)) return FMX_E_ARG;
    *bytes = ws_bytes_of(n, pos_bytes);
    return FMX_OK;
}

fmx_status fmx_locate_batch_async(fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                  uint32_t flags, void *d_counts, uint64_t *d_loc_offsets, void *d_locs,
                                  uint64_t cap, uint64_t *d_needed, void *d_ws, uint64_t ws_bytes, void *stream) {
    if (!ix || !d_loc_offsets || !d_needed || (n && (!d_bytes || !d_offsets)) || (cap && !d_locs)) return FMX_E_ARG;
    if (!d_ws || ws_bytes < kWsHeader + 16) return FMX_E_ARG;
    if (((uintptr_t)d_ws & 15) != 0) return FMX_E_ARG;  // (the grouped passes' 16-B vectors: fmx.h)
    hipStream_t s = stream ? (hipStream_t)stream : ix->stream;
    DeviceGuard dg(ix->device);
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_loc_offsets, 0, 8, s);
        if (e == hipSuccess) e = hipMemsetAsync(d_needed, 0, 8, s);
        return dev_err(e);
    }
    if (ws_bytes < ws_bytes_for(ix, n)) return FMX_E_ARG;
    uint8_t *ws = (uint8_t *)d_ws;
    const uint64_t G = locate_tiles_cap(n);
    return with_status(ix, s, [&](uint32_t *status) {
        return dev_err(timed(ix, "locate", s, n, [&] {
            return launch_locate(ix, d_bytes, d_offsets, n, flags, d_counts, d_loc_offsets, d_locs, cap, d_needed,
                                 (uint64_t *)(ws + kWsHeader), G, status, s);
        }));
    });
}

fmx_status fmx_locate_jobs_async(fmx_index *ix, const fmx_locate_job *jobs, uint64_t n_jobs) {
    if (!ix || (n_jobs && !jobs)) return FMX_E_ARG;
    for (uint64_t i = 0; i < n_jobs; ++i) {
        const fmx_locate_job &j = jobs[i];
        const fmx_status st =
            fmx_locate_batch_async(ix, j.d_bytes, j.d_offsets, j.n_patterns, j.flags, j.d_counts, j.d_loc_offsets,
                                   j.d_locs, j.cap, j.d_needed, j.d_workspace, j.workspace_bytes, j.stream);
        if (st) return st;
    }
    return FMX_OK;
}

fmx_status fmx_locate_group_async(fmx_index *ix, const fmx_locate_job *jobs, uint64_t n_jobs, void *stream) {
    if (!ix || (n_jobs && !jobs)) return FMX_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : ix->stream;
    for (uint64_t i = 0; i < n_jobs; ++i) {
        const fmx_locate_job &j = jobs[i];
        if (!j.d_loc_offsets || !j.d_needed || (j.n_patterns && (!j.d_bytes || !j.d_offsets)) ||
            (j.cap && !j.d_locs) || !j.d_workspace || j.workspace_bytes < ws_bytes_for(ix, j.n_patterns) ||
            ((uintptr_t)j.d_workspace & 15) != 0 || j.reserved != 0)
            return FMX_E_ARG;
        for (uint64_t k = 0; k < i; ++k)
            if (jobs[k].d_workspace == j.d_workspace) return FMX_E_ARG;  // the batches run concurrently
    }
    DeviceGuard dg(ix->device);
    return with_status(ix, s, [&](uint32_t *status) -> fmx_status {
    // up to kMaxMega non-empty batches per launch, as groups of kMaxGroup (one
    // grouped launch over all of them, or one launch in launch order per
    // group: launch_locate_groups); empty ones get their zero offset and total
    // directly
    constexpr uint32_t kGroups = kMaxMega / kMaxGroup;
    std::unique_ptr<LocateGroup[]> grps(new (std::nothrow) LocateGroup[kGroups]);
    if (!grps) return FMX_E_DEVICE;
    uint64_t i = 0;
    while (i < n_jobs) {
        uint32_t ng = 0, stage = 0;
        uint64_t units = 0;
        group_reset(grps[0]);
        uint32_t tiles = 0;
        for (; i < n_jobs; ++i) {
            const fmx_locate_job &j = jobs[i];
            if (j.n_patterns == 0) {
                hipError_t e = hipMemsetAsync(j.d_loc_offsets, 0, 8, s);
                if (e == hipSuccess) e = hipMemsetAsync(j.d_needed, 0, 8, s);
                if (e != hipSuccess) return FMX_E_DEVICE;
                continue;
            }
            if (grps[ng].n == kMaxGroup) {  // the next group
                if (ng + 1 == kGroups) break;
                group_reset(grps[++ng]);
                tiles = 0;
            }
            LocateGroup &grp = grps[ng];
            const uint64_t G = locate_tiles_cap(j.n_patterns);
            grp.tile_begin[grp.n] = tiles;
            grp.b[grp.n++] = LocateBatch{j.d_bytes, j.d_offsets, j.n_patterns, j.d_counts, j.d_loc_offsets,
                                         j.d_locs, j.cap, j.d_needed, (uint64_t *)((uint8_t *)j.d_workspace + kWsHeader),
                                         (j.flags & FMX_PATTERN_REVERSED) ? 1u : 0u, j.flags >> 16};
            tiles += (uint32_t)G;
            units += j.n_patterns;
            // the launch stages with the largest hint of its batches
            const uint32_t kb = (j.flags >> 8) & 0xffu, kbs = (stage >> 8) & 0xffu;
            if (kb > kbs) stage = (stage & ~0xff00u) | (kb << 8);
            stage |= j.flags & FMX_HINT_LONG_PATTERNS;
        }
        if (grps[0].n == 0) continue;
        const uint32_t ngroups = grps[ng].n ? ng + 1 : ng;
        // (A/B) the persistent grid's tile counter: batch 0's workspace header
        if (ngroups == 1 && ix->search_persistent && ix->occ_mode == FMX_OCC_INTERLEAVED && !ix->qa.dlut &&
            !ix->qa.safull && !ix->qa.text)
            grps[0].tile_ctr =
                reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(grps[0].b[0].tiles) - kWsHeader);
        const fmx_status st = dev_err(timed_split(ix, "locate", "locate.search", "locate.emit", s, units,
                                                  [&](hipEvent_t mid) {
            return launch_locate_groups(ix, grps.get(), ngroups, stage, status, s, mid);
        }));
        if (st) return st;
    }
    return FMX_OK;
    });
}

fmx_status fmx_sync(fmx_index *ix, void *stream) {
    if (!ix) return FMX_E_ARG;
    DeviceGuard dg(ix->device);
    return read_status(ix, stream ? (hipStream_t)stream : ix->stream);
}

fmx_status fmx_stream_release(fmx_index *ix, void *stream) {
    if (!ix) return FMX_E_ARG;
    DeviceGuard dg(ix->device);
    hipStream_t s = stream ? (hipStream_t)stream : ix->stream;
    const fmx_status st = read_status(ix, s);
    std::lock_guard<std::mutex> g(ix->status_mu);
    auto it = ix->status_of.find((const void *)s);
    if (it != ix->status_of.end() && !ix->slots[it->second].pinned && ix->slots[it->second].inflight == 0) {
        StatusSlot &sl = ix->slots[it->second];
        sl.key = nullptr;
        sl.launched = false;
        sl.maybe_busy = false;
        ix->free_slots.push_back(it->second);
        ix->status_of.erase(it);
        // pressure mode ends once most words are free again
        if (ix->free_slots.size() >= ix->slots.size() / 2) ix->status_pressure = false;
    }
    return st;
}

// ----------------------------------------------------------- host buffers

static fmx_status check_patterns(const uint64_t *offsets, uint64_t n) {
    if (n && offsets[0] != 0) return FMX_E_ARG;
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) return FMX_E_ARG;
        if (offsets[i + 1] == offsets[i]) return FMX_E_EMPTY_PATTERN;  // count_array.rs:211 panics
    }
    return FMX_OK;
}

// The hints for a host batch (they replace the caller's): FMX_HINT_STAGE_KB
// = the most bytes any 256-pattern tile spans, rounded up to whole KB (tiles
// past 56 KB read their patterns from HBM), and FMX_HINT_FIXED_LEN when every
// pattern has the same length.
static uint32_t stage_hint(const uint64_t *offsets, uint64_t n) {
    uint64_t most = 0;
    for (uint64_t t = 0; t < n; t += 256) most = std::max(most, offsets[std::min(n, t + 256)] - offsets[t]);
    const uint64_t kb = std::min<uint64_t>(std::max<uint64_t>((most + 1023) / 1024, 1), kStageBytesLong / 1024);
    const uint64_t m = offsets[1] - offsets[0];
    bool fixed = m <= 0xffffu;
    for (uint64_t i = 1; fixed && i < n; ++i) fixed = offsets[i + 1] - offsets[i] == m;
    return FMX_HINT_STAGE_KB(kb) | (fixed ? FMX_HINT_FIXED_LEN(m) : 0u);
}

fmx_status fmx_count_batch(fmx_index *ix, const uint8_t *bytes, const uint64_t *offsets, uint64_t n,
                           uint32_t flags, void *out_counts) {
    if (!ix || (n && (!offsets || !out_counts))) return FMX_E_ARG;
    if (n == 0) return FMX_OK;
    std::lock_guard<std::mutex> g(ix->mu);
    fmx_status st = check_patterns(offsets, n);
    if (st) return st;
    DeviceGuard dg(ix->device);
    const uint64_t nb = offsets[n], pb = ix->bv.L.pos_bytes;
    const uint64_t o_off = align_up(nb, 256), o_cnt = o_off + align_up((n + 1) * 8, 256);
    st = ensure_scratch(ix, o_cnt + n * pb);
    if (st) return st;
    hipStream_t s = ix->stream;
    uint8_t *d = ix->d_scratch;
    hipError_t e = ix->stage.h2d(d, bytes, nb, s);
    if (e == hipSuccess) e = ix->stage.h2d(d + o_off, offsets, (n + 1) * 8, s);
    if (e != hipSuccess) return FMX_E_DEVICE;
    flags = (flags & 0xffu) | stage_hint(offsets, n);
    st = fmx_count_batch_async(ix, d, (uint64_t *)(d + o_off), n, flags, d + o_cnt, s);
    if (st) return st;
    if (ix->stage.d2h(out_counts, d + o_cnt, n * pb, s) != hipSuccess) return FMX_E_DEVICE;
    return read_status(ix, s);
}

// The host-API locate workspace lives in the index, zeroed when (re)allocated.
static fmx_status ensure_ws(fmx_index *ix, uint64_t n) {
    const uint64_t need = ws_bytes_for(ix, n);
    if (ix->ws_bytes >= need) return FMX_OK;
    if (ix->d_ws) hipFree(ix->d_ws);
    ix->d_ws = nullptr;
    ix->ws_bytes = 0;
    const uint64_t want = std::max<uint64_t>(need, 1 << 16);
    if (hipMalloc(&ix->d_ws, want) != hipSuccess) return FMX_E_DEVICE;
    // zeroed on the index's own (non-blocking) stream, which the host-API
    // launches use (a plain hipMemset runs on the null stream, unordered with
    // it); only the persistent-grid A/B variant's tile counter needs it (a
    // grouped launch zeroes its own key counters)
    if (hipMemsetAsync(ix->d_ws, 0, want, ix->stream) != hipSuccess) return FMX_E_DEVICE;
    if (hipStreamSynchronize(ix->stream) != hipSuccess) return FMX_E_DEVICE;
    ix->ws_bytes = want;
    return FMX_OK;
}

fmx_status fmx_locate_batch(fmx_index *ix, const uint8_t *bytes, const uint64_t *offsets, uint64_t n,
                            uint32_t flags, uint64_t *out_loc_offsets, void *out_locs, uint64_t cap,
                            uint64_t *needed) {
    if (!ix || !out_loc_offsets || (n && !offsets) || (cap && !out_locs)) return FMX_E_ARG;
    if (needed) *needed = 0;
    if (n == 0) { out_loc_offsets[0] = 0; return FMX_OK; }
    std::lock_guard<std::mutex> g(ix->mu);
    fmx_status st = check_patterns(offsets, n);
    if (st) return st;
    DeviceGuard dg(ix->device);
    const uint64_t nb = offsets[n], pb = ix->bv.L.pos_bytes;
    flags = (flags & 0xffu) | stage_hint(offsets, n);
    st = ensure_ws(ix, n);
    if (st) return st;
    const uint64_t o_off = align_up(nb, 256);
    const uint64_t o_loff = o_off + align_up((n + 1) * 8, 256);
    const uint64_t o_need = o_loff + align_up((n + 1) * 8, 256);
    const uint64_t o_locs = o_need + 256;
    hipStream_t s = ix->stream;
    // Guess the output size (one occurrence per pattern, or what scratch
    // already holds); if the patterns have more occurrences, grow and rerun.
    uint64_t dcap = std::min<uint64_t>(cap, std::max<uint64_t>(n, ix->scratch_bytes > o_locs
                                                                       ? (ix->scratch_bytes - o_locs) / pb : 0));
    for (int pass = 0; pass < 2; ++pass) {
        st = ensure_scratch(ix, o_locs + std::max<uint64_t>(dcap, 1) * pb);
        if (st) return st;
        uint8_t *d = ix->d_scratch;
        hipError_t e = ix->stage.h2d(d, bytes, nb, s);
        if (e == hipSuccess) e = ix->stage.h2d(d + o_off, offsets, (n + 1) * 8, s);
        if (e != hipSuccess) return FMX_E_DEVICE;
        st = fmx_locate_batch_async(ix, d, (uint64_t *)(d + o_off), n, flags, nullptr, (uint64_t *)(d + o_loff),
                                    d + o_locs, dcap, (uint64_t *)(d + o_need), ix->d_ws, ix->ws_bytes, s);
        if (st) return st;
        uint64_t total = 0;
        if (ix->stage.d2h(&total, d + o_need, 8, s) != hipSuccess) return FMX_E_DEVICE;
        st = read_status(ix, s);
        if (st) return st;
        if (needed) *needed = total;
        if (total > cap) {
            if (ix->stage.d2h(out_loc_offsets, d + o_loff, (n + 1) * 8, s) != hipSuccess) return FMX_E_DEVICE;
            return FMX_E_CAPACITY;
        }
        if (total <= dcap) {
            e = ix->stage.d2h(out_loc_offsets, d + o_loff, (n + 1) * 8, s);
            if (e == hipSuccess && total) e = ix->stage.d2h(out_locs, d + o_locs, total * pb, s);
            return dev_err(e);
        }
        dcap = total;  // second pass with room for every location
    }
    return FMX_E_DEVICE;
}

// ---------------------------------------------------------------- timing

fmx_status fmx_timing_enable(fmx_index *ix, int enable) {
    if (!ix) return FMX_E_ARG;
    if (enable < 0) return FMX_E_ARG;
    std::lock_guard<std::mutex> g(ix->timing_mu);
    if (enable) {  // a fresh measurement: totals (and spans not read yet) start from zero
        for (const TimedSpan &sp : ix->spans) {
            if (hipEventSynchronize(sp.b) != hipSuccess) return FMX_E_DEVICE;
            ix->event_pool.push_back(sp.a);
            ix->event_pool.push_back(sp.b);
            if (sp.m) ix->event_pool.push_back(sp.m);
        }
        ix->spans.clear();
        for (auto &t : ix->timers) {
            t.launches = 0;
            t.ms = 0.0;
            t.units = 0;
        }
    }
    ix->timing = enable != 0;
    ix->timing_every = enable > 0 ? (uint32_t)enable : 1u;
    ix->timing_seq = 0;
    return FMX_OK;
}

fmx_status fmx_timing_read(fmx_index *ix, fmx_kernel_timing *out, int max_entries, int *n_entries) {
    if (!ix || !n_entries) return FMX_E_ARG;
    std::lock_guard<std::mutex> g(ix->timing_mu);
    while (!ix->spans.empty()) {
        if (hipEventSynchronize(ix->spans.front().b) != hipSuccess) return FMX_E_DEVICE;
        fold_span(ix, ix->spans.front());
        ix->spans.pop_front();
    }
    int k = 0;
    for (auto &t : ix->timers) {
        if (out && k < max_entries) {
            memset(&out[k], 0, sizeof(out[k]));
            snprintf(out[k].name, sizeof(out[k].name), "%s", t.name.c_str());
            out[k].launches = t.launches;
            out[k].total_ms = t.ms;
            out[k].units = t.units;
        }
        ++k;
    }
    *n_entries = k;
    return FMX_OK;
}

// --------------------------------------------------------------- builder

fmx_status fmx_build_blob_size(uint64_t text_len, uint32_t symbol_count, fmx_layout layout, uint32_t kmer_size,
                               uint32_t sampling_ratio, uint64_t *out_size) {
    if (!out_size) return FMX_E_ARG;
    BlobSizes S;
    fmx_status st = blob_sizes(text_len, symbol_count, layout, kmer_size, sampling_ratio, &S);
    if (st) return st;
    *out_size = S.total;
    return FMX_OK;
}

fmx_status fmx_build_device(const uint8_t *d_text, uint64_t text_len, const uint8_t *table, uint32_t symbol_count,
                            fmx_layout layout, uint32_t kmer_size, uint32_t sampling_ratio, uint8_t *d_blob,
                            uint64_t blob_len, int device) {
    if (!d_blob || (text_len && !d_text)) return FMX_E_ARG;
    DeviceGuard dg(device);
    if (!dg.ok) return FMX_E_DEVICE;
    // d_text may still be being written by work queued on any stream of the
    // device (the caller's): this synchronous call starts after all of it
    if (hipDeviceSynchronize() != hipSuccess) return FMX_E_DEVICE;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return FMX_E_DEVICE;
    fmx_status st = build_device(d_text, text_len, table, symbol_count, layout, kmer_size, sampling_ratio, d_blob,
                                 blob_len, s);
    hipStreamSynchronize(s);
    hipStreamDestroy(s);
    return st;
}

fmx_status fmx_build(const uint8_t *text, uint64_t text_len, const uint8_t *table, uint32_t symbol_count,
                     fmx_layout layout, uint32_t kmer_size, uint32_t sampling_ratio, uint8_t *blob,
                     uint64_t blob_len, int device) {
    if (!blob || (text_len && !text)) return FMX_E_ARG;
    if (((uintptr_t)blob) % align_of(layout) != 0) return FMX_E_ALIGN;  // BuildError::NotAlignedBlob
    DeviceGuard dg(device);
    if (!dg.ok) return FMX_E_DEVICE;
    uint8_t *dt = nullptr, *db = nullptr;
    if (hipMalloc(&dt, std::max<uint64_t>(text_len, 1)) != hipSuccess) return FMX_E_DEVICE;
    if (hipMalloc(&db, std::max<uint64_t>(blob_len, 16)) != hipSuccess) { hipFree(dt); return FMX_E_DEVICE; }
    fmx_status st = FMX_OK;
    {
        // the caller's text and blob through a pinned stage (no DMA on their
        // pageable pages); fmx_build_device starts after the text's copies
        // (hipDeviceSynchronize) and has finished when it returns
        Stage io(32ull << 20);
        if (text_len && io.h2d(dt, text, text_len, nullptr) != hipSuccess) st = FMX_E_DEVICE;
        if (!st) st = fmx_build_device(dt, text_len, table, symbol_count, layout, kmer_size, sampling_ratio, db,
                                       blob_len, device);
        if (!st && io.d2h(blob, db, blob_len, nullptr) != hipSuccess) st = FMX_E_DEVICE;
    }
    hipFree(dt);
    hipFree(db);
    return st;
}

}  // extern "C"
