// TEST INFRASTRUCTURE — the runtime behind tests/simt/shim/hip/hip_runtime.h:
// runs the engine's kernels on the CPU, one fiber per work-item.
//
//   * workgroups run one at a time, in a random order;
//   * inside a workgroup a random runnable work-item runs until it reaches a
//     barrier, a wave operation, an atomic (a switch point with probability
//     SIMT_YIELD, default 0.5) or its end: the interleaving between barriers,
//     and so the order in which atomics return, is random;
//   * __syncthreads() releases when every live work-item of the workgroup has
//     arrived; a wave operation when every live lane of its 64-lane wave has
//     (lanes that have returned contribute random bits, as inactive lanes do
//     on the GPU); arrivals whose per-item barrier counts differ (a barrier
//     or wave operation in divergent code) and workgroups that cannot finish
//     (a barrier some work-items never reach) fail the launch;
//   * LDS (the simt_lds section plus the dynamic buffer) is refilled with
//     random bytes before every workgroup, and hipMalloc'd memory is random
//     until written: a read of memory nobody wrote gives a random answer.
//
// The host API is synchronous (a launch has finished when it returns), with
// one exception that mirrors the HIP/CUDA contract: a host-to-device
// hipMemcpy (the null stream) returns once its source is staged, and the
// copy lands later — before the next null-stream operation or device-wide
// synchronisation, and at a random later launch on any other stream (a
// non-blocking stream is not ordered after the null stream).  A kernel on
// such a stream that reads the destination without a synchronisation reads
// whatever was there before.
// Deferred streams (simt_defer(), SIMT_DEFER=1): work on a non-null stream —
// kernels, copies, memsets, event records, waits on events — is queued and
// runs in stream order at a random later time (at random points of later
// host API calls), and at the latest when the host synchronises with it
// (hipStreamSynchronize, hipEventSynchronize, a completed hipEventQuery,
// hipDeviceSynchronize, hipFree).  A copy reads its source and writes its
// destination when it runs, as a DMA engine does: a host buffer reused before
// the copy that reads it has run, or read before the copy that fills it has
// run, gives wrong bytes.  A deferred kernel's failure is reported by the
// next synchronisation of its stream.
// SIMT_SEED sets the random stream (simt_config() from a test).
#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <signal.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <deque>
#include <cstdlib>
#include <mutex>
#include <random>
#include <string>
#include <vector>

extern "C" void simt_defer(int on, double progress);

extern "C" {
extern char __start_simt_lds[] __attribute__((weak, visibility("hidden")));
extern char __stop_simt_lds[] __attribute__((weak, visibility("hidden")));
void simt_switch(void **save_sp, void *to_sp) __attribute__((visibility("hidden")));
void simt_fiber_start() __attribute__((visibility("hidden")));
void simt_fiber_main() __attribute__((visibility("hidden"), used));
}

// x86-64 context switch: callee-saved registers on the old stack, stack
// pointer swapped; a new fiber's stack holds six zero registers and
// simt_fiber_start as its return address.
asm(R"(
    .text
    .globl simt_switch
    .hidden simt_switch
    .type simt_switch,@function
simt_switch:
    pushq %rbp
    pushq %rbx
    pushq %r12
    pushq %r13
    pushq %r14
    pushq %r15
    movq %rsp, (%rdi)
    movq %rsi, %rsp
    popq %r15
    popq %r14
    popq %r13
    popq %r12
    popq %rbx
    popq %rbp
    ret
    .size simt_switch,.-simt_switch
    .globl simt_fiber_start
    .hidden simt_fiber_start
    .type simt_fiber_start,@function
simt_fiber_start:
    andq $-16, %rsp
    call simt_fiber_main
    ud2
    .size simt_fiber_start,.-simt_fiber_start
)");

namespace simt {
namespace {

constexpr size_t kStack = 512 * 1024;  // per work-item (kernel arguments are copied per call: ~28 KB)
constexpr uint32_t kMaxItems = 1024;

enum State { kRun, kBlockBar, kWaveBar, kDone };

struct Xfer {
    uint64_t v[64];
    uint64_t live;
};

struct Fiber {
    void *sp = nullptr;
    uint8_t *stack = nullptr;  // lowest address (a guard page below)
    uint32_t tid = 0, wave = 0, lane = 0;
    State st = kRun;
    uint64_t nbar = 0, nwave = 0;  // barriers / wave operations passed
    std::shared_ptr<Xfer> xfer;
};

struct Wave {
    uint32_t alive = 0, arrived = 0;
    uint64_t present = 0, slot[64] = {};
    uint64_t site = 0;
    bool site_set = false;
    std::vector<uint32_t> waiters;
};

std::recursive_mutex g_mu;          // one grid at a time
std::mutex g_rng_mu;                // host-side random fills
std::mt19937_64 g_rng(0x5eed);
double g_yield = 0.5;
bool g_ordered = false;  // workgroups in index order (simt_block_order)
bool g_inited = false;
std::vector<Fiber> g_fibers;
std::vector<Wave> g_waves;
std::vector<uint32_t> g_runnable;
void *g_sched_sp = nullptr;
Fiber *g_cur = nullptr;
const std::function<void()> *g_body = nullptr;
dim3 g_tid_dummy, g_bid, g_grid, g_block;
std::vector<dim3> g_tids;
std::vector<uint8_t> g_dyn;
uint32_t g_alive = 0, g_arrived = 0;
std::vector<uint32_t> g_bar_waiters;
uint64_t g_bar_site = 0;
bool g_bar_site_set = false;
std::string g_fail;
hipError_t g_last = hipSuccess;
uint64_t g_grids = 0, g_items = 0, g_switches = 0;

// A fault inside a kernel (an out-of-bounds access the GPU might not have
// caught) prints the work-item, the workgroup and a backtrace (resolve the
// frames with llvm-symbolizer / addr2line against libfmx_simt.so).
void on_fault(int sig) {
    char buf[256];
    const int n = snprintf(buf, sizeof buf, "simt: signal %d in work-item %u of workgroup (%u,%u,%u)\n", sig,
                           g_cur ? g_cur->tid : ~0u, g_bid.x, g_bid.y, g_bid.z);
    if (n > 0) (void)!write(2, buf, (size_t)n);
    void *fr[64];
    const int k = backtrace(fr, 64);
    backtrace_symbols_fd(fr, k, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

void init_once() {
    if (g_inited) return;
    g_inited = true;
    static std::vector<uint8_t> alt(1 << 16);
    stack_t ss{};
    ss.ss_sp = alt.data();
    ss.ss_size = alt.size();
    sigaltstack(&ss, nullptr);
    struct sigaction sa{};
    sa.sa_handler = on_fault;
    sa.sa_flags = SA_ONSTACK;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
    if (const char *s = getenv("SIMT_SEED")) g_rng.seed(strtoull(s, nullptr, 0));
    if (const char *y = getenv("SIMT_YIELD")) g_yield = atof(y);
    if (const char *d = getenv("SIMT_DEFER")) simt_defer(atoi(d), 0.25);
}

uint64_t rnd() { return g_rng(); }

void fill_random(void *p, size_t n, std::mt19937_64 &r) {
    uint8_t *b = static_cast<uint8_t *>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = r();
        std::memcpy(b + i, &x, 8);
    }
    if (i < n) {
        const uint64_t x = r();
        std::memcpy(b + i, &x, n - i);
    }
}

void ensure_fibers(uint32_t n) {
    while (g_fibers.size() < n) {
        Fiber f;
        const size_t guard = 4096;
        void *m = mmap(nullptr, kStack + guard, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                       -1, 0);
        if (m == MAP_FAILED) {
            fprintf(stderr, "simt: cannot map a fiber stack\n");
            abort();
        }
        mprotect(m, guard, PROT_NONE);
        f.stack = static_cast<uint8_t *>(m) + guard;
        g_fibers.push_back(std::move(f));
    }
}

void to_scheduler() {
    ++g_switches;
    simt_switch(&g_cur->sp, g_sched_sp);
}

void fail(const std::string &why) {
    if (g_fail.empty()) g_fail = why;
}

void release_block() {
    for (uint32_t t : g_bar_waiters) {
        g_fibers[t].st = kRun;
        g_runnable.push_back(t);
    }
    g_bar_waiters.clear();
    g_arrived = 0;
    g_bar_site_set = false;
}

void release_wave(Wave &W) {
    auto x = std::make_shared<Xfer>();
    for (int l = 0; l < 64; ++l) x->v[l] = ((W.present >> l) & 1) ? W.slot[l] : rnd();
    x->live = W.present;
    for (uint32_t t : W.waiters) {
        g_fibers[t].xfer = x;
        g_fibers[t].st = kRun;
        g_runnable.push_back(t);
    }
    W.waiters.clear();
    W.arrived = 0;
    W.present = 0;
    W.site_set = false;
}

}  // namespace

const dim3 &thread_idx() { return g_tids[g_cur->tid]; }
const dim3 &block_idx() { return g_bid; }
const dim3 &grid_dim() { return g_grid; }
const dim3 &block_dim() { return g_block; }
uint8_t *dyn_lds() { return g_dyn.data(); }
uint32_t lane_id() { return g_cur->lane; }

uint64_t wall_ticks() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count() / 10;
}

void syncthreads() {
    Fiber &f = *g_cur;
    ++f.nbar;
    if (!g_bar_site_set) {
        g_bar_site = f.nbar;
        g_bar_site_set = true;
    } else if (g_bar_site != f.nbar) {
        fail("__syncthreads reached at different barrier counts (divergent barrier)");
    }
    f.st = kBlockBar;
    g_bar_waiters.push_back(f.tid);
    if (++g_arrived == g_alive) release_block();
    to_scheduler();
}

void wave_exchange(uint64_t bits, uint64_t *out, uint64_t *live) {
    Fiber &f = *g_cur;
    Wave &W = g_waves[f.wave];
    ++f.nwave;
    if (!W.site_set) {
        W.site = f.nwave;
        W.site_set = true;
    } else if (W.site != f.nwave) {
        fail("wave operation reached at different counts by the lanes of a wave (divergent)");
    }
    W.slot[f.lane] = bits;
    W.present |= 1ull << f.lane;
    f.st = kWaveBar;
    W.waiters.push_back(f.tid);
    if (++W.arrived == W.alive) release_wave(W);
    to_scheduler();
    std::memcpy(out, f.xfer->v, sizeof(f.xfer->v));
    *live = f.xfer->live;
    f.xfer.reset();
}

void maybe_yield() {
    if (!g_cur) return;
    if (std::uniform_real_distribution<double>(0.0, 1.0)(g_rng) >= g_yield) return;
    g_runnable.push_back(g_cur->tid);
    to_scheduler();
}

void set_last_error(hipError_t e) { g_last = e; }

hipError_t run_grid(dim3 grid, dim3 block, size_t dyn_bytes, const std::function<void()> &body) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    init_once();
    const uint64_t nb = (uint64_t)grid.x * grid.y * grid.z;
    const uint64_t nt = (uint64_t)block.x * block.y * block.z;
    if (nb == 0 || nt == 0 || nt > kMaxItems || grid.x > 0x7fffffffu || dyn_bytes > 160 * 1024)
        return hipErrorInvalidConfiguration;
    ensure_fibers((uint32_t)nt);
    ++g_grids;
    g_grid = grid;
    g_block = block;
    g_body = &body;
    g_tids.resize(nt);
    for (uint32_t t = 0; t < nt; ++t) g_tids[t] = dim3(t % block.x, (t / block.x) % block.y, t / (block.x * block.y));
    // blocks in a random order (simt_block_order(1): in index order)
    std::vector<uint64_t> order(nb);
    for (uint64_t i = 0; i < nb; ++i) order[i] = i;
    if (!g_ordered) std::shuffle(order.begin(), order.end(), g_rng);
    const uint32_t nwaves = (uint32_t)((nt + 63) / 64);
    g_fail.clear();
    for (uint64_t bi : order) {
        g_bid = dim3((uint32_t)(bi % grid.x), (uint32_t)((bi / grid.x) % grid.y), (uint32_t)(bi / ((uint64_t)grid.x * grid.y)));
        if (+__start_simt_lds && +__stop_simt_lds > +__start_simt_lds)
            fill_random(__start_simt_lds, (size_t)(__stop_simt_lds - __start_simt_lds), g_rng);
        g_dyn.resize(dyn_bytes + 16);
        fill_random(g_dyn.data(), g_dyn.size(), g_rng);
        g_waves.assign(nwaves, Wave{});
        g_runnable.clear();
        g_bar_waiters.clear();
        g_arrived = 0;
        g_bar_site_set = false;
        g_alive = (uint32_t)nt;
        for (uint32_t t = 0; t < nt; ++t) {
            Fiber &f = g_fibers[t];
            f.tid = t;
            f.wave = t / 64;
            f.lane = t % 64;
            f.st = kRun;
            f.nbar = f.nwave = 0;
            f.xfer.reset();
            g_waves[f.wave].alive++;
            // fresh stack: six zero registers under simt_fiber_start
            void **top = reinterpret_cast<void **>(f.stack + kStack);
            *--top = nullptr;  // (alignment pad)
            *--top = reinterpret_cast<void *>(&simt_fiber_start);
            for (int r = 0; r < 6; ++r) *--top = nullptr;
            f.sp = top;
            g_runnable.push_back(t);
        }
        while (!g_runnable.empty()) {
            const size_t k = (size_t)(rnd() % g_runnable.size());
            const uint32_t t = g_runnable[k];
            g_runnable[k] = g_runnable.back();
            g_runnable.pop_back();
            g_cur = &g_fibers[t];
            ++g_switches;
            simt_switch(&g_sched_sp, g_cur->sp);
            g_cur = nullptr;
            if (!g_fail.empty()) break;
        }
        if (g_fail.empty() && g_alive != 0) {
            char buf[160];
            snprintf(buf, sizeof buf, "workgroup (%u,%u,%u) cannot finish: %u work-items wait at a barrier (%u arrived)",
                     g_bid.x, g_bid.y, g_bid.z, g_alive, g_arrived);
            fail(buf);
        }
        if (!g_fail.empty()) {
            fprintf(stderr, "simt: launch failed: %s\n", g_fail.c_str());
            g_body = nullptr;
            return hipErrorLaunchFailure;
        }
        g_items += nt;
    }
    g_body = nullptr;
    return hipSuccess;
}

}  // namespace simt

using namespace simt;

extern "C" void simt_fiber_main() {
    (*g_body)();
    Fiber &f = *g_cur;
    f.st = kDone;
    --g_alive;
    Wave &W = g_waves[f.wave];
    --W.alive;
    if (W.arrived > 0 && W.arrived == W.alive) release_wave(W);
    if (g_arrived > 0 && g_arrived == g_alive) release_block();
    simt_switch(&f.sp, g_sched_sp);
    abort();  // (never resumed)
}

extern "C" {
// TEST hooks: reseed the schedule / memory fills, set the atomic switch probability.
void simt_config(uint64_t seed, double yield_p) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    init_once();
    g_rng.seed(seed);
    g_yield = yield_p;
}
// TEST hook (fault injection): the next zeroing memset of exactly `size`
// bytes leaves these words at its start instead of zeros (e.g. a grouped
// launch's key counters left dirty by a launch cut short).
static std::vector<uint32_t> g_memset_fault;
static uint64_t g_memset_fault_size = 0;
void simt_memset_fault(uint64_t size, const uint32_t *words, uint64_t n_words) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_memset_fault.assign(words, words + n_words);
    g_memset_fault_size = size;
}
// TEST hook: workgroups in index order (1), as the GPU dispatches them, or
// shuffled (0, the default).
void simt_block_order(int ordered) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    g_ordered = ordered != 0;
}
void simt_stats(uint64_t *grids, uint64_t *items, uint64_t *switches) {
    *grids = g_grids;
    *items = g_items;
    *switches = g_switches;
}
}

// ---------------------------------------------------------------- host API
namespace {
std::mt19937_64 g_host_rng(0xfeed);
struct Tag {};
struct Pending {
    void *dst;
    std::vector<uint8_t> bytes;
};
std::mutex g_pend_mu;
std::vector<Pending> g_pending;  // staged null-stream H2D copies not landed yet
void land_pending() {
    std::lock_guard<std::mutex> g(g_pend_mu);
    for (Pending &p : g_pending) std::memcpy(p.dst, p.bytes.data(), p.bytes.size());
    g_pending.clear();
}
bool null_stream(hipStream_t s) { return s == nullptr; }
}  // namespace

// ------------------------------------------------------- deferred streams
struct simt_stream {
    std::deque<std::function<void()>> q;  // queued, not run yet (deferred mode)
    uint64_t issued = 0, done = 0;        // operations queued / run so far
    hipError_t err = hipSuccess;          // a deferred kernel's failure, until the next sync
};
struct simt_event {
    simt_stream *s = nullptr;  // null: complete
    uint64_t seq = 0;          // complete once s->done >= seq
};

namespace {
std::recursive_mutex g_q_mu;
bool g_defer = false;
double g_progress = 0.25;  // chance that a host API call runs some queued work
std::mt19937_64 g_q_rng(0xdefe);
std::vector<simt_stream *> g_streams;  // (never freed: events may outlive their stream)
int g_q_depth = 0;

void drain(simt_stream *s, uint64_t upto) {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    ++g_q_depth;
    while (s->done < upto && !s->q.empty()) {
        std::function<void()> f = std::move(s->q.front());
        s->q.pop_front();
        ++s->done;
        f();
    }
    --g_q_depth;
}

void drain_all() {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    for (size_t i = 0; i < g_streams.size(); ++i) drain(g_streams[i], g_streams[i]->issued);
}

// at random points of host API calls: a random stream runs a random prefix of its queue
void maybe_progress() {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    if (!g_defer || g_q_depth || g_streams.empty()) return;
    if (std::uniform_real_distribution<double>(0.0, 1.0)(g_q_rng) >= g_progress) return;
    simt_stream *s = g_streams[g_q_rng() % g_streams.size()];
    if (s->q.empty()) return;
    drain(s, s->done + 1 + g_q_rng() % s->q.size());
}

// run f now (immediate mode, the null stream) or queue it on s
void submit(hipStream_t s, std::function<void()> f) {
    std::unique_lock<std::recursive_mutex> g(g_q_mu);
    if (!g_defer || null_stream(s)) {
        if (s) { ++s->issued; ++s->done; }
        g.unlock();
        f();
        return;
    }
    s->q.push_back(std::move(f));
    ++s->issued;
    maybe_progress();
}
}  // namespace

namespace simt {
hipError_t submit_launch(hipStream_t s, std::function<hipError_t()> launch) {
    {
        std::lock_guard<std::recursive_mutex> g(g_q_mu);
        if (!g_defer || null_stream(s)) {
            if (s) { ++s->issued; ++s->done; }
        } else {
            s->q.push_back([s, launch]() {
                const hipError_t e = launch();
                if (e != hipSuccess && s->err == hipSuccess) s->err = e;
            });
            ++s->issued;
            maybe_progress();
            return hipSuccess;
        }
    }
    return launch();
}
}  // namespace simt

extern "C" {
// TEST hook: deferred streams on / off (from now on; queued work is run first)
// and the chance that a host API call runs some queued work.
void simt_defer(int on, double progress) {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    drain_all();
    g_defer = on != 0;
    g_progress = progress;
}
// TEST hook: the deferred-stream model itself (0 = as specified): a queued
// host-to-device copy reads its source when it runs, a queued device-to-host
// copy has not written its destination before the host synchronises, an
// event orders both.
int simt_selftest_defer() {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    const bool was = g_defer;
    const double p = g_progress;
    g_defer = true;
    g_progress = 0.0;
    int bad = 0;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    void *dv = nullptr;
    hipMallocRaw(&dv, 64);
    uint8_t *d = static_cast<uint8_t *>(dv), h[64], o[64];
    std::memset(h, 1, 64);
    hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s);
    std::memset(h, 2, 64);  // reused before the copy has run
    hipStreamSynchronize(s);
    bad |= d[0] != 2 ? 1 : 0;
    std::memset(o, 0, 64);
    hipMemcpyAsync(o, d, 64, hipMemcpyDeviceToHost, s);
    bad |= o[63] != 0 ? 2 : 0;  // not written before the host waits for it
    hipEvent_t e;
    hipEventCreate(&e);
    hipEventRecord(e, s);
    bad |= s->done == s->issued ? 4 : 0;
    hipEventSynchronize(e);
    bad |= o[63] != 2 ? 8 : 0;
    hipEventDestroy(e);
    g_defer = was;
    g_progress = p;
    free(dv);
    return bad;
}
}

namespace simt {
// before a launch: on the null stream every staged copy lands first; on
// another stream each lands with probability 1/2
void land_before_launch(hipStream_t s) {
    if (null_stream(s)) {
        land_pending();
        return;
    }
    std::lock_guard<std::mutex> g(g_pend_mu);
    std::vector<Pending> keep;
    for (Pending &p : g_pending) {
        if (g_rng() & 1) std::memcpy(p.dst, p.bytes.data(), p.bytes.size());
        else keep.push_back(std::move(p));
    }
    g_pending.swap(keep);
}
}  // namespace simt

hipError_t hipGetLastError() {
    const hipError_t e = g_last;
    g_last = hipSuccess;
    return e;
}
const char *hipGetErrorString(hipError_t e) {
    switch (e) {
        case hipSuccess: return "hipSuccess";
        case hipErrorInvalidValue: return "hipErrorInvalidValue";
        case hipErrorOutOfMemory: return "hipErrorOutOfMemory";
        case hipErrorInvalidConfiguration: return "hipErrorInvalidConfiguration";
        case hipErrorLaunchFailure: return "hipErrorLaunchFailure";
        default: return "hipError";
    }
}
hipError_t hipMallocRaw(void **p, size_t n) {
    *p = nullptr;
    void *m = aligned_alloc(256, (std::max<size_t>(n, 1) + 255) & ~size_t(255));
    if (!m) return hipErrorOutOfMemory;
    {
        std::lock_guard<std::mutex> g(g_rng_mu);
        fill_random(m, n, g_host_rng);
    }
    *p = m;
    return hipSuccess;
}
hipError_t hipFree(void *p) {
    drain_all();     // (hipFree synchronises the device)
    land_pending();
    free(p);
    return hipSuccess;
}
hipError_t hipHostMallocRaw(void **p, size_t n, unsigned) { return hipMallocRaw(p, n); }
hipError_t hipHostFree(void *p) { return hipFree(p); }
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind k) {
    land_pending();  // (a null-stream operation: earlier null-stream work is done)
    if (n && k == hipMemcpyHostToDevice) {  // staged; lands later (see the header)
        std::lock_guard<std::mutex> g(g_pend_mu);
        g_pending.push_back(Pending{d, std::vector<uint8_t>(static_cast<const uint8_t *>(s),
                                                             static_cast<const uint8_t *>(s) + n)});
        return hipSuccess;
    }
    if (n) std::memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t st) {
    if (null_stream(st)) return hipMemcpy(d, s, n, k);
    submit(st, [d, s, n]() {
        if (n) std::memmove(d, s, n);
    });
    return hipSuccess;
}
hipError_t hipMemcpyPeer(void *d, int, const void *s, int, size_t n) { return hipMemcpy(d, s, n, hipMemcpyDefault); }
static void memset_or_fault(void *d, int v, size_t n) {
    if (n) std::memset(d, v, n);
    if (v == 0 && g_memset_fault_size && n == g_memset_fault_size) {
        std::memcpy(d, g_memset_fault.data(), std::min<size_t>(n, 4 * g_memset_fault.size()));
        g_memset_fault_size = 0;
    }
}
hipError_t hipMemset(void *d, int v, size_t n) {
    land_pending();
    memset_or_fault(d, v, n);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t st) {
    if (null_stream(st)) return hipMemset(d, v, n);
    submit(st, [d, v, n]() { memset_or_fault(d, v, n); });
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    *s = new simt_stream;
    g_streams.push_back(*s);
    return hipSuccess;
}
hipError_t hipStreamCreate(hipStream_t *s) { return hipStreamCreateWithFlags(s, 0); }
hipError_t hipStreamDestroy(hipStream_t s) {
    if (s) drain(s, s->issued);  // (its work completes; the record stays for events that name it)
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    if (null_stream(s)) {
        land_pending();
        return hipSuccess;
    }
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    drain(s, s->issued);
    const hipError_t e = s->err;
    s->err = hipSuccess;
    return e;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
    if (!e || !e->s) return hipSuccess;
    simt_stream *es = e->s;
    const uint64_t seq = e->seq;
    if (null_stream(s)) {
        drain(es, seq);
        return hipSuccess;
    }
    submit(s, [es, seq]() { drain(es, seq); });  // (s runs on once es has reached the event)
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t *e) {
    *e = new simt_event;
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    if (null_stream(s)) {
        e->s = nullptr;
        e->seq = 0;
        return hipSuccess;
    }
    e->s = s;
    e->seq = s->issued + 1;
    submit(s, [] {});
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
    if (e && e->s) drain(e->s, e->seq);
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
    std::lock_guard<std::recursive_mutex> g(g_q_mu);
    if (!e || !e->s || e->s->done >= e->seq) return hipSuccess;
    if (g_q_rng() & 1) return hipErrorNotReady;
    drain(e->s, e->seq);
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b) {
    if (hipEventQuery(a) != hipSuccess || hipEventQuery(b) != hipSuccess) return hipErrorNotReady;
    *ms = 0.001f;
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    return hipSuccess;
}
hipError_t hipDeviceSynchronize() {
    drain_all();
    land_pending();
    return hipSuccess;
}
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidValue; }
hipError_t hipGetDevice(int *d) {
    *d = 0;
    return hipSuccess;
}
hipError_t hipGetDeviceCount(int *n) {
    *n = 1;
    return hipSuccess;
}
hipError_t hipMemGetInfo(size_t *f, size_t *t) {
    *f = 16ull << 30;
    *t = 32ull << 30;
    return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t a, int) {
    *v = a == hipDeviceAttributeWallClockRate ? 100000 : 256;  // (kHz)
    return hipSuccess;
}
