// TEST INFRASTRUCTURE — a host-only stand-in for <hip/hip_runtime.h> under
// which the engine's own sources (sview-fmindex_amd/csrc: fmx_api.cpp,
// fmx_query.hip, fmx_layout.hip, fmx_kernels.hpp, fmx_device.hpp) compile as
// plain C++ and run on the CPU (tests/simt/libfmx_simt.so).  Kernels run as
// one fiber per work-item (tests/simt/simt_rt.cpp): workgroups in a shuffled
// order, the work-items of a workgroup interleaved at random between
// barriers, wave operations (__shfl*, __all, readfirstlane) exchanged per
// 64-lane wave, every atomic a possible switch point, LDS and hipMalloc'd
// memory filled with random bytes, a null-stream host-to-device hipMemcpy
// landing late for work on other streams.  A schedule-dependent result, a
// read of memory nobody wrote (or nobody waited for), a barrier some
// work-items skip: each shows up as a wrong answer or a reported deadlock on
// the CPU.  Not a product path: only
// tests/ load the library.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <tuple>
#include <type_traits>
#include <utility>

#define __host__
#define __device__
#define __global__
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
// LDS: one static per variable (workgroups run one at a time), all in one
// section that simt_rt fills with random bytes before every workgroup
#define __shared__ static __attribute__((section("simt_lds")))
#define FMX_DYN_LDS(name) uint8_t *name = ::simt::dyn_lds()

struct dim3 {
    uint32_t x, y, z;
    constexpr dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};

enum hipError_t {
    hipSuccess = 0,
    hipErrorInvalidValue = 1,
    hipErrorOutOfMemory = 2,
    hipErrorInvalidConfiguration = 9,
    hipErrorNotReady = 600,
    hipErrorLaunchFailure = 719,
};
enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4
};
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 63, hipDeviceAttributeWallClockRate = 90 };
enum hipStreamCaptureStatus { hipStreamCaptureStatusNone = 0, hipStreamCaptureStatusActive = 1 };
typedef struct simt_stream *hipStream_t;
typedef struct simt_event *hipEvent_t;
#define hipStreamNonBlocking 1u
#define hipStreamDefault 0u
#define hipEventDisableTiming 2u
#define hipEventDefault 0u
#define hipHostMallocDefault 0u

namespace simt {

// ---------------------------------------------------------------- device side
const dim3 &thread_idx();
const dim3 &block_idx();
const dim3 &grid_dim();
const dim3 &block_dim();
uint8_t *dyn_lds();
void syncthreads();
void maybe_yield();  // an atomic's switch point
// wave exchange: every live lane of the wave contributes `bits`; returns the
// 64 slots (dead / absent lanes hold random bits) and the live-lane mask
void wave_exchange(uint64_t bits, uint64_t *out, uint64_t *live);
uint32_t lane_id();
uint64_t wall_ticks();  // 100 MHz, as the GPU's wall clock

template <class T>
inline uint64_t to_bits(T v) {
    static_assert(sizeof(T) <= 8 && std::is_trivially_copyable_v<T>);
    uint64_t b = 0;
    std::memcpy(&b, &v, sizeof(T));
    return b;
}
template <class T>
inline T from_bits(uint64_t b) {
    T v;
    std::memcpy(&v, &b, sizeof(T));
    return v;
}
template <class T>
inline T shfl_from(T v, uint32_t (*src)(uint32_t lane, uint32_t arg), uint32_t arg) {
    uint64_t slots[64], live;
    wave_exchange(to_bits(v), slots, &live);
    return from_bits<T>(slots[src(lane_id(), arg) & 63u]);
}
inline uint32_t src_abs(uint32_t, uint32_t a) { return a; }
inline uint32_t src_up(uint32_t l, uint32_t d) { return l >= d ? l - d : l; }
inline uint32_t src_xor(uint32_t l, uint32_t m) { return l ^ m; }

template <class T>
inline T readfirstlane(T v) {
    uint64_t slots[64], live;
    wave_exchange(to_bits(v), slots, &live);
    return from_bits<T>(slots[__builtin_ctzll(live)]);
}

template <class T>
inline T atomic_add(T *p, T v) {
    const T old = *p;
    *p = old + v;
    maybe_yield();
    return old;
}
template <class T>
inline T atomic_or(T *p, T v) {
    const T old = *p;
    *p = old | v;
    maybe_yield();
    return old;
}

// ---------------------------------------------------------------- launches
hipError_t run_grid(dim3 grid, dim3 block, size_t dyn_lds_bytes, const std::function<void()> &body);
void set_last_error(hipError_t e);
void land_before_launch(hipStream_t s);

// Runs `launch` now, or (deferred streams, simt_defer) queues it on s:
// then a failure is reported by the next synchronisation of s, as on the GPU.
hipError_t submit_launch(hipStream_t s, std::function<hipError_t()> launch);

template <class... KP, class... A>
hipError_t launch_kernel(void (*k)(KP...), dim3 g, dim3 b, size_t lds, hipStream_t s, A &&...a) {
    static_assert(sizeof...(KP) == sizeof...(A), "kernel argument count");
    auto args = std::make_shared<std::tuple<std::decay_t<KP>...>>(std::forward<A>(a)...);
    const hipError_t e = submit_launch(s, [k, args, g, b, lds, s]() {
        land_before_launch(s);
        return run_grid(g, b, lds, [k, args]() { std::apply(k, *args); });
    });
    if (e != hipSuccess) set_last_error(e);
    return e;
}

}  // namespace simt

#define threadIdx (::simt::thread_idx())
#define blockIdx (::simt::block_idx())
#define gridDim (::simt::grid_dim())
#define blockDim (::simt::block_dim())
#define __syncthreads() ::simt::syncthreads()
#define __builtin_amdgcn_readfirstlane(x) ::simt::readfirstlane(x)
#define hipLaunchKernelGGL(K, G, B, L, S, ...) (void)::simt::launch_kernel(K, G, B, L, S, __VA_ARGS__)

template <class T>
inline T __shfl(T v, int src, int = 64) { return ::simt::shfl_from(v, ::simt::src_abs, (uint32_t)src); }
template <class T>
inline T __shfl_up(T v, unsigned d, int = 64) { return ::simt::shfl_from(v, ::simt::src_up, d); }
template <class T>
inline T __shfl_xor(T v, int m, int = 64) { return ::simt::shfl_from(v, ::simt::src_xor, (uint32_t)m); }
inline int __all(int p) {
    uint64_t slots[64], live;
    ::simt::wave_exchange(p != 0, slots, &live);
    for (int l = 0; l < 64; ++l)
        if (((live >> l) & 1) && !slots[l]) return 0;
    return 1;
}
inline uint32_t atomicAdd(uint32_t *p, uint32_t v) { return ::simt::atomic_add(p, v); }
inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) { return ::simt::atomic_add(p, v); }
inline uint64_t atomicAdd(uint64_t *p, uint64_t v) { return ::simt::atomic_add(p, v); }
inline int atomicAdd(int *p, int v) { return ::simt::atomic_add(p, v); }
inline uint32_t atomicOr(uint32_t *p, uint32_t v) { return ::simt::atomic_or(p, v); }

// k_locate's hand-off (fmx_kernels.hpp, FMX_HANDOFF): plain accesses, each a
// possible switch point; the wall clock in 10 ns ticks.  Workgroups run one at
// a time, so a workgroup that waits for another still to run waits out its
// bound (simt_block_order(1): workgroups in index order, as the GPU
// dispatches them).
#define FMX_HANDOFF 1
inline uint64_t ld_agent(const uint64_t *p) {
    ::simt::maybe_yield();
    return __atomic_load_n(p, __ATOMIC_RELAXED);
}
inline void st_agent(uint64_t *p, uint64_t v) {
    __atomic_store_n(p, v, __ATOMIC_RELAXED);
    ::simt::maybe_yield();
}
inline void st_agent32(uint32_t *p, uint32_t v) {
    __atomic_store_n(p, v, __ATOMIC_RELAXED);
    ::simt::maybe_yield();
}
inline void drain_stores() {}
inline void poll_pause() { ::simt::maybe_yield(); }
inline void after_poll() {}
inline uint64_t wall_ticks() { return ::simt::wall_ticks(); }

// ---------------------------------------------------------------- host API
hipError_t hipGetLastError();
const char *hipGetErrorString(hipError_t e);
hipError_t hipMallocRaw(void **p, size_t n);
template <class T>
inline hipError_t hipMalloc(T **p, size_t n) { return hipMallocRaw(reinterpret_cast<void **>(p), n); }
hipError_t hipFree(void *p);
hipError_t hipHostMallocRaw(void **p, size_t n, unsigned flags);
template <class T>
inline hipError_t hipHostMalloc(T **p, size_t n, unsigned flags = 0) {
    return hipHostMallocRaw(reinterpret_cast<void **>(p), n, flags);
}
hipError_t hipHostFree(void *p);
hipError_t hipMemcpy(void *dst, const void *src, size_t n, hipMemcpyKind k);
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s = nullptr);
hipError_t hipMemcpyPeer(void *dst, int ddev, const void *src, int sdev, size_t n);
hipError_t hipMemset(void *dst, int v, size_t n);
hipError_t hipMemsetAsync(void *dst, int v, size_t n, hipStream_t s = nullptr);
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned flags);
hipError_t hipStreamCreate(hipStream_t *s);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
inline hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus *st) {
    *st = hipStreamCaptureStatusNone;
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned flags = 0);
hipError_t hipEventCreate(hipEvent_t *e);
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned flags);
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s = nullptr);
hipError_t hipEventSynchronize(hipEvent_t e);
hipError_t hipEventQuery(hipEvent_t e);
hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b);
hipError_t hipEventDestroy(hipEvent_t e);
hipError_t hipDeviceSynchronize();
hipError_t hipSetDevice(int d);
hipError_t hipGetDevice(int *d);
hipError_t hipGetDeviceCount(int *n);
hipError_t hipMemGetInfo(size_t *free_b, size_t *total_b);
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t a, int dev);
template <class F>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int *n, F, int, size_t) {
    *n = 2;
    return hipSuccess;
}
