// What a large by-value kernel argument costs a small kernel (k_emit of one
// 100k batch: 98 workgroups, ~25 KB LocateGroup argument, 12-14 us in the
// round-5 trace where a trivial kernel boundary is ~2 us).  Four kernels of
// 98 x 256 threads, each reading one 16-B record per lane from a buffer and
// writing it back, differing only in how they get their pointers:
//   small    pointers as plain arguments (~40 B of kernarg)
//   big_s    the same pointers inside a 26 KB struct passed by value, read
//            with scalar loads (a workgroup-uniform field, as k_emit does)
//   big_v    the same, plus a per-lane read of the struct (k_emit's sC copy of
//            QueryArgs::C: vector loads from the kernarg segment)
//   table    the 26 KB struct in device memory, its pointer the argument
// Each runs 2,000 times back to back on one stream; rocprofv3 --kernel-trace
// --stats gives the per-kernel durations, hipEvents the per-launch wall, the
// host clock around the launch loop the host's enqueue cost per launch.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

struct Entry {
    const uint4 *src;
    uint4 *dst;
    unsigned long long n, pad[8];
};
struct Big {
    Entry e[256];
    unsigned int first[256], second[256];
    unsigned long long c[65];
};

__global__ __launch_bounds__(256) void k_small(const uint4 *src, uint4 *dst, unsigned long long n) {
    const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
    if (i < n) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void k_big_s(const Big g) {
    const Entry &E = g.e[0];
    const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
    if (i < E.n) E.dst[i] = E.src[i];
}
__global__ __launch_bounds__(256) void k_big_v(const Big g) {
    __shared__ unsigned long long sc[65];
    if (threadIdx.x < 65) sc[threadIdx.x] = g.c[threadIdx.x];
    __syncthreads();
    const Entry &E = g.e[0];
    const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
    if (i < E.n) {
        uint4 v = E.src[i];
        v.x += (unsigned)sc[threadIdx.x & 63];
        E.dst[i] = v;
    }
}
__global__ __launch_bounds__(256) void k_table(const Big *__restrict__ g) {
    const Entry &E = g->e[0];
    const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
    if (i < E.n) E.dst[i] = E.src[i];
}

int main() {
    const unsigned long long n = 100000;
    const unsigned grid = (unsigned)((n + 255) / 256 + 3) / 4;  // 98, like k_emit's 4 tiles per workgroup
    uint4 *src, *dst;
    Big *d_big;
    if (hipMalloc(&src, n * 16) || hipMalloc(&dst, n * 16) || hipMalloc(&d_big, sizeof(Big))) return 2;
    hipMemset(src, 1, n * 16);
    static Big h{};
    h.e[0] = Entry{src, dst, grid * 256ull, {}};
    for (int i = 0; i < 65; ++i) h.c[i] = i;
    hipMemcpy(d_big, &h, sizeof(Big), hipMemcpyHostToDevice);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[4] = {"small", "big_s", "big_v", "table"};
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 4; ++k) {
            hipEventRecord(a, s);
            const auto h0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 2000; ++it) {
                if (k == 0) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, src, dst, grid * 256ull);
                if (k == 1) hipLaunchKernelGGL(k_big_s, dim3(grid), dim3(256), 0, s, h);
                if (k == 2) hipLaunchKernelGGL(k_big_v, dim3(grid), dim3(256), 0, s, h);
                if (k == 3) hipLaunchKernelGGL(k_table, dim3(grid), dim3(256), 0, s, (const Big *)d_big);
            }
            const double host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 1)
                printf("{\"kernel\": \"%s\", \"kernarg_bytes\": %zu, \"us_per_launch\": %.3f, "
                       "\"host_enqueue_us_per_launch\": %.3f}\n",
                       names[k], k == 0 ? sizeof(void *) * 3 : k == 3 ? sizeof(void *) : sizeof(Big), ms * 1e3 / 2000,
                       host_us / 2000);
        }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
