// Does a kernel pay for fetching its code on every launch?  k_emit of one
// 100k batch (98 workgroups, 12.5 KB of code) takes 13 us in the round-5
// trace, a 98-workgroup copy kernel of a few hundred bytes 2.6 us.  Two
// kernels of 98 x 256 threads each run a long straight-line body (NOPS
// dependent integer ops spread over ~12 KB of code) and store one word:
//   AAAA  the same kernel back to back (its code warm after the first launch)
//   ABAB  two different kernels alternating (each launch follows the other)
//   tiny  the copy-sized kernel, for the floor
// rocprofv3 --kernel-trace --stats gives the kernel durations.
#include <hip/hip_runtime.h>

#include <cstdio>

#ifndef NOPS
#define NOPS 1500
#endif

template <int SALT>
__global__ __launch_bounds__(256) void k_long(unsigned *out, unsigned seed) {
    unsigned x = seed + threadIdx.x + SALT;
#pragma unroll
    for (int i = 0; i < NOPS; ++i) {
        x ^= x >> 13;
        x = x * 0x5bd1e995u + (unsigned)(i ^ SALT);
    }
    out[blockIdx.x * 256u + threadIdx.x] = x;
}
__global__ __launch_bounds__(256) void k_tiny(unsigned *out, unsigned seed) {
    out[blockIdx.x * 256u + threadIdx.x] = seed + threadIdx.x;
}

int main() {
    const unsigned grid = 98;
    unsigned *out;
    if (hipMalloc(&out, grid * 256 * 4)) return 2;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            hipEventRecord(a, s);
            for (int it = 0; it < 1000; ++it) {
                if (mode == 0) hipLaunchKernelGGL(k_long<0>, dim3(grid), dim3(256), 0, s, out, (unsigned)it);
                if (mode == 1) {
                    if (it & 1) hipLaunchKernelGGL(k_long<1>, dim3(grid), dim3(256), 0, s, out, (unsigned)it);
                    else hipLaunchKernelGGL(k_long<2>, dim3(grid), dim3(256), 0, s, out, (unsigned)it);
                }
                if (mode == 2) hipLaunchKernelGGL(k_tiny, dim3(grid), dim3(256), 0, s, out, (unsigned)it);
            }
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const char *names[3] = {"AAAA", "ABAB", "tiny"};
            if (rep == 1) printf("{\"mode\": \"%s\", \"us_per_launch\": %.3f}\n", names[mode], ms * 1e3 / 1000);
        }
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
