// Microbenchmark: dependent random-load latency on one MI355X versus the size
// of the buffer the loads land in (TLB reach) and the number of chains in
// flight.  Each lane chases R pointers through uniformly random 64-B lines of
// a buffer of S bytes; ns per step = kernel time / R.  Few lanes: unloaded
// latency; 100k lanes: the k_locate regime (one chain per pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ void fill(uint64_t *b, uint64_t words) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = mix(i);
}

__global__ void chase(const uint64_t *__restrict__ b, uint64_t mask, uint64_t n, int R, uint64_t seed, uint64_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t pos = mix(t ^ seed) & mask;
    for (int r = 0; r < R; ++r) pos = (__builtin_nontemporal_load(&b[pos * 8]) >> 7) & mask;
    if (pos == 42) out[0] = pos;
}

int main() {
    const uint64_t sizes_mb[] = {64, 1024, 8192, 32768, 65536};
    const uint64_t lanes[] = {64, 4096, 100000};
    const int R = 64;
    uint64_t *out;
    CK(hipMalloc(&out, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint64_t mb : sizes_mb) {
        const uint64_t bytes = mb << 20, words = bytes / 8, lines = bytes / 64;
        uint64_t *b;
        if (hipMalloc(&b, bytes) != hipSuccess) { printf("alloc %llu MB failed\n", (unsigned long long)mb); continue; }
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, words);
        CK(hipDeviceSynchronize());
        for (uint64_t n : lanes) {
            const uint64_t mask = lines - 1;
            const dim3 grid((unsigned)((n + 255) / 256));
            const dim3 block(n < 256 ? (unsigned)n : 256u);
            hipLaunchKernelGGL(chase, grid, block, 0, 0, b, mask, n, R, 1ull, out);
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(chase, grid, block, 0, 0, b, mask, n, R, 100ull + rep, out);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("{\"buffer_mb\": %llu, \"lanes\": %llu, \"steps\": %d, \"ms\": %.4f, \"ns_per_step\": %.1f, "
                   "\"glines_per_s\": %.2f}\n",
                   (unsigned long long)mb, (unsigned long long)n, R, best, best * 1e6 / R,
                   (double)n * R / (best * 1e-3) / 1e9);
            fflush(stdout);
        }
        CK(hipFree(b));
    }
    return 0;
}
