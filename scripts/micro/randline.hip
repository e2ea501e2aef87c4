// Microbenchmark: the random-line request rate of one MI355X — the ceiling a
// dependent-gather kernel like k_locate runs against.  Each lane makes R
// 8-byte loads at uniformly random 64-B lines of a buffer of S bytes, either
// independent (addresses from a hash, all in flight at once) or dependent
// (each address from the previous load's value: a pointer chase, like the LF
// loop).  Prints lines/s and the equivalent GB/s at 64 B per line.
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

template <int R>
__global__ void indep(const uint64_t *__restrict__ b, uint64_t mask, uint64_t n, uint64_t seed, uint64_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t x = mix(t ^ seed), acc = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc ^= b[((x >> 7) & mask) * 8];
        x = mix(x);
    }
    if (acc == 42) out[0] = acc;
}

template <int R>
__global__ void dep(const uint64_t *__restrict__ b, uint64_t mask, uint64_t n, uint64_t seed, uint64_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t pos = mix(t ^ seed) & mask;
    for (int r = 0; r < R; ++r) pos = (b[pos * 8] >> 7) & mask;
    if (pos == 42) out[0] = pos;
}

int main(int argc, char **argv) {
    const int R = 8;
    uint64_t sizes_gb[] = {1, 8, 32, 128};
    uint64_t threads[] = {100000, 1000000, 4000000};
    uint64_t *out;
    CK(hipMalloc(&out, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint64_t gb : sizes_gb) {
        const uint64_t bytes = gb << 30, words = bytes / 8, lines = bytes / 64;
        uint64_t *b;
        if (hipMalloc(&b, bytes) != hipSuccess) { printf("alloc %llu GB failed\n", (unsigned long long)gb); continue; }
        fill<<<4096, 256>>>(b, words);
        CK(hipDeviceSynchronize());
        for (uint64_t n : threads) {
            for (int kind = 0; kind < 2; ++kind) {
                const uint32_t grid = (uint32_t)((n + 255) / 256);
                float best = 1e30f;
                for (int it = 0; it < 6; ++it) {
                    CK(hipEventRecord(e0));
                    if (kind == 0) indep<R><<<grid, 256>>>(b, lines - 1, n, it * 977, out);
                    else dep<R><<<grid, 256>>>(b, lines - 1, n, it * 977, out);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (it > 0 && ms < best) best = ms;
                }
                const double rate = (double)n * R / (best * 1e-3);
                printf("{\"buffer_gb\": %llu, \"lanes\": %llu, \"loads_per_lane\": %d, \"kind\": \"%s\", "
                       "\"ms\": %.4f, \"glines_per_s\": %.2f, \"gbps_at_64B\": %.0f}\n",
                       (unsigned long long)gb, (unsigned long long)n, R, kind ? "dependent" : "independent", best,
                       rate * 1e-9, rate * 64e-9);
            }
        }
        CK(hipFree(b));
    }
    return 0;
}
