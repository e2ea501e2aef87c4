// Microbenchmark: dependent chains of random 64-B record reads where each
// lane reads NC (1..4) of its record's 16-B chunks (NC dwordx4 loads to the
// same line).  Question it answers: does the rank query's chunk count per
// record (C2's interleaved record: 2 chunks for c < 2, 3 otherwise) set the
// line rate?  Footprints 1 GB (C2's occ records) and 4 GB.
// Build: hipcc -O3 --offload-arch=gfx950 chunks.hip -o chunks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using V4 = uint32_t __attribute__((ext_vector_type(4)));

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

template <int NC>
__global__ __launch_bounds__(256) void chase(const uint8_t *__restrict__ b, uint64_t recs, uint64_t chains, int R,
                                             uint64_t seed, uint32_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= chains) return;
    uint64_t pos = mix(t ^ seed) % recs;
    uint32_t acc = 0;
    for (int r = 0; r < R; ++r) {
        const V4 *p = reinterpret_cast<const V4 *>(b + pos * 64);
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const V4 v = p[i];
            x ^= v[i & 3];
        }
        acc ^= x;
        pos = mix(pos ^ x) % recs;
    }
    if (acc == 42u) out[0] = acc;
}

template <int NC>
static void run(const uint8_t *b, uint64_t bytes, uint64_t chains, uint32_t *out, hipEvent_t e0, hipEvent_t e1) {
    const int R = 8;
    const uint64_t recs = bytes / 64;
    const uint32_t grid = (uint32_t)((chains + 255) / 256);
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0));
        chase<NC><<<grid, 256>>>(b, recs, chains, R, it * 977, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
    }
    printf("{\"chunks\": %d, \"footprint_gb\": %.1f, \"chains\": %llu, \"ms\": %.4f, \"grecords_per_s\": %.2f}\n", NC,
           bytes / 1073741824.0, (unsigned long long)chains, best, (double)chains * R / (best * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t maxb = 4ull << 30;
    uint8_t *b;
    CK(hipMalloc(&b, maxb));
    fill<<<4096, 256>>>((uint64_t *)b, maxb / 8);
    CK(hipDeviceSynchronize());
    for (uint64_t bytes : {1ull << 30, 4ull << 30})
        for (uint64_t chains : {800000ull, 2000000ull}) {
            run<1>(b, bytes, chains, out, e0, e1);
            run<2>(b, bytes, chains, out, e0, e1);
            run<3>(b, bytes, chains, out, e0, e1);
            run<4>(b, bytes, chains, out, e0, e1);
        }
    return 0;
}
