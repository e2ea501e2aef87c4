// Microbenchmark: what one random HBM record read costs by its shape — the
// question behind the interleaved occ record layout.  Each lane reads R
// records at uniformly random G-byte aligned slots of an S-byte buffer, each
// record as A 16-B loads (dwordx4) at offsets 0, 16, ... (all A loads of a
// record issued together, records independent).  Prints records/s and
// 16-B accesses/s.  Build: hipcc -O3 --offload-arch=gfx950 shapes.hip -o shapes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

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

// R records per lane, each A dwordx4 loads; G = record slot bytes.  Records
// are a dependent chain (the next slot comes from the loaded words), as in the
// LF loop.
template <int A, int G>
__global__ __launch_bounds__(256) void chase(const uint8_t *__restrict__ b, uint64_t slots, uint64_t n, int R,
                                             uint64_t seed, uint64_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t pos = mix(t ^ seed) % slots;
    uint32_t acc = 0;
    for (int r = 0; r < R; ++r) {
        const V4 *p = reinterpret_cast<const V4 *>(b + pos * G);
        V4 v[A];
#pragma unroll
        for (int a = 0; a < A; ++a) v[a] = p[a];
        uint32_t x = 0;
#pragma unroll
        for (int a = 0; a < A; ++a) x ^= v[a][0] ^ v[a][3];
        acc ^= x;
        pos = mix(pos ^ x) % slots;
    }
    if (acc == 42u) out[0] = acc;
}

template <int A, int G>
static void run(const uint8_t *b, uint64_t bytes, uint64_t n, uint64_t *out, hipEvent_t e0, hipEvent_t e1,
                double gb) {
    const int R = 8;
    const uint64_t slots = bytes / G;
    const uint32_t grid = (uint32_t)((n + 255) / 256);
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0));
        chase<A, G><<<grid, 256>>>(b, slots, n, R, it * 977, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
    }
    const double recs = (double)n * R / (best * 1e-3);
    printf("{\"buffer_gb\": %.3f, \"lanes\": %llu, \"slot_bytes\": %d, \"loads_per_record\": %d, \"ms\": %.4f, "
           "\"grecords_per_s\": %.2f, \"gaccesses_per_s\": %.2f}\n",
           gb, (unsigned long long)n, G, A, best, recs / 1e9, recs * A / 1e9);
    fflush(stdout);
}

int main(int argc, char **argv) {
    // argv: buffer sizes in MB (default 1024 8192); a size list selects the
    // one-record-per-line shapes only (footprint sweep)
    uint64_t *out;
    CK(hipMalloc(&out, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> sizes_mb = {1024, 8192};
    if (argc > 1) {
        sizes_mb.clear();
        for (int i = 1; i < argc; ++i) sizes_mb.push_back(strtoull(argv[i], nullptr, 10));
    }
    const uint64_t lanes[] = {500000, 2000000};
    for (uint64_t mb : sizes_mb) {
        const uint64_t bytes = mb << 20;
        const double gb = (double)mb / 1024.0;
        uint8_t *b;
        CK(hipMalloc(&b, bytes));
        fill<<<4096, 256>>>((uint64_t *)b, bytes / 8);
        CK(hipDeviceSynchronize());
        for (uint64_t n : lanes) {
            if (argc > 1) {
                run<1, 128>(b, bytes, n, out, e0, e1, gb);
                run<2, 64>(b, bytes, n, out, e0, e1, gb);
                continue;
            }
            run<1, 64>(b, bytes, n, out, e0, e1, (double)gb);
            run<2, 64>(b, bytes, n, out, e0, e1, (double)gb);
            run<4, 64>(b, bytes, n, out, e0, e1, (double)gb);
            run<1, 128>(b, bytes, n, out, e0, e1, (double)gb);
            run<2, 128>(b, bytes, n, out, e0, e1, (double)gb);
            run<4, 128>(b, bytes, n, out, e0, e1, (double)gb);
            run<8, 128>(b, bytes, n, out, e0, e1, (double)gb);
            run<1, 256>(b, bytes, n, out, e0, e1, (double)gb);
        }
        CK(hipFree(b));
    }
    return 0;
}
