// Microbenchmark: can a random 64-B record be fetched from HBM as one 64-B
// request instead of a 128-B line?  Dependent chains of random record reads
// over a 4 GB buffer, in four shapes:
//   lane   : each lane reads its record's first 16 B (one dwordx4)
//   lane4  : each lane reads its whole 64-B record (four dwordx4)
//   quad   : four consecutive lanes read one record's four 16-B chunks
//            together (one coalesced 64-B access per quad)
// each with plain or non-temporal (nt) loads.  Prints records/s; run under
// rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum to see the
// request sizes.  Build: hipcc -O3 --offload-arch=gfx950 fetch64.hip -o fetch64
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

template <bool NT>
__device__ __forceinline__ V4 ld(const V4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// SHAPE 0: lane, 1: lane4, 2: quad
template <int SHAPE, bool NT>
__global__ __launch_bounds__(256) void chase(const uint8_t *__restrict__ b, uint64_t recs, uint64_t chains, int R,
                                             uint64_t seed, uint32_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t chain = SHAPE == 2 ? t / 4 : t;
    if (chain >= chains) return;
    const uint32_t sub = SHAPE == 2 ? (uint32_t)(t & 3) : 0u;
    uint64_t pos = mix(chain ^ seed) % recs;
    uint32_t acc = 0;
    for (int r = 0; r < R; ++r) {
        const V4 *p = reinterpret_cast<const V4 *>(b + pos * 64);
        uint32_t x;
        if constexpr (SHAPE == 0) {
            const V4 v = ld<NT>(p);
            x = v[0] ^ v[3];
        } else if constexpr (SHAPE == 1) {
            const V4 v0 = ld<NT>(p), v1 = ld<NT>(p + 1), v2 = ld<NT>(p + 2), v3 = ld<NT>(p + 3);
            x = v0[0] ^ v1[1] ^ v2[2] ^ v3[3];
        } else {
            const V4 v = ld<NT>(p + sub);
            x = v[0] ^ v[3];
            // the quad's four chunks combined (every lane gets the record's hash)
            x ^= __shfl_xor(x, 1);
            x ^= __shfl_xor(x, 2);
        }
        acc ^= x;
        pos = mix(pos ^ x) % recs;
    }
    if (acc == 42u) out[0] = acc;
}

template <int SHAPE, bool NT>
static void run(const uint8_t *b, uint64_t bytes, uint64_t chains, uint32_t *out, hipEvent_t e0, hipEvent_t e1) {
    const int R = 8;
    const uint64_t recs = bytes / 64;
    const uint64_t threads = SHAPE == 2 ? chains * 4 : chains;
    const uint32_t grid = (uint32_t)((threads + 255) / 256);
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0));
        chase<SHAPE, NT><<<grid, 256>>>(b, recs, chains, R, it * 977, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
    }
    const char *names[] = {"lane16", "lane64", "quad64"};
    printf("{\"shape\": \"%s\", \"nt\": %d, \"chains\": %llu, \"ms\": %.4f, \"grecords_per_s\": %.2f}\n", names[SHAPE],
           NT ? 1 : 0, (unsigned long long)chains, best, (double)chains * R / (best * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t bytes = 4ull << 30;
    uint8_t *b;
    CK(hipMalloc(&b, bytes));
    fill<<<4096, 256>>>((uint64_t *)b, bytes / 8);
    CK(hipDeviceSynchronize());
    for (uint64_t chains : {500000ull, 2000000ull}) {
        run<0, false>(b, bytes, chains, out, e0, e1);
        run<0, true>(b, bytes, chains, out, e0, e1);
        run<1, false>(b, bytes, chains, out, e0, e1);
        run<1, true>(b, bytes, chains, out, e0, e1);
        run<2, false>(b, bytes, chains, out, e0, e1);
        run<2, true>(b, bytes, chains, out, e0, e1);
    }
    return 0;
}
