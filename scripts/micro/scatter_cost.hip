// Random 8-B writes vs random 8-B reads at the grouped search's scale (one
// result per pattern of a 25.6 M-pattern launch into a 205 MB array): does a
// scattered write cost more than a scattered read (partial-line writes)?  If
// so, writing the grouped search's results in sorted order and gathering them
// in pattern order afterwards (an inverse permutation written by the place
// pass) would pay; if not, it only moves the random access.
//   scatter_w : out[perm[i]] = v[i]   (perm read in order, writes random)
//   gather_r  : out[i] = v[perm[i]]   (reads random, writes in order)
//   seq       : out[i] = v[i]         (both in order: the streaming floor)
// 25.6 M elements of 8 B, a random permutation; each kernel 20 times.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void k_scatter(const unsigned *__restrict__ perm, const unsigned long long *__restrict__ v,
                                                 unsigned long long *__restrict__ out, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[perm[i]] = v[i];
}
__global__ __launch_bounds__(256) void k_gather(const unsigned *__restrict__ perm, const unsigned long long *__restrict__ v,
                                                unsigned long long *__restrict__ out, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = v[perm[i]];
}
__global__ __launch_bounds__(256) void k_seq(const unsigned *__restrict__ perm, const unsigned long long *__restrict__ v,
                                             unsigned long long *__restrict__ out, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = v[i] + perm[i];
}

int main() {
    const unsigned n = 25600000;
    std::vector<unsigned> h(n);
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937_64(5));
    unsigned *perm;
    unsigned long long *v, *out;
    if (hipMalloc(&perm, n * 4ull) || hipMalloc(&v, n * 8ull) || hipMalloc(&out, n * 8ull)) return 2;
    hipMemcpy(perm, h.data(), n * 4ull, hipMemcpyHostToDevice);
    hipMemset(v, 1, n * 8ull);
    hipMemset(out, 0, n * 8ull);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[3] = {"scatter_w", "gather_r", "seq"};
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 3; ++k) {
            hipEventRecord(a, 0);
            for (int it = 0; it < 20; ++it) {
                if (k == 0) hipLaunchKernelGGL(k_scatter, dim3((n + 255) / 256), dim3(256), 0, 0, perm, v, out, n);
                if (k == 1) hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, 0, perm, v, out, n);
                if (k == 2) hipLaunchKernelGGL(k_seq, dim3((n + 255) / 256), dim3(256), 0, 0, perm, v, out, n);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 1)
                printf("{\"kernel\": \"%s\", \"elements\": %u, \"us_per_launch\": %.1f, \"g_elements_per_s\": %.2f}\n",
                       names[k], n, ms * 1e3 / 20, n * 20.0 / (ms * 1e-3) / 1e9);
        }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
