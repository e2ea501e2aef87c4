// Does a kernel take an 8 KB by-value argument on this ROCm (kernarg segment limit)?
#include <hip/hip_runtime.h>
#include <cstdio>
#ifndef WORDS
#define WORDS 1024
#endif
struct Big { unsigned long long v[WORDS]; };  // WORDS x 8 B
__global__ void k_big(const Big b, unsigned long long *out) {
    unsigned long long s = 0;
    for (int i = threadIdx.x; i < WORDS; i += 64) s += b.v[i];
    atomicAdd(out, s);
}
int main() {
    Big b;
    unsigned long long want = 0;
    for (int i = 0; i < WORDS; ++i) { b.v[i] = i * 3 + 1; want += b.v[i]; }
    unsigned long long *d = nullptr, got = 0;
    if (hipMalloc(&d, 8) != hipSuccess) return 2;
    hipMemset(d, 0, 8);
    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, 0, b, d);
    hipError_t e = hipGetLastError();
    hipError_t e2 = hipDeviceSynchronize();
    hipMemcpy(&got, d, 8, hipMemcpyDeviceToHost);
    printf("launch=%s sync=%s got=%llu want=%llu %s\n", hipGetErrorString(e), hipGetErrorString(e2), got, want,
           got == want ? "OK" : "MISMATCH");
    return got == want ? 0 : 1;
}
