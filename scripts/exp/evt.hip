#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
__global__ void spin(long long cycles, int* out) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}
int main() {
    hipStream_t a, b;
    hipStreamCreate(&a); hipStreamCreate(&b);
    int* out; hipMalloc(&out, 1 << 20);
    hipEvent_t e0, e1, x0, x1;
    hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&x0); hipEventCreate(&x1);
    for (int it = 0; it < 3; it++) {
        // occupy the whole GPU on stream a for a while (many long blocks)
        spin<<<256 * 8, 1024, 0, a>>>(2000000, out);
        // short kernel on b: plain events
        hipEventRecord(e0, b);
        spin<<<64, 64, 0, b>>>(100000, out);
        hipEventRecord(e1, b);
        // short kernel on b: hipExtLaunchKernelGGL events
        hipExtLaunchKernelGGL(spin, dim3(64), dim3(64), 0, b, x0, x1, 0, 100000LL, out);
        hipDeviceSynchronize();
        float ms1, ms2;
        hipEventElapsedTime(&ms1, e0, e1);
        hipEventElapsedTime(&ms2, x0, x1);
        printf("plain events %.3f ms, ext-launch events %.3f ms\n", ms1, ms2);
    }
    // alone
    hipEventRecord(e0, b);
    spin<<<64, 64, 0, b>>>(100000, out);
    hipEventRecord(e1, b);
    hipExtLaunchKernelGGL(spin, dim3(64), dim3(64), 0, b, x0, x1, 0, 100000LL, out);
    hipDeviceSynchronize();
    float ms1, ms2;
    hipEventElapsedTime(&ms1, e0, e1);
    hipEventElapsedTime(&ms2, x0, x1);
    printf("alone: plain %.3f ms, ext %.3f ms\n", ms1, ms2);
    return 0;
}
