// Cross-stream gate probe: when does a kernel behind hipStreamWaitEvent on
// stream B start, relative to the kernel before the event's record (K1) and the
// kernel enqueued after it (K2) on stream A? Device clock stamps (100 MHz).
//   mode 0: event (timing off), B's wait enqueued after K2
//   mode 1: event (timing off), B's wait enqueued before K2
//   mode 2: event (timing on),  B's wait enqueued after K2
//   mode 3: hipStreamWriteValue32 after K1 / hipStreamWaitValue32 on B, after K2
//           (the word from hipExtMallocWithFlags(hipMallocSignalMemory))
//   mode 4: as 3, the word written by a one-wave kernel (release store)
// Build: hipcc --offload-arch=gfx950 -O2 gate_probe.hip -o gate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_spin(unsigned long long* stamp, int slot, long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while ((long long)(wall_clock64() - t0) < ticks) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        stamp[2 * slot] = t0;
        stamp[2 * slot + 1] = wall_clock64();
    }
}

__global__ void k_signal(uint32_t* w, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

int main() {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    unsigned long long* st;
    CK(hipMalloc(&st, 64 * sizeof(unsigned long long)));
    uint32_t* flag = nullptr;
    const hipError_t fe_ = hipExtMallocWithFlags((void**)&flag, 8, hipMallocSignalMemory);
    if (fe_ != hipSuccess) printf("signal memory: %s\n", hipGetErrorString(fe_));
    if (flag) CK(hipMemset(flag, 0, 8));
    hipEvent_t ev_nt, ev_t;
    CK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
    CK(hipEventCreate(&ev_t));
    for (int mode = 0; mode < (flag ? 5 : 3); mode++) {
        for (int rep = 0; rep < 3; rep++) {
            CK(hipDeviceSynchronize());
            CK(hipMemset(st, 0, 64 * 8));
            hipEvent_t ev = mode == 2 ? ev_t : ev_nt;
            const uint32_t val = (uint32_t)(mode * 10 + rep + 1);
            // keep B busy briefly so its wait is enqueued on a live queue
            k_spin<<<1, 64, 0, a>>>(st, 0, 100000);  // K1: 1 ms
            if (mode == 3)
                CK(hipStreamWriteValue32(a, flag, val, 0));
            else if (mode == 4)
                k_signal<<<1, 64, 0, a>>>(flag, val);
            else
                CK(hipEventRecord(ev, a));
            if (mode == 1) {
                CK(hipStreamWaitEvent(b, ev, 0));
                k_spin<<<1, 64, 0, b>>>(st, 2, 100);  // K3
            }
            k_spin<<<1, 64, 0, a>>>(st, 1, 200000);  // K2: 2 ms
            if (mode == 0 || mode == 2) {
                CK(hipStreamWaitEvent(b, ev, 0));
                k_spin<<<1, 64, 0, b>>>(st, 2, 100);
            } else if (mode >= 3) {
                CK(hipStreamWaitValue32(b, flag, val, hipStreamWaitValueGte, 0xffffffffu));
                k_spin<<<1, 64, 0, b>>>(st, 2, 100);
            }
            CK(hipDeviceSynchronize());
            unsigned long long h[6];
            CK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
            const double k1e = h[1] * 1e-2, k2e = h[3] * 1e-2, k3s = h[4] * 1e-2;
            printf("mode %d rep %d: K3 start - K1 end %.1f us, K3 start - K2 end %.1f us\n", mode, rep, k3s - k1e,
                   k3s - k2e);
        }
    }
    return 0;
}
