// Micro-benchmark: wake-up latency of a cross-stream wait that is actively
// blocking.  Stream b runs a kernel that spins for `us` microseconds (stop
// event, or a marker event after it); stream a runs a short kernel, waits for
// b's event, then a kernel whose first workgroup stamps s_memrealtime.  Gap =
// a's stamp - b's end stamp (100 MHz clock).  Timing only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_spin(unsigned long long* t, unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0 && blockIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();
}
__global__ void k_stamp(unsigned long long* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}
__global__ void k_short(int* p) { if (threadIdx.x == 0) p[0] += 1; }

int main() {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    unsigned long long* t; CK(hipMalloc(&t, 64));
    int* p; CK(hipMalloc(&p, 64));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence));
    for (int mode = 0; mode < 4; ++mode) {
        for (int us : {5, 20, 50}) {
            double sum = 0, mx = 0; const int R = 20;
            for (int r = 0; r < R; ++r) {
                CK(hipDeviceSynchronize());
                if (mode == 0 || mode == 2) {
                    hipExtLaunchKernelGGL(k_spin, dim3(mode == 2 ? 512 : 1), dim3(64), 0, b, nullptr, ev, 0, t, (unsigned long long)us * 100);
                } else {
                    hipLaunchKernelGGL(k_spin, dim3(mode == 3 ? 512 : 1), dim3(64), 0, b, t, (unsigned long long)us * 100);
                    CK(hipEventRecord(ev, b));
                }
                hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, a, p);
                CK(hipStreamWaitEvent(a, ev, 0));
                hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, t);
                CK(hipDeviceSynchronize());
                unsigned long long h[2]; CK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost));
                const double g = ((double)h[1] - (double)h[0]) / 100.0;
                sum += g; if (g > mx) mx = g;
            }
            printf("%-28s spin %3d us: gap mean %6.2f us max %6.2f\n",
                   mode == 0 ? "ext stop event, 1 WG" : mode == 1 ? "marker event, 1 WG" : mode == 2 ? "ext stop event, 512 WG" : "marker event, 512 WG",
                   us, sum / R, mx);
        }
    }
    // same stream for comparison
    double sum = 0; const int R = 20;
    for (int r = 0; r < R; ++r) {
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, t, 2000ull);
        hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, t);
        CK(hipDeviceSynchronize());
        unsigned long long h[2]; CK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost));
        sum += ((double)h[1] - (double)h[0]) / 100.0;
    }
    printf("same stream: gap mean %6.2f us\n", sum / R);
    return 0;
}
