// Micro-benchmark: cost of a cross-stream wait (hipStreamWaitEvent on an
// event completed long before) between back-to-back streaming kernels, and of
// the dirty-L2 write-back a streaming writer leaves at its boundary.  Timing only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_write(double* b, size_t n, double v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = v;
}
__global__ void k_write_nt(double* b, size_t n, double v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(v, &b[i]);
}
__global__ void k_small(int* p) { if (threadIdx.x == 0) p[0] += 1; }

int main() {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    const size_t n = (size_t)250 << 20 >> 3;   // 250 MB of doubles
    double* buf; CK(hipMalloc(&buf, n * 8));
    int* p; CK(hipMalloc(&p, 64));
    hipEvent_t e0, e1, eb, ebx;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&ebx, hipEventDisableTiming | hipEventDisableSystemFence));
    hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, b, p);
    CK(hipEventRecord(eb, b));
    hipExtLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, b, nullptr, ebx, 0, p);
    CK(hipDeviceSynchronize());
    const int R = 40;
    const unsigned G = 256 * 8;
    auto run = [&](const char* name, auto body) {
        for (int i = 0; i < 3; ++i) body();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, a));
        for (int i = 0; i < R; ++i) body();
        CK(hipEventRecord(e1, a));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-52s %8.2f us/iter\n", name, ms * 1e3 / R);
        return 0;
    };
    run("write 250MB", [&] { hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    run("write 250MB nt", [&] { hipLaunchKernelGGL(k_write_nt, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    run("wait(old marker event) + write", [&] { hipStreamWaitEvent(a, eb, 0); hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    run("wait(old ext stop event) + write", [&] { hipStreamWaitEvent(a, ebx, 0); hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    run("wait(old event) + write nt", [&] { hipStreamWaitEvent(a, eb, 0); hipLaunchKernelGGL(k_write_nt, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    run("write + small (same stream)", [&] { hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, buf, n, 1.0); hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, a, p); });
    run("write + ext-stop-event write", [&] { hipExtLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, nullptr, ebx, 0, buf, n, 1.0); });
    // live cross-stream: b runs a small kernel each iteration, a waits for it
    run("b: small+record; a: wait + write", [&] {
        hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, b, p); hipEventRecord(eb, b);
        hipStreamWaitEvent(a, eb, 0); hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, a, buf, n, 1.0); });
    return 0;
}
