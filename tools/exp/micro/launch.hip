// Micro-benchmark: per-launch cost of small kernels (empty, host-pinned store,
// 1024-thread single workgroup, back-to-back chains).  Timing only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_empty(int* p) { if (p && threadIdx.x == 9999) p[0] = 1; }
__global__ void k_host_relaxed(unsigned* h, unsigned v) {
    if (threadIdx.x == 0) { __hip_atomic_store(h, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
}
__global__ void k_host_release(unsigned* h, unsigned v) {
    if (threadIdx.x == 0) { __hip_atomic_store(h, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM); }
}
__global__ void k_dev_store(unsigned* d, unsigned v) { d[threadIdx.x] = v; }
__global__ void k_load_store(const unsigned* a, unsigned* b, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) b[i] = a[i] + 1;
}
__global__ void k_stream(const float4* a, float4* b, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* h; CK(hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned* dh; CK(hipHostGetDevicePointer((void**)&dh, h, 0));
    unsigned *d, *d2; CK(hipMalloc(&d, 1 << 20)); CK(hipMalloc(&d2, 1 << 20));
    size_t nbig = (size_t)64 << 20; float4 *A, *B; CK(hipMalloc(&A, nbig)); CK(hipMalloc(&B, nbig));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch, int reps) {
        for (int i = 0; i < 5; ++i) launch();
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.2f us/launch\n", name, ms * 1e3 / reps);
    };
    const int R = 200;
    run("empty 1x64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr); }, R);
    run("empty 1x1024", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(1024), 0, s, nullptr); }, R);
    run("empty 4096x256", [&] { hipLaunchKernelGGL(k_empty, dim3(4096), dim3(256), 0, s, nullptr); }, R);
    run("host store relaxed 1x1024", [&] { hipLaunchKernelGGL(k_host_relaxed, dim3(1), dim3(1024), 0, s, dh, 1u); }, R);
    run("host store release 1x1024", [&] { hipLaunchKernelGGL(k_host_release, dim3(1), dim3(1024), 0, s, dh, 1u); }, R);
    run("dev store 1x1024", [&] { hipLaunchKernelGGL(k_dev_store, dim3(1), dim3(1024), 0, s, d, 1u); }, R);
    run("load+store 16KB 1x1024", [&] { hipLaunchKernelGGL(k_load_store, dim3(1), dim3(1024), 0, s, d, d2, 4096); }, R);
    size_t n4 = nbig / 16;
    run("stream 64MB (copy)", [&] { hipLaunchKernelGGL(k_stream, dim3((n4 + 255) / 256), dim3(256), 0, s, A, B, n4); }, 20);
    run("stream 64MB + empty", [&] { hipLaunchKernelGGL(k_stream, dim3((n4 + 255) / 256), dim3(256), 0, s, A, B, n4);
                                     hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr); }, 20);
    run("stream 64MB + load+store 1x1024", [&] { hipLaunchKernelGGL(k_stream, dim3((n4 + 255) / 256), dim3(256), 0, s, A, B, n4);
                                     hipLaunchKernelGGL(k_load_store, dim3(1), dim3(1024), 0, s, d, d2, 4096); }, 20);
    run("stream 64MB + host release", [&] { hipLaunchKernelGGL(k_stream, dim3((n4 + 255) / 256), dim3(256), 0, s, A, B, n4);
                                     hipLaunchKernelGGL(k_host_release, dim3(1), dim3(1024), 0, s, dh, 1u); }, 20);
    return 0;
}
