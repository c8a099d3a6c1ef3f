// Micro-benchmark: LDS atomicAdd throughput by address pattern (all lanes one
// address / 4 addresses / 16 / distinct) and a wave-aggregated form (one
// atomic per distinct address via ballot).  Timing only.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ void k_atom(unsigned* out, int iters, int groups) {
    __shared__ unsigned h[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int bin = (lane / (64 / groups)) * 7 + (threadIdx.x >> 6) * 97;
    for (int it = 0; it < iters; ++it) {
        const int b = (bin + it * 13) & 4095;
        if (MODE == 0) {
            atomicAdd(&h[b], 1u);
        } else {   // aggregated: leader per distinct bin
            unsigned long long todo = __ballot(1);
            while (todo) {
                const int src = __builtin_ctzll(todo);
                const int lb = __builtin_amdgcn_readlane(b, src);
                const unsigned long long m = __ballot(b == lb);
                if (lane == src) atomicAdd(&h[lb], (unsigned)__popcll(m));
                todo &= ~m;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = h[bin & 4095];
}

int main() {
    unsigned* o; CK(hipMalloc(&o, 1 << 20));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int iters = 2000;
    for (int mode = 0; mode < 2; ++mode)
        for (int g : {1, 4, 16, 64}) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(k_atom<0>, dim3(1024), dim3(256), 0, 0, o, iters, g);
                else hipLaunchKernelGGL(k_atom<1>, dim3(1024), dim3(256), 0, 0, o, iters, g);
            };
            launch(); CK(hipDeviceSynchronize());
            CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            const double waveops = 1024.0 * 4 * iters;
            printf("%s distinct addrs/wave %2d: %7.3f ms  %6.1f ns per wave-instr per CU\n", mode ? "aggregated" : "plain     ",
                   g, ms, ms * 1e6 / (waveops / 256));
        }
    return 0;
}
