// Microbenchmarks (diagnostic, not product): binary64 VALU latency/throughput
// and the cost of the bit-exact tanh+atanh pair on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
#include "../../qkd_ldpc_amd/csrc/qkd_math.h"

template <int ILP>
__device__ void chain_body(double* out, int iters, double a, double b) {
    double x[ILP];
    for (int u = 0; u < ILP; ++u) x[u] = threadIdx.x * 1e-3 + u;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int u = 0; u < ILP; ++u) x[u] = x[u] * a + b;   // contract off: mul + add
    double s = 0;
    for (int u = 0; u < ILP; ++u) s += x[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ILP>
__global__ void k_pair(double* out, int iters) {
    double x[ILP];
    for (int u = 0; u < ILP; ++u) x[u] = (threadIdx.x % 97) * 0.13 - 6.0 + u;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int u = 0; u < ILP; ++u) {
            const double t = qkdm::tanh_flat(x[u] * 0.5);
            x[u] = 2.0 * qkdm::atanh_flat(t * 0.97);
        }
    double s = 0;
    for (int u = 0; u < ILP; ++u) s += x[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
float run(K k, int blocks, int threads, double* d, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

template <int ILP>
__global__ void k_chain_w(double* out, int iters) { chain_body<ILP>(out, iters, 0.999999, 1e-9); }

int main() {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double* d; hipMalloc(&d, 256ull * 1024 * 64 * sizeof(double));
    const int it = 4096;
    for (int wps : {1, 2, 4, 8}) {            // waves per SIMD
        const int threads = 256;               // 4 waves / block -> 1 wave per SIMD per block
        const int blocks = cus * wps;
        for (int ilp : {1, 2, 4}) {
            float ms = ilp == 1 ? run(k_chain_w<1>, blocks, threads, d, it)
                     : ilp == 2 ? run(k_chain_w<2>, blocks, threads, d, it) : run(k_chain_w<4>, blocks, threads, d, it);
            const double ops = 2.0 * it * ilp * blocks * threads / 64.0;      // wave-instructions (mul+add)
            const double per_simd = ops / (cus * 4.0);
            printf("chain waves/SIMD %d ILP %d: %.3f ms, %.2f ns per wave-instr per SIMD\n", wps, ilp, ms,
                   ms * 1e6 / per_simd);
        }
    }
    const int it2 = 256;
    for (int wps : {1, 2, 4, 8}) {
        const int threads = 256, blocks = cus * wps;
        for (int ilp : {1, 2}) {
            float ms = ilp == 1 ? run(k_pair<1>, blocks, threads, d, it2) : run(k_pair<2>, blocks, threads, d, it2);
            const double pairs = (double)it2 * ilp * blocks * threads;
            printf("tanh+atanh waves/SIMD %d ILP %d: %.3f ms, %.3f ns per pair per lane-chip -> %.1f G pairs/s\n",
                   wps, ilp, ms, ms * 1e6 / pairs, pairs / ms / 1e6);
        }
    }
    return 0;
}
