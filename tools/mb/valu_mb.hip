// Microbenchmark (diagnostic, not product): issue cost of the binary32 VALU
// instructions the speculative check phase is made of, at the decoder's
// occupancy (one 1024-thread workgroup per CU = 4 waves per SIMD), 8
// independent chains per lane. Prints ns per wave-instruction per SIMD and
// the ratio to v_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ILP = 8;

template <int OP>
__global__ __launch_bounds__(1024) void k(float* out, int iters, float a, float b) {
    float x[ILP];
    f2 y[ILP];
    for (int u = 0; u < ILP; ++u) { x[u] = threadIdx.x * 1e-6f + u * 0.1f + 0.5f; y[u] = f2{x[u], x[u] + 0.25f}; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < ILP; ++u) {
            if constexpr (OP == 0) x[u] = __builtin_fmaf(x[u], a, b);
            if constexpr (OP == 1) y[u] = __builtin_elementwise_fma(y[u], f2{a, a}, f2{b, b});
            if constexpr (OP == 2) x[u] = __builtin_amdgcn_exp2f(x[u]);
            if constexpr (OP == 3) x[u] = __builtin_amdgcn_logf(x[u]);
            if constexpr (OP == 4) x[u] = __builtin_amdgcn_rcpf(x[u]);
            if constexpr (OP == 5) x[u] = __builtin_amdgcn_fmed3f(x[u], a, b);
            if constexpr (OP == 6) x[u] = x[u] + a;
            if constexpr (OP == 7) y[u] = y[u] + f2{a, b};
            if constexpr (OP == 8) { double d = (double)x[u]; d = __builtin_fma(d, (double)a, (double)b); x[u] = (float)d; }
            if constexpr (OP == 9) x[u] = __builtin_bit_cast(float, __builtin_amdgcn_ubfe(__builtin_bit_cast(uint32_t, x[u]), 3, 20) | 0x3f000000u);
        }
    }
    float s = 0;
    for (int u = 0; u < ILP; ++u) s += x[u] + y[u].x + y[u].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
float run(float* d, int cus, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(1024), 0, 0, d, iters, 0.999f, 1e-7f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(1024), 0, 0, d, iters, 0.999f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* d; hipMalloc(&d, (size_t)cus * 1024 * sizeof(float));
    const int it = 1 << 14;
    // wave-instructions per SIMD: 4 waves x iters x ILP
    const double winst = 4.0 * it * ILP;
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_med3_f32",
                           "v_add_f32", "v_pk_add_f32", "cvt+fma_f64+cvt", "v_bfe_u32+or"};
    float ms[10];
    ms[0] = run<0>(d, cus, it); ms[1] = run<1>(d, cus, it); ms[2] = run<2>(d, cus, it);
    ms[3] = run<3>(d, cus, it); ms[4] = run<4>(d, cus, it); ms[5] = run<5>(d, cus, it);
    ms[6] = run<6>(d, cus, it); ms[7] = run<7>(d, cus, it); ms[8] = run<8>(d, cus, it);
    ms[9] = run<9>(d, cus, it);
    for (int i = 0; i < 10; ++i)
        printf("%-18s %.3f ms  %.3f ns/wave-inst/SIMD  x%.2f of v_fma_f32\n", names[i], ms[i], ms[i] * 1e6 / winst,
               ms[i] / ms[0]);
    return 0;
}
