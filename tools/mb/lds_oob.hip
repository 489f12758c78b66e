// Probe: what a DS access past the workgroup's LDS allocation does on gfx950
// (the encoded message-slot words of decode_split.hip rely on it: reads give
// 0, writes are dropped, no wrap-around into the allocation).
//   hipcc --offload-arch=gfx950 -O2 lds_oob.hip -o lds_oob && ./lds_oob
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void probe(uint32_t alloc, uint32_t far, uint64_t* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t t = threadIdx.x;
    uint64_t* in = reinterpret_cast<uint64_t*>(smem);
    const uint32_t n = alloc / 8;
    for (uint32_t i = t; i < n; i += blockDim.x) in[i] = 0x1111111100000000ull | i;
    __syncthreads();
    // writes past the allocation: at alloc + 8 t and at far + 8 t
    volatile uint64_t* w0 = reinterpret_cast<volatile uint64_t*>(smem + alloc + 8 * t);
    volatile uint64_t* w1 = reinterpret_cast<volatile uint64_t*>(smem + far + 8 * t);
    *w0 = 0xdeadbeef00000000ull | t;
    *w1 = 0xfeedface00000000ull | t;
    __syncthreads();
    // reads past the allocation
    out[t * 4 + 0] = *w0;
    out[t * 4 + 1] = *w1;
    // did anything inside the allocation change?
    uint64_t bad = 0;
    for (uint32_t i = t; i < n; i += blockDim.x) bad += in[i] != (0x1111111100000000ull | i);
    out[t * 4 + 2] = bad;
    // a read with the sign bit set in the address (encoded words keep it)
    volatile uint64_t* w2 = reinterpret_cast<volatile uint64_t*>(smem + (0x80000000u | (8 * t)));
    out[t * 4 + 3] = *w2;
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 256 * 4 * 8);
    const uint32_t allocs[] = {65536, 163840 - 4096, 163840};
    for (uint32_t alloc : allocs) {
        for (uint32_t far : {0x40000u, 0x80000u, 0x100000u}) {
            hipMemset(d, 0x55, 256 * 4 * 8);
            hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, alloc);
            hipLaunchKernelGGL(probe, dim3(1), dim3(256), alloc, 0, alloc, far, d);
            hipError_t e = hipDeviceSynchronize();
            uint64_t h[256 * 4];
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            uint64_t nz0 = 0, nz1 = 0, bad = 0, nz2 = 0;
            for (int t = 0; t < 256; ++t) {
                nz0 += h[t * 4] != 0;
                nz1 += h[t * 4 + 1] != 0;
                bad += h[t * 4 + 2];
                nz2 += h[t * 4 + 3] != 0;
            }
            printf("alloc %u far 0x%x: %s  nonzero reads at alloc: %llu, at far: %llu, corrupted in-range: %llu, "
                   "sign-bit reads nonzero: %llu (t0 %016llx %016llx %016llx)\n",
                   alloc, far, hipGetErrorString(e), (unsigned long long)nz0, (unsigned long long)nz1,
                   (unsigned long long)bad, (unsigned long long)nz2, (unsigned long long)h[0],
                   (unsigned long long)h[1], (unsigned long long)h[3]);
        }
    }
    return 0;
}
