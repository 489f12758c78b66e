// Memory microbenchmark for the long-code store question: what
// a check phase's slot traffic costs in
//   (a) the frame-interleaved store: one 128-byte line = one slot of 16 frames,
//       a 16-lane group reads and writes a whole line (lines in a random
//       order, ILP U lines per group), the whole batch (4096 frames) resident;
//   (b) the same store walked in line order (the bit phase's rows);
//   (c) the one-frame-per-workgroup store: 8-byte slots at random positions of
//       a 0.96 MB region per workgroup (the current split kernel's global part).
// Timed with HIP events; prints GB/s of bytes moved (read + write, useful bytes).
//   hipcc --offload-arch=gfx950 -O3 tools/mb/interleave_mb.hip -o tools/mb/interleave_mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

constexpr int U = 6;   // lines in flight per group (a degree-6 check's slots)

// (a)/(b): 64 groups of 16 lanes per workgroup; lane = frame
template <bool RANDOM>
__global__ __launch_bounds__(1024) void lines_rmw(double* base, uint32_t lines, int passes) {
    double* r = base + (size_t)blockIdx.x * lines * 16;
    const uint32_t grp = threadIdx.x >> 4, f = threadIdx.x & 15;
    for (int p = 0; p < passes; ++p)
        for (uint32_t l0 = grp * U; l0 < lines; l0 += 64 * U) {
            uint32_t li[U];
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t l = l0 + u;
                li[u] = RANDOM ? mix(l * 2654435761u + p * 40503u + blockIdx.x) % lines : (l < lines ? l : lines - 1);
                v[u] = r[(size_t)li[u] * 16 + f];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) r[(size_t)li[u] * 16 + f] = v[u] * 0.5 + 1.0;
        }
}

// (c): every lane its own random 8-byte slot of the workgroup's region
__global__ __launch_bounds__(1024) void slots_rmw(double* base, uint32_t slots, int passes) {
    double* r = base + (size_t)blockIdx.x * slots;
    for (int p = 0; p < passes; ++p)
        for (uint32_t s0 = threadIdx.x * U; s0 < slots; s0 += 1024 * U) {
            uint32_t si[U];
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                si[u] = mix((s0 + u) * 2654435761u + p * 40503u + blockIdx.x) % slots;
                v[u] = r[si[u]];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) r[si[u]] = v[u] * 0.5 + 1.0;
        }
}

int main() {
    const uint32_t lines = 122880;               // 3 x n_pad slots, N = 40000
    const int wgs = 256, passes = 2;
    const size_t bytes_a = (size_t)wgs * lines * 128;        // 4.03 GB
    double* buf;
    CK(hipMalloc(&buf, bytes_a));
    CK(hipMemset(buf, 0, bytes_a));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0));
        lines_rmw<true><<<wgs, 1024>>>(buf, lines, passes);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("interleaved random lines  footprint %.2f GB  %.3f ms  %.0f GB/s\n", bytes_a / 1e9, ms,
               2.0 * passes * bytes_a / ms / 1e6);
        CK(hipEventRecord(e0));
        lines_rmw<false><<<wgs, 1024>>>(buf, lines, passes);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("interleaved line order    footprint %.2f GB  %.3f ms  %.0f GB/s\n", bytes_a / 1e9, ms,
               2.0 * passes * bytes_a / ms / 1e6);
        // (a) with fewer frames per workgroup region (footprint / 4: 1 GB; / 16: 252 MB)
        for (uint32_t div : {4u, 16u}) {
            CK(hipEventRecord(e0));
            lines_rmw<true><<<wgs, 1024>>>(buf, lines / div, passes);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("interleaved random lines  footprint %.2f GB  %.3f ms  %.0f GB/s\n", bytes_a / div / 1e9, ms,
                   2.0 * passes * bytes_a / div / ms / 1e6);
        }
        const uint32_t slots = 122880;            // one frame's slots per workgroup
        CK(hipEventRecord(e0));
        slots_rmw<<<wgs, 1024>>>(buf, slots, passes);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double useful = 2.0 * passes * (double)wgs * slots * 8;
        printf("per-frame random slots    footprint %.2f GB  %.3f ms  %.0f GB/s useful\n",
               (double)wgs * slots * 8 / 1e9, ms, useful / ms / 1e6);
    }
    CK(hipFree(buf));
    return 0;
}
