// LDS bank-conflict probe of the split decoder's access streams (gfx950).
// Replays, in a 1024-thread workgroup per CU with a 160 KB allocation, the
// check phase's slot accesses of the real config-2 plan (one ds_read_b64 and
// one ds_write_b64 per lane and task, tasks wave, wave + 16, ..., global slots'
// lanes at their out-of-range LDS addresses as in the kernel) and the bit
// phase's syndrome XORs (ds_xor_b32 on the xsyn words of each bit's checks),
// in variants that isolate one stream each. Run under rocprofv3 --pmc
// SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS: each variant is its own
// kernel (template argument), so the counters attribute per dispatch; the
// in-kernel shader-clock cycles per pass are printed too.
//   python tools/mb/gen_lds_stream.py   (needs the built library; writes lds_stream.bin)
//   hipcc --offload-arch=gfx950 -O3 lds_bank_mb.hip -o lds_bank_mb && ./lds_bank_mb lds_stream.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

enum Variant : int {
    kReadWrite = 0,     // the check phase: read then write each lane's slot
    kRead = 1,          // reads only
    kWrite = 2,         // writes only
    kReadNoOob = 3,     // reads, out-of-range lanes moved to a broadcast address
    kWriteNoOob = 4,    // writes, the same
    kReadLinear = 5,    // reads at lane-linear addresses (no conflict possible)
    kXorHalf = 6,       // bit phase: ds_xor_b32 for the bits with a 1 decision (~half)
    kXorAll = 7,        // the same with every lane active
    kReadOobOnly = 8,   // only the out-of-range lanes read (the others masked off)
};

constexpr int kBlock = 1024;
constexpr int kReps = 20;

__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

template <int V>
__global__ __launch_bounds__(kBlock) void probe(const uint32_t* slot_addr, int n_tasks, const uint32_t* syn_addr,
                                                int n_pad, uint64_t* sink, unsigned long long* cycles) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef __attribute__((address_space(3))) double LdsD;
    typedef __attribute__((address_space(3))) uint32_t LdsU;
    for (int i = threadIdx.x; i < 160 * 1024 / 8; i += kBlock) reinterpret_cast<double*>(smem)[i] = (double)i;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double acc = 0.0;
    uint32_t xacc = 0;
    const long long t0 = clock64();
    for (int rep = 0; rep < kReps; ++rep) {
        if (V <= kReadLinear || V == kReadOobOnly) {
            for (int t = wave; t < n_tasks; t += kBlock / 64) {
                uint32_t a = slot_addr[t * 64 + lane];
                const bool oob = a >= 0x28000u;
                if (V == kReadNoOob || V == kWriteNoOob) a = oob ? 8u * (uint32_t)wave : a;
                if (V == kReadLinear) a = 8u * (uint32_t)(wave * 64 + lane);
                a = opaque(a);
                if (V == kRead || V == kReadWrite || V == kReadNoOob || V == kReadLinear ||
                    (V == kReadOobOnly && oob))
                    acc += *reinterpret_cast<LdsD*>((size_t)a);
                if (V == kWrite || V == kReadWrite || V == kWriteNoOob)
                    *reinterpret_cast<LdsD*>((size_t)a) = acc + (double)t;
            }
        } else {
            for (int r = 0; r * kBlock < n_pad; ++r) {
                const int i = threadIdx.x + r * kBlock;
                if (i >= n_pad) break;
                // a bit's decision: any fixed pseudo-random half of the bits
                const bool z = V == kXorAll || ((i * 2654435761u) >> 31) != 0;
                if (z) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t a = opaque(syn_addr[i * 3 + k]);
                        __hip_atomic_fetch_xor(reinterpret_cast<LdsU*>((size_t)a), 1u << (i & 31),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
        __syncthreads();
    }
    const long long t1 = clock64();
    xacc = *reinterpret_cast<LdsU*>((size_t)(threadIdx.x * 4));
    sink[blockIdx.x * kBlock + threadIdx.x] = __builtin_bit_cast(uint64_t, acc) ^ xacc;
    if (threadIdx.x == 0) atomicAdd(cycles, (unsigned long long)(t1 - t0));
}

template <int V>
static void run(const char* name, const uint32_t* d_slot, int n_tasks, const uint32_t* d_syn, int n_pad,
                uint64_t* d_sink, unsigned long long* d_cyc, int grid) {
    hipFuncSetAttribute((const void*)probe<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipMemset(d_cyc, 0, 8);
    hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(kBlock), 160 * 1024, 0, d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc);
    hipDeviceSynchronize();
    unsigned long long cyc = 0;
    hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
    const double per_pass = (double)cyc / grid / kReps;
    printf("%-14s cycles per pass (one workgroup) %10.0f\n", name, per_pass);
}

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "tools/mb/lds_stream.bin";
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); return 1; }
    uint32_t hdr[2];
    if (fread(hdr, 4, 2, f) != 2) return 1;
    const int n_tasks = (int)hdr[0], n_pad = (int)hdr[1];
    std::vector<uint32_t> slot((size_t)n_tasks * 64), syn((size_t)n_pad * 3);
    if (fread(slot.data(), 4, slot.size(), f) != slot.size()) return 1;
    if (fread(syn.data(), 4, syn.size(), f) != syn.size()) return 1;
    fclose(f);
    // every address inside the allocation, or past it (>= 0x40000) as the kernel's
    for (uint32_t a : slot) if (!(a < 160 * 1024 - 8 || a >= 0x40000)) { fprintf(stderr, "bad addr %u\n", a); return 1; }
    for (uint32_t a : syn) if (a >= 160 * 1024) { fprintf(stderr, "bad syn addr %u\n", a); return 1; }
    uint32_t *d_slot, *d_syn;
    uint64_t* d_sink;
    unsigned long long* d_cyc;
    const int grid = 256;
    hipMalloc(&d_slot, slot.size() * 4);
    hipMalloc(&d_syn, syn.size() * 4);
    hipMalloc(&d_sink, (size_t)grid * kBlock * 8);
    hipMalloc(&d_cyc, 8);
    hipMemcpy(d_slot, slot.data(), slot.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_syn, syn.data(), syn.size() * 4, hipMemcpyHostToDevice);
    printf("tasks %d, n_pad %d, %d workgroups x %d passes\n", n_tasks, n_pad, grid, kReps);
    run<kReadLinear>("read_linear", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kRead>("read", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kReadNoOob>("read_no_oob", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kReadOobOnly>("read_oob_only", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kWrite>("write", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kWriteNoOob>("write_no_oob", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kReadWrite>("read_write", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kXorHalf>("xor_half", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    run<kXorAll>("xor_all", d_slot, n_tasks, d_syn, n_pad, d_sink, d_cyc, grid);
    const hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
