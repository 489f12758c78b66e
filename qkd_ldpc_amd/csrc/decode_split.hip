// decode_split.hip — the sum-product decoder with a split message store.
//
// Same algorithm and the same binary64 (or binary32) operations as
// decode_kernel (decode.hip; reference src/qkd_ldpc_algorithm.cpp:175-345 and
// :3-173), organised around the reference's own two-message formulation
// instead of the bit totals:
//
//   check phase  (:220-249)  per edge: t = tanh(b2c / 2), the in-check
//                product, c2b = clamp(2 atanh(P / t)); the edge's slot
//                holds b2c on entry and c2b on exit
//   bit phase    (:256-267, :303-316)  per bit: total = LLR + c2b_0 + c2b_1
//                + ... (ascending checks), hard decision and its syndrome,
//                then b2c_k = clamp(total - c2b_k) back into slot k
//
// so each edge has ONE slot that both phases read and rewrite in place, and
// nothing else per bit or per edge has to persist between phases: the bit
// totals live only in registers, the hard decision as one bit per bit in LDS.
// That leaves almost the whole LDS for message slots. The slot of the k-th
// check of bit i is x = k * n_pad + i (bit-major: the bit phase's accesses are
// coalesced); slots x < S live in LDS, the rest in the workgroup's global
// region, x - S. For N = 10240 (fp64): S = 18.5k of 30.9k slots, so the
// per-frame global footprint is 99 KB instead of the classic store's 247 KB,
// and 32 frames per XCD fit the 4 MB L2. binary32 messages
// fit LDS entirely (S = all slots): the kRuleSp32 variant touches no global
// scratch at all.
//
// QKD path tables (first_check_phase / second_table_fill in decode.hip and
// qkd_decode.h): the first check phase is always folded into the first bit
// phase (messages rebuilt from one sign bit per check). With the second table
// in use, that bit phase stores in each slot, instead of b2c, the table index
// of the edge's second-iteration tanh (an integer in the slot's bits), and
// the second check phase looks it up.
#include <hip/hip_runtime.h>

#include "qkd_decode.h"

namespace qkd {

// One workgroup's message slots: x < S in LDS, the rest in global memory
// through a buffer descriptor. Every access issues both an LDS and a buffer
// instruction and selects: lanes whose slot is in LDS give the buffer an
// out-of-range offset (the hardware returns 0 and drops stores, no memory is
// touched), lanes whose slot is global read LDS word 0 and write their own
// trash slot (S + lane). Branching on x < S instead lets the compiler merge
// the two accesses into one FLAT instruction, which waits for both the
// vector-memory and the LDS counters to drain and so serialises the
// check phase's software pipeline.
template <typename T> struct BufIo;
template <> struct BufIo<double> {
    static __device__ __forceinline__ double ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
    }
    static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
        using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V, v), r, (int)off, 0, 0);
    }
};
template <> struct BufIo<float> {
    static __device__ __forceinline__ float ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
    }
    static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0, 0);
    }
};

template <typename T>
struct SplitStore {
    T* l;                        // LDS slots [0, S) and the trash slots [S, S + 64)
    __amdgpu_buffer_rsrc_t g;    // global slots S.. of this workgroup
    uint32_t S;
    static constexpr uint32_t kOob = 0x7ffffff0u;
    __device__ __forceinline__ T ld(uint32_t x) const {
        const bool in = x < S;
        const T vl = l[in ? x : 0u];
        const T vg = BufIo<T>::ld(g, in ? kOob : (x - S) * (uint32_t)sizeof(T));
        return in ? vl : vg;
    }
    __device__ __forceinline__ void st(uint32_t x, T v) const {
        const bool in = x < S;
        l[in ? x : S + (threadIdx.x & 63u)] = v;
        BufIo<T>::st(g, in ? kOob : (x - S) * (uint32_t)sizeof(T), v);
    }
    // slots x .. x + 63 of a wave's 64 consecutive lanes (xw = the wave's
    // first slot, wave-uniform): one kind of access when the wave's slots are
    // all in LDS or all global
    __device__ __forceinline__ T ld_row(uint32_t xw, uint32_t x) const {
        if (xw + 64u <= S) return l[x];
        if (xw >= S) return BufIo<T>::ld(g, (x - S) * (uint32_t)sizeof(T));
        return ld(x);
    }
    __device__ __forceinline__ void st_row(uint32_t xw, uint32_t x, T v) const {
        if (xw + 64u <= S)
            l[x] = v;
        else if (xw >= S)
            BufIo<T>::st(g, (x - S) * (uint32_t)sizeof(T), v);
        else
            st(x, v);
    }
};

// Check phase of one iteration for one wave (tasks wave, wave + NW, ...):
// per edge the incoming b2c (or, SRC == kSrcTable, its table index) from the
// edge's slot, the outgoing c2b back into it. Software-pipelined exactly as
// check_phase (decode.hip): the plan word two tasks ahead and the slot one
// task ahead are loaded before this task's arithmetic; stores trail by one
// task. Slots of different tasks are distinct (idle lanes share the dummy
// column's slot, whose value nothing reads).
template <int SRC, bool CLAMP, int DC, int RULE, typename T>
__device__ __forceinline__ void split_check_phase(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                  const double* tab2, const SplitStore<T>& ms, T* row,
                                                  int n_tasks, uint32_t n_pad, T thr, int wave, int lane) {
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const uint2* pl = plan + lane;
    auto slot = [&](uint2 p) -> uint32_t { return pw_row(p) * n_pad + pw_bit(p); };
    auto sbit = [&](uint2 p) -> uint32_t {
        const uint32_t j = pw_chk(p);
        return (tsyn[j >> 5] >> (j & 31)) & 1u;
    };
    auto edge = [&](T x, uint2 w) -> T {
        T a;
        if constexpr (SRC == kSrcTable && RULE == kRuleSp64)
            a = tab2[qkdm::lo32(x)];
        else
#ifdef QKD_EXP_NO_MATH
            a = x * (T)0.5;
#else
            a = RuleMath<RULE>::tanh_half(x);                      // (:224)
#endif
        row[lane] = a;
        wave_lds_sync();
        return edge_out<CLAMP, DC, RULE>(a, w, sbit(w), lane, thr, row, 0.0f);
    };
    uint2 wa = pl[t * 64];
    uint2 wb = pl[(t + NW) * 64];
    T xa = ms.ld(slot(wa));
    uint32_t pend = 0xffffffffu;    // slot of the previous task's message, not yet stored
    T pv = 0;
    for (;;) {
        if (pend != 0xffffffffu) ms.st(pend, pv);
        const uint2 wc = pl[(t + 2 * NW) * 64];
        const T xb = ms.ld(slot(wb));
        pv = edge(xa, wa);
        pend = slot(wa);
        t += NW;
        if (t >= n_tasks) break;
        ms.st(pend, pv);
        wa = pl[(t + 2 * NW) * 64];
        xa = ms.ld(slot(wc));
        pv = edge(xb, wb);
        pend = slot(wb);
        t += NW;
        if (t >= n_tasks) break;
        wb = wa;
        wa = wc;
    }
    ms.st(pend, pv);
}

// Flooding sum-product decode of whole frames, one frame per workgroup at a
// time, frames from the device queue (as decode_kernel). RULE is kRuleSp64
// (the reference, bit-exact) or kRuleSp32 (the binary32 variant).
template <int MODE, int RULE, int DC, bool CLAMP>
__global__ __launch_bounds__(kDecodeBlock) void decode_split_kernel(DecodeArgs a) {
    using T = typename RuleMsg<RULE>::T;
    constexpr bool TABLES = MODE == kModeKeys && RULE == kRuleSp64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const DeviceCode& c = a.code;
    const SplitLds L(c.n_pad, (c.n + 63) / 64, c.m, c.max_dv, DC, a.tab2_entries, (int)sizeof(T), a.lds_budget);
    const int m_words = decode_m_words(c.m);
    uint32_t* tsyn = reinterpret_cast<uint32_t*>(smem + L.tsyn);
    uint32_t* xsyn = reinterpret_cast<uint32_t*>(smem + L.xsyn);
    uint32_t* qsyn = reinterpret_cast<uint32_t*>(smem + L.qsyn);
    uint64_t* zw = reinterpret_cast<uint64_t*>(smem + L.zw);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + L.ctl);
    double* ctab = reinterpret_cast<double*>(smem + L.ctab);
    double* tab2 = reinterpret_cast<double*>(smem + L.tab2);
    const SplitStore<T> ms{
        reinterpret_cast<T*>(smem + L.msg),
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<T*>(a.c2b) + (size_t)blockIdx.x * a.c2b_stride, (short)0,
                                          (int)(a.c2b_stride * sizeof(T)), 0x00020000),
        L.S};
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    T* row = reinterpret_cast<T*>(smem + L.tval) + wave * (64 + DC);
    const int n_tasks = c.n_tasks;
    const uint32_t n_pad = (uint32_t)c.n_pad;
    const T thr = (T)a.thr;
    const T llr_p = (T)a.log_p;
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;     // sign bit of log_p
    // the first check phase is folded into the first bit phase (QKD path;
    // the fold rebuilds the unrolled rows only)
    const bool fold1 = TABLES && a.first_table && c.max_dv <= kDvUnroll;
    const bool tab2_on = fold1 && a.tab2_entries;
    uint32_t any_k = 0;
    if (tid == 0) { ctl[2] = 0; ctl[3] = 0; }
    if (TABLES && tid <= kFirstTableDeg) ctab[tid] = a.first_c2b[tid];
    if (tab2_on) {
        __syncthreads();
        second_table_fill<CLAMP>(c, ctab, a.log_p, a.thr, tab2, a.tab2_entries);
    }
    PhaseClock pc(a.phase);

    for (;;) {
        pc.mark(4);
        if (tid == 0) ctl[0] = atomicAdd(a.counter, 1u);
        for (int w = tid; w < m_words; w += kDecodeBlock) xsyn[w] = 0;
        __syncthreads();
        const uint32_t f = ctl[0];
        if (f >= a.n_frames) break;

        // ---- prologue: the frame's Alice and Bob words staged in LDS (the
        //      product rows are free until the first check phase)
        const uint64_t* sw = reinterpret_cast<const uint64_t*>(smem + L.tval);   // [alice | bob]
        if (MODE == kModeKeys) {
            uint64_t* w = reinterpret_cast<uint64_t*>(smem + L.tval);
            for (int q = tid; q < (int)a.words; q += kDecodeBlock) {
                w[q] = a.alice_w[(size_t)f * a.words + q];
                w[a.words + q] = a.bob_w[(size_t)f * a.words + q];
            }
            __syncthreads();
        }
        // Bob's bits of this thread's bit-phase rounds (round r: bit tid + r *
        // kDecodeBlock; N <= 32 * kDecodeBlock, kMaxBitsLds). Without the fold
        // the first check phase reads b2c = LLR_i (:188) from every slot.
        uint32_t bobmask = 0;
        {
            int r = 0;
            for (int i = tid; i < c.n; i += kDecodeBlock, ++r) {
                T l;
                if (MODE == kModeLlr) {
                    l = (T)a.llr[(size_t)f * c.n + i];
                } else {
                    const uint32_t bb = (uint32_t)((sw[a.words + (i >> 6)] >> (i & 63)) & 1u);
                    bobmask |= bb << r;
                    l = bb ? -llr_p : llr_p;
                }
                if (!fold1) {
                    const int deg = c.bit_deg[i];
                    for (int k = 0; k < deg; ++k) ms.st((uint32_t)k * n_pad + i, l);
                }
            }
            // the dummy column's slot (idle plan lanes): a finite value, and
            // table index 0 for the second check phase
            if (tid == 0) ms.st((uint32_t)c.n, (T)0);
        }
        // ---- prologue: target syndrome bits per check (tsyn) and, on the QKD
        //      path, each check's first-product sign (qsyn); thread per check
        for (int j0 = wave * 64; j0 < c.m; j0 += kDecodeBlock) {
            const int j = j0 + lane;
            const bool ok = j < c.m;
            int sj = 0, qj = 0;
            if (MODE == kModeLlr) {
                sj = ok ? (a.syn[(size_t)f * c.m + j] != 0) : 0;
            } else {
                // calculate_syndrome_irregular on Alice's key (:413-414), and
                // q_j = s_j ^ syn(bob)_j ^ (deg_j & sign(log_p))
                uint32_t pa = 0, pb = 0, deg = 0;
                for (int k = 0; k < c.max_dc; ++k) {
                    const int bit = ok ? c.chk_bits[k * c.m_pad + j] : -1;
                    if (bit >= 0) {
                        pa ^= (uint32_t)(sw[bit >> 6] >> (bit & 63));
                        pb ^= (uint32_t)(sw[a.words + (bit >> 6)] >> (bit & 63));
                        deg++;
                    }
                }
                sj = (int)(pa & 1u);
                qj = (int)((pa ^ pb ^ (lsign & deg)) & 1u);
            }
            const uint64_t sm = __ballot(sj);
            const uint64_t qm = __ballot(qj);
            if (lane == 0) {
                tsyn[j0 >> 5] = (uint32_t)sm;
                tsyn[(j0 >> 5) + 1] = (uint32_t)(sm >> 32);
                qsyn[j0 >> 5] = (uint32_t)qm;
                qsyn[(j0 >> 5) + 1] = (uint32_t)(qm >> 32);
            }
        }
        __syncthreads();
        pc.mark(0);

        // ---- iterations (:212-330)
        bool done = false;
        uint32_t it = 0;
        for (; it < a.max_it; ++it) {
            const bool folded = fold1 && it == 0;
            if (!folded) {
                if (TABLES && it == 1 && tab2_on)
                    split_check_phase<kSrcTable, CLAMP, DC, RULE>(c.plan, tsyn, tab2, ms, row, n_tasks, n_pad, thr,
                                                                   wave, lane);
                else
                    split_check_phase<kSrcFirst, CLAMP, DC, RULE>(c.plan, tsyn, tab2, ms, row, n_tasks, n_pad, thr,
                                                                   wave, lane);
                __syncthreads();
            }
            pc.mark((TABLES && it < 2 && fold1) ? 5 + (int)it : 1);
            // the b2c of this bit phase are read only by a next iteration
            const bool keep = it + 1 < a.max_it;
            // bit phase: total_i = LLR_i + sum_k c2b[k][i], ascending checks (:256-267),
            // the hard decision's syndrome (:277, calculate_syndrome_irregular :476-486),
            // then b2c_k = clamp(total_i - c2b_k) (:303-316) into slot k.
            for (int r0 = 0; r0 * kDecodeBlock < c.n; r0 += kBitChunk) {
                T v[kBitChunk][kDvUnroll];
                int32_t jc[kBitChunk][kDvUnroll];
                int dg[kBitChunk];
#pragma unroll
                for (int u = 0; u < kBitChunk; ++u) {
                    const int i = tid + (r0 + u) * kDecodeBlock;
                    const bool ok = i < c.n;
                    dg[u] = ok ? c.bit_deg[i] : 0;
                    // the wave's 64 bits are consecutive: row k's slots start at
                    // xw (wave-uniform). Slots past the bit's degree (or past N)
                    // are read harmlessly (holes, or out of the buffer's range:
                    // 0) and never summed.
                    const uint32_t iw = (uint32_t)((r0 + u) * kDecodeBlock + wave * 64);
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) {
                        const bool ld = ok && k < c.max_dv;
                        const uint32_t x = (uint32_t)k * n_pad + i;
                        v[u][k] = folded ? (T)0 : ms.ld_row((uint32_t)k * n_pad + iw, x);
                        jc[u][k] = ld ? c.bit_chk[k * n_pad + i] : 0;
                    }
                }
#pragma unroll
                for (int u = 0; u < kBitChunk; ++u) {
                    const int r = r0 + u;
                    if (r * kDecodeBlock >= c.n) break;            // block-uniform
                    const int i = tid + r * kDecodeBlock;
                    const uint32_t iw = (uint32_t)(r * kDecodeBlock + wave * 64);
                    const bool ok = i < c.n;
                    const int deg = dg[u];
                    T acc;
                    if (MODE == kModeLlr) acc = ok ? (T)a.llr[(size_t)f * c.n + i] : (T)0;
                    else acc = ((bobmask >> r) & 1u) ? -llr_p : llr_p;
                    if constexpr (TABLES) if (folded && ok) {
                        // fold_first_message: message of the k-th check j of bit i is
                        // +-C_{d_j} with sign = sign(P_j) ^ sign(LLR_i) (first_check_phase)
                        const uint32_t sgi = ((bobmask >> r) & 1u) ^ lsign;
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k) {
                            if (k < deg) {
                                const int j = jc[u][k];
                                const uint32_t sp = (qsyn[j >> 5] >> (j & 31)) & 1u;
                                const double cm = ctab[c.chk_deg[j]];
                                v[u][k] = (sp ^ sgi) ? -cm : cm;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) acc = k < deg ? acc + v[u][k] : acc;
                    for (int k = kDvUnroll; k < deg; ++k) acc = acc + ms.ld((uint32_t)k * n_pad + i);
                    // hard decision z_i = total_i <= 0 (NaN -> 0), one ballot word per wave
                    const bool z = ok && acc <= 0;
                    const uint64_t zb = __ballot(z);
                    if (lane == 0 && r * kDecodeBlock + wave * 64 < c.n) zw[(r * kDecodeBlock >> 6) + wave] = zb;
#ifdef QKD_EXP_NO_SYN
                    if (false) {
#else
                    if (z) {
#endif
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k)
                            if (k < deg) atomicXor(&xsyn[jc[u][k] >> 5], 1u << (jc[u][k] & 31));
                        for (int k = kDvUnroll; k < deg; ++k) {
                            const int j = c.bit_chk[k * n_pad + i];
                            atomicXor(&xsyn[j >> 5], 1u << (j & 31));
                        }
                    }
                    if (!keep || !ok) continue;
                    if (TABLES && folded && tab2_on) {
                        // second_table_index: Bob's bit and the signs of the first
                        // messages; the slot of row k keeps the index of its entry
                        uint32_t code = (bobmask >> r) & 1u;
#pragma unroll
                        for (int k = 0; k < kTab2MaxDv; ++k)
                            if (k < deg) code |= ((uint32_t)qkdm::hi32(v[u][k]) >> 31) << (1 + k);
                        const uint32_t base = (uint32_t)(c.bit_pat[i] * tab2_stride(c.max_dv)) + code * c.max_dv;
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k)
                            if (k < deg)
                                ms.st_row((uint32_t)k * n_pad + iw, (uint32_t)k * n_pad + i,
                                          (T)qkdm::from_bits(base + k));
                    } else {
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k) {
                            if (k < deg) {
                                T b = acc - v[u][k];
                                if (CLAMP) b = clamp_msg(b, thr);
                                ms.st_row((uint32_t)k * n_pad + iw, (uint32_t)k * n_pad + i, b);
                            }
                        }
                        for (int k = kDvUnroll; k < deg; ++k) {
                            const uint32_t x = (uint32_t)k * n_pad + i;
                            T b = acc - ms.ld(x);
                            if (CLAMP) b = clamp_msg(b, thr);
                            ms.st(x, b);
                        }
                    }
                }
            }
            __syncthreads();
            pc.mark(2);
            // syndrome test (:285): any word differing from the target
            bool mismatch = false;
            for (int w = tid; w < m_words; w += kDecodeBlock) {
                mismatch |= xsyn[w] != tsyn[w];
                xsyn[w] = 0;
            }
            const bool any_mismatch = block_any(mismatch, ctl + 2, any_k);
            pc.mark(3);
#ifndef QKD_EXP_NO_STOP
            if (!any_mismatch) {
                done = true;
                break;
            }
#endif
        }

        // ---- outputs: SP_result + last hard decision (+ keys_match)
        bool key_mismatch = false;
        for (int i = tid; i < c.n; i += kDecodeBlock) {
            const uint8_t d = (uint8_t)((zw[i >> 6] >> (i & 63)) & 1u);
            if (a.bits_out) a.bits_out[(size_t)f * c.n + i] = d;
            if (MODE == kModeKeys) {
                const uint64_t w = a.alice_w[(size_t)f * a.words + (i >> 6)];
                key_mismatch |= (uint8_t)((w >> (i & 63)) & 1u) != d;
            }
        }
        if (MODE == kModeKeys) {
            __syncthreads();
            const bool km = block_any(key_mismatch, ctl + 2, any_k);
            if (tid == 0 && a.key_ok) a.key_ok[f] = km ? 0 : 1;   // arrays_equal (:433)
        }
        if (tid == 0) {
            a.iters[f] = done ? it + 1 : a.max_it;
            a.sp_ok[f] = done ? 1 : 0;
        }
        __syncthreads();
    }
    pc.flush();
}

template <int MODE, int RULE, bool CLAMP>
static DecodeFn pick_split_dc(int max_dc, int* dc) {
    if (max_dc <= 4) { *dc = 4; return decode_split_kernel<MODE, RULE, 4, CLAMP>; }
    if (max_dc <= 6) { *dc = 6; return decode_split_kernel<MODE, RULE, 6, CLAMP>; }
    if (max_dc <= 8) { *dc = 8; return decode_split_kernel<MODE, RULE, 8, CLAMP>; }
    if (max_dc <= 16) { *dc = 16; return decode_split_kernel<MODE, RULE, 16, CLAMP>; }
    *dc = 64;
    return decode_split_kernel<MODE, RULE, 64, CLAMP>;
}

template <int MODE, int RULE>
static DecodeFn pick_split_clamp(bool clamp, int max_dc, int* dc) {
    return clamp ? pick_split_dc<MODE, RULE, true>(max_dc, dc) : pick_split_dc<MODE, RULE, false>(max_dc, dc);
}

template <int MODE>
static DecodeFn pick_split_rule(int rule, bool clamp, int max_dc, int* dc) {
    if (rule == kRuleSp32) return pick_split_clamp<MODE, kRuleSp32>(clamp, max_dc, dc);
    return pick_split_clamp<MODE, kRuleSp64>(clamp, max_dc, dc);
}

DecodeFn pick_split_decode(int mode, int rule, bool clamp, int max_dc, int* dc) {
    return mode == kModeLlr ? pick_split_rule<kModeLlr>(rule, clamp, max_dc, dc)
                            : pick_split_rule<kModeKeys>(rule, clamp, max_dc, dc);
}

}  // namespace qkd
