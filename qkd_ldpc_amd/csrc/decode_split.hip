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

#include <type_traits>

#include "qkd_decode.h"
#include "qkd_spec.h"

namespace qkd {

// Running syndrome (QKD_RUN_SYN): xsyn holds H * (the current hard
// decision) across iterations -- initialised per frame to H * bob (keys path;
// from frame_syn's words) or 0 (LLR path, decision words 0) -- and each bit
// phase XORs into it only the decisions that changed against the packed
// words of the last one (zw), instead of every 1 decision into a zeroed xsyn:
// at QBER 0.02 a few percent of the bits change per iteration, where about
// half of them are 1, and the LDS atomics run ~8-way bank-conflicted
// (tools/mb/lds_bank_mb.hip).
#ifndef QKD_RUN_SYN
#define QKD_RUN_SYN 1
#endif
constexpr bool kRunSyn = QKD_RUN_SYN != 0;

// The weight of row entry k in the extrinsic sum of a lane at position p
// (= lane - start) of a segment of degree deg (qkd_decode.h seg_weight_entries).
template <int DC>
struct SegWeights {
    const float* w;         // DC <= 8: wtab row of (deg, p)
    uint64_t mask;          // otherwise: bit k = weight of entry k
    __device__ __forceinline__ SegWeights(const float* wtab, int deg, int p) {
        if constexpr (DC <= 8) {
            // (idle lanes: a degree-1 segment starting at lane 0, p = lane;
            // any p >= 1 gives their only weight, entry 0)
            w = wtab + (deg * 8 + min(p, DC - 1)) * DC;
            mask = 0;
        } else {
            // 64-bit: deg reaches 64 in the widest bucket and p (= lane - start)
            // any lane 0..63 for idle lanes; both shifts stay below 64
            w = nullptr;
            const uint64_t seg = deg >= 64 ? ~0ull : ((1ull << (uint32_t)deg) - 1ull);
            mask = seg & ~(1ull << ((uint32_t)p & 63u));
        }
    }
    __device__ __forceinline__ float operator[](int k) const {
        if constexpr (DC <= 8) return w[k];
        else return (float)(uint32_t)((mask >> (uint32_t)k) & 1ull);
    }
};

// A lane's segment and target bit from an encoded plan word (encode_seg).
__device__ __forceinline__ int seg_start(uint2 w) { return (int)((w.y >> kSegStartShift) & 63u); }
__device__ __forceinline__ uint32_t seg_wi(uint2 w) { return (w.y >> kSegWiShift) & 255u; }
template <int DC>
__device__ __forceinline__ int seg_deg(uint2 w) {
    if constexpr (DC <= 8) return (int)((w.y >> (kSegWiShift + 3)) & 15u);
    return DC <= 16 ? (int)(seg_wi(w) / (uint32_t)DC) + 1 : (int)seg_wi(w) + 1;
}
template <int DC>
__device__ __forceinline__ SegWeights<DC> seg_weights(const float* wtab, uint2 w, int lane) {
    if constexpr (DC <= 8) {
        SegWeights<DC> r(wtab, 1, 0);
        r.w = wtab + seg_wi(w) * DC;
        return r;
    } else {
        return SegWeights<DC>(wtab, seg_deg<DC>(w), lane - seg_start(w));
    }
}
// the check's target bit: its syndrome word read from LDS address 0 on (tsyn
// leads the layout, SplitLds, and the dynamic LDS starts at 0)
__device__ __forceinline__ uint32_t seg_sbit(uint2 w) {
    typedef __attribute__((address_space(3))) const uint32_t LdsU32;
    const uint32_t word = *reinterpret_cast<LdsU32*>((size_t)(w.y >> kSegWordShift));
    return (word >> (w.y & 31u)) & 1u;
}
// parity of the segment's bits in a wave ballot (seg_parity of qkd_decode.h)
// xor the low bits of add (two one-bit terms at most): the popcount's own
// accumulator (v_bcnt_u32_b32) takes the sum, no separate xors (-0.7 % per
// config-2 batch, profiles/r06_ab.txt)
template <int DC>
__device__ __forceinline__ uint32_t seg_parity_acc(uint64_t ballot, uint2 w, uint32_t add) {
    const uint64_t sh = ballot >> seg_start(w);
    const uint32_t deg = (uint32_t)seg_deg<DC>(w);
    if constexpr (DC < 32) return ((uint32_t)__popc(__builtin_amdgcn_ubfe((uint32_t)sh, 0, deg)) + add) & 1u;
    const uint64_t m = deg >= 64 ? ~0ull : ((1ull << deg) - 1ull);
    return ((uint32_t)__popcll(sh & m) + add) & 1u;
}
template <int DC>
__device__ __forceinline__ uint32_t seg_parity_enc(uint64_t ballot, uint2 w) {
    const uint64_t sh = ballot >> seg_start(w);
    const uint32_t deg = (uint32_t)seg_deg<DC>(w);
    if constexpr (DC < 32) return (uint32_t)__popc(__builtin_amdgcn_ubfe((uint32_t)sh, 0, deg)) & 1u;
    const uint64_t m = deg >= 64 ? ~0ull : ((1ull << deg) - 1ull);
    return (uint32_t)__popcll(sh & m) & 1u;
}

// The extrinsic interval sum of a speculative check phase: sum over k < DC of
// row[start + k] times its weight (0 or 1, exact), in ascending order (a
// pairwise tree, depth ~log2(DC) for two more operations, measured no faster:
// DESIGN.md §4.3). The caller charges its rounding relative to the sum.
#ifndef QKD_SEG_BATCH
#define QKD_SEG_BATCH 1
#endif
template <int DC>
__device__ __forceinline__ qkds::f2 seg_sum(const double* row, int start, const SegWeights<DC>& wk) {
    qkds::f2 sum = qkds::f2{0.0f, 0.0f};
    if constexpr (QKD_SEG_BATCH && DC <= 8) {
        // every row entry and weight read before the first use (a scheduling
        // barrier: left alone, the scheduler reuses registers and serialises
        // the reads into DC / 2 LDS round trips)
        qkds::f2 v[DC];
        float w[DC];
#pragma unroll
        for (int k = 0; k < DC; ++k) v[k] = qkds::unpack_iv(row[start + k]);
#pragma unroll
        for (int k = 0; k < DC; ++k) w[k] = wk[k];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < DC; ++k) sum = __builtin_elementwise_fma(v[k], qkds::f2(w[k]), sum);
        return sum;
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) sum = __builtin_elementwise_fma(qkds::unpack_iv(row[start + k]), qkds::f2(wk[k]), sum);
    return sum;
}

// Lane `lane`'s word of plan task t through a buffer descriptor: the task's
// offset is a scalar operand and the lane's a loop-invariant VGPR, so a load
// costs no vector address arithmetic (a pointer form becomes a 64-bit VGPR
// induction variable, two adds per load). t is wave-uniform; readfirstlane
// says so where the compiler cannot prove it (else it emits a waterfall loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plan_rsrc(const uint2* plan) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2*>(plan), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ uint2 plan_word(__amdgpu_buffer_rsrc_t plan, int t, int lane) {
    using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(plan, 0, 0, 0));
    const V v = __builtin_amdgcn_raw_buffer_load_b64(plan, (int)((uint32_t)lane * 8u),
                                                       __builtin_amdgcn_readfirstlane(t * 64 * 8), 0);
    return __builtin_bit_cast(uint2, v);
}

// a wave mask folded to 32 bits, nonzero iff the mask is (scalar ors)
__device__ __forceinline__ uint32_t fold64(uint64_t m) { return (uint32_t)m | (uint32_t)(m >> 32); }

// [lo, hi] negated: [-hi, -lo] when neg. Written per element, so each half is
// one v_cndmask_b32 with a negated source (the vector form costs a packed
// negation and a swap besides).
__device__ __forceinline__ qkds::f2 neg_iv_if(bool neg, qkds::f2 v) {
    return qkds::f2{neg ? -v.y : v.x, neg ? -v.x : v.y};
}

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
    // a lane offset plus a wave-uniform one (soffset: scalar arithmetic only)
    static __device__ __forceinline__ double ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
    }
    static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double v) {
        using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V, v), r, (int)voff, (int)soff, 0);
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

// ALL: every slot is in LDS (the host launches that instantiation only when
// they fit): plain LDS accesses.
template <typename T, bool ALL = false>
struct SplitStore {
    T* l;                        // LDS slots [0, S) and the trash slots [S, S + 64)
    uint32_t S;
    // The global slots S.. of this workgroup: ONE buffer descriptor, gw below
    // (the check phases' encoded words address it directly; a slot index x >=
    // S is at byte offset x * size + goff, goff = kSlotGlobalBase - S * size).
    // One descriptor instead of two: 4 SGPRs fewer in a kernel whose uniform
    // values already spill to VGPR lanes, read back by v_readlane in the hot
    // loops (-1.9 % per config-2 batch with the epilogue below, A/B).
    // (for x < S the offset is kSlotLds: past the descriptor's range, the
    // load gives 0 and the store is dropped)
    __device__ __forceinline__ uint32_t gofs(uint32_t x) const { return x * (uint32_t)sizeof(T) + goff; }
    __device__ __forceinline__ T ld(uint32_t x) const {
        if constexpr (ALL) return l[x];
        const bool in = x < S;
        const T vl = l[in ? x : 0u];
        const T vg = BufIo<T>::ld(gw, in ? kSlotLds : gofs(x));
        return in ? vl : vg;
    }
    // The check phases address slots by encoded words (encode_slot,
    // qkd_decode.h; DecodeArgs::plan_enc): an LDS slot's word is its byte
    // address with kSlotLds set, which the buffer range check rejects; a
    // global slot's word is its byte offset in the region past
    // kSlotGlobalBase, an LDS address past any allocation (the hardware
    // returns 0 and drops the store there, tools/mb/lds_oob.hip). So both
    // accesses take the word as it is (the LDS one without its top bit), and
    // a load is the OR of the two halves: no compare, no select.
    __amdgpu_buffer_rsrc_t gw;   // the region, kSlotGlobalBase bytes before its start
    uint32_t goff;
    // ld_w in two halves for a software pipeline: ld_raw issues both accesses,
    // pick (at the value's first use, a loop iteration later) combines them
    struct Raw {
        T vl, vg;
    };
    // (the byte addresses are absolute: the dynamic LDS starts at address 0,
    // the split kernels having no static LDS, which the host checks)
    typedef __attribute__((address_space(3))) T LdsT;
    __device__ __forceinline__ LdsT* lds_of(uint32_t w) const {
        return reinterpret_cast<LdsT*>((size_t)(w & ~kSlotLds));
    }
    __device__ __forceinline__ Raw ld_raw(uint32_t w) const {
        return Raw{*lds_of(w), BufIo<T>::ld(gw, w)};
    }
    __device__ __forceinline__ T pick(const Raw& r) const {
        if constexpr (sizeof(T) == 8)
            return __builtin_bit_cast(T, __builtin_bit_cast(uint64_t, r.vl) | __builtin_bit_cast(uint64_t, r.vg));
        else
            return __builtin_bit_cast(T, __builtin_bit_cast(uint32_t, r.vl) | __builtin_bit_cast(uint32_t, r.vg));
    }
    __device__ __forceinline__ T ld_w(uint32_t w) const { return pick(ld_raw(w)); }
    __device__ __forceinline__ void st_w(uint32_t w, T v) const {
        *lds_of(w) = v;
        BufIo<T>::st(gw, w, v);
    }
    __device__ __forceinline__ void st(uint32_t x, T v) const {
        if constexpr (ALL) {
            l[x] = v;
            return;
        }
        const bool in = x < S;
        l[in ? x : S + (threadIdx.x & 63u)] = v;
        BufIo<T>::st(gw, in ? kSlotLds : gofs(x), v);
    }
    // slots x .. x + 63 of a wave's 64 consecutive lanes (xw = the wave's
    // first slot, wave-uniform, a multiple of 64 as S is: SplitLds): all in
    // LDS or all global, one kind of access
    __device__ __forceinline__ T ld_row(uint32_t xw, uint32_t x) const {
        if (ALL || xw < S) return l[x];
        return BufIo<T>::ld(gw, gofs(x));
    }
    __device__ __forceinline__ void st_row(uint32_t xw, uint32_t x, T v) const {
        if (ALL || xw < S)
            l[x] = v;
        else
            BufIo<T>::st(gw, gofs(x), v);
    }
};

// Check phase of one iteration for one wave (tasks wave, wave + NW, ...):
// per edge the incoming b2c (or, SRC == kSrcTable, its table index) from the
// edge's slot, the outgoing c2b back into it. Software-pipelined exactly as
// check_phase (decode.hip): the plan word two tasks ahead and the slot one
// task ahead are loaded before this task's arithmetic; stores trail by one
// task. Slots of different tasks are distinct (idle lanes share the dummy
// column's slot, whose value nothing reads).
template <int SRC, bool CLAMP, int DC, int RULE, typename T, typename MS>
__device__ __forceinline__ void split_check_phase(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                  const double* tab2, const MS& ms, T* row,
                                                  int n_tasks, uint32_t n_pad, T thr, int wave, int lane) {
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const __amdgpu_buffer_rsrc_t prs = plan_rsrc(plan);
    auto slot = [&](uint2 p) -> uint32_t { return pw_slot(p); };
    auto edge = [&](T x, uint2 w) -> T {
        T a;
        if constexpr (SRC == kSrcTable && RULE == kRuleSp64)
            a = tab2[qkdm::lo32(x)];
        else
            a = RuleMath<RULE>::tanh_half(x);                      // (:224)
        row[lane] = a;
        wave_lds_sync();
        // (edge_out reads the segment from a plan word of the unencoded form)
        const uint2 wo = make_uint2(w.x, ((uint32_t)seg_start(w) << 20) | ((uint32_t)(seg_deg<DC>(w) - 1) << 26));
        return edge_out<CLAMP, DC, RULE>(a, wo, seg_sbit(w), lane, thr, row, 0.0f);
    };
    uint2 wa = plan_word(prs, t, lane);
    uint2 wb = plan_word(prs, t + NW, lane);
    auto xa = ms.ld_raw(slot(wa));
    uint32_t pend = 0xffffffffu;    // slot of the previous task's message, not yet stored
    T pv = 0;
    for (;;) {
        if (pend != 0xffffffffu) ms.st_w(pend, pv);
        const uint2 wc = plan_word(prs, t + 2 * NW, lane);
        const auto xb = ms.ld_raw(slot(wb));
        pv = edge(ms.pick(xa), wa);
        pend = slot(wa);
        t += NW;
        if (t >= n_tasks) break;
        ms.st_w(pend, pv);
        wa = plan_word(prs, t + 2 * NW, lane);
        xa = ms.ld_raw(slot(wc));
        pv = edge(ms.pick(xb), wb);
        pend = slot(wb);
        t += NW;
        if (t >= n_tasks) break;
        wb = wa;
        wa = wc;
    }
    ms.st_w(pend, pv);
}

// ---- the binary32 variant (kRuleSp32; specification: tests/test_variants.py) 
// Check phase of the binary32 rule (edge_out's Gallager form, bit for bit):
// psi(|b2c|) of the NEXT task's edge and phi of this task's extrinsic sum in
// one packed evaluation (RuleMath<kRuleSp32>::pair), the message sign as the
// segment parity of one ballot. The row holds the magnitudes |psi|; the sum
// adds them in ascending lane order with weight 0 for this lane and for lanes
// past the segment (x + 0 * y = x exactly), as edge_out skips them. Every slot
// is in LDS (SplitStore<float, true>). Otherwise pipelined as
// spec_check_phase_paired.
template <bool CLAMP, int DC, typename MS>
__device__ __forceinline__ void sp32_check_phase(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                 const MS& ms, float* row, const float* wtab, int n_tasks,
                                                 uint32_t n_pad, float thr, int wave, int lane) {
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const __amdgpu_buffer_rsrc_t prs = plan_rsrc(plan);
    if (lane < DC) row[64 + lane] = 0.0f;
    auto slot = [&](uint2 p) -> uint32_t { return pw_slot(p); };
    uint2 wt = plan_word(prs, t, lane);
    uint2 wn = plan_word(prs, t + NW, lane);
    uint2 wnn = plan_word(prs, t + 2 * NW, lane);
    float xt = ms.ld(slot(wt));
    row[lane] = __builtin_fabsf(RuleMath<kRuleSp32>::tanh_half(xt));
    uint64_t sgn_t = __ballot(xt < 0.0f);
    bool neg_t = xt < 0.0f;
    float xn = ms.ld(slot(wn));
    for (;;) {
        const uint2 w3 = plan_word(prs, t + 3 * NW, lane);
        const float xnn = ms.ld(slot(wnn));
        wave_lds_sync();
        const int start = pw_start(wt);
        const int deg = pw_deg(wt);
        const SegWeights<DC> wk(wtab, deg, lane - start);
        float S = 0.0f;
#pragma unroll
        for (int k = 0; k < DC; ++k) S = __builtin_fmaf(row[start + k], wk[k], S);
        const qkds::f2 pv = RuleMath<kRuleSp32>::pair(xn, S);
        const uint32_t j = pw_chk(wt);
        const uint32_t neg = ((tsyn[j >> 5] >> (j & 31)) & 1u) ^
                             (uint32_t)(DC < 32 ? seg_parity32(sgn_t, wt) : seg_parity(sgn_t, wt)) ^
                             (neg_t ? 1u : 0u);
        // pv.y >= +0 is never NaN (the sum enters through fminf), so clamp_msg
        // of +-pv.y is +-med3(pv.y, 0, thr) (thr > 0: check_decode_params)
        const float m = CLAMP ? __builtin_amdgcn_fmed3f(pv.y, 0.0f, thr) : pv.y;
        ms.st(slot(wt), neg ? -m : m);
        row[lane] = pv.x;
        sgn_t = __ballot(xn < 0.0f);
        neg_t = xn < 0.0f;
        t += NW;
        if (t >= n_tasks) break;
        wt = wn;
        wn = wnn;
        wnn = w3;
        xn = xnn;
    }
}

// ---- min-sum on the split skeleton (kRuleMinSumSplit / kRuleMinSumSplitSc) --
// The binary32 rules' all-LDS store (4 bytes per edge, SplitStore<float,
// true>) and their bit phase (sp32_bit_phase); the check phase per edge
// (the min-sum specification tests/test_variants.py checks, bit for bit):
//   c2b = (-1)^(s_j + #negative other b2c) * max(scale * min |other b2c| - off, 0),
//   clamped (:246-249)
// The extrinsic min reads the task's row of |b2c| through an additive mask
// table (mtab: 0 for the segment's other lanes, +inf for this lane and past
// the segment), so it is one add and one min per row entry (v_min3 pairs),
// NaN magnitudes ignored as fminf does; the sign is the segment parity of one
// ballot, as sp32_check_phase's.
// SC (Savin's self-correction, QKD_MINSUM_SELF_CORRECT): a b2c whose sign
// differs from the edge's previous b2c, both nonzero, is erased to 0 before
// the rule. The previous b2c of every edge is two ballot words per task in
// LDS (scw[2 t]: negative, scw[2 t + 1]: nonzero), read and rewritten by the
// task's wave. sc_mode: 0 the frame's first check phase (no previous b2c), 1
// the previous b2c from scw, 2 the check phase after the folded first
// iteration, whose b2c were the channel LLRs: negative iff Bob's bit of the
// edge (bwl, the frame's key words) differs from the sign of log_p (lsign),
// nonzero (the fold needs log_p != 0); the edge's bit is its slot index
// (the plan word's LDS address, msg the first slot's) modulo n_pad.
template <bool CLAMP, int DC, bool SC, bool OFF, typename MS>
__device__ __forceinline__ void ms_split_check_phase(const uint2* __restrict__ plan, const MS& ms, float* row,
                                                     const float* mtab, uint64_t* scw, int sc_mode,
                                                     const uint64_t* bwl, uint32_t msg, uint32_t n_pad,
                                                     uint32_t lsign, int n_tasks, float thr, float scale, float off,
                                                     int wave, int lane) {
    static_assert(DC <= 8, "min-sum split buckets: check degree <= 8 (the mask table)");
    typedef __attribute__((address_space(3))) float LdsF;
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const __amdgpu_buffer_rsrc_t prs = plan_rsrc(plan);
    // (entries past lane 63 are read by segments ending there, masked: finite)
    if (lane < DC) row[64 + lane] = 0.0f;
    // the plan is encoded for this layout (plan_for_layout, binary32): the
    // slot's LDS byte address, and encode_seg's pre-decoded segment fields
    auto slot = [](uint2 p) -> LdsF* { return reinterpret_cast<LdsF*>((size_t)p.x); };
    // b2c of task tt's edge after the self-correction; records it as the
    // edge's previous b2c
    auto input = [&](float x, uint2 w, int tt) -> float {
        if constexpr (SC) {
            if (sc_mode != 0) {
                bool pn, pz;      // the previous b2c: negative, nonzero
                if (sc_mode == 1) {
                    pn = ((scw[2 * tt] >> lane) & 1ull) != 0;
                    pz = ((scw[2 * tt + 1] >> lane) & 1ull) != 0;
                } else {
                    uint32_t i = (w.x - msg) >> 2;          // (bit degree <= 3: bit_code)
                    i = i >= n_pad ? i - n_pad : i;
                    i = i >= n_pad ? i - n_pad : i;
                    pn = ((uint32_t)(bwl[i >> 6] >> (i & 63u)) & 1u) != lsign;
                    pz = true;
                }
                const bool er = pz && x != 0.0f && (x < 0.0f) != pn;
                x = er ? 0.0f : x;
            }
            const uint64_t nneg = __ballot(x < 0.0f), nnz = __ballot(x != 0.0f);
            if (lane == 0) {
                scw[2 * tt] = nneg;
                scw[2 * tt + 1] = nnz;
            }
        }
        return x;
    };
    uint2 wt = plan_word(prs, t, lane);
    uint2 wn = plan_word(prs, t + NW, lane);
    uint2 wnn = plan_word(prs, t + 2 * NW, lane);
    float xt = input(*slot(wt), wt, t);
    row[lane] = __builtin_fabsf(xt);
    uint64_t sgn_t = __ballot(xt < 0.0f);
    bool neg_t = xt < 0.0f;
    // One task: task t's c2b from the row, then task t + NW's row entry from
    // its slot (read a task earlier); loads the plan word three tasks ahead
    // (w_ld) and the slot of task t + 2 NW (x_ld). Unrolled four times over
    // rotating registers: no copies, so no load is waited for early.
    auto step = [&](const uint2 w_t, const uint2 w_n, const uint2 w_nn, uint2& w_ld, const float x_n,
                    float& x_ld) -> bool {
        w_ld = plan_word(prs, t + 3 * NW, lane);
        x_ld = *slot(w_nn);
        wave_lds_sync();
        const int start = seg_start(w_t);
        const float* mk = mtab + seg_wi(w_t) * DC;
        float mn = __builtin_inff();
#pragma unroll
        for (int k = 0; k < DC; ++k) mn = __builtin_fminf(mn, row[start + k] + mk[k]);
        float v = scale * mn;
        if constexpr (OFF) v = __builtin_fmaxf(v - off, 0.0f);
        const uint32_t neg = seg_sbit(w_t) ^ seg_parity_enc<DC>(sgn_t, w_t) ^ (neg_t ? 1u : 0u);
        // v >= +0 is never NaN (the chain starts at +inf), so clamp_msg of +-v
        // is +-med3(v, 0, thr)
        const float m = CLAMP ? __builtin_amdgcn_fmed3f(v, 0.0f, thr) : v;
        *slot(w_t) = neg ? -m : m;
        t += NW;
        if (t >= n_tasks) return false;
        // the next task's row (after this task's row reads: a wave's LDS
        // accesses complete in order)
        const float xc = input(x_n, w_n, t);
        row[lane] = __builtin_fabsf(xc);
        sgn_t = __ballot(xc < 0.0f);
        neg_t = xc < 0.0f;
        return true;
    };
    float xa = *slot(wn), xb;
    uint2 wd;
    for (;;) {
        if (!step(wt, wn, wnn, wd, xa, xb)) break;
        if (!step(wn, wnn, wd, wt, xb, xa)) break;
        if (!step(wnn, wd, wt, wn, xa, xb)) break;
        if (!step(wd, wt, wn, wnn, xb, xa)) break;
    }
}

// Bit phase of the binary32 rule over DeviceCode::bit_code (one load per bit
// for its checks and their degrees): total = LLR + c2b_0 + c2b_1 + ...
// ascending (:256-267), the hard decision and its syndrome, b2c_k =
// clamp(total - c2b_k) (:303-316); FOLD: the first iteration's messages
// +-C_d (fold_first_message). The operations of the generic bit phase.
constexpr int kSp32Chunk = 3;     // bit-phase rounds per load batch
static_assert(kSp32Chunk - 1 <= kBitPadRounds, "per-bit arrays padded past the last load batch (host.cpp)");
// DV3: every bit has exactly kDvUnroll (3) checks (the reference's N = 10240
// code): no per-row degree guards, so a round's loads, sums and stores are
// straight-line code (the guarded form compiled each row's store to an
// exec-mask branch; the min-sum rule spends 40 % of its time here). Whole
// batches of full rounds skip the per-round bounds tests (as spec_bit_phase).
template <bool FOLD, int MODE, bool CLAMP, bool DV3, typename MS>
__device__ __forceinline__ void sp32_bit_phase(const DeviceCode& c, const DecodeArgs& a, const MS& ms,
                                               const uint32_t* qsyn, const double* ctab, uint32_t* xsyn,
                                               uint64_t* zw, uint64_t bobmask, bool keep, uint32_t f, int tid,
                                               int wave, int lane) {
    // (the code's sizes as scalars: through the DecodeArgs reference they are
    // not known to be uniform)
    const uint32_t n_pad = __builtin_amdgcn_readfirstlane((uint32_t)c.n_pad);
    const int cn = __builtin_amdgcn_readfirstlane(c.n);
    const int max_dv = __builtin_amdgcn_readfirstlane(c.max_dv);
    const float llr_p = (float)a.log_p;
    const float thr = (float)a.thr;
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;
    auto batch = [&](auto fullc, int r0) {
        constexpr bool FULLC = decltype(fullc)::value;
        float v[kSp32Chunk][kDvUnroll];
        uint64_t bc[kSp32Chunk];
#pragma unroll
        for (int u = 0; u < kSp32Chunk; ++u) {
            const int i = tid + (r0 + u) * kDecodeBlock;
            // (bit_code is padded to whole rounds, host.cpp build_code; rows
            // k < max_dv of any i < n_pad are store slots: unconditional loads)
            bc[u] = c.bit_code[i];
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k)     // (rows past max_dv have no slots)
                v[u][k] = (FOLD || (!DV3 && k >= max_dv)) ? 0.0f : ms.ld((uint32_t)k * n_pad + (uint32_t)i);
        }
#pragma unroll
        for (int u = 0; u < kSp32Chunk; ++u) {
            const int r = r0 + u;
            if (!FULLC && r * kDecodeBlock >= cn) break;            // block-uniform
            const int i = tid + r * kDecodeBlock;
            const bool ok = FULLC || i < cn;
            const int deg = DV3 ? kDvUnroll : (int)(bc[u] >> 48) & 3;
            int32_t jc[kDvUnroll];
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) jc[k] = (int32_t)(bc[u] >> (16 * k)) & 0xffff;
            const uint32_t bob = (uint32_t)(bobmask >> r) & 1u;
            float acc;
            if constexpr (MODE == kModeLlr) acc = ok ? (float)a.llr[(size_t)f * c.n + c.perm[i]] : 0.0f;
            else acc = bob ? -llr_p : llr_p;
            if (FOLD) {
                const uint32_t sgi = bob ^ lsign;
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    const int j = jc[k];
                    const uint32_t sp = (qsyn[j >> 5] >> (j & 31)) & 1u;
                    const float cm = (float)ctab[((uint32_t)(bc[u] >> (50 + 4 * k)) & 15u) + 1u];
                    v[u][k] = (sp ^ sgi) ? -cm : cm;
                }
            }
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) acc = (DV3 || k < deg) ? acc + v[u][k] : acc;
            const bool z = ok && acc <= 0.0f;
            const uint64_t zb = __ballot(z);
            const bool flip =
                kRunSyn ? (ok && z != (((zw[(r * kDecodeBlock >> 6) + wave] >> lane) & 1ull) != 0)) : z;
            if (lane == 0 && (FULLC || r * kDecodeBlock + wave * 64 < cn)) zw[(r * kDecodeBlock >> 6) + wave] = zb;
            if (flip) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k)
                    if (DV3 || k < deg) atomicXor(&xsyn[jc[k] >> 5], 1u << (jc[k] & 31));
            }
            if (!keep) continue;
            // (lanes past N store into their own padding slots: no guard in
            // full rounds; rows past a bit's degree are not stored)
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) {
                if (DV3 || (ok && k < deg)) {
                    float b = acc - v[u][k];
                    // keys path: b is finite (LLR +-log_p, clamped messages), where
                    // v_med3_f32 is clamp_msg exactly; LLR input may carry NaN
                    if (CLAMP) b = MODE == kModeKeys ? __builtin_amdgcn_fmed3f(b, -thr, thr) : clamp_msg(b, thr);
                    if (DV3 && !FULLC) {
                        if (ok) ms.st((uint32_t)k * n_pad + (uint32_t)i, b);
                    } else {
                        ms.st((uint32_t)k * n_pad + (uint32_t)i, b);
                    }
                }
            }
        }
    };
    using Full = std::integral_constant<bool, true>;
    using Part = std::integral_constant<bool, false>;
    for (int r0 = 0; __builtin_amdgcn_readfirstlane(r0 * kDecodeBlock) < cn; r0 += kSp32Chunk) {
        if ((r0 + kSp32Chunk) * kDecodeBlock <= cn) batch(Full{}, r0);
        else batch(Part{}, r0);
    }
}

// ---- speculative interval iterations (qkd_spec.h) ---------------------------
// Check phase on intervals: each slot holds [lo, hi] of the edge's b2c on
// entry and of its c2b on exit (two binary32 in the 8-byte slot). The
// message's sign is exact (s_j and the signs of the other b2c, which the
// intervals must certify); its magnitude is bounded in the phi domain
// (qkd_spec.h). A b2c interval that does not exclude 0 (or is too
// close to 0, or a sum too large, to certify) raises the abort bit of the
// round. Two forms: spec_check_phase_paired (below) for b2c intervals, and
// this one for the iteration after the folded first one, whose slots hold
// the psi bounds of exact b2c already (psi_of_exact, spec_bit_phase), so only
// the output bound is evaluated per edge. Pipelined as
// spec_check_phase_paired: each task's row (its psi bounds) is written at the
// end of the task before, from its slot loaded a task earlier still, so the
// row reads of a task follow its start with no LDS write in between.
template <int DC>
__device__ __forceinline__ void spec_check_phase_psi(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                 const SplitStore<double>& ms, double* row, const float* wtab,
                                                 int n_tasks,
                                                 uint32_t n_pad, uint32_t dummy, float thr_dn, float thr_up,
                                                 uint32_t* round_word, int wave, int lane) {
    using qkds::f2;
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const __amdgpu_buffer_rsrc_t prs = plan_rsrc(plan);
    // lanes that could not certify (wave masks: scalar ors, no per-lane flag)
    uint32_t bad = 0;
    // the row's DC entries past lane 63 are read (times 0) by segments ending
    // there: keep them finite (the prologue stages key words in this region)
    if (lane < DC) row[64 + lane] = 0.0;
    auto slot = [&](uint2 p) -> uint32_t { return pw_slot(p); };
    // phi(|b2c|) / ln 2 with the sign of b2c in the low word, NaN when the
    // sign is not certain (psi_of_exact); idle lanes (the dummy column) do
    // not count. The row entry is the magnitude's bounds (0 when uncertain).
    auto input = [&](double xv, uint2 w, bool& neg) -> f2 {
        const f2 bv = qkds::unpack_iv(xv);
        neg = bv.x < 0.0f;
        const bool ok = bv.x == bv.x;
        // (an uncertain entry stays NaN in the row: the round aborts on it, so
        // what it does to the other lanes' sums never stands; the dummy
        // column's entry is finite. Two ballots of plain compares: a ballot of
        // their conjunction materialises it as 0 / 1 and compares it back)
        bad |= fold64(__ballot(!ok) & __ballot(pw_slot(w) != dummy));
        return neg_iv_if(neg, bv);
    };
    uint2 wt = plan_word(prs, t, lane);
    uint2 wn = plan_word(prs, t + NW, lane);
    uint2 wnn = plan_word(prs, t + 2 * NW, lane);
    bool neg_t;
    row[lane] = qkds::pack_iv(input(ms.ld_w(slot(wt)), wt, neg_t));
    uint64_t sgn_t = __ballot(neg_t);
    uint32_t sb_t = seg_sbit(wt);
    using Raw = SplitStore<double>::Raw;
    // One task (as spec_check_phase_paired's step): task t's c2b from the row,
    // then task t + NW's row entry from its slot (loaded a task earlier).
    auto step = [&](const uint2 w_t, const uint2 w_n, const uint2 w_nn, uint2& w_ld, const Raw& x_n,
                    Raw& x_ld) -> bool {
        w_ld = plan_word(prs, t + 3 * NW, lane);
        x_ld = ms.ld_raw(slot(w_nn));
        const uint32_t sb_n = seg_sbit(w_n);
        bool neg_n;
        const f2 ph_n = input(ms.pick(x_n), w_n, neg_n);
        wave_lds_sync();
        const int deg = seg_deg<DC>(w_t);
        // extrinsic sum over the other lanes of the segment (a subtraction of
        // the own term would widen the interval by the own term's width)
        const f2 sum = seg_sum<DC>(row, seg_start(w_t), seg_weights<DC>(wtab, w_t, lane));
        // widened by the binary32 roundings (relative to the sum; small
        // buckets charge every segment the bucket's count) and the
        // reference's binary64 roundings (absolute, qkd_spec.h)
        const float nr = DC <= 8 ? (float)(DC + 2) : (float)(deg + 2);
        const float mg = __builtin_fmaf(sum.y, nr * qkds::kSumRel, qkds::kRefSumAbs);
        f2 ext = sum + f2{-mg, mg};
        ext.x = ext.x > 0.0f ? ext.x : 0.0f;
        bad |= fold64(__ballot(!(ext.y < qkds::kPsiSumMax)));      // the reference's product would underflow
        f2 m = qkds::phi_bounds_out(ext.x, ext.y);
        // threshold_matrix (:246-249) on the magnitude
        // (m >= 0, not NaN: med3 with 0 is the min, without the per-edge
        // canonicalisation fminf needs for a kernel argument)
        m.x = __builtin_amdgcn_fmed3f(m.x, 0.0f, thr_dn);
        m.y = __builtin_amdgcn_fmed3f(m.y, 0.0f, thr_up);
        const uint32_t sigma = seg_parity_acc<DC>(sgn_t, w_t, sb_t + (neg_t ? 1u : 0u));
        ms.st_w(slot(w_t), qkds::pack_iv(neg_iv_if(sigma != 0u, m)));
        row[lane] = qkds::pack_iv(ph_n);
        sgn_t = __ballot(neg_n);
        neg_t = neg_n;
        sb_t = sb_n;
        t = __builtin_amdgcn_readfirstlane(t + NW);
        return t < n_tasks;
    };
    Raw xa = ms.ld_raw(slot(wn)), xb;
    uint2 wd;
    for (;;) {
        if (!step(wt, wn, wnn, wd, xa, xb)) break;
        if (!step(wn, wnn, wd, wt, xb, xa)) break;
        if (!step(wnn, wd, wt, wn, xa, xb)) break;
        if (!step(wd, wt, wn, wnn, xb, xa)) break;
    }
    if (bad != 0 && lane == 0) atomicOr(round_word, 2u);
}

// The same check phase with the input bound of the NEXT task's edge and the
// output bound of this task's edge evaluated together (qkds::phi_pair: one
// packed binary32 evaluation instead of two scalar ones). Per task t, in
// order: the next task's b2c unpacked; this task's extrinsic sums from the
// wave's row (written one iteration earlier); the pair; this task's c2b
// stored; the next task's bounds into the row (after this task's row reads:
// a wave's LDS accesses complete in order). Slots are loaded one task ahead
// of their input bound, plan words two.
template <int DC>
__device__ __forceinline__ void spec_check_phase_paired(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                        const SplitStore<double>& ms, double* row, const float* wtab,
                                                        int n_tasks,
                                                        uint32_t n_pad, uint32_t dummy, float thr_dn, float thr_up,
                                                        uint32_t* round_word, int wave, int lane) {
    using qkds::f2;
    constexpr int NW = kDecodeBlock / 64;
    int t = wave;
    if (t >= n_tasks) return;
    const __amdgpu_buffer_rsrc_t prs = plan_rsrc(plan);
    // lanes that could not certify (wave masks: scalar ors, no per-lane flag)
    uint32_t bad = 0;
    if (lane < DC) row[64 + lane] = 0.0;
    auto slot = [&](uint2 p) -> uint32_t { return pw_slot(p); };
    // |b2c| of an edge, its sign and whether the interval certifies it
    // (idle lanes, the dummy column, do not count)
    auto input = [&](double xv, uint2 w, bool& neg, f2& ab) -> bool {
        const f2 bv = qkds::unpack_iv(xv);
        neg = bv.y < 0.0f;
        ab = neg_iv_if(neg, bv);
        // certified: the interval excludes 0 by a margin ((neg || lo > 0) &&
        // |.|lo > 1e-30, of which the second alone decides: |.|lo is -hi
        // when neg, lo otherwise; NaN fails either way)
        const bool ok = ab.x > 1.0e-30f;
        bad |= fold64(__ballot(!ok) & __ballot(pw_slot(w) != dummy));
        return ok;
    };
    // (the plan has kPlanPadTasks idle tasks past n_tasks: loads ahead need no test)
    uint2 wt = plan_word(prs, t, lane);
    uint2 wn = plan_word(prs, t + NW, lane);
    uint2 wnn = plan_word(prs, t + 2 * NW, lane);
    bool neg_t;
    {
        f2 ab;
        const bool ok = input(ms.ld_w(slot(wt)), wt, neg_t, ab);
        row[lane] = qkds::pack_iv(ok ? qkds::phi_bounds(ab.x, ab.y) : f2{0.0f, 0.0f});
    }
    uint64_t sgn_t = __ballot(neg_t);
    // the target bit of a task's check is read one task ahead (its LDS round
    // trip then shares the wait of the row reads)
    uint32_t sb_t = seg_sbit(wt);
    using Raw = SplitStore<double>::Raw;
    // One task: task t's c2b from the row and the input bound of task t + NW
    // (its slot x_n, loaded one task earlier) into the row; loads the plan
    // word three tasks ahead (into w_ld) and the slot of task t + 2 NW (into
    // x_ld). The loop runs it unrolled four times over four plan-word and two
    // slot registers, so nothing is copied between tasks and each slot's
    // select waits one task after its load (SplitStore::pick).
    auto step = [&](const uint2 w_t, const uint2 w_n, const uint2 w_nn, uint2& w_ld, const Raw& x_n,
                    Raw& x_ld) -> bool {
        w_ld = plan_word(prs, t + 3 * NW, lane);
        x_ld = ms.ld_raw(slot(w_nn));
        const uint32_t sb_n = seg_sbit(w_n);
        bool neg_n;
        f2 ab_n;
        input(ms.pick(x_n), w_n, neg_n, ab_n);
        // this task's extrinsic sums (as spec_check_phase_psi)
        wave_lds_sync();
        const int start = seg_start(w_t);
        const int deg = seg_deg<DC>(w_t);
        const f2 sum = seg_sum<DC>(row, start, seg_weights<DC>(wtab, w_t, lane));
        const float nr = DC <= 8 ? (float)(DC + 2) : (float)(deg + 2);
        const float mg = __builtin_fmaf(sum.y, nr * qkds::kSumRel, qkds::kRefSumAbs);
        f2 ext = sum + f2{-mg, mg};
        ext.x = ext.x > 0.0f ? ext.x : 0.0f;
        bad |= fold64(__ballot(!(ext.y < qkds::kPsiSumMax)));
        f2 ph_n, m;
        qkds::phi_pair(ab_n.x, ab_n.y, ext.x, ext.y, ph_n, m);
        // this task's c2b: threshold_matrix (:246-249) on the magnitude, the sign
        m.x = __builtin_amdgcn_fmed3f(m.x, 0.0f, thr_dn);
        m.y = __builtin_amdgcn_fmed3f(m.y, 0.0f, thr_up);
        const uint32_t sigma = seg_parity_acc<DC>(sgn_t, w_t, sb_t + (neg_t ? 1u : 0u));
        ms.st_w(slot(w_t), qkds::pack_iv(neg_iv_if(sigma != 0u, m)));
        // the next task's input bounds into the row: an uncertified entry as
        // phi_pair left it -- finite for the dummy column's 0 (phi_pair
        // evaluates at no less than kPhiTiny), anything for the others, whose
        // round aborts (no select: -3 VALU per task with the ballots above)
        row[lane] = qkds::pack_iv(ph_n);
        sgn_t = __ballot(neg_n);
        neg_t = neg_n;
        sb_t = sb_n;
        t = __builtin_amdgcn_readfirstlane(t + NW);
        return t < n_tasks;
    };
    Raw xa = ms.ld_raw(slot(wn)), xb;
    uint2 wd;
    for (;;) {
        if (!step(wt, wn, wnn, wd, xa, xb)) break;
        if (!step(wn, wnn, wd, wt, xb, xa)) break;
        if (!step(wnn, wd, wt, wn, xa, xb)) break;
        if (!step(wd, wt, wn, wnn, xb, xa)) break;
    }
    if (bad != 0 && lane == 0) atomicOr(round_word, 2u);
}

// The folded first iteration as a table (speculative kernel, QKD path): its
// messages are +-C_d (first_check_phase), so a bit's exact total and the psi
// bounds of its b2c (spec_bit_phase, FOLD) depend only on its degree pattern
// p, Bob's bit and the signs of its three messages: entry
//   ftab[(p * 16 + code) * 4 + k],  code = bob | sign_k << (1 + k)
// holds psi_of_exact(clamp(total - c_k)) for row k < 3 (packed) and, at k = 3,
// whether total <= 0 (the hard decision), each computed with the binary64
// operations of the per-bit form in the same order (tests/test_spec.py runs
// both forms).
// Entry (p, code) sits at position p * 16 + (code ^ (p & 15)): the hot codes
// (0 and 15: Bob's bit with every message sign agreeing) of the 8 patterns
// of a (3, 5|6) code would otherwise all fall on two of the eight 32-byte
// bank groups of an LDS row (iteration 1 measured 0.53 bank-conflict cycles
// per LDS-active cycle in round 5).
__device__ __forceinline__ uint32_t fold_tab_pos(uint32_t p, uint32_t code) { return p * 16u + (code ^ (p & 15u)); }
__device__ void fold_table_fill(const DeviceCode& c, const double* ctab, double log_p, double thr, double* ftab,
                                int entries) {
    static_assert(kFoldTabPat == 64, "16 codes x 4 entries");
    for (int e = threadIdx.x; e < entries; e += kDecodeBlock) {
        const int p = e / kFoldTabPat;
        const uint32_t code = ((uint32_t)e >> 2) & 15u;
        const int k = e & 3;
        const uint32_t at = fold_tab_pos((uint32_t)p, code) * 4u + (uint32_t)k;
        const uint8_t* degs = c.pat_deg + p * c.max_dv;
        double acc = (code & 1u) ? -log_p : log_p;
        double cv[kDvUnroll];
        int dv = 0;
#pragma unroll
        for (int m = 0; m < kDvUnroll; ++m) {
            const int d = m < c.max_dv ? (int)degs[m] : 0;
            if (d != 0 && dv == m) dv = m + 1;
            const double cm = ctab[d];
            cv[m] = ((code >> (1 + m)) & 1u) ? -cm : cm;
        }
#pragma unroll
        for (int m = 0; m < kDvUnroll; ++m) acc = m < dv ? acc + cv[m] : acc;
        double v = 0.0;
        if (k == kDvUnroll) {
            v = __builtin_bit_cast(double, (unsigned long long)(acc <= 0 ? 1 : 0));
        } else if (k < dv) {
            const double ck = k == 0 ? cv[0] : (k == 1 ? cv[1] : cv[2]);
            v = qkds::pack_iv(qkds::psi_of_exact(clamp_msg(acc - ck, thr)));
        }
        ftab[at] = v;
    }
    __syncthreads();
}

// Bit phase on intervals. FOLD (the first iteration): the messages are the
// exact +-C_d of first_check_phase, so the totals are computed in binary64
// exactly as the exact path does and the b2c are stored as enclosing
// intervals. Otherwise: total in L + sum c_k (intervals) and each b2c_k =
// clamp(total - c2b_k) (:303-316) as the extrinsic sum L + sum_{m != k} c_m, widened by
// the binary32 and the reference's binary64 rounding allowances, clamped with
// med3. A hard decision whose sign the interval leaves open marks its checks
// in xunc (the syndrome test then decides whether the round can stand).
// Needs DeviceCode::bit_code (bit degree <= 3, M <= 65536, check degree <= 16).
#ifndef QKD_IV_CHUNK
#define QKD_IV_CHUNK 2
#endif
// rounds per load batch (2: measured -1 % per config-2 batch against 3, the
// registers go to the check phases)
constexpr int kIvChunk = QKD_IV_CHUNK;
static_assert(kIvChunk - 1 <= kBitPadRounds, "per-bit arrays padded past the last load batch (host.cpp)");
// DV3: every bit has exactly kDvUnroll (3) checks (a column-weight-3 code,
// like the reference's N = 10240 one): no per-degree guards, so the round is
// straight-line code except one branch around the hard decision's syndrome
// updates (and a rare one around the uncertainty marks). The general form
// guards every row by the bit's degree.
template <bool FOLD, int MODE, bool DV3>
__device__ __forceinline__ void spec_bit_phase(const DeviceCode& c, const DecodeArgs& a, const SplitStore<double>& ms,
                                               const uint32_t* qsyn, const double* ctab, const double* ftab,
                                               uint32_t* xsyn,
                                               uint32_t* xunc, uint64_t* zw, uint64_t bobmask, bool keep,
                                               uint32_t f, int tid, int wave, int lane) {
    using qkds::f2;
    static_assert(!DV3 || kDvUnroll == 3, "DV3 unrolls three rows");
    // the code's sizes as scalars (read through the DecodeArgs reference they
    // are not known to be uniform, and every row's LDS / global choice, k *
    // n_pad + iw < S, then compiles to a divergent branch)
    const uint32_t n_pad = __builtin_amdgcn_readfirstlane((uint32_t)c.n_pad);
    const int cn = __builtin_amdgcn_readfirstlane(c.n);
    const double llr_p = a.log_p;
    // Fixed rows (FX): row 0 wholly in LDS and row 2 wholly global (n_pad <=
    // S <= 2 n_pad, the config-2 layout): only row 1's rounds choose, so
    // four of a round's six slot accesses need no branch (a branch per access
    // also waits for every load issued before it, breaking the load batch).
#ifndef QKD_FIXED_ROWS
#define QKD_FIXED_ROWS 1
#endif
    const bool fixed_rows = QKD_FIXED_ROWS && DV3 && n_pad <= ms.S && ms.S <= 2 * n_pad;
    // fx: 0 every row chooses per round (ld_row / st_row); 1 fixed rows, row 1
    // chooses per round; 2 / 3 fixed rows with row 1 in LDS / global for the
    // whole batch (run picks them per batch: the wave's rounds of row 1 are in
    // LDS up to a wave-uniform round and global after it, so most batches need
    // no branch at all -- a branch per access also waits for every load issued
    // before it)
#ifndef QKD_R1_SPLIT
#define QKD_R1_SPLIT 1
#endif
    // a fixed global row's slot as the lane's byte offset, loop-invariant,
    // plus the wave-uniform rest in soffset: no per-access vector address
    // arithmetic (iw = the wave's first bit of the round)
    const uint32_t vlane = (uint32_t)lane * 8u;
    auto gsoff = [&](int k, uint32_t iw) -> uint32_t {
        return ms.gofs((uint32_t)k * n_pad + iw);
    };
    auto ld_k = [&](auto fx, int k, uint32_t iw, uint32_t i) -> double {
        const uint32_t x = (uint32_t)k * n_pad + i;
        if constexpr (decltype(fx)::value >= 1) {
            if (k == 0) return ms.l[x];
            if (k == 2) return BufIo<double>::ld(ms.gw, vlane, gsoff(k, iw));
            if constexpr (decltype(fx)::value == 2) return ms.l[x];
            if constexpr (decltype(fx)::value == 3) return BufIo<double>::ld(ms.gw, vlane, gsoff(k, iw));
        }
        return ms.ld_row((uint32_t)k * n_pad + iw, x);
    };
    auto st_k = [&](auto fx, int k, uint32_t iw, uint32_t i, double v) {
        const uint32_t x = (uint32_t)k * n_pad + i;
        if constexpr (decltype(fx)::value >= 1) {
            if (k == 0) { ms.l[x] = v; return; }
            if (k == 2) { BufIo<double>::st(ms.gw, vlane, gsoff(k, iw), v); return; }
            if constexpr (decltype(fx)::value == 2) { ms.l[x] = v; return; }
            if constexpr (decltype(fx)::value == 3) { BufIo<double>::st(ms.gw, vlane, gsoff(k, iw), v); return; }
        }
        ms.st_row((uint32_t)k * n_pad + iw, x, v);
    };
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;
    // the LLR interval's bounds as a VGPR pair made once (as kernel arguments
    // they spilled to VGPR lanes and every round read them back with
    // v_readlane and moved them into VGPRs for its select: -15 % of the bit
    // rounds' VALU with the soffset slots above, profiles/r06_ab.txt)
    qkds::f2 lpv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lpv.x) : "s"(a.lp_dn));
    asm volatile("v_mov_b32 %0, %1" : "=v"(lpv.y) : "s"(a.lp_up));
    // one batch of kIvChunk rounds: its loads, then its rounds
    typedef double VB[kIvChunk][kDvUnroll];
    auto batch_load = [&](auto fx, int r0, VB& v, uint64_t (&bc)[kIvChunk], uint32_t (&pat)[kIvChunk]) {
#pragma unroll
        for (int u = 0; u < kIvChunk; ++u) {
            const int i = tid + (r0 + u) * kDecodeBlock;
            const bool ok = i < cn;
            // (bit_code and bit_pat are padded to whole rounds, host.cpp
            // build_code: an unconditional load, no exec-mask branch around it)
            bc[u] = c.bit_code[i];
            pat[u] = (FOLD && ftab) ? (uint32_t)c.bit_pat[i] : 0u;
            // (wave-uniform, said so: left to itself loop strength reduction
            // rebuilds it from the per-lane bit index, and every row's LDS /
            // global choice becomes a divergent branch with exec-mask shuffling)
            const uint32_t iw = __builtin_amdgcn_readfirstlane((uint32_t)((r0 + u) * kDecodeBlock + wave * 64));
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k)
                v[u][k] = FOLD ? 0.0 : ld_k(fx, k, iw, (uint32_t)i);
            (void)ok;
        }
    };
    // fullc: every round of the batch is full (compile time: no per-round
    // bounds tests at all)
    auto batch_compute = [&](auto fx, auto fullc, int r0, VB& v, uint64_t (&bc)[kIvChunk],
                             uint32_t (&pat)[kIvChunk]) {
        constexpr bool FULLC = decltype(fullc)::value;
#pragma unroll
        for (int u = 0; u < kIvChunk; ++u) {
            const int r = r0 + u;
            if (!FULLC && r * kDecodeBlock >= cn) break;            // block-uniform
            const int i = tid + r * kDecodeBlock;
            const uint32_t iw = __builtin_amdgcn_readfirstlane((uint32_t)(r * kDecodeBlock + wave * 64));
            // a full round (block-uniform): every lane's bit exists
            const bool full = FULLC || (r + 1) * kDecodeBlock <= cn;
            const bool ok = full || i < cn;
            const int deg = DV3 ? kDvUnroll : (int)(bc[u] >> 48) & 3;
            int32_t jc[kDvUnroll];
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) jc[k] = (int32_t)(bc[u] >> (16 * k)) & 0xffff;
            const uint32_t bob = (uint32_t)(bobmask >> r) & 1u;
            bool z, unc = false;
            f2 bo[kDvUnroll];
            if (FOLD && ftab) {
                // the same from the table (fold_table_fill): the code of Bob's
                // bit and the message signs picks the bit's psi bounds and decision
                const uint32_t sgi = bob ^ lsign;
                uint32_t code = bob;
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    const int j = jc[k];
                    code |= (((qsyn[j >> 5] >> (j & 31)) & 1u) ^ sgi) << (1 + k);
                }
                const double* e = ftab + fold_tab_pos(pat[u], code) * 4u;
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) bo[k] = qkds::unpack_iv(e[k]);
                z = ok && __builtin_bit_cast(unsigned long long, e[kDvUnroll]) != 0ull;
            } else if (FOLD) {
                // the exact first iteration (fold_first_message, then :256-267, :303-316)
                const uint32_t sgi = bob ^ lsign;
                double acc = bob ? -llr_p : llr_p;
                double cv[kDvUnroll];
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    const int j = jc[k];
                    const uint32_t sp = (qsyn[j >> 5] >> (j & 31)) & 1u;
                    const double cm = ctab[((uint32_t)(bc[u] >> (50 + 4 * k)) & 15u) + 1u];
                    cv[k] = (DV3 || k < deg) ? ((sp ^ sgi) ? -cm : cm) : 0.0;
                }
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) acc = (DV3 || k < deg) ? acc + cv[k] : acc;
                z = ok && acc <= 0;
                static_assert(kDvUnroll == 3, "rows 0 and 1 paired, row 2 alone");
                qkds::psi_of_exact2(clamp_msg(acc - cv[0], a.thr), clamp_msg(acc - cv[1], a.thr), bo[0], bo[1]);
                bo[2] = qkds::psi_of_exact(clamp_msg(acc - cv[2], a.thr));
            } else {
                f2 L;
                if constexpr (MODE == kModeLlr) L = qkds::iv_of(ok ? a.llr[(size_t)f * c.n + c.perm[i]] : 0.0);
                else L = bob ? f2{-lpv.y, -lpv.x} : lpv;
                f2 cs[kDvUnroll];
                f2 T = L;
                // max(|lo|, |hi|) of an interval lo <= hi is max(hi, -lo) (med3
                // with +inf: a max without canonicalising its operands)
                // (+inf from a kernel argument: with a literal one LLVM folds
                // the med3 into a maxnum, which in IEEE mode canonicalises both
                // operands first, three instructions for one)
                const float pinf = a.pinf;
                auto amax = [pinf](f2 x) { return __builtin_amdgcn_fmed3f(x.y, -x.x, pinf); };
                float mag = amax(L);
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    cs[k] = (DV3 || k < deg) ? qkds::unpack_iv(v[u][k]) : f2{0.0f, 0.0f};
                    T = T + cs[k];
                    mag = mag + amax(cs[k]);
                }
                // binary32 roundings (the sum here and the subtraction below)
                // and the reference's binary64 ones, relative to the magnitudes
                // (one fma: kSumRel carries twice the rounding it covers, so the
                // single rounding of the fused form is covered as the two of
                // the product-then-sum were)
                const float mg = __builtin_fmaf(mag, (float)(kDvUnroll + 2) * qkds::kSumRel, 1.0e-30f);
                T = T + f2{-mg, mg};
                // z = total <= 0 (:259), certain only if the interval says so
                const bool z1 = T.y <= 0.0f;
                unc = ok && !(z1 || T.x > 0.0f);
                z = ok && z1;
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    // the extrinsic sum L + sum_{m != k} c_m (no dependency widening)
                    f2 e = L + f2{-mg, mg};
#pragma unroll
                    for (int m = 0; m < kDvUnroll; ++m)
                        if (m != k) e = e + cs[m];
                    // clamp (:313-316) with binary32 bounds of thr
                    bo[k] = f2{__builtin_amdgcn_fmed3f(e.x, -a.thr_up, a.thr_dn),
                               __builtin_amdgcn_fmed3f(e.y, -a.thr_dn, a.thr_up)};
                }
            }
            const uint64_t zb = __ballot(z);
            const bool wave_in = FULLC || r * kDecodeBlock + wave * 64 < cn;
            // (running syndrome: the decisions that changed; this round's word
            // of the last decision is read before lane 0 overwrites it: one
            // wave's LDS accesses complete in order)
            // (lanes past N never flip: their word may lie past zw's end)
            const bool flip =
                kRunSyn ? (ok && z != (((zw[(r * kDecodeBlock >> 6) + wave] >> lane) & 1ull) != 0)) : z;
            if (lane == 0 && wave_in) zw[(r * kDecodeBlock >> 6) + wave] = zb;
            // (each check's word and bit formed inside the branch, behind an
            // empty asm: hoisted above it, they cost every round their VALU
            // although many rounds of a wave flip no decision; -0.7 %)
            if (flip) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    int32_t j = jc[k];
                    asm volatile("" : "+v"(j));
                    if (DV3 || k < deg) atomicXor(&xsyn[j >> 5], 1u << (j & 31));
                }
            }
            if (unc) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    int32_t j = jc[k];
                    asm volatile("" : "+v"(j));
                    if (DV3 || k < deg) atomicOr(&xunc[j >> 5], 1u << (j & 31));
                }
            }
            if (!keep) continue;
            if (DV3 && full) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) st_k(fx, k, iw, (uint32_t)i, qkds::pack_iv(bo[k]));
            } else if (ok) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k)
                    if (k < deg) ms.st_row((uint32_t)k * n_pad + iw, (uint32_t)k * n_pad + i, qkds::pack_iv(bo[k]));
            }
        }
    };
    using NoFx = std::integral_constant<int, 0>;
    using Fx = std::integral_constant<int, 1>;
    using FxL = std::integral_constant<int, 2>;
    using FxG = std::integral_constant<int, 3>;
    using Full = std::integral_constant<bool, true>;
    using Part = std::integral_constant<bool, false>;
    auto batch = [&](auto fx, auto fullc, int r0) {
        VB v;
        uint64_t bc[kIvChunk];                 // the bits' packed words (DeviceCode::bit_code)
        uint32_t pat[kIvChunk];                // FOLD with ftab: the bits' degree patterns
        batch_load(fx, r0, v, bc, pat);
        batch_compute(fx, fullc, r0, v, bc, pat);
    };
    if (fixed_rows) {
        for (int r0 = 0; __builtin_amdgcn_readfirstlane(r0 * kDecodeBlock) < cn; r0 += kIvChunk) {
            // row 1 of the batch's first / last round (wave-uniform; S and
            // n_pad are multiples of 64, so a wave's 64 slots are one kind)
            const uint32_t x0 = n_pad + __builtin_amdgcn_readfirstlane((uint32_t)(r0 * kDecodeBlock + wave * 64));
            const uint32_t x1 = x0 + (uint32_t)(kIvChunk - 1) * kDecodeBlock;
            // (whole batches of full rounds: every bit of every round exists)
            const bool full = (r0 + kIvChunk) * kDecodeBlock <= cn;
            if (QKD_R1_SPLIT && full && x1 < ms.S)
                batch(FxL{}, Full{}, r0);
            else if (QKD_R1_SPLIT && full && x0 >= ms.S)
                batch(FxG{}, Full{}, r0);
            else
                batch(Fx{}, Part{}, r0);
        }
    } else {
        for (int r0 = 0; __builtin_amdgcn_readfirstlane(r0 * kDecodeBlock) < cn; r0 += kIvChunk)
            batch(NoFx{}, Part{}, r0);
    }
}

// The workgroup's global slot region. QKD_XCD_REGIONS (default): the regions
// of one XCD's workgroups (blockIdx % 8 = XCD when dispatched round-robin; a
// placement assumption for speed only, any mapping is correct) adjacent in
// memory, so each XCD's L2 holds one contiguous range: L2 misses per launch
// 1.94M -> 0.41M, -1 % per config-2 batch.
#ifndef QKD_XCD_REGIONS
#define QKD_XCD_REGIONS 1
#endif
__device__ __forceinline__ uint32_t region_of_block() {
    if (QKD_XCD_REGIONS && (gridDim.x & 7u) == 0)
        return (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    return blockIdx.x;
}

// Flooding sum-product decode of whole frames, one frame per workgroup at a
// time, frames from the device queue (as decode_kernel). RULE is kRuleSp64
// (the reference, bit-exact) or kRuleSp32 (the binary32 variant).
//
// SPEC (QKD path, binary64 rule, clamp on): each frame first runs interval
// iterations (qkd_spec.h); a frame the intervals cannot certify (or that
// reaches spec_cap) restarts at once with the exact iterations, which this
// instantiation compiles with a shorter bit-phase load batch (kBitChunkSpec)
// to leave the registers to the interval phases. The replay policy (ctl[6])
// can send a frame straight to the exact iterations.
// SPEC 2 (checkpointed, keys path, for QBERs where most frames fail the
// above): the exact iterations come first; once one leaves at most
// a.ckpt_unsat checks unsatisfied the message store is saved (a.ckpt) and
// the iterations go on with intervals; a frame they cannot certify within
// spec_cap iterations resumes exactly from the saved messages.
// (experiment builds: QKD_SPLIT_WAVES_PER_EU=8 asks for two workgroups per
// CU, 64 VGPRs; run with QKD_SPLIT_BUDGET halving the LDS. DESIGN.md §4.3)
#ifdef QKD_SPLIT_WAVES_PER_EU
#define QKD_SPLIT_BOUNDS __launch_bounds__(kDecodeBlock, QKD_SPLIT_WAVES_PER_EU)
#else
#define QKD_SPLIT_BOUNDS __launch_bounds__(kDecodeBlock)
#endif
// LONG: codes past kMaxBitsSplit bits (up to kMaxBitsSplitLong), the exact
// keys-path kernel only (the frame-interleaved decoder's hand-offs): Bob's
// bits of rounds 64 and up come from the frame's key words kept in LDS (the
// ftab region, DecodeArgs::ftab_entries >= words) instead of bobmask.
template <int MODE, int RULE, int DC, bool CLAMP, int SPEC, bool LONG = false>
__global__ QKD_SPLIT_BOUNDS void decode_split_kernel(DecodeArgs a) {
    static_assert(!LONG || (MODE == kModeKeys && RULE == kRuleSp64 && SPEC == 0), "long codes: exact keys path");
    using T = typename RuleMsg<RULE>::T;
    // QKD path: the first check phase folds into the first bit phase for both
    // sum-product rules (every b2c is +-log_p, so every message is +-C_d:
    // ctab); the second-iteration tanh table is the binary64 rule's only
    // (min-sum: the self-corrected rule has no fold, its first check phase
    // records every edge's b2c)
    constexpr bool MSR = RULE == kRuleMinSumSplit || RULE == kRuleMinSumSplitSc;   // min-sum rules
    constexpr bool MSC = RULE == kRuleMinSumSplitSc;
    constexpr bool F32 = RULE != kRuleSp64;       // binary32 slots, all in LDS
    constexpr bool FOLDS = MODE == kModeKeys && (RULE == kRuleSp64 || RULE == kRuleSp32 || MSR);
    constexpr bool TABLES = MODE == kModeKeys && RULE == kRuleSp64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const DeviceCode& c = a.code;
    const SplitLds L(c.n_pad, (c.n + 63) / 64, c.m, c.max_dv, DC, a.tab2_entries, a.ftab_entries, (int)sizeof(T),
                     a.lds_budget);
    const int m_words = decode_m_words(c.m);
    uint32_t* tsyn = reinterpret_cast<uint32_t*>(smem + L.tsyn);
    uint32_t* xsyn = reinterpret_cast<uint32_t*>(smem + L.xsyn);
    uint32_t* qsyn = reinterpret_cast<uint32_t*>(smem + L.qsyn);
    uint32_t* xunc = reinterpret_cast<uint32_t*>(smem + L.xunc);
    uint64_t* zw = reinterpret_cast<uint64_t*>(smem + L.zw);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + L.ctl);
    double* ctab = reinterpret_cast<double*>(smem + L.ctab);
    double* tab2 = reinterpret_cast<double*>(smem + L.tab2);
    float* wtab = reinterpret_cast<float*>(smem + L.wtab);
    // (min-sum: the additive masks of ms_split_check_phase, 0 / +inf)
    for (int e = threadIdx.x; e < seg_weight_entries(DC); e += kDecodeBlock) {
        const int k = e % DC;
        const int p = (e / DC) % 8, deg = e / (DC * 8);      // (rows deg * 8 + p, encode_seg)
        const bool in = k < deg && k != p;
        wtab[e] = MSR ? (in ? 0.0f : __builtin_inff()) : (in ? 1.0f : 0.0f);
    }
    using MS = SplitStore<T, F32>;
    T* const region = reinterpret_cast<T*>(a.c2b) + (size_t)region_of_block() * a.c2b_stride;
    const MS ms{
        reinterpret_cast<T*>(smem + L.msg),
        L.S,
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(region) - kSlotGlobalBase, (short)0,
                                          (int)(kSlotGlobalBase + a.c2b_stride * sizeof(T)), 0x00020000),
        kSlotGlobalBase - L.S * (uint32_t)sizeof(T)};
    // the check phases' plan: encoded slot words for this layout (binary64
    // rule: DecodeArgs::plan_enc, built by the host from L), slot indices for
    // the all-LDS binary32 rule; the dummy column's slot in the same form
    const uint2* const plan = (RULE == kRuleSp64 || MSR) ? a.plan_enc : c.plan_slot;
    const uint32_t dummy_w = encode_slot((uint32_t)c.n, L.S, (uint32_t)L.msg, (uint32_t)sizeof(T));
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
    const bool fold1 = FOLDS && a.first_table && c.max_dv <= kDvUnroll;
    // column weight 3 throughout (the speculative bit phase's straight-line form)
    const bool dv3 = c.min_dv == kDvUnroll && c.max_dv == kDvUnroll;
    const bool tab2_on = fold1 && a.tab2_entries;
    uint32_t rnd = 0;    // rounds (iterations of any frame) run by this workgroup
    if (tid == 0) { ctl[2] = 0; ctl[3] = 0; ctl[4] = 0; ctl[5] = 0; ctl[6] = 1; ctl[7] = 0; }
    static_assert(!SPEC || (RULE == kRuleSp64 && CLAMP), "speculation: binary64 rule, clamped messages");
    constexpr bool CKPT = SPEC == 2;
    static_assert(!CKPT || MODE == kModeKeys, "checkpointed speculation: keys path");
#ifndef QKD_EXACT_CHUNK
#define QKD_EXACT_CHUNK kBitChunk
#endif
    constexpr int BC = SPEC ? kBitChunkSpec : QKD_EXACT_CHUNK;      // exact bit phase load batch
    if (TABLES && tid <= kFirstTableDeg) ctab[tid] = a.first_c2b[tid];
    if constexpr (RULE == kRuleSp32 && FOLDS) {
        // the binary32 rule's first messages by check degree d, evaluated exactly
        // as split_check_phase would on d inputs of equal magnitude |float(log_p)|:
        // S = ((0 + p) + p) + ... over the d - 1 other edges, C_d = phi(S ln 2)
        if (tid <= kFirstTableDeg) {
            const float p = __builtin_fabsf(RuleMath<kRuleSp32>::tanh_half((float)a.log_p));
            float S = 0.0f;
            for (int k = 1; k < tid; ++k) S = S + p;
            float v = RuleMath<kRuleSp32>::two_atanh(S);
            if (CLAMP) v = clamp_msg(v, (float)a.thr);
            ctab[tid] = (double)v;
        }
    }
    if constexpr (MSR && FOLDS) {
        // the min-sum rule's first messages (every |b2c| = |float(log_p)|):
        // scale * |log_p| - off, floored at 0, clamped, for every degree >= 2;
        // degree 1 has no other edge (min over nothing: +inf)
        if (tid <= kFirstTableDeg) {
            float v = tid <= 1 ? __builtin_inff() : a.ms_scale * __builtin_fabsf((float)a.log_p);
            if (a.ms_offset > 0.0f) v = __builtin_fmaxf(v - a.ms_offset, 0.0f);
            if (CLAMP) v = clamp_msg(v, (float)a.thr);
            ctab[tid] = (double)v;
        }
    }
    // self-corrected min-sum: the previous b2c of each edge, two ballot words
    // per task (ms_split_check_phase), then the frame's Bob words (keys path),
    // in the ftab region (host: ftab_entries)
    uint64_t* const scw = MSC ? reinterpret_cast<uint64_t*>(smem + L.ftab) : nullptr;
    uint64_t* const bwl = MSC ? scw + 2 * c.n_tasks : (LONG ? reinterpret_cast<uint64_t*>(smem + L.ftab) : nullptr);
    if (tab2_on) {
        __syncthreads();
        second_table_fill<CLAMP>(c, ctab, a.log_p, a.thr, tab2, a.tab2_entries);
    }
    double* ftab = nullptr;
    if constexpr (SPEC == 1) {
        if (fold1 && a.ftab_entries) {
            ftab = reinterpret_cast<double*>(smem + L.ftab);
            __syncthreads();
            fold_table_fill(c, ctab, a.log_p, a.thr, ftab, a.ftab_entries);
        }
    }
    PhaseClock pc(a.phase);

    // frames from the queue: each frame's successor is claimed when the frame
    // starts (thread 0 keeps it in a register until the frame's end), so the
    // atomic's round trip overlaps the prologue's loads
    // the in-launch replay policy for frame fr (SPEC kernels; DecodeArgs::win):
    // whether window fr / W - win_lag replayed at most a sixth of its frames,
    // waiting (thread 0, between frames) until that window has completed. A
    // wait cannot deadlock: every frame of a waited-on window is done, being
    // decoded, or claimed by a workgroup that waits on a strictly earlier window.
    // A window is ONE 64-bit word (completed frames in the low half, replay
    // events in the high half) updated by one relaxed atomic add, so its two
    // counts are always read together and no release / acquire ordering is
    // needed: at agent scope those compile to a write-back (buffer_wbl2) and
    // an invalidation (buffer_inv) of the whole L2, which the frame loop can
    // not afford (measured +21 % per config-2 batch).
    unsigned long long* const win64 = reinterpret_cast<unsigned long long*>(a.win);
    // window_of(fr): the window frame fr's policy reads, or -1 (none: always on)
    auto window_of = [&](uint32_t fr) -> int {
        if (!SPEC || a.spec_always || fr >= a.n_frames) return -1;
        const uint32_t wn = fr >> a.win_shift;
        return wn < a.win_lag ? -1 : (int)(wn - a.win_lag);
    };
    // v: that window's word as read earlier (the frame's start, so the load's
    // latency overlaps the frame; almost always complete by then), polled again
    // only while incomplete
    auto spec_policy = [&](uint32_t fr, unsigned long long v) -> uint32_t {
        const int k = window_of(fr);
        if (k < 0) return 1u;
        const uint32_t W = 1u << a.win_shift;
        // (bounded, ~1 s: a defensive exit, never expected to be reached)
        for (uint32_t polls = 0; (uint32_t)v < W; ++polls) {
            if (polls >= (1u << 24)) return 1u;
            __builtin_amdgcn_s_sleep(2);
            v = __hip_atomic_load(win64 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return (uint32_t)(v >> 32) * 6u <= W ? 1u : 0u;     // kSpecReplayMax
    };
    auto window_peek = [&](uint32_t fr) -> unsigned long long {
        const int k = window_of(fr);
        return k < 0 ? 0ull : __hip_atomic_load(win64 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // the next frame of the queue: frame k, or with a frame list (the
    // interleaved decoder's hand-offs, decode_ilv.hip) its k-th entry
    auto claim = [&]() -> uint32_t {
        const uint32_t k = atomicAdd(a.counter, 1u);
        if (a.frame_list == nullptr) return k;
        return k < *a.frame_count ? a.frame_list[k] : a.n_frames;
    };
    if (tid == 0) {
        ctl[1] = claim();
        ctl[6] = spec_policy(ctl[1], window_peek(ctl[1]));
    }
    uint32_t next_f = 0;
    for (;;) {
        pc.mark(4);
        for (int w = tid; w < m_words; w += kDecodeBlock) {
            xsyn[w] = 0;
            xunc[w] = 0;
        }
        __syncthreads();
        const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane((int)ctl[1]);   // (uniform to the compiler)
        if (f >= a.n_frames) break;
        if (tid == 0) next_f = claim();
        // this frame's replay events (thread 0; the policy's window count)
        uint32_t frame_replays = 0;

        // ---- prologue. Keys path: the frame's Bob words, in the internal
        //      bit order (frame_syn_kernel permuted them), staged in LDS (the
        //      product rows are free until the first check phase) and its
        //      syndrome words from frame_syn_kernel.
        const uint64_t* bw = reinterpret_cast<const uint64_t*>(smem + L.tval);
        if (MODE == kModeKeys) {
            uint64_t* w = reinterpret_cast<uint64_t*>(smem + L.tval);
            uint64_t* aw = reinterpret_cast<uint64_t*>(smem + L.aw);
            const bool ka = a.key_ok != nullptr;
            for (int q = tid; q < (int)a.words; q += kDecodeBlock) {
                const uint64_t bv = a.bob_w[(size_t)f * a.words + q];
                const uint64_t av = ka ? a.alice_w[(size_t)f * a.words + q] : 0ull;
                w[q] = bv;
                aw[q] = av;
                if constexpr (MSC || LONG) bwl[q] = bv;
            }
            const uint32_t* sy = a.synw + (size_t)f * 2 * m_words;
            for (int q = tid; q < m_words; q += kDecodeBlock) {
                tsyn[q] = sy[q];
                qsyn[q] = sy[m_words + q];
            }
            __syncthreads();
        }
        // Bob's bits of this thread's bit-phase rounds (round r: internal bit
        // i = tid + r * kDecodeBlock; N <= 64 * kDecodeBlock, kMaxBitsSplit).
        // Without the fold the first check phase reads b2c = LLR_i (:188),
        // i.e. the caller's LLR of bit c.perm[i], from every slot.
        // (the speculative kernel's replay policy for this frame: ctl[6])
        const bool spec0 = SPEC == 1 && ctl[6] != 0;
        uint64_t bobmask = 0;
        // the first check phase's b2c = LLR_i in every slot (:188), as enclosing
        // intervals when speculating (the LLR path has no folded first iteration)
        auto init_slots = [&](bool as_interval) {
            int r = 0;
            for (int i = tid; i < c.n; i += kDecodeBlock, ++r) {
                T l;
                if (MODE == kModeLlr) {
                    l = (T)a.llr[(size_t)f * c.n + c.perm[i]];
                } else {
                    const uint32_t bb = (uint32_t)((bw[i >> 6] >> (i & 63)) & 1u);
                    if (!LONG || r < 64) bobmask |= (uint64_t)bb << r;
                    l = bb ? -llr_p : llr_p;
                }
                if (!fold1) {
                    T sv = l;
                    if constexpr (SPEC) if (as_interval) sv = qkds::pack_iv(qkds::iv_of((double)l));
                    const int deg = c.bit_deg[i];
                    for (int k = 0; k < deg; ++k) ms.st((uint32_t)k * n_pad + i, sv);
                }
            }
            // the dummy column's slot (idle plan lanes): a finite value, and
            // table index 0 for the second check phase
            if (tid == 0) ms.st((uint32_t)c.n, (T)0);
        };
        init_slots(spec0);
        // Bob's bit of this thread's round r (LONG: past round 63 from LDS)
        auto bob_r = [&](int r) -> uint32_t {
            if constexpr (LONG)
                if (r >= 64) return (uint32_t)(bwl[(r * kDecodeBlock >> 6) + wave] >> lane) & 1u;
            return (uint32_t)(bobmask >> r) & 1u;
        };
        // running syndrome (kRunSyn): the last decision = Bob's key (keys path,
        // the words staged above) or 0 (LLR path), and xsyn = H * it: from
        // frame_syn's words, q_j = s_j ^ (H bob)_j ^ (deg_j & sign(log_p))
        if constexpr (kRunSyn) {
            const int zwords = (int)(n_pad >> 6);
            for (int q = tid; q < zwords; q += kDecodeBlock)
                zw[q] = (MODE == kModeKeys && q < (int)a.words) ? bw[q] : 0ull;
            if (MODE == kModeKeys) {
                for (int w = tid; w < m_words; w += kDecodeBlock)
                    xsyn[w] = tsyn[w] ^ qsyn[w] ^ (lsign ? c.chk_odd[w] : 0u);
            }
        }
        // ---- prologue, LLR path: target syndrome bits per check (tsyn), thread per check
        if (MODE == kModeLlr) {
            for (int j0 = wave * 64; j0 < c.m; j0 += kDecodeBlock) {
                const int j = j0 + lane;
                const int sj = j < c.m ? (a.syn[(size_t)f * c.m + j] != 0) : 0;
                const uint64_t sm = __ballot(sj);
                if (lane == 0) {
                    tsyn[j0 >> 5] = (uint32_t)sm;
                    tsyn[(j0 >> 5) + 1] = (uint32_t)(sm >> 32);
                }
            }
        }
        __syncthreads();
        pc.mark(0);
        // (thread 0: the next frame's policy window, read here, after the
        // prologue has waited out next_f's atomic, so the load's latency
        // overlaps this frame's iterations)
        unsigned long long next_win = 0;
        if (SPEC && tid == 0) next_win = window_peek(next_f);

        // ---- iterations (:212-330): interval iterations (qkd_spec.h) in the
        //      speculative launch, the reference's binary64 ones otherwise
        bool spec = spec0;
        // a frame the policy keeps off the speculation counts as replayed (so
        // the policy, once on, stays on, and the call's count reports it)
        if (SPEC == 1 && !spec && tid == 0) {
            atomicAdd(a.replay_count, 1u);
            frame_replays++;
        }
        bool done = false;
        uint32_t it = 0;
        // checkpointed speculation: the iteration the saved messages feed, and
        // the unsatisfied-check count below which this frame takes its next
        // checkpoint (halved after each restore; 0 once the policy, ctl[6], is off)
        uint32_t it_ck = 0;
        uint32_t ck_lim = (CKPT && ctl[6] != 0) ? a.ckpt_unsat : 0u;
        // save (and turn into enclosing intervals) or restore every slot
        auto ckpt_io = [&](bool save) {
            if constexpr (CKPT) {
                double* bk = a.ckpt + (size_t)blockIdx.x * a.ckpt_stride;
                const uint32_t tot = (uint32_t)c.max_dv * n_pad;
                for (uint32_t x = tid; x < tot; x += kDecodeBlock) {
                    if (save) {
                        const T v = ms.ld(x);
                        bk[x] = v;
                        ms.st(x, qkds::pack_iv(qkds::iv_of(v)));
                    } else {
                        ms.st(x, bk[x]);
                    }
                }
            }
        };
        for (;;) {
            if (it >= a.max_it) break;
            const bool folded = fold1 && it == 0;
            uint32_t* rw = ctl + 4 + (rnd & 1u);
            if (SPEC && spec) {
                if constexpr (SPEC) {
                    // (iteration 2 after the folded first one: the slots hold
                    // the phi bounds of exact b2c, psi_of_exact)
                    if (!folded && fold1 && it == 1) {
                        spec_check_phase_psi<DC>(plan, tsyn, ms, row, wtab, n_tasks, n_pad, dummy_w,
                                                 a.thr_dn, a.thr_up, rw, wave, lane);
                        __syncthreads();
                    } else if (!folded) {
                        spec_check_phase_paired<DC>(plan, tsyn, ms, row, wtab, n_tasks, n_pad, dummy_w, a.thr_dn,
                                                    a.thr_up, rw, wave, lane);
                        __syncthreads();
                    }
                }
            } else if (!folded) {
                if constexpr (MSR) {
                    const int sc_mode = it == 0 ? 0 : (fold1 && it == 1 ? 2 : 1);
                    if (a.ms_offset > 0.0f)
                        ms_split_check_phase<CLAMP, DC, MSC, true>(plan, ms, row, wtab, scw, sc_mode, bwl,
                                                                   (uint32_t)L.msg, n_pad, lsign, n_tasks, (float)thr,
                                                                   a.ms_scale, a.ms_offset, wave, lane);
                    else
                        ms_split_check_phase<CLAMP, DC, MSC, false>(plan, ms, row, wtab, scw, sc_mode, bwl,
                                                                    (uint32_t)L.msg, n_pad, lsign, n_tasks, (float)thr,
                                                                    a.ms_scale, a.ms_offset, wave, lane);
                } else if constexpr (RULE == kRuleSp32)
                    sp32_check_phase<CLAMP, DC>(c.plan_slot, tsyn, ms, row, wtab, n_tasks, n_pad, thr, wave, lane);
                else if (TABLES && it == 1 && tab2_on)
                    split_check_phase<kSrcTable, CLAMP, DC, RULE>(plan, tsyn, tab2, ms, row, n_tasks, n_pad, thr,
                                                                   wave, lane);
                else
                    split_check_phase<kSrcFirst, CLAMP, DC, RULE>(plan, tsyn, tab2, ms, row, n_tasks, n_pad, thr,
                                                                   wave, lane);
                __syncthreads();
            }
            pc.mark((FOLDS && it < 2 && fold1) ? 5 + (int)it : 1);
            // the b2c of this bit phase are read only by a next iteration
            const bool keep = it + 1 < a.max_it;
            // bit phase: total_i = LLR_i + sum_k c2b[k][i], ascending checks (:256-267),
            // the hard decision's syndrome (:277, calculate_syndrome_irregular :476-486),
            // then b2c_k = clamp(total_i - c2b_k) (:303-316) into slot k.
            if (SPEC && spec) {
                if constexpr (SPEC) {
                    if (dv3) {
                        if (folded)
                            spec_bit_phase<true, MODE, true>(c, a, ms, qsyn, ctab, ftab, xsyn, xunc, zw, bobmask, keep,
                                                             f, tid, wave, lane);
                        else
                            spec_bit_phase<false, MODE, true>(c, a, ms, qsyn, ctab, ftab, xsyn, xunc, zw, bobmask, keep,
                                                              f, tid, wave, lane);
                    } else {
                        if (folded)
                            spec_bit_phase<true, MODE, false>(c, a, ms, qsyn, ctab, ftab, xsyn, xunc, zw, bobmask, keep,
                                                              f, tid, wave, lane);
                        else
                            spec_bit_phase<false, MODE, false>(c, a, ms, qsyn, ctab, ftab, xsyn, xunc, zw, bobmask, keep,
                                                               f, tid, wave, lane);
                    }
                }
            } else if (F32 && c.bit_code != nullptr) {
                if constexpr (F32) {
                    if (dv3) {
                        if (folded)
                            sp32_bit_phase<true, MODE, CLAMP, true>(c, a, ms, qsyn, ctab, xsyn, zw, bobmask, keep, f,
                                                                    tid, wave, lane);
                        else
                            sp32_bit_phase<false, MODE, CLAMP, true>(c, a, ms, qsyn, ctab, xsyn, zw, bobmask, keep, f,
                                                                     tid, wave, lane);
                    } else {
                        if (folded)
                            sp32_bit_phase<true, MODE, CLAMP, false>(c, a, ms, qsyn, ctab, xsyn, zw, bobmask, keep, f,
                                                                     tid, wave, lane);
                        else
                            sp32_bit_phase<false, MODE, CLAMP, false>(c, a, ms, qsyn, ctab, xsyn, zw, bobmask, keep,
                                                                      f, tid, wave, lane);
                    }
                }
            } else
            for (int r0 = 0; r0 * kDecodeBlock < c.n; r0 += BC) {
                T v[BC][kDvUnroll];
                int32_t jc[BC][kDvUnroll];
                int dg[BC];
#pragma unroll
                for (int u = 0; u < BC; ++u) {
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
                for (int u = 0; u < BC; ++u) {
                    const int r = r0 + u;
                    if (r * kDecodeBlock >= c.n) break;            // block-uniform
                    const int i = tid + r * kDecodeBlock;
                    const uint32_t iw = (uint32_t)(r * kDecodeBlock + wave * 64);
                    const bool ok = i < c.n;
                    const int deg = dg[u];
                    T acc;
                    if (MODE == kModeLlr) acc = ok ? (T)a.llr[(size_t)f * c.n + c.perm[i]] : (T)0;
                    else acc = bob_r(r) ? -llr_p : llr_p;
                    if constexpr (FOLDS) if (folded && ok) {
                        // fold_first_message: message of the k-th check j of bit i is
                        // +-C_{d_j} with sign = sign(P_j) ^ sign(LLR_i) (first_check_phase)
                        const uint32_t sgi = bob_r(r) ^ lsign;
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k) {
                            if (k < deg) {
                                const int j = jc[u][k];
                                const uint32_t sp = (qsyn[j >> 5] >> (j & 31)) & 1u;
                                const T cm = (T)ctab[c.chk_deg[j]];
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
                    const bool flip =
                        kRunSyn ? (ok && z != (((zw[(r * kDecodeBlock >> 6) + wave] >> lane) & 1ull) != 0)) : z;
                    if (lane == 0 && r * kDecodeBlock + wave * 64 < c.n) zw[(r * kDecodeBlock >> 6) + wave] = zb;
                    if (flip) {
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
                        uint32_t code = bob_r(r);
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
            // round flags: bit 0 a check certainly unsatisfied, bit 1 speculation
            // abort, bit 2 some check's parity uncertain (speculative rounds).
            // The next round's word was last read before this round's phases
            // and is next written after the barrier below.
            if (tid == 0) {
                ctl[4 + ((rnd + 1) & 1u)] = 0;
                if (CKPT) ctl[2 + ((rnd + 1) & 1u)] = 0;
            }
            // syndrome test (:285): any word differing from the target
            bool mismatch = false, uncertain = false;
            uint32_t nbad = 0;      // checkpointed speculation: unsatisfied checks
            for (int w = tid; w < m_words; w += kDecodeBlock) {
                const uint32_t u = xunc[w];
                const uint32_t d = (xsyn[w] ^ tsyn[w]) & ~u;
                mismatch |= d != 0;
                if (CKPT) nbad += __builtin_popcount(d);
                uncertain |= u != 0;
                if (!kRunSyn) xsyn[w] = 0;
                xunc[w] = 0;
            }
            const uint32_t wv = __builtin_amdgcn_readfirstlane(
                (uint32_t)(__any(mismatch) ? 1u : 0u) | (uint32_t)(__any(uncertain) ? 4u : 0u));
            if (wv && lane == 0) atomicOr(rw, wv);
            if (CKPT && nbad) atomicAdd(ctl + 2 + (rnd & 1u), nbad);
            __syncthreads();
            const uint32_t fl = *rw;
            const uint32_t unsat = CKPT ? ctl[2 + (rnd & 1u)] : 0u;
            rnd++;
            pc.mark(3);
            // A speculative round stands if no sign was lost on the way (bit 1)
            // and its outcome is certain: a certainly unsatisfied check (bit 0;
            // the reference iterates on), unless this was the last iteration,
            // whose hard decision is the output and must then be certain too;
            // or no uncertainty at all (bit 2 clear: the decision is exact).
            if (spec && ((fl & 2u) || ((fl & 4u) && (!(fl & 1u) || it + 1 >= a.max_it)))) {
                // decode the frame exactly (from its checkpoint)
                spec = false;
                it = it_ck;
                if (CKPT) {
                    ckpt_io(false);
                    __syncthreads();
                    ck_lim >>= 1;
                } else if (!fold1) {    // the LLR path starts from LLR_i in every slot again
                    init_slots(false);
                    __syncthreads();
                } else if (tid == 0) {
                    // the dummy column's slot back to table index 0 (the
                    // interval phases' idle lanes wrote it; read next by the
                    // second check phase, after the folded bit phase's barrier)
                    ms.st((uint32_t)c.n, (T)0);
                }
                if (tid == 0) {
                    atomicAdd(a.replay_count, 1u);
                    atomicAdd(a.spec_replays, 1ull);
                    frame_replays++;
                }
                continue;
            }
            if (!(fl & 1u)) {
                done = true;
                break;
            }
            ++it;
            if (spec && it >= it_ck + a.spec_cap && it < a.max_it) {
                spec = false;
                it = it_ck;
                if (CKPT) {
                    ckpt_io(false);
                    __syncthreads();
                    ck_lim >>= 1;
                } else if (!fold1) {
                    init_slots(false);
                    __syncthreads();
                } else if (tid == 0) {
                    ms.st((uint32_t)c.n, (T)0);    // (as above)
                }
                if (tid == 0) {
                    atomicAdd(a.replay_count, 1u);
                    atomicAdd(a.spec_replays, 1ull);
                    frame_replays++;
                }
            } else if (CKPT && !spec && it >= 2 && it + 1 < a.max_it && unsat < ck_lim) {
                // (exact round: iteration it - 1 left its b2c in the slots, and
                // iteration it can read intervals of them; iteration 1's slots
                // are table indices)
                ckpt_io(true);
                __syncthreads();
                spec = true;
                it_ck = it;
            }
        }

        // ---- outputs: SP_result and the last hard decision (keys path:
        //      packed, for key_match_kernel's arrays_equal, :433)
        if (MODE == kModeKeys) {
            // keys_match = arrays_equal(alice, decoded) (:433, :96-106), fused
            // here: this thread's word of the last hard decision against Alice's
            // (block-wide OR through ctl[7], no static LDS: the dynamic
            // allocation may take the whole 160 KB)
            if (a.key_ok) {
                // (Alice's word read here rather than held in registers
                // through the frame's iterations; both words in the internal
                // bit order)
                const uint64_t* aw = reinterpret_cast<const uint64_t*>(smem + L.aw);
                bool mis = false;
                if (tid < (int)a.words) {
                    uint64_t d = zw[tid] ^ aw[tid];
                    if ((tid + 1) * 64 > c.n) d &= (1ull << (c.n - tid * 64)) - 1ull;
                    mis = d != 0;
                }
                if (__any(mis) && lane == 0) atomicOr(ctl + 7, 1u);
            }
            // the packed decision for bits_out, internal order
            // (zout_unpack_kernel puts the bits back in place)
            if (a.bits_out)
                for (int q = tid; q < (int)a.words; q += kDecodeBlock) a.zout[(size_t)f * a.words + q] = zw[q];
        } else if (a.bits_out) {
            for (int i = tid; i < c.n; i += kDecodeBlock)
                a.bits_out[(size_t)f * c.n + c.perm[i]] = (uint8_t)((zw[i >> 6] >> (i & 63)) & 1u);
        }
        if (tid == 0) {
            a.iters[f] = done ? it + 1 : a.max_it;
            a.sp_ok[f] = done ? 1 : 0;
            ctl[1] = next_f;
            if (SPEC) {
                // this frame into its window (its completion and its replay
                // events in one add), then the next frame's policy
                __hip_atomic_fetch_add(win64 + (f >> a.win_shift), ((unsigned long long)frame_replays << 32) | 1ull,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ctl[6] = spec_policy(next_f, next_win);
            }
        }
        __syncthreads();
        if (MODE == kModeKeys && a.key_ok && tid == 0) {
            a.key_ok[f] = ctl[7] ? 0 : 1;
            ctl[7] = 0;
        }
    }
    pc.flush();
}

// ---- keys path: the kernels around decode_split_kernel ---------------------
// frame_syn_kernel: per frame the target syndrome s_A = H * alice
// (calculate_syndrome_irregular, array_and_matrix_operations.cpp:476-486, on
// Alice's key, qkd_ldpc_algorithm.cpp:413-414) and the sign of each check's
// first-iteration product, q_j = s_j ^ (H * bob)_j ^ (deg_j & sign(log_p))
// (first_check_phase), one bit per check in whole 64-check groups. kSynFrames
// frames per workgroup share each load of a check's row.
#ifndef QKD_SYN_FRAMES
#define QKD_SYN_FRAMES 4
#endif
constexpr int kSynFrames = QKD_SYN_FRAMES;
constexpr int kSynBlock = 256;
constexpr int kSynRow = 8;
//
// It also rewrites the frames' two keys in place in the split decoder's
// internal bit order (DeviceCode::perm: internal bit q holds original bit
// perm[q]), from the copies it staged: the decoder then reads Bob's bits and
// compares Alice's word by word with no gathers of its own.
__global__ __launch_bounds__(kSynBlock) void frame_syn_kernel(DeviceCode c, uint64_t* alice_w, uint64_t* bob_w,
                                                              uint32_t words, uint32_t n_frames, uint32_t lsign,
                                                              uint32_t* synw, uint32_t* counter, uint32_t* win,
                                                              uint32_t win_words) {
    // [kSynFrames][2 * words] pairs (Alice's 32-bit word, Bob's 32-bit word):
    // one 8-byte LDS read gives both keys' bit
    extern __shared__ uint2 kw[];
    // the decoder's frame queue and replay count (decode.hip launch_decode:
    // this kernel runs first on the stream, in place of a memset)
    if (blockIdx.x == 0 && threadIdx.x < 2) counter[threadIdx.x] = 0;
    for (uint32_t i = blockIdx.x * kSynBlock + threadIdx.x; i < win_words; i += gridDim.x * kSynBlock) win[i] = 0;
    const uint32_t w32 = 2 * words;
    const uint32_t f0 = blockIdx.x * kSynFrames;
    const uint32_t nf = min((uint32_t)kSynFrames, n_frames - f0);
    for (uint32_t q = threadIdx.x; q < nf * words; q += kSynBlock) {
        const uint32_t fr = q / words;
        const uint32_t w = q - fr * words;
        const uint64_t av = alice_w[(size_t)(f0 + fr) * words + w];
        const uint64_t bv = bob_w[(size_t)(f0 + fr) * words + w];
        kw[fr * w32 + 2 * w] = make_uint2((uint32_t)av, (uint32_t)bv);
        kw[fr * w32 + 2 * w + 1] = make_uint2((uint32_t)(av >> 32), (uint32_t)(bv >> 32));
    }
    __syncthreads();
    const int m_words = decode_m_words(c.m);
    const int lane = threadIdx.x & 63;
    for (int j0 = (int)(threadIdx.x & ~63u); j0 < c.m; j0 += kSynBlock) {
        const int j = j0 + lane;
        uint32_t pa[kSynFrames], pb[kSynFrames];
#pragma unroll
        for (int fr = 0; fr < kSynFrames; ++fr) pa[fr] = pb[fr] = 0;
        uint32_t deg = 0;
        auto take = [&](int bit) {
            if (bit < 0) return;
            deg++;
            const uint32_t wi = (uint32_t)bit >> 5, sh = (uint32_t)bit & 31u;
#pragma unroll
            for (int fr = 0; fr < kSynFrames; ++fr) {
                const uint2 v = kw[fr * w32 + wi];
                pa[fr] ^= v.x >> sh;
                pb[fr] ^= v.y >> sh;
            }
        };
        if (j < c.m) {
            // the row's first kSynRow entries loaded together (their latencies
            // overlap), the rest one by one
            int bits[kSynRow];
#pragma unroll
            for (int k = 0; k < kSynRow; ++k) bits[k] = k < c.max_dc ? c.chk_bits[k * c.m_pad + j] : -1;
#pragma unroll
            for (int k = 0; k < kSynRow; ++k) take(bits[k]);
            for (int k = kSynRow; k < c.max_dc; ++k) take(c.chk_bits[k * c.m_pad + j]);
        }
#pragma unroll
        for (int fr = 0; fr < kSynFrames; ++fr) {
            const uint64_t sm = __ballot(pa[fr] & 1u);
            const uint64_t qm = __ballot((pa[fr] ^ pb[fr] ^ (lsign & deg)) & 1u);
            if (lane == 0 && (uint32_t)fr < nf) {
                uint32_t* o = synw + (size_t)(f0 + fr) * 2 * m_words;
                o[j0 >> 5] = (uint32_t)sm;
                o[(j0 >> 5) + 1] = (uint32_t)(sm >> 32);
                o[m_words + (j0 >> 5)] = (uint32_t)qm;
                o[m_words + (j0 >> 5) + 1] = (uint32_t)(qm >> 32);
            }
        }
    }
    // the keys in the internal order: word w of a frame gathers bits
    // perm[64 w + lane] (one perm load serves the workgroup's frames). A wave
    // takes kSynPermBatch consecutive words at a time, issues their perm loads
    // first, and lane u keeps word u's ballots, so each key's words leave as
    // one coalesced store per frame.
    constexpr uint32_t kSynPermBatch = 8;
    constexpr uint32_t NWS = kSynBlock / 64;
    for (uint32_t w0 = (threadIdx.x >> 6) * kSynPermBatch; w0 < words; w0 += NWS * kSynPermBatch) {
        uint32_t ob[kSynPermBatch];
#pragma unroll
        for (uint32_t u = 0; u < kSynPermBatch; ++u) {
            const uint32_t q = (w0 + u) * 64 + (uint32_t)lane;
            ob[u] = q < (uint32_t)c.n ? (uint32_t)c.perm[q] : 0xffffffffu;
        }
#pragma unroll
        for (int fr = 0; fr < kSynFrames; ++fr) {
            uint64_t mya = 0, myb = 0;
#pragma unroll
            for (uint32_t u = 0; u < kSynPermBatch; ++u) {
                const bool in = ob[u] != 0xffffffffu;
                const uint32_t o = in ? ob[u] : 0u;
                const uint2 v = kw[fr * w32 + (o >> 5)];
                const uint64_t am = __ballot(in && ((v.x >> (o & 31u)) & 1u));
                const uint64_t bm = __ballot(in && ((v.y >> (o & 31u)) & 1u));
                if ((uint32_t)lane == u) {
                    mya = am;
                    myb = bm;
                }
            }
            const uint32_t w = w0 + (uint32_t)lane;
            if ((uint32_t)lane < kSynPermBatch && w < words && (uint32_t)fr < nf) {
                alice_w[(size_t)(f0 + fr) * words + w] = mya;
                bob_w[(size_t)(f0 + fr) * words + w] = myb;
            }
        }
    }
}

// bits_out[f][bit] from the decoder's packed decisions in the internal bit
// order (DeviceCode::inv)
__global__ void zout_unpack_kernel(const uint64_t* zout, const int32_t* inv, uint32_t n, uint32_t words,
                                   uint32_t n_frames, uint8_t* out) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (size_t)n_frames * n) return;
    const size_t f = gid / n;
    const uint32_t q = (uint32_t)inv[gid - f * n];
    out[gid] = (uint8_t)((zout[f * words + (q >> 6)] >> (q & 63)) & 1u);
}

// frame_syn_kernel's work bit-sliced over frames: a workgroup takes 16
// frames and first transposes their keys into 32-bit slices T[i] (bit f =
// Alice's bit i of frame f, bit 16 + f = Bob's; one ballot gives two bit
// positions: lanes 0-31 hold word w of the 16 frames' two keys, lanes 32-63
// word w + 1). A check's parities for all 16 frames and both keys are then
// one XOR of its row's slices, and each internal-order key word one slice read
// per lane followed by a ballot per frame and key. Per frame this reads LDS
// ~15x less than frame_syn_kernel (an 8-byte read per row entry and frame).
// LDS: words * 64 slices of 4 bytes (N <= 40960 in 160 KB).
constexpr int kSlicedFrames = 16;
constexpr int kSlicedBlock = 1024;
constexpr int kSlicedPre = 8;        // key-word pairs a wave loads ahead
// A bit transpose within each 32-lane half of the wave: afterwards lane 32 h +
// c holds in bit r what lane 32 h + r held in bit c. Five butterfly stages
// (s = 16 ... 1): lane l takes its partner l ^ s's value through ds_swizzle,
// rotates it by s toward the bit block it trades (one v_alignbit_b32) and
// keeps its own other block (one v_bfi_b32) -- 2 VALU and a swizzle per stage
// where a ballot per bit and a lane select per bit took ~15 VALU per bit.
template <int S, uint32_t MASK>
__device__ __forceinline__ uint32_t transpose_stage(uint32_t x, uint32_t lane) {
    const uint32_t y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (S << 10));   // lane ^ S
    const bool hi = (lane & (uint32_t)S) != 0;
    const uint32_t ys = __builtin_amdgcn_alignbit(y, y, hi ? (uint32_t)S : 32u - (uint32_t)S);
    const uint32_t k = hi ? ~MASK : MASK;
    return (x & k) | (ys & ~k);
}
__device__ __forceinline__ uint32_t wave_transpose32(uint32_t x, uint32_t lane) {
    x = transpose_stage<16, 0x0000FFFFu>(x, lane);
    x = transpose_stage<8, 0x00FF00FFu>(x, lane);
    x = transpose_stage<4, 0x0F0F0F0Fu>(x, lane);
    x = transpose_stage<2, 0x33333333u>(x, lane);
    return transpose_stage<1, 0x55555555u>(x, lane);
}
// BYTES (qkd_qkd_ldpc_batch's byte keys, N % 8 == 0, rows 8-byte aligned): the
// slices come straight from the caller's 0/1 bytes, and alice_w / bob_w are
// only written (step 3), so no packing kernel runs before this one: per
// thread and pass 8 positions of every frame and key, one 8-byte load each;
// (v & 0x01010101) << f gathers 8 frames' bits of 4 positions into the 4
// bytes of one word, and v_perm_b32 assembles each position's slice from the
// four words (Alice frames 0-7 / 8-15, Bob frames 0-7 / 8-15).
template <bool BYTES>
__global__ __launch_bounds__(kSlicedBlock) void frame_syn_sliced_kernel(DeviceCode c, uint64_t* alice_w,
                                                                        uint64_t* bob_w, uint32_t words,
                                                                        uint32_t n_frames, uint32_t lsign,
                                                                        uint32_t* synw, uint32_t* counter,
                                                                        uint32_t* win, uint32_t win_words,
                                                                        const uint8_t* alice_b,
                                                                        const uint8_t* bob_b) {
    extern __shared__ uint32_t T[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));   // (uniform to the compiler)
    constexpr uint32_t NW = kSlicedBlock / 64;
    if (blockIdx.x == 0 && tid < 2) counter[tid] = 0;     // (the decoder's queue, as frame_syn_kernel)
    for (uint32_t i = blockIdx.x * kSlicedBlock + tid; i < win_words; i += gridDim.x * kSlicedBlock) win[i] = 0;
    const uint32_t f0 = blockIdx.x * kSlicedFrames;
    const uint32_t nf = min((uint32_t)kSlicedFrames, n_frames - f0);
    const uint32_t fr = lane & 15u;
    const bool bob_lane = (lane & 16u) != 0;
    const uint32_t half = lane >> 5;                      // which word of the pair
    const uint32_t pairs = (words + 1) / 2;
    // 1. slices: wave takes word pairs p = wave, wave + NW, ..., loading up to
    //    kSlicedPre of them ahead; lane b keeps the ballot of bit b: the
    //    slices of positions 64 (2p) + b (low half) and 64 (2p + 1) + b (high)
    auto load_pair = [&](uint32_t p) -> uint64_t {
        const uint32_t w = 2 * p + half;
        if (p >= pairs || w >= words || fr >= nf) return 0;
        return (bob_lane ? bob_w : alice_w)[(size_t)(f0 + fr) * words + w];
    };
    auto slice_pair = [&](uint32_t p, uint64_t v) {
        // the lanes of half h hold word 2p + h of the 16 frames' keys (lane
        // 16 key + frame): transposed, lane 32 h + c holds the slice of that
        // word's bit c (low 32 bits) or bit 32 + c (high)
        const uint32_t tlo = wave_transpose32((uint32_t)v, lane);
        const uint32_t thi = wave_transpose32((uint32_t)(v >> 32), lane);
        const uint32_t w = 2 * p + half, b = lane & 31u;
        if (w < words) {
            T[(size_t)w * 64 + b] = tlo;
            T[(size_t)w * 64 + 32 + b] = thi;
        }
    };
    if constexpr (BYTES) {
        const uint32_t n = (uint32_t)c.n;
        for (uint32_t p = tid; p * 8 < n; p += kSlicedBlock) {
            uint2 va[kSlicedFrames], vb[kSlicedFrames];
#pragma unroll
            for (uint32_t f = 0; f < (uint32_t)kSlicedFrames; ++f) {
                const size_t off = (size_t)(f0 + f) * n + 8 * p;
                va[f] = f < nf ? *reinterpret_cast<const uint2*>(alice_b + off) : make_uint2(0, 0);
                vb[f] = f < nf ? *reinterpret_cast<const uint2*>(bob_b + off) : make_uint2(0, 0);
            }
            // x[key][frame half][position half]: byte k bit f' = that key's bit
            // at position 4 * (position half) + k of frame 8 * (frame half) + f'
            uint32_t x[2][2][2] = {};
#pragma unroll
            for (uint32_t f = 0; f < (uint32_t)kSlicedFrames; ++f) {
                const uint32_t h = f >> 3, sh = f & 7u;
                x[0][h][0] |= (va[f].x & 0x01010101u) << sh;
                x[0][h][1] |= (va[f].y & 0x01010101u) << sh;
                x[1][h][0] |= (vb[f].x & 0x01010101u) << sh;
                x[1][h][1] |= (vb[f].y & 0x01010101u) << sh;
            }
            uint32_t sl[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t ph = k >> 2, b = k & 3u;
                // bytes 0-1: Alice frames 0-7 / 8-15; 2-3: Bob's (selector 12: 0x00)
                const uint32_t lo = __builtin_amdgcn_perm(x[0][1][ph], x[0][0][ph], b | ((b + 4) << 8) | 0x0c0c0000u);
                const uint32_t hi = __builtin_amdgcn_perm(x[1][1][ph], x[1][0][ph], 0x0c0cu | (b << 16) | ((b + 4) << 24));
                sl[k] = lo | hi;
            }
            // (positions past N are never read: rows and perm hold bits < N)
            *reinterpret_cast<uint4*>(T + 8 * p) = make_uint4(sl[0], sl[1], sl[2], sl[3]);
            *reinterpret_cast<uint4*>(T + 8 * p + 4) = make_uint4(sl[4], sl[5], sl[6], sl[7]);
        }
    } else {
        for (uint32_t p0 = wave; p0 < pairs; p0 += NW * kSlicedPre) {
            uint64_t v[kSlicedPre];
#pragma unroll
            for (int k = 0; k < kSlicedPre; ++k) v[k] = load_pair(p0 + (uint32_t)k * NW);
#pragma unroll
            for (int k = 0; k < kSlicedPre; ++k)
                if (p0 + (uint32_t)k * NW < pairs) slice_pair(p0 + (uint32_t)k * NW, v[k]);
        }
    }
    __syncthreads();
    // 2. syndromes: lane = check; 64 checks per wave and pass, then per frame
    //    two ballots (target s_j, first-product sign q_j) that lane f keeps
    const int m_words = decode_m_words(c.m);
    const int rs = c.chk_rs;
    for (uint32_t j0 = wave * 64; j0 < (uint32_t)c.m; j0 += kSlicedBlock) {
        const uint32_t j = j0 + lane;
        uint32_t P = 0, deg = 0;
        if (j < (uint32_t)c.m) {
            const uint16_t* row = c.chk_rows16 + (size_t)j * rs;
            for (int h = 0; h < rs; h += 8) {
                const uint4 r = *reinterpret_cast<const uint4*>(row + h);
                const uint32_t e[8] = {r.x & 0xffffu, r.x >> 16, r.y & 0xffffu, r.y >> 16,
                                       r.z & 0xffffu, r.z >> 16, r.w & 0xffffu, r.w >> 16};
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (e[k] != 0xffffu) {
                        P ^= T[e[k]];
                        deg++;
                    }
            }
        }
        const uint32_t Q = P ^ (P >> 16) ^ ((lsign & deg) ? 0xffffu : 0u);   // low 16: q bits
        // transposed, lane f < 16 holds frame f's target bits of the 64 checks
        // (its own value the low word, lane 32 + f's the high) and lane 16 + f
        // its q bits; both go out as one 8-byte store (m_words and j0 / 32 even)
        const uint32_t tr = wave_transpose32((P & 0xffffu) | (Q << 16), lane);
        const uint32_t up = (uint32_t)__shfl_xor((int)tr, 32);
        const uint32_t g = lane & 15u;
        if (lane < 32 && g < nf) {
            uint32_t* o = synw + (size_t)(f0 + g) * 2 * m_words + (lane < 16 ? 0 : m_words) + (j0 >> 5);
            *reinterpret_cast<uint2*>(o) = make_uint2(tr, up);
        }
    }
    // 3. the keys in the internal order (DeviceCode::perm), in place: word w's
    //    lane l reads the slice of original bit perm[64 w + l] (the perm entry
    //    of the wave's next word loaded a word ahead, through a clamped index:
    //    no branch around the load); transposed, lane f < 16 holds Alice's word
    //    of frame f (high half from lane 32 + f), lane 16 + f Bob's
    const uint32_t cn = (uint32_t)c.n;
    auto perm_at = [&](uint32_t w) -> uint32_t {
        const uint32_t q = w * 64 + lane;
        return c.perm[q < cn ? q : 0u];
    };
    uint32_t pq = perm_at(wave < (uint32_t)words ? wave : 0u);
    for (uint32_t w = wave; w < words; w += NW) {
        const uint32_t wn = w + NW;
        const uint32_t pn = perm_at(wn < (uint32_t)words ? wn : w);
        const uint32_t S = w * 64 + lane < cn ? T[pq] : 0u;
        const uint32_t tr = wave_transpose32(S, lane);
        const uint32_t up = (uint32_t)__shfl_xor((int)tr, 32);
        const uint32_t g = lane & 15u;
        if (lane < 32 && g < nf)
            (lane < 16 ? alice_w : bob_w)[(size_t)(f0 + g) * words + w] = ((uint64_t)up << 32) | tr;
        pq = pn;
    }
}

hipError_t launch_frame_syn(const DecodeArgs& a, hipStream_t stream, bool gather, bool pack_first) {
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;
    // the bit-sliced form when its slices fit LDS and the compact rows exist
    // (gather, the QKD_SYN_SLICED option 0: frame_syn_kernel; tests compare the two)
    const size_t slds = (size_t)a.words * 64 * sizeof(uint32_t);
    const bool sliced = a.code.chk_rows16 && slds <= 160 * 1024 && !gather;
    // byte keys (qkd_qkd_ldpc_batch): packed by the sliced kernel itself when
    // their rows allow 8-byte loads (pack_first, the QKD_SYN_BYTES option 0: pack_kernel first;
    // tests compare the two), else by pack_kernel
    const bool bytes = a.alice_b && sliced && a.code.n % 8 == 0 &&
                       ((reinterpret_cast<uintptr_t>(a.alice_b) | reinterpret_cast<uintptr_t>(a.bob_b)) & 7u) == 0 &&
                       !pack_first;
    if (a.alice_b && !bytes) {
        const hipError_t e = launch_pack_keys(a, stream);
        if (e != hipSuccess) return e;
    }
    if (sliced) {
        const void* fn = bytes ? (const void*)frame_syn_sliced_kernel<true> : (const void*)frame_syn_sliced_kernel<false>;
        // (the attribute on every launch, for the current device, as decode_grid
        // does for the decoder: no process-wide flag to race on or to skip for
        // a second device)
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        const dim3 grid((a.n_frames + kSlicedFrames - 1) / kSlicedFrames);
        if (bytes)
            hipLaunchKernelGGL(frame_syn_sliced_kernel<true>, grid, dim3(kSlicedBlock), slds, stream, a.code,
                               const_cast<uint64_t*>(a.alice_w), const_cast<uint64_t*>(a.bob_w), a.words,
                               a.n_frames, lsign, const_cast<uint32_t*>(a.synw), a.counter, a.win,
                               2 * a.win_count, a.alice_b, a.bob_b);
        else
            hipLaunchKernelGGL(frame_syn_sliced_kernel<false>, grid, dim3(kSlicedBlock), slds, stream, a.code,
                               const_cast<uint64_t*>(a.alice_w), const_cast<uint64_t*>(a.bob_w), a.words,
                               a.n_frames, lsign, const_cast<uint32_t*>(a.synw), a.counter, a.win,
                               2 * a.win_count, nullptr, nullptr);
        return hipGetLastError();
    }
    const size_t lds = (size_t)kSynFrames * 2 * a.words * sizeof(uint64_t);
    hipLaunchKernelGGL(frame_syn_kernel, dim3((a.n_frames + kSynFrames - 1) / kSynFrames), dim3(kSynBlock), lds,
                       stream, a.code, const_cast<uint64_t*>(a.alice_w), const_cast<uint64_t*>(a.bob_w), a.words,
                       a.n_frames, lsign, const_cast<uint32_t*>(a.synw), a.counter, a.win, 2 * a.win_count);
    return hipGetLastError();
}

hipError_t launch_key_match(const DecodeArgs& a, hipStream_t stream) {
    // (decode_split_kernel compares the keys itself: keys_match needs no launch)
    if (a.bits_out) {
        const size_t total = (size_t)a.n_frames * a.code.n;
        hipLaunchKernelGGL(zout_unpack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, a.zout,
                           a.code.inv, (uint32_t)a.code.n, a.words, a.n_frames, a.bits_out);
    }
    return hipGetLastError();
}

template <int MODE, int RULE, bool CLAMP, int SPEC = 0>
static DecodeFn pick_split_dc(int max_dc, int* dc) {
    if (max_dc <= 4) { *dc = 4; return decode_split_kernel<MODE, RULE, 4, CLAMP, SPEC>; }
    if (max_dc <= 6) { *dc = 6; return decode_split_kernel<MODE, RULE, 6, CLAMP, SPEC>; }
    if (max_dc <= 8) { *dc = 8; return decode_split_kernel<MODE, RULE, 8, CLAMP, SPEC>; }
    if (max_dc <= 16) { *dc = 16; return decode_split_kernel<MODE, RULE, 16, CLAMP, SPEC>; }
    *dc = 64;
    return decode_split_kernel<MODE, RULE, 64, CLAMP, SPEC>;
}

DecodeFn pick_split_spec(int mode, int max_dc, bool ckpt, int* dc) {
    if (ckpt) return pick_split_dc<kModeKeys, kRuleSp64, true, 2>(max_dc, dc);
    return mode == kModeLlr ? pick_split_dc<kModeLlr, kRuleSp64, true, 1>(max_dc, dc)
                            : pick_split_dc<kModeKeys, kRuleSp64, true, 1>(max_dc, dc);
}

template <int MODE, int RULE>
static DecodeFn pick_split_clamp(bool clamp, int max_dc, int* dc) {
    return clamp ? pick_split_dc<MODE, RULE, true>(max_dc, dc) : pick_split_dc<MODE, RULE, false>(max_dc, dc);
}

// the min-sum rules' buckets (the host takes them for check degree <= 8
// only: the additive mask table)
template <int MODE, int RULE, bool CLAMP>
static DecodeFn pick_split_ms_dc(int max_dc, int* dc) {
    if (max_dc <= 4) { *dc = 4; return decode_split_kernel<MODE, RULE, 4, CLAMP, 0>; }
    if (max_dc <= 6) { *dc = 6; return decode_split_kernel<MODE, RULE, 6, CLAMP, 0>; }
    *dc = 8;
    return decode_split_kernel<MODE, RULE, 8, CLAMP, 0>;
}
template <int MODE, int RULE>
static DecodeFn pick_split_ms(bool clamp, int max_dc, int* dc) {
    return clamp ? pick_split_ms_dc<MODE, RULE, true>(max_dc, dc) : pick_split_ms_dc<MODE, RULE, false>(max_dc, dc);
}

template <int MODE>
static DecodeFn pick_split_rule(int rule, bool clamp, int max_dc, int* dc) {
    if (rule == kRuleMinSumSplit) return pick_split_ms<MODE, kRuleMinSumSplit>(clamp, max_dc, dc);
    if (rule == kRuleMinSumSplitSc) return pick_split_ms<MODE, kRuleMinSumSplitSc>(clamp, max_dc, dc);
    if (rule == kRuleSp32) return pick_split_clamp<MODE, kRuleSp32>(clamp, max_dc, dc);
    return pick_split_clamp<MODE, kRuleSp64>(clamp, max_dc, dc);
}

// the exact keys-path kernel for codes past kMaxBitsSplit (LONG)
DecodeFn pick_split_long(bool clamp, int max_dc, int* dc) {
    if (max_dc <= 4) { *dc = 4; return clamp ? decode_split_kernel<kModeKeys, kRuleSp64, 4, true, 0, true>
                                             : decode_split_kernel<kModeKeys, kRuleSp64, 4, false, 0, true>; }
    if (max_dc <= 6) { *dc = 6; return clamp ? decode_split_kernel<kModeKeys, kRuleSp64, 6, true, 0, true>
                                             : decode_split_kernel<kModeKeys, kRuleSp64, 6, false, 0, true>; }
    if (max_dc <= 8) { *dc = 8; return clamp ? decode_split_kernel<kModeKeys, kRuleSp64, 8, true, 0, true>
                                             : decode_split_kernel<kModeKeys, kRuleSp64, 8, false, 0, true>; }
    *dc = 16;
    return clamp ? decode_split_kernel<kModeKeys, kRuleSp64, 16, true, 0, true>
                 : decode_split_kernel<kModeKeys, kRuleSp64, 16, false, 0, true>;
}

DecodeFn pick_split_decode(int mode, int rule, bool clamp, int max_dc, int* dc) {
    return mode == kModeLlr ? pick_split_rule<kModeLlr>(rule, clamp, max_dc, dc)
                            : pick_split_rule<kModeKeys>(rule, clamp, max_dc, dc);
}

}  // namespace qkd
