// decode.hip — gfx950 kernels and launchers of the QKD LDPC decoder.
//
// Hot path: flooding sum-product decoding, reference
// src/qkd_ldpc_algorithm.cpp:175-345 (irregular) / :3-173 (regular, the same
// arithmetic for a regular code), reached through QKD_LDPC_* (:347-447) and
// run_trial (src/simulation.cpp:161-189).
//
// MI355X mapping
//   * One 1024-thread workgroup owns one frame at a time; workgroups are
//     persistent (grid = resident workgroups) and pull frames from a device
//     queue (one atomic per frame), so frames with 2 and 50 iterations mix
//     without tail stalls.
//   * Per-frame state is the reference's two message arrays collapsed to one:
//     c2b messages (E binary64, slot-major per check, in HBM/L2/MALL) plus the
//     bit totals (N binary64) in LDS. The reference's b2c message for edge
//     (j,i) is exactly total_i - c2b(j,i) clamped (its :303-316), so it is
//     recomputed inside the check update instead of being stored: same bits,
//     half the message traffic.
//   * Check phase: thread per check, slot-major coalesced c2b read/write, the
//     d_c tanh values in registers, the extrinsic product by division (keeps
//     the reference's 0/0 -> NaN behaviour). Bit phase: thread per bit,
//     gathers its d_v c2b in ascending check order (the reference's
//     std::accumulate order). Syndrome test: thread per check over LDS totals,
//     block-wide OR.
//   * tanh/atanh are the bit-exact restatements in qkd_math.h; the whole
//     library builds with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <cstring>

#include "qkd_internal.h"
#include "qkd_math.h"
#include "qkd_plan.h"
#include "qkd_rng.h"
#include "qkd_decode.h"
#include "qkd_spec.h"

namespace qkd {

// The check phase of one iteration for one wave: tasks wave, wave + NW, ...
// Per edge (qkd_ldpc_algorithm.cpp:220-249):
//   b2c = FIRST ? LLR_i : clamp(total_i - c2b)                  (:188, :303-316)
//   t   = tanh(b2c / 2)                                         (:224)
//   P   = (s_j ? -1 : 1) * t_0 * t_1 * ...  (ascending bits)    (:231-235)
//   c2b = clamp(2 * atanh(P / t))                               (:239-249)
// Software-pipelined and unrolled by two so that no loaded value is copied
// across the loop back-edge. Each half-trip does, in this order:
//   store the previous task's message  |  issue the look-ahead loads (plan
//   word two tasks ahead, bit total and stored message one task ahead)  |
//   compute this task (its operands were loaded one half-trip earlier).
// vmcnt counts loads and stores in issue order, so a task only ever waits
// for memory operations that had a whole task of arithmetic to complete.
// The plan is padded with idle tasks (qkd_plan.h): no bounds tests on the
// look-ahead loads.
//
// Measured (config 2, three iterations): removing the tanh /
// atanh arithmetic saves only 12 % of the kernel, making the message
// gathers/scatters coalesced saves 24 %: the phase is bound by the two
// together, not by fp64 latency (working on two tasks at once, to interleave
// two dependency chains, measured no gain).
template <int SRC, bool CLAMP, int DC, int RULE, typename T>
__device__ __forceinline__ void check_phase(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                            const T* total, const uint16_t* t2idx, const double* tab2,
                                            T* __restrict__ c2b, T* row, int n_tasks, int n_pad, T thr,
                                            int wave, int lane, float ms_scale, float ms_offset) {
    constexpr int NW = kDecodeBlock / 64;
    constexpr bool FIRST = SRC != kSrcGeneral;    // no stored message is read
    int t = wave;
    if (t >= n_tasks) return;
    const uint2* pl = plan + lane;
    auto msg = [&](uint2 p) -> T* { return c2b + pw_row(p) * n_pad + pw_bit(p); };
    // the incoming value: a bit total, or (kSrcTable) the tabulated tanh
    auto src = [&](uint2 p) -> T {
        if constexpr (SRC == kSrcTable) return tab2[t2idx[pw_bit(p)] + pw_row(p)];
        else return total[pw_bit(p)];
    };
    // the target syndrome bit of the lane's check
    auto sbit = [&](uint2 p) -> uint32_t {
        const uint32_t j = pw_chk(p);
        return (tsyn[j >> 5] >> (j & 31)) & 1u;
    };
    auto edge = [&](T x, T o, uint2 w) -> T {
        const T a = edge_in<SRC, CLAMP, RULE>(x, o, thr);
        row[lane] = a;
        wave_lds_sync();
        return edge_out<CLAMP, DC, RULE>(a, w, sbit(w), lane, thr, row, ms_scale, ms_offset);
    };
    uint2 wa = pl[t * 64];
    uint2 wb = pl[(t + NW) * 64];
    T xa = src(wa);
    T oa = FIRST ? (T)0 : *msg(wa);
    T* pend = nullptr;      // message computed by the previous task, not yet stored
    T pv = 0;
    for (;;) {
        if (pend) msg_store(pend, pv);
        const uint2 wc = pl[(t + 2 * NW) * 64];
        const T xb = src(wb);
        const T ob = FIRST ? (T)0 : *msg(wb);
        pv = edge(xa, oa, wa);
        pend = msg(wa);
        t += NW;
        if (t >= n_tasks) break;
        msg_store(pend, pv);
        wa = pl[(t + 2 * NW) * 64];
        xa = src(wc);
        oa = FIRST ? (T)0 : *msg(wc);
        pv = edge(xb, ob, wb);
        pend = msg(wb);
        t += NW;
        if (t >= n_tasks) break;
        wb = wa;
        wa = wc;
    }
    *pend = pv;
}

// ---- min-sum with the message state in LDS (kRuleMinSumLds) -----------------
// Every min-sum message of a check j is a function of four words (ms_state):
//   x  min1 = min_k |b2c_k|                (binary32 bits)
//   y  min2 = min over k != idx1 of |b2c_k|
//   z  sign bits, bit k = (b2c_k < 0)
//   w  idx1 (bits 0..7; 0xff: none) | par << 31,   par = s_j ^ parity(z)
// and, self-corrected (QKD_MINSUM_SELF_CORRECT), a fifth word czf[j]: bit k =
// (b2c_k == 0). z and czf are then also the previous iteration's b2c signs
// and erasures, which the next check phase compares with (Savin's
// self-corrected min-sum: a b2c whose sign flipped, both nonzero, becomes 0).
// The message to the edge at position k is scale * (k == idx1 ? min2 : min1),
// negated when par ^ z_k, then clamped: the same binary32 operations, on the
// same values, as edge_out's min-sum branch (and tests/test_variants.py's model), so the
// two kernels agree bit for bit. (min over the others of the |b2c| is min2 for
// the argmin and min1 for everyone else, ties included; NaN magnitudes never
// win a comparison, as fminf ignores them.) 16 bytes per check instead of 4
// bytes per edge: the frame's whole message state (m * 16 B) and its bit
// totals (n * 4 B) stay in LDS, and the decode touches no global memory but
// the code's own (L2-resident) arrays.
template <bool CLAMP>
__device__ __forceinline__ float ms_msg(uint4 st, uint32_t pos, float scale, float off, float thr) {
    const float m = pos == (st.w & 0xffu) ? __uint_as_float(st.y) : __uint_as_float(st.x);
    float v = scale * m;
    if (off > 0.0f) v = fmaxf(v - off, 0.0f);
    const uint32_t neg = (st.w >> 31) ^ ((st.z >> pos) & 1u);
    v = neg ? -v : v;
    if (CLAMP) v = clamp_msg(v, thr);
    return v;
}

// Check phase of kRuleMinSumLds for one wave: per lane (edge), b2c from the
// bit total and the check's previous state; the segment's first lane then
// folds the segment's b2c (through the wave's LDS row) into the new state.
// Check phase of kRuleMinSumLds: one THREAD per check (rounds of 1024
// checks). The min-sum check rule costs a handful of operations per edge, so
// unlike the sum-product phase (one edge per lane, to spread the per-edge
// transcendentals) a thread walks its check's row itself: bit totals from
// LDS, the previous state from LDS, the row's bits from the code's ELL array
// (coalesced across threads, L2-resident), the next round's row loaded ahead.
//   b2c_k = FIRST ? total : clamp(total - message_k(previous state))
//   state = (min |b2c|, second min, argmin, signs, s_j ^ parity)
template <int SRC, bool CLAMP, int DC>
__device__ __forceinline__ void ms_check_phase(const DeviceCode& c, const uint32_t* tsyn, const float* total,
                                               uint4* cst, uint32_t* czf, bool sc, float thr, float scale,
                                               float off) {
    const int m = c.m;
    int j = threadIdx.x;
    if (j >= m) return;
    int nb[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) nb[k] = k < c.max_dc ? c.chk_bits[k * c.m_pad + j] : -1;
    for (;;) {
        int bl[DC];
#pragma unroll
        for (int k = 0; k < DC; ++k) bl[k] = nb[k];
        const int jn = j + kDecodeBlock;
        if (jn < m) {
#pragma unroll
            for (int k = 0; k < DC; ++k) nb[k] = k < c.max_dc ? c.chk_bits[k * c.m_pad + jn] : -1;
        }
        uint4 st = make_uint4(0, 0, 0, 0);
        uint32_t zp = 0;
        if (SRC == kSrcGeneral) {
            st = cst[j];
            if (sc) zp = czf[j];
        }
        float m1 = __builtin_inff(), m2 = __builtin_inff();
        uint32_t idx = 0xffu, sg = 0, zf = 0;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (bl[k] >= 0) {
                float x = total[bl[k]];
                if (SRC == kSrcGeneral) {
                    x = x - ms_msg<CLAMP>(st, (uint32_t)k, scale, off, thr);
                    if (CLAMP) x = clamp_msg(x, thr);
                    // self-correction: the previous b2c nonzero, this one too,
                    // signs differ -> erased
                    if (sc && !((zp >> k) & 1u) && x != 0.0f && (x < 0.0f) != (((st.z >> k) & 1u) != 0u)) x = 0.0f;
                }
                const float a = fabsf(x);
                sg |= (x < 0.0f ? 1u : 0u) << k;
                zf |= (x == 0.0f ? 1u : 0u) << k;
                if (a < m1) {
                    m2 = m1;
                    m1 = a;
                    idx = (uint32_t)k;
                } else if (a < m2) {
                    m2 = a;
                }
            }
        }
        const uint32_t sbit = (tsyn[j >> 5] >> (j & 31)) & 1u;
        const uint32_t par = sbit ^ ((uint32_t)__popc(sg) & 1u);
        cst[j] = make_uint4(__float_as_uint(m1), __float_as_uint(m2), sg, idx | (par << 31));
        if (sc) czf[j] = zf;
        j = jn;
        if (j >= m) break;
    }
}


// fold_first_message: when the second table is also in use, nothing reads the
// first iteration's stored messages (the second check phase takes its inputs
// from the table), so the first check phase is skipped and the first bit phase
// rebuilds each message from one sign bit per check (qsyn, the sign of P_j,
// computed in the prologue from Bob's bits) and the bit's own LLR sign.
//
// First check phase of the QKD path (QKD_LDPC_irregular, :398-425 -> :220-249
// at it = 0), where b2c = LLR_i = bob_i ? -log_p : +log_p for every edge. Then
//   t_i = tanh(LLR_i / 2) = sign_i * T,  T = |tanh(log_p / 2)|  (tanh is odd)
//   P   = (s_j ? -1 : 1) * t_0 * ... * t_{d-1}: binary64 products round on
//         magnitudes only, so |P| = M_d = (((T * T) * T) ...) and
//         sign(P) = s_j ^ sign_0 ^ ... ^ sign_{d-1}
//   c2b = clamp(2 atanh(P / t_i)) = sign(P) ^ sign_i times
//         C_d = clamp(2 atanh(M_d / T))            (atanh and clamp are odd)
// so every first-iteration message is +-C_d, bit for bit; the host evaluates
// C_d with the same tanh/atanh restatement (decode_keys). sign_i is the sign
// bit of the LLR in `total` (also right for log_p <= 0 and for +-0).
__device__ __forceinline__ void first_check_phase(const uint2* __restrict__ plan, const uint32_t* tsyn,
                                                  const double* total, const double* ctab,
                                                  double* __restrict__ c2b, int n_tasks, int n_pad, int wave,
                                                  int lane) {
    constexpr int NW = kDecodeBlock / 64;
    // kPlanGroup tasks per trip: their plan words are loaded together (the
    // plan is padded, so the loads need no bounds test); stores are predicated.
    for (int t0 = wave; t0 < n_tasks; t0 += NW * kPlanGroup) {
        uint2 w[kPlanGroup];
#pragma unroll
        for (int u = 0; u < kPlanGroup; ++u) w[u] = plan[(t0 + u * NW) * 64 + lane];
#pragma unroll
        for (int u = 0; u < kPlanGroup; ++u) {
            const int t = t0 + u * NW;
            if (t >= n_tasks) break;
            const uint32_t bit = pw_bit(w[u]);
            const uint32_t j = pw_chk(w[u]);
            const uint32_t sg = (uint32_t)qkdm::hi32(total[bit]) >> 31;
            const uint32_t sp = ((tsyn[j >> 5] >> (j & 31)) & 1u) ^ (uint32_t)seg_parity(__ballot(sg), w[u]);
            const double cm = ctab[pw_deg(w[u])];
            c2b[pw_row(w[u]) * n_pad + bit] = (sp ^ sg) ? -cm : cm;
        }
    }
}

// Flooding sum-product decode of whole frames, one frame per workgroup at a
// time (reference sum_product_decoding_irregular, qkd_ldpc_algorithm.cpp:175-345;
// the regular twin :3-173 is the same arithmetic).
//
// Message store: the c2b messages of the frame live bit-major in global memory,
// c2b[k * n_pad + i] = message from the k-th check (ascending) of bit i, i.e.
// the reference's c2b[i][k] layout transposed for coalescing (:192-205). The
// check phase's gather/scatter of it overlaps its transcendental arithmetic;
// the bit phase streams it. (A plan-order store, coalesced in the check phase
// and gathered in the bit phase, measured 10 % slower overall: the gathers
// then stall a phase with nothing to overlap.)
//
// Per iteration:
//  check phase (check_phase above), one edge per lane, wave tasks of whole
//    checks (qkd_plan.h)
//  bit phase (:256-267), one bit per lane, coalesced rows:
//    total_i = LLR_i + c2b[0][i] + c2b[1][i] + ...  (ascending check order)
//    hard decision z_i = total_i <= 0; if z_i, XOR it into the syndrome bit of
//    each of its checks (LDS bit array; XOR is order-free, so exact)
//  syndrome test (:277-285): compare with the target words, block-wide any()
//
// GT (large codes, N beyond what LDS holds): the bit totals live in global
// scratch instead of LDS; everything else is the same kernel. The tables of
// the QKD path (per-bit LDS indices) and the LDS-state min-sum are not used.
template <int MODE, int RULE, int DC, bool CLAMP, bool GT>
__global__ __launch_bounds__(kDecodeBlock) void decode_kernel(DecodeArgs a) {
    using T = typename RuleMsg<RULE>::T;
    // the exact QKD-path shortcuts (first/second-iteration tables) exist for
    // the reference rule only
    constexpr bool TABLES = MODE == kModeKeys && RULE == kRuleSp64 && !GT;
    constexpr bool MSL = RULE == kRuleMinSumLds || RULE == kRuleMinSumLdsSc;
    constexpr bool SC = RULE == kRuleMinSumLdsSc;      // self-corrected min-sum
    static_assert(!(MSL && GT), "the LDS-state min-sum keeps its totals in LDS");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const DeviceCode& c = a.code;
    const DecodeLds L(c.n_pad, (c.n + 63) / 64, c.m, DC, a.tab2_entries, GT ? 0 : (int)sizeof(T),
                      MSL ? c.m : 0, (int)sizeof(T), SC);
    uint4* cst = reinterpret_cast<uint4*>(smem + L.cst);
    uint32_t* czf = reinterpret_cast<uint32_t*>(smem + L.czf);
    const int m_words = decode_m_words(c.m);
    T* total;
    if constexpr (GT)
        total = reinterpret_cast<T*>(a.totals + (size_t)blockIdx.x * a.totals_stride);
    else
        total = reinterpret_cast<T*>(smem);
    uint32_t* tsyn = reinterpret_cast<uint32_t*>(smem + L.tsyn);
    uint32_t* xsyn = reinterpret_cast<uint32_t*>(smem + L.xsyn);
    uint32_t* qsyn = reinterpret_cast<uint32_t*>(smem + L.qsyn);
    // QKD path with both tables: the first check phase is folded into the
    // first bit phase (fold_first_message)
    const bool fold1 = TABLES && a.first_table && a.tab2_entries;
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;     // sign bit of log_p
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + L.ctl);
    double* ctab = reinterpret_cast<double*>(smem + L.ctab);
    double* tab2 = reinterpret_cast<double*>(smem + L.tab2);
    uint16_t* t2idx = reinterpret_cast<uint16_t*>(smem + L.t2idx);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave index as a scalar: task loops and plan addresses stay in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    T* row = reinterpret_cast<T*>(smem + L.tval) + wave * (64 + DC);
    const int n_tasks = c.n_tasks;
    const int n_pad = c.n_pad;
    const uint2* plan = c.plan;
    T* c2b = reinterpret_cast<T*>(a.c2b + (size_t)blockIdx.x * a.c2b_stride);
    const T thr = (T)a.thr;
    const T llr_p = (T)a.log_p;
    uint32_t any_k = 0;
    if (tid == 0) { ctl[2] = 0; ctl[3] = 0; }
    if (TABLES && tid <= kFirstTableDeg) ctab[tid] = a.first_c2b[tid];
    if (TABLES && a.tab2_entries) {
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

        // ---- prologue: the frame's Alice and Bob words staged in LDS (the tanh
        //      rows are free until the first check phase)
        const uint64_t* sw = reinterpret_cast<const uint64_t*>(smem + L.tval);   // [alice | bob]
        if (MODE == kModeKeys) {
            uint64_t* w = reinterpret_cast<uint64_t*>(smem + L.tval);
            for (int q = tid; q < (int)a.words; q += kDecodeBlock) {
                w[q] = a.alice_w[(size_t)f * a.words + q];
                w[a.words + q] = a.bob_w[(size_t)f * a.words + q];
            }
            __syncthreads();
        }
        // ---- prologue: channel LLRs into LDS (:188 / :400-405); the dummy
        //      column n of idle plan lanes gets 0
        // Bob's bits of this thread's bit-phase rounds (round r: bit tid + r *
        // kDecodeBlock), N <= 32 * kDecodeBlock; the large-code kernels read
        // them from the packed key instead (any N)
        uint32_t bobmask = 0;
        {
            int r = 0;
            for (int i = tid; i < c.n; i += kDecodeBlock, ++r) {
                T l;
                if (MODE == kModeLlr) {
                    l = (T)a.llr[(size_t)f * c.n + i];
                } else {
                    const uint32_t bb = (uint32_t)((sw[a.words + (i >> 6)] >> (i & 63)) & 1u);
                    if (!GT) bobmask |= bb << r;
                    l = bb ? -llr_p : llr_p;
                }
                total[i] = l;
            }
            if (tid == 0) {
                total[c.n] = 0;
                if (TABLES && a.tab2_entries) t2idx[c.n] = 0;   // idle lanes' table reads
            }
        }
        // ---- prologue: target syndrome bits per check (tsyn) and, on the QKD
        //      path, each check's first-product sign (qsyn, fold_first_message);
        //      thread per check, 64 consecutive checks per wave -> one ballot.
        //      ELL pad entries are -1, so the row loads do not wait for the degree.
        for (int j0 = wave * 64; j0 < c.m; j0 += kDecodeBlock) {
            const int j = j0 + lane;
            const bool ok = j < c.m;
            int sj = 0, qj = 0;
            if (MODE == kModeLlr) {
                sj = ok ? (a.syn[(size_t)f * c.m + j] != 0) : 0;
            } else {
                // calculate_syndrome_irregular on Alice's key (:413-414), and
                // q_j = s_j ^ syn(bob)_j ^ (deg_j & sign(log_p))
                int bl[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) bl[k] = (ok && k < c.max_dc) ? c.chk_bits[k * c.m_pad + j] : -1;
                uint32_t pa = 0, pb = 0, deg = 0;
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    const int bit = bl[k];
                    if (bit >= 0) {
                        pa ^= (uint32_t)(sw[bit >> 6] >> (bit & 63));
                        pb ^= (uint32_t)(sw[a.words + (bit >> 6)] >> (bit & 63));
                        deg++;
                    }
                }
                if (ok && DC < c.max_dc) {
                    for (int k = DC; k < c.max_dc; ++k) {
                        const int bit = c.chk_bits[k * c.m_pad + j];
                        if (bit >= 0) {
                            pa ^= (uint32_t)(sw[bit >> 6] >> (bit & 63));
                            pb ^= (uint32_t)(sw[a.words + (bit >> 6)] >> (bit & 63));
                            deg++;
                        }
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
            bool tabled = false;
            if constexpr (MSL) {
                tabled = true;
                if (it == 0)
                    ms_check_phase<kSrcFirst, CLAMP, DC>(c, tsyn, total, cst, czf, SC, thr, a.ms_scale,
                                                         a.ms_offset);
                else
                    ms_check_phase<kSrcGeneral, CLAMP, DC>(c, tsyn, total, cst, czf, SC, thr, a.ms_scale,
                                                           a.ms_offset);
            }
            if constexpr (TABLES) {
                tabled = true;
                if (it == 0 && fold1)
                    ;   // messages rebuilt from signs in the bit phase (fold_first_message)
                else if (it == 0 && a.first_table)
                    first_check_phase(plan, tsyn, total, ctab, c2b, n_tasks, n_pad, wave, lane);
                else if (it == 1 && a.tab2_entries)
                    check_phase<kSrcTable, CLAMP, DC, RULE>(plan, tsyn, total, t2idx, tab2, c2b, row, n_tasks,
                                                            n_pad, thr, wave, lane, a.ms_scale, a.ms_offset);
                else
                    tabled = false;
            }
            if constexpr (!MSL) {
                if (!tabled) {
                    if (it == 0)
                        check_phase<kSrcFirst, CLAMP, DC, RULE>(plan, tsyn, total, t2idx, tab2, c2b, row, n_tasks,
                                                                n_pad, thr, wave, lane, a.ms_scale, a.ms_offset);
                    else
                        check_phase<kSrcGeneral, CLAMP, DC, RULE>(plan, tsyn, total, t2idx, tab2, c2b, row,
                                                                  n_tasks, n_pad, thr, wave, lane, a.ms_scale, a.ms_offset);
                }
            }
            __syncthreads();
            pc.mark((TABLES && it < 2 && a.first_table) ? 5 + (int)it : 1);
            // bit phase: total_i = LLR_i + sum_k c2b[k][i], ascending checks (:256-267),
            // and the hard decision's syndrome (:277, calculate_syndrome_irregular :476-486).
            // kBitChunk rounds at a time: all their message rows and check indices
            // are loaded before any of them is summed.
            for (int r0 = 0; r0 * kDecodeBlock < c.n; r0 += kBitChunk) {
                T v[kBitChunk][kDvUnroll];
                int32_t jc[kBitChunk][kDvUnroll];
                uint32_t ps[kBitChunk][kDvUnroll];     // MSL: positions in the checks
                int dg[kBitChunk];
#pragma unroll
                for (int u = 0; u < kBitChunk; ++u) {
                    const int i = tid + (r0 + u) * kDecodeBlock;
                    const bool ok = i < c.n;
                    dg[u] = ok ? c.bit_deg[i] : 0;
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) {
                        const bool ld = ok && k < c.max_dv;
                        if constexpr (MSL) {
                            v[u][k] = 0;
                            ps[u][k] = ld ? c.bit_pos[k * n_pad + i] : 0u;
                        } else {
                            v[u][k] = (ld && !(fold1 && it == 0)) ? c2b[k * n_pad + i] : (T)0;
                        }
                        jc[u][k] = ld ? c.bit_chk[k * n_pad + i] : 0;
                    }
                }
#pragma unroll
                for (int u = 0; u < kBitChunk; ++u) {
                    const int r = r0 + u;
                    const int i = tid + r * kDecodeBlock;
                    if (i >= c.n) break;
                    const int deg = dg[u];
                    T acc;
                    if (MODE == kModeLlr) acc = (T)a.llr[(size_t)f * c.n + i];
                    else if constexpr (GT)
                        acc = ((a.bob_w[(size_t)f * a.words + (i >> 6)] >> (i & 63)) & 1u) ? -llr_p : llr_p;
                    else
                        acc = ((bobmask >> r) & 1u) ? -llr_p : llr_p;
                    if constexpr (TABLES) if (fold1 && it == 0) {
                        // fold_first_message: message of the k-th check j of bit i is
                        // +-C_{d_j} with sign = sign(P_j) ^ sign(LLR_i) (first_check_phase)
                        const uint32_t sgi = ((bobmask >> r) & 1u) ^ lsign;
                        const uint8_t* pd = c.pat_deg + c.bit_pat[i] * c.max_dv;
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k) {
                            if (k < deg) {
                                const int j = jc[u][k];
                                const uint32_t sp = (qsyn[j >> 5] >> (j & 31)) & 1u;
                                const double cm = ctab[pd[k]];
                                v[u][k] = (sp ^ sgi) ? -cm : cm;
                            }
                        }
                    }
                    if constexpr (MSL) {
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k)
                            if (k < deg) v[u][k] = ms_msg<CLAMP>(cst[jc[u][k]], ps[u][k], a.ms_scale, a.ms_offset, thr);
                    }
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) acc = k < deg ? acc + v[u][k] : acc;
                    if constexpr (MSL) {
                        for (int k = kDvUnroll; k < deg; ++k)
                            acc = acc + ms_msg<CLAMP>(cst[c.bit_chk[k * n_pad + i]], c.bit_pos[k * n_pad + i],
                                                      a.ms_scale, a.ms_offset, thr);
                    } else {
                        for (int k = kDvUnroll; k < deg; ++k) acc = acc + c2b[k * n_pad + i];
                    }
                    total[i] = acc;
                    if constexpr (TABLES) if (a.tab2_entries && it == 0) {
                        // second_table_index: bob bit and the signs of the first messages
                        uint32_t code = (bobmask >> r) & 1u;
#pragma unroll
                        for (int k = 0; k < kTab2MaxDv; ++k)
                            if (k < deg) code |= ((uint32_t)qkdm::hi32(v[u][k]) >> 31) << (1 + k);
                        t2idx[i] = (uint16_t)(c.bit_pat[i] * tab2_stride(c.max_dv) + code * c.max_dv);
                    }
                    if (acc <= 0) {
#pragma unroll
                        for (int k = 0; k < kDvUnroll; ++k)
                            if (k < deg) atomicXor(&xsyn[jc[u][k] >> 5], 1u << (jc[u][k] & 31));
                        for (int k = kDvUnroll; k < deg; ++k) {
                            const int j = c.bit_chk[k * n_pad + i];
                            atomicXor(&xsyn[j >> 5], 1u << (j & 31));
                        }
                    }
                }
            }
            __syncthreads();
            pc.mark(2);
            if constexpr (RULE == kRuleSp64) {
                // TRACE_SUM_PRODUCT (:250-275): this iteration's clamped c2b ("E") and totals ("L")
                if (a.trace) {
                    double* tr = a.trace + (size_t)it * a.trace_stride;
                    const int nm = c.max_dv * n_pad;
                    for (int q = tid; q < nm; q += kDecodeBlock) tr[q] = c2b[q];
                    for (int q = tid; q < c.n; q += kDecodeBlock) tr[nm + q] = total[q];
                }
            }
            // syndrome test (:285): any word differing from the target
            bool mismatch = false;
            for (int w = tid; w < m_words; w += kDecodeBlock) {
                mismatch |= xsyn[w] != tsyn[w];
                xsyn[w] = 0;
            }
            const bool any_mismatch = block_any(mismatch, ctl + 2, any_k);
            pc.mark(3);
            if (!any_mismatch) {
                done = true;
                break;
            }
        }

        // ---- outputs: SP_result + last hard decision (+ keys_match)
        bool key_mismatch = false;
        for (int i = tid; i < c.n; i += kDecodeBlock) {
            const uint8_t d = total[i] <= 0 ? 1 : 0;
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

// ---- syndrome ---------------------------------------------------------------
__global__ void syndrome_kernel(DeviceCode c, const uint8_t* bits, uint32_t n_frames, uint8_t* syn) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (size_t)n_frames * c.m) return;
    const size_t f = gid / c.m;
    const int j = (int)(gid - f * c.m);
    const int deg = c.chk_deg[j];
    int s = 0;
    for (int k = 0; k < deg; ++k) s ^= bits[f * c.n + c.chk_bits[k * c.m_pad + j]] & 1;
    syn[gid] = (uint8_t)s;
}

// ---- bit packing ------------------------------------------------------------
// One lane per 8 key bytes -> one packed byte (little-endian words, so the
// byte array is the uint64 word array); bits past n are 0. 8-byte loads when
// every frame row is 8-byte aligned (n % 8 == 0), byte loads otherwise.
__global__ void pack_kernel(const uint8_t* bytes0, const uint8_t* bytes1, uint32_t n, uint32_t words,
                            uint32_t n_frames, uint64_t* out0, uint64_t* out1, uint32_t wide) {
    // wide (the host's choice: n % 32 == 0 and both arrays 16-byte aligned): 32
    // key bytes -> 4 packed bytes per thread (two 16-byte loads); else one
    // packed byte per thread
    const uint8_t* bytes = blockIdx.y ? bytes1 : bytes0;
    uint64_t* out = blockIdx.y ? out1 : out0;
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per_frame = (size_t)words * 8;
    if (wide) {
        const size_t per4 = per_frame / 4;            // 4-byte output groups per frame
        if (gid >= (size_t)n_frames * per4) return;
        const size_t f = gid / per4;
        const uint32_t b = (uint32_t)(gid - f * per4);   // output bytes 4b .. 4b+3
        uint32_t m = 0;
        if ((size_t)b * 32 < n) {
            const uint4* src = reinterpret_cast<const uint4*>(bytes + f * n + (size_t)b * 32);
            const uint4 v0 = src[0], v1 = src[1];
            const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t t = w[k] & 0x01010101u;            // byte q's LSB at bit 8q
                m |= ((t * 0x01020408u) >> 24 & 0xfu) << (4 * k); // byte q -> bit 24 + q
            }
        }
        reinterpret_cast<uint32_t*>(out)[gid] = m;
        return;
    }
    if (gid >= (size_t)n_frames * per_frame) return;
    const size_t f = gid / per_frame;
    const uint32_t b = (uint32_t)(gid - f * per_frame);
    const uint8_t* src = bytes + f * n;
    uint32_t m = 0;
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t i = b * 8 + k;
        if (i < n) m |= (uint32_t)(src[i] & 1u) << k;
    }
    reinterpret_cast<uint8_t*>(out)[gid] = (uint8_t)m;
}

hipError_t launch_pack_keys(const DecodeArgs& a, hipStream_t stream) {
    const uint32_t n = (uint32_t)a.code.n;
    const size_t nw = (size_t)a.n_frames * a.words;
    // Alice's and Bob's keys in one launch (grid.y selects the key; the wide
    // form needs both arrays 16-byte aligned)
    const bool wide = (n % 32) == 0 &&
                      ((reinterpret_cast<uintptr_t>(a.alice_b) | reinterpret_cast<uintptr_t>(a.bob_b)) & 15u) == 0;
    const size_t threads = wide ? nw * 2 : nw * 8;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((threads + 255) / 256), 2), dim3(256), 0, stream,
                       a.alice_b, a.bob_b, n, a.words, a.n_frames, const_cast<uint64_t*>(a.alice_w),
                       const_cast<uint64_t*>(a.bob_w), wide ? 1u : 0u);
    return hipGetLastError();
}

__global__ void unpack_kernel(const uint64_t* words_in, uint32_t n, uint32_t words, uint32_t n_frames,
                              uint8_t* out) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (size_t)n_frames * n) return;
    const size_t f = gid / n;
    const uint32_t i = (uint32_t)(gid - f * n);
    out[gid] = (uint8_t)((words_in[f * words + (i >> 6)] >> (i & 63)) & 1u);
}

// ---- key generation: one thread per frame ------------------------------------
// generate_random_bit_array + introduce_errors (array_and_matrix_operations.cpp:424-460)
__global__ void keygen_kernel(const uint64_t* seeds, uint64_t offset, uint32_t n_frames, uint32_t n,
                              uint32_t words, uint32_t ne, uint64_t* alice_w, uint64_t* bob_w,
                              uint32_t* low_scratch, double* exact_q) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    qkdr::Xoshiro256pp g;
    g.seed(seeds[f] + offset);
    uint64_t* A = alice_w + (size_t)f * words;
    uint64_t* B = bob_w + (size_t)f * words;
    for (uint32_t w = 0; w < words; ++w) {
        const uint32_t nb = min(64u, n - w * 64);
        uint64_t v = 0;
        for (uint32_t b = 0; b < nb; ++b) v |= (g.next() >> 63) << b;
        A[w] = v;
        B[w] = v;
    }
    uint32_t* low = low_scratch + (size_t)f * ne;
    qkdr::shuffle_low_positions(g, n, ne, low);
    for (uint32_t p = 0; p < ne; ++p) {
        const uint32_t pos = low[p];
        B[pos >> 6] ^= 1ull << (pos & 63);
    }
    if (exact_q) exact_q[f] = (double)ne / (double)n;
}

// ---- key generation: kKeygenLanes lanes per frame (jump-ahead) ---------------
// Same key pair as keygen_kernel, drawn in parallel; kKeygenFrames frames per
// workgroup, each on its own kKeygenLanes-lane slice of it. The
// trial's draw stream (qkdr::trial_draws) is cut into kKeygenLanes chunks of
// `chunk` draws; lane l of a frame jumps the seeded state by l * chunk draws
// (jump[b] = T^(chunk * 2^b), applied for the set bits of l: a jump is a
// 256x256 GF(2) product per level and lane, so fewer lanes per frame mean fewer
// levels and less work per frame) and then steps through its chunk:
//   draws [0, N)      Alice's bits (whole words per lane: chunk % 64 == 0)
//   draw N (even N)   the lone swap of std::shuffle
//   the rest          one Lemire draw per shuffle pair (i, i+1)
// Shuffle steps with index < ne need the exact swap sequence: their draws are
// parked in LDS and replayed by the frame's lane 0 (qkdr::shuffle_low_positions,
// steps i < ne). Steps >= ne only ever write "low[x] = i", so the last such
// writer of each low position is found with an LDS atomicMax. A Lemire rejection
// (probability ~ range / 2^64 per draw) shifts every later draw: such a frame
// is regenerated serially by its lane 0 from its seed.
// R32 (N <= 65536): every pair's range (i + 1)(i + 2) < 2^32, so the Lemire
// products are 64 x 32 bits and the pair split x / (i + 2) a binary32
// reciprocal product with one exact integer correction (the lanes of a frame
// diverge between Alice's bits and the shuffle draws, so the wave pays both
// paths on every draw: the binary64 division was most of it).
template <bool R32>
__global__ __launch_bounds__(kKeygenBlock) void keygen_fast_kernel(const uint64_t* seeds, uint64_t offset, uint32_t n,
                                                         uint32_t words, uint32_t ne, uint32_t chunk,
                                                         uint32_t n_frames, const uint64_t* __restrict__ jump,
                                                         const uint64_t* __restrict__ jpoly,
                                                         uint64_t* alice_w, uint64_t* bob_w, double* exact_q,
                                                         uint32_t force_serial) {
    extern __shared__ uint32_t kg_lds[];
    __shared__ uint32_t s_lone[kKeygenFrames], s_reject[kKeygenFrames];
    const uint32_t slot = threadIdx.x / kKeygenLanes;          // this frame's slice of the workgroup
    const uint32_t lane = threadIdx.x % kKeygenLanes;
    // per frame (an even number of words, so every park is 8-byte aligned):
    // low[ne], last[ne], park[ne / 2 + 1]
    const uint32_t frame_words = 2 * ne + 2 * (ne / 2 + 1);
    uint32_t* low = kg_lds + (size_t)slot * frame_words;     // ne: replayed positions
    uint32_t* last = low + ne;                               // ne: last step >= ne writing here (0 = none)
    uint2* park = (uint2*)(last + ne);                       // ne / 2 + 1 parked pair draws

    const uint32_t f = blockIdx.x * kKeygenFrames + slot;
    const bool live = f < n_frames;                          // (the last workgroup may hold fewer frames)
    const bool even = (n & 1u) == 0;
    const uint64_t pair0 = even ? (uint64_t)n + 1 : (uint64_t)n;  // draw index of the first pair
    const uint32_t i0 = even ? 2u : 1u;                             // its step index
    const uint64_t draws = qkdr::trial_draws(n);

    qkdr::Xoshiro256pp g;
    g.seed(live ? seeds[f] + offset : 0);
    uint64_t st[4] = {g.s0, g.s1, g.s2, g.s3};
    if (jpoly) {
        // the lane's jump as a polynomial in T (qkd_rng.h jump_poly_apply):
        // 256 state steps, no matrix reads
        const uint64_t p[4] = {jpoly[lane * 4 + 0], jpoly[lane * 4 + 1], jpoly[lane * 4 + 2], jpoly[lane * 4 + 3]};
        qkdr::jump_poly_apply(p, st);
    } else {
        for (int b = 0; b < kKeygenLevels; ++b) {
            uint64_t t[4] = {st[0], st[1], st[2], st[3]};
            qkdr::jump_apply(jump + (size_t)b * 1024, t);
            if ((lane >> b) & 1u) {
                st[0] = t[0]; st[1] = t[1]; st[2] = t[2]; st[3] = t[3];
            }
        }
    }
    g.s0 = st[0]; g.s1 = st[1]; g.s2 = st[2]; g.s3 = st[3];

    for (uint32_t p = lane; p < ne; p += kKeygenLanes) {
        low[p] = p;
        last[p] = 0;
    }
    if (lane == 0) {
        s_lone[slot] = 0;
        s_reject[slot] = force_serial;
    }
    __syncthreads();

    uint64_t* A = alice_w + (size_t)f * words;
    uint64_t* B = bob_w + (size_t)f * words;
    const uint64_t first = (uint64_t)lane * chunk;
    const uint64_t end = live ? min(first + chunk, draws) : first;
    uint64_t acc = 0;
    for (uint64_t d = first; d < end; ++d) {
        const uint64_t r = g.next();
        if (d < n) {
            acc |= (r >> 63) << (d & 63);
            if ((d & 63) == 63 || d + 1 == n) {
                A[d >> 6] = acc;
                B[d >> 6] = acc;
                acc = 0;
            }
        } else if (d < pair0) {
            s_lone[slot] = (uint32_t)(r >> 63);
        } else {
            const uint32_t i = i0 + 2u * (uint32_t)(d - pair0);
            const uint64_t b1 = (uint64_t)i + 2;
            const uint64_t range = ((uint64_t)i + 1) * b1;
            uint32_t qa, qb;
            if constexpr (R32) {
                // r * range = p1 * 2^32 + p0 with range < 2^32: the low 64 bits
                // (Lemire's test) and the high ones (x < range < 2^32)
                const uint32_t rg = (uint32_t)range, bb = (uint32_t)b1;
                const uint64_t p0 = (uint64_t)(uint32_t)r * rg;
                const uint64_t p1 = (uint64_t)(uint32_t)(r >> 32) * rg;
                const uint64_t lo = p0 + (p1 << 32);
                if (lo < range) {
                    if (lo < (0 - range) % range) s_reject[slot] = 1;
                }
                const uint32_t x = (uint32_t)((p1 + (p0 >> 32)) >> 32);
                // x / bb < 2^16 to 2^-21 relative: off by at most one
                uint32_t q = (uint32_t)((float)x * __builtin_amdgcn_rcpf((float)bb));
                int32_t rem = (int32_t)(x - q * bb);
                if (rem < 0) { --q; rem += (int32_t)bb; }
                else if (rem >= (int32_t)bb) { ++q; rem -= (int32_t)bb; }
                qa = q;
                qb = (uint32_t)rem;
            } else {
                const uint64_t lo = r * range;
                if (lo < range && lo < (0 - range) % range) s_reject[slot] = 1;
                const uint64_t x = qkdr::mul_hi64(r, range);
                // quotient through binary64, corrected to the exact integer one
                uint64_t a = (uint64_t)((double)x / (double)b1);
                if (a * b1 > x) --a;
                else if (x - a * b1 >= b1) ++a;
                qa = (uint32_t)a;
                qb = (uint32_t)(x - a * b1);
            }
            if (i < ne) {
                park[(i - i0) >> 1] = make_uint2(qa, qb);
            } else {
                if (qa < ne) atomicMax(&last[qa], i);
                if (qb < ne) atomicMax(&last[qb], i + 1);
            }
        }
    }
    __syncthreads();

    if (live && s_reject[slot]) {
        // exact serial regeneration of this frame (never observed in practice)
        if (lane == 0) {
            qkdr::Xoshiro256pp h;
            h.seed(seeds[f] + offset);
            for (uint32_t w = 0; w < words; ++w) {
                const uint32_t nb = min(64u, n - w * 64);
                uint64_t v = 0;
                for (uint32_t b = 0; b < nb; ++b) v |= (h.next() >> 63) << b;
                A[w] = v;
                B[w] = v;
            }
            qkdr::shuffle_low_positions(h, n, ne, low);
            for (uint32_t p = 0; p < ne; ++p) B[low[p] >> 6] ^= 1ull << (low[p] & 63);
            if (exact_q) exact_q[f] = (double)ne / (double)n;
        }
    } else if (live && lane == 0) {
        // replay of the steps with index < ne (shuffle_low_positions' step())
        auto step = [&](uint32_t si, uint32_t x) {
            if (si < ne) {
                const uint32_t v = low[x];
                low[x] = si;
                low[si] = v;
            } else if (x < ne) {
                low[x] = si;
            }
        };
        if (n > 1) {
            if (even) step(1, s_lone[slot]);
            for (uint32_t i = i0; i < ne && i < n; i += 2) {
                const uint2 q = park[(i - i0) >> 1];
                step(i, q.x);
                step(i + 1, q.y);
            }
        }
        if (exact_q) exact_q[f] = (double)ne / (double)n;
    }
    __syncthreads();
    if (live && !s_reject[slot]) {
        for (uint32_t p = lane; p < ne; p += kKeygenLanes) {
            const uint32_t pos = last[p] ? last[p] : low[p];
            atomicXor((unsigned long long*)&B[pos >> 6], 1ull << (pos & 63));
        }
    }
}

// The error positions without replaying the shuffle (keygen_split_kernel).
// Step s of the forward shuffle (introduce_errors, qkd_ldpc_algorithm.cpp)
// swaps a[s] with a[x_s], x_s <= s, and a[s] is still s when it does (earlier
// steps touch only lower indices), so afterwards a[x_s] = s. Hence a[q]
// (q < ne) is the last step s with x_s = q (last[q], an LDS atomicMax over
// all steps) when there is one; otherwise the last step to touch q is step q
// itself, which left there the value position x_q held just before it: the
// last step s in [x_q, q) with x_s = x_q, or failing that (recursively) the
// value x_q received from its own step. Position 0 is no step's index (its
// value is 0 until a step writes it). Such positions (no later writer) are
// ~q/N of them, ~2 per config-2 frame: the whole wave resolves each in turn,
// scanning 64 steps per ballot. Every argument is wave-uniform.
template <class XS>
__device__ __forceinline__ uint32_t kg_resolve_wave(uint32_t q, const XS& xs, uint32_t lane) {
    uint32_t t = q, p = xs(q);
    for (;;) {
        const int lo = p > 1u ? (int)p : 1;
        for (int base = (int)t - 1; base >= lo; base -= 64) {
            const int st = base - (int)lane;
            const bool hit = st >= lo && xs((uint32_t)st) == p;
            const uint64_t hb = __ballot(hit);
            if (hb) return (uint32_t)(base - (__ffsll((unsigned long long)hb) - 1));
        }
        if (p == 0) return 0;
        t = p;
        p = xs(p);
    }
}

// The same key pair by two waves per workgroup (the default generator): in the
// one-wave form every lane's chunk mixes Alice's bits and shuffle draws, so
// the wave runs both loop bodies on every draw. Here wave 0 draws only Alice's
// bits (a frame's lane l: draws [l * cb, (l + 1) * cb), cb a multiple of 32,
// written as whole 32-bit LDS words) and wave 1 only the shuffle's
// (lane l: from draw N + l * cs): each lane jumps once (its own polynomial,
// c->d_jpoly2), every loop is uniform. A frame takes kKgSplitLanes lanes of
// each wave, so a workgroup holds kKgSplitFrames frames: fewer lanes per
// frame mean longer chunks but fewer 256-step jumps per frame. Every step's
// swap partner below ne goes into last[] (LDS atomicMax), the low steps'
// partners also into park[]; the error positions then follow without a serial
// replay (kg_resolve_wave). The flips land in a mask beside Alice's words,
// and both keys leave as whole coalesced words (Bob's as Alice ^ mask).
// LDS per frame: low[ne] (the serial path's), last[ne], park[ne / 2 + 1],
// alice[words], flips[words].
template <bool R32>
__global__ __launch_bounds__(kKgBlock) void keygen_split_kernel(const uint64_t* seeds, uint64_t offset, uint32_t n,
                                                           uint32_t words, uint32_t ne, uint32_t cb, uint32_t cs,
                                                           uint32_t n_frames, const uint64_t* __restrict__ jpoly,
                                                           uint64_t* alice_w, uint64_t* bob_w, double* exact_q,
                                                           uint32_t force_serial) {
    constexpr uint32_t KL = kKgSplitLanes, FPW = kKgSplitFrames;
    extern __shared__ uint64_t ks_lds[];
    __shared__ uint32_t s_lone[FPW], s_reject[FPW];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    // (the wave index through readfirstlane: the compiler then knows it, and a
    // frame's seed, wave-uniform, so the jumps' state steps stay scalar)
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const bool shuffle_wave = (wv & 1u) != 0;
    const uint32_t slot = (wv >> 1) * (64 / KL) + lane / KL;   // this lane's frame in the workgroup
    const uint32_t l = lane % KL;                               // and its lane in that frame
    // (per frame an even number of 32-bit words before the key words)
    const uint32_t frame_u64 = (2 * ne + 2 * (ne / 2 + 1)) / 2 + 2 * words;
    auto frame_lds = [&](uint32_t sl) { return ks_lds + (size_t)sl * frame_u64; };
    uint32_t* low = reinterpret_cast<uint32_t*>(frame_lds(slot));
    uint32_t* last = low + ne;
    uint2* park = reinterpret_cast<uint2*>(last + ne);
    uint64_t* aw = reinterpret_cast<uint64_t*>(park + ne / 2 + 1);
    const uint32_t f = blockIdx.x * FPW + slot;
    const bool live = f < n_frames;                             // (the last workgroup may hold fewer)
    const bool even = (n & 1u) == 0;
    const uint64_t pair0 = even ? (uint64_t)n + 1 : (uint64_t)n;
    const uint32_t i0 = even ? 2u : 1u;
    const uint64_t draws = qkdr::trial_draws(n);

    qkdr::Xoshiro256pp g;
    g.seed(live ? seeds[f] + offset : 0);
    {
        uint64_t st[4] = {g.s0, g.s1, g.s2, g.s3};
        const uint32_t pi = (shuffle_wave ? KL : 0u) + l;
        const uint64_t p[4] = {jpoly[pi * 4 + 0], jpoly[pi * 4 + 1], jpoly[pi * 4 + 2], jpoly[pi * 4 + 3]};
        qkdr::jump_poly_apply(p, st);
        g.s0 = st[0]; g.s1 = st[1]; g.s2 = st[2]; g.s3 = st[3];
    }
    for (uint32_t sl = 0; sl < FPW; ++sl) {
        uint32_t* lo = reinterpret_cast<uint32_t*>(frame_lds(sl));
        uint64_t* a = reinterpret_cast<uint64_t*>(reinterpret_cast<uint2*>(lo + 2 * ne) + ne / 2 + 1);
        for (uint32_t q = tid; q < ne; q += kKgBlock) lo[ne + q] = 0;
        for (uint32_t w = tid; w < 2 * words; w += kKgBlock) a[w] = 0;   // Alice's words, then the flip mask
    }
    if (tid < FPW) {
        s_lone[tid] = 0;
        s_reject[tid] = force_serial;
    }
    __syncthreads();

    if (!shuffle_wave) {
        // Alice's bits: cb is a multiple of 32 (host.cpp), so a lane's chunk
        // is whole 32-bit words of the key, written by that lane alone. A
        // block of 32 draws shifts each draw's top bit into a register from
        // the right (one v_alignbit_b32) and reverses it at the end, so draw
        // d lands on bit d & 31.
        const uint32_t first = l * cb;
        const uint32_t end = live ? min(first + cb, n) : first;
        uint32_t* aw32 = reinterpret_cast<uint32_t*>(aw);
        for (uint32_t d = first; d < end; d += 32) {
            uint32_t acc = 0;
            const uint32_t cnt = min(32u, end - d);
            if (cnt == 32) {
#pragma unroll 8
                for (int k = 0; k < 32; ++k)
                    acc = __builtin_amdgcn_alignbit(acc, (uint32_t)(g.next_fast() >> 32), 31);
                aw32[d >> 5] = __builtin_bitreverse32(acc);
            } else {
                for (uint32_t k = 0; k < cnt; ++k)
                    acc = __builtin_amdgcn_alignbit(acc, (uint32_t)(g.next_fast() >> 32), 31);
                aw32[d >> 5] = __builtin_bitreverse32(acc) >> (32 - cnt);
            }
        }
    } else if constexpr (R32) {
        // The shuffle's pair draws, N <= 65536: every range (i + 1)(i + 2) <
        // 2^32 (kept up to date by one add per draw). Lemire's product r *
        // range in 32-bit pieces: x = its high 64 bits is A_hi + carry(A_lo +
        // B_hi) for A = r_hi * range, B = r_lo * range; its low 64 bits are
        // below range (the rejection test, probability ~2^-32) only if A_lo +
        // B_hi wraps to 0, and only then is B_lo needed. The pair split x /
        // (i + 2) as a binary32 reciprocal product with one exact correction
        // (checked on the host for every divisor), its remainder by a 24-bit
        // multiply (q, i + 2 < 2^17).
        uint64_t d = (uint64_t)n + (uint64_t)l * cs;
        const uint64_t end = live ? min(d + cs, draws) : d;
        if (d < end && d < pair0) {                      // the lone draw (even N): lane 0
            const uint32_t x = (uint32_t)(g.next_fast() >> 63);
            s_lone[slot] = x;
            if (x < ne) atomicMax(&last[x], 1u);
            ++d;
        }
        uint32_t i = i0 + 2u * (uint32_t)(d - pair0);
        uint32_t rg = (i + 1u) * (i + 2u);
        for (; d < end; ++d) {
            const uint64_t r = g.next_fast();
            const uint32_t rl = (uint32_t)r, rh = (uint32_t)(r >> 32);
            const uint32_t alo = rh * rg, ahi = __umulhi(rh, rg), bhi = __umulhi(rl, rg);
            const uint32_t t = alo + bhi;
            const uint32_t x = ahi + (t < alo ? 1u : 0u);
            if (t == 0u) {
                const uint32_t blo = rl * rg;
                if (blo < rg && (uint64_t)blo < (0ull - (uint64_t)rg) % (uint64_t)rg) s_reject[slot] = 1;
            }
            const uint32_t bb = i + 2u;
            const uint32_t q0 = (uint32_t)((float)x * __builtin_amdgcn_rcpf((float)bb));
            const int32_t r0 = (int32_t)(x - __umul24(q0, bb));
            // (the correction as selects, no divergent branch)
            const bool lo = r0 < 0, hi = r0 >= (int32_t)bb;
            const uint32_t q = q0 + (hi ? 1u : 0u) - (lo ? 1u : 0u);
            const int32_t rem = r0 + (lo ? (int32_t)bb : 0) - (hi ? (int32_t)bb : 0);
            if (i < ne) park[(i - i0) >> 1] = make_uint2(q, (uint32_t)rem);
            if (q < ne) atomicMax(&last[q], i);
            if ((uint32_t)rem < ne) atomicMax(&last[rem], i + 1);
            rg += 4u * i + 10u;                          // (i + 3)(i + 4)
            i += 2u;
        }
    } else {
        const uint64_t first = (uint64_t)n + (uint64_t)l * cs;
        const uint64_t end = live ? min(first + cs, draws) : first;
        for (uint64_t d = first; d < end; ++d) {
            const uint64_t r = g.next();
            if (d < pair0) {
                const uint32_t x = (uint32_t)(r >> 63);
                s_lone[slot] = x;
                if (x < ne) atomicMax(&last[x], 1u);
                continue;
            }
            const uint32_t i = i0 + 2u * (uint32_t)(d - pair0);
            const uint64_t b1 = (uint64_t)i + 2;
            const uint64_t range = ((uint64_t)i + 1) * b1;
            uint32_t qa, qb;
            {
                const uint64_t lo = r * range;
                if (lo < range && lo < (0 - range) % range) s_reject[slot] = 1;
                const uint64_t x = qkdr::mul_hi64(r, range);
                uint64_t a = (uint64_t)((double)x / (double)b1);
                if (a * b1 > x) --a;
                else if (x - a * b1 >= b1) ++a;
                qa = (uint32_t)a;
                qb = (uint32_t)(x - a * b1);
            }
            if (i < ne) park[(i - i0) >> 1] = make_uint2(qa, qb);
            if (qa < ne) atomicMax(&last[qa], i);
            if (qb < ne) atomicMax(&last[qb], i + 1);
        }
    }
    __syncthreads();

    uint64_t* A = alice_w + (size_t)f * words;
    uint64_t* B = bob_w + (size_t)f * words;
    const bool rej = live && s_reject[slot];
    if (rej && !shuffle_wave && l == 0) {
        // exact serial regeneration of this frame (never observed in practice)
        qkdr::Xoshiro256pp h;
        h.seed(seeds[f] + offset);
        for (uint32_t w = 0; w < words; ++w) {
            const uint32_t nb = min(64u, n - w * 64);
            uint64_t v = 0;
            for (uint32_t b = 0; b < nb; ++b) v |= (h.next() >> 63) << b;
            A[w] = v;
            B[w] = v;
        }
        qkdr::shuffle_low_positions(h, n, ne, low);
        for (uint32_t q = 0; q < ne; ++q) B[low[q] >> 6] ^= 1ull << (low[q] & 63);
        if (exact_q) exact_q[f] = (double)ne / (double)n;
    }
    if (live && !rej && shuffle_wave && l == 0 && exact_q) exact_q[f] = (double)ne / (double)n;
    // (the rest per frame slot, all kKgBlock threads; a rejected frame is done):
    // the flips into a mask beside Alice's words, Bob's key = Alice's ^ mask
    for (uint32_t sl = 0; sl < FPW; ++sl) {
        const uint32_t fs = blockIdx.x * FPW + sl;
        if (fs >= n_frames || s_reject[sl]) continue;                // (workgroup-uniform)
        uint32_t* lo = reinterpret_cast<uint32_t*>(frame_lds(sl));
        const uint2* pk = reinterpret_cast<const uint2*>(lo + 2 * ne);
        uint64_t* b = reinterpret_cast<uint64_t*>(reinterpret_cast<uint2*>(lo + 2 * ne) + ne / 2 + 1) + words;
        // x_s: the position step s (1 <= s < ne) swaps with
        auto xs = [&](uint32_t st) -> uint32_t {
            if (even && st == 1) return s_lone[sl];
            const uint2 pr = pk[(st - i0) >> 1];
            return ((st - i0) & 1u) ? pr.y : pr.x;
        };
        for (uint32_t q0 = 0; q0 < ne; q0 += kKgBlock) {       // (uniform trip count: the scans use every lane)
            const uint32_t q = q0 + tid;
            uint32_t pos = q < ne ? lo[ne + q] : 1u;
            uint64_t rare = __ballot(pos == 0 && q > 0);
            while (rare) {
                const uint32_t src = (uint32_t)(__ffsll((unsigned long long)rare) - 1);
                rare &= rare - 1;
                const uint32_t r = kg_resolve_wave(q0 + (tid & ~63u) + src, xs, lane);
                if (lane == src) pos = r;
            }
            if (q < ne) atomicXor(reinterpret_cast<unsigned long long*>(&b[pos >> 6]), 1ull << (pos & 63u));
        }
    }
    __syncthreads();
    for (uint32_t sl = 0; sl < FPW; ++sl) {
        const uint32_t fs = blockIdx.x * FPW + sl;
        if (fs >= n_frames || s_reject[sl]) continue;
        const uint64_t* a = reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint2*>(
                                reinterpret_cast<const uint32_t*>(frame_lds(sl)) + 2 * ne) + ne / 2 + 1);
        for (uint32_t w = tid; w < words; w += kKgBlock) {
            alice_w[(size_t)fs * words + w] = a[w];
            bob_w[(size_t)fs * words + w] = a[w] ^ a[words + w];
        }
    }
}

// ---- batch reduction (simulation.cpp:252-312) ----------------------------------
__global__ void counters_kernel(const uint32_t* iters, const uint8_t* sp, const uint8_t* ko,
                                uint32_t n_frames, qkd_counters* out) {
    __shared__ unsigned long long s_sum[5];
    __shared__ uint32_t s_min, s_max;
    if (threadIdx.x < 5) s_sum[threadIdx.x] = 0;
    if (threadIdx.x == 0) { s_min = 0xffffffffu; s_max = 0; }
    __syncthreads();
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < n_frames) {
        atomicAdd(&s_sum[0], 1ull);
        if (sp[f]) {
            const unsigned long long it = iters[f];
            atomicAdd(&s_sum[1], 1ull);
            if (!ko || ko[f]) atomicAdd(&s_sum[2], 1ull);
            atomicAdd(&s_sum[3], it);
            atomicAdd(&s_sum[4], it * it);
            atomicMin(&s_min, (uint32_t)it);
            atomicMax(&s_max, (uint32_t)it);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd((unsigned long long*)&out->frames, s_sum[0]);
        atomicAdd((unsigned long long*)&out->sp_ok, s_sum[1]);
        atomicAdd((unsigned long long*)&out->ldpc_ok, s_sum[2]);
        atomicAdd((unsigned long long*)&out->sum_iters, s_sum[3]);
        atomicAdd((unsigned long long*)&out->sum_iters_sq, s_sum[4]);
        atomicMin(&out->min_iters, s_min);
        atomicMax(&out->max_iters, s_max);
    }
}

// One workgroup over every frame (batches up to kCountersOneBlock frames): the
// reduction and the record's initialisation in one launch.
constexpr uint32_t kCountersOneBlock = 1u << 16;
__global__ __launch_bounds__(1024) void counters_one_kernel(const uint32_t* iters, const uint8_t* sp,
                                                            const uint8_t* ko, uint32_t n_frames,
                                                            qkd_counters* out) {
    __shared__ unsigned long long s_sum[5];
    __shared__ uint32_t s_min, s_max;
    if (threadIdx.x < 5) s_sum[threadIdx.x] = 0;
    if (threadIdx.x == 0) { s_min = 0xffffffffu; s_max = 0; }
    __syncthreads();
    unsigned long long c1 = 0, c2 = 0, c3 = 0, c4 = 0;
    uint32_t mn = 0xffffffffu, mx = 0;
    // (every load unconditional and kCntBatch frames' loads issued together:
    // a load behind the sp[f] branch made each frame two dependent round trips)
    constexpr uint32_t kCntBatch = 4;
    for (uint32_t f0 = threadIdx.x; f0 < n_frames; f0 += kCntBatch * blockDim.x) {
        uint32_t itv[kCntBatch];
        uint8_t spv[kCntBatch], kov[kCntBatch];
#pragma unroll
        for (uint32_t u = 0; u < kCntBatch; ++u) {
            const uint32_t f = f0 + u * blockDim.x;
            const bool in = f < n_frames;
            itv[u] = in ? iters[f] : 0u;
            spv[u] = in ? sp[f] : (uint8_t)0;
            kov[u] = (in && ko) ? ko[f] : (uint8_t)1;
        }
#pragma unroll
        for (uint32_t u = 0; u < kCntBatch; ++u) {
            if (spv[u]) {
                const unsigned long long it = itv[u];
                c1++;
                if (kov[u]) c2++;
                c3 += it;
                c4 += it * it;
                mn = min(mn, (uint32_t)it);
                mx = max(mx, (uint32_t)it);
            }
        }
    }
    // wave reductions first: one LDS atomic per wave and quantity
    for (int o = 32; o > 0; o >>= 1) {
        c1 += __shfl_xor(c1, o);
        c2 += __shfl_xor(c2, o);
        c3 += __shfl_xor(c3, o);
        c4 += __shfl_xor(c4, o);
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_sum[1], c1);
        atomicAdd(&s_sum[2], c2);
        atomicAdd(&s_sum[3], c3);
        atomicAdd(&s_sum[4], c4);
        atomicMin(&s_min, mn);
        atomicMax(&s_max, mx);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        out->frames = n_frames;
        out->sp_ok = s_sum[1];
        out->ldpc_ok = s_sum[2];
        out->sum_iters = s_sum[3];
        out->sum_iters_sq = s_sum[4];
        out->min_iters = s_min;
        out->max_iters = s_max;
    }
}

// counters <- the reduction of F frames' outputs (one launch up to kCountersOneBlock)
static hipError_t launch_counters(const uint32_t* iters, const uint8_t* sp, const uint8_t* ko, size_t n_frames,
                                  qkd_counters* c, hipStream_t stream);

__global__ void counters_init_kernel(qkd_counters* c) {
    c->frames = c->sp_ok = c->ldpc_ok = c->sum_iters = c->sum_iters_sq = 0;
    c->min_iters = 0xffffffffu;
    c->max_iters = 0;
}

static hipError_t launch_counters(const uint32_t* iters, const uint8_t* sp, const uint8_t* ko, size_t n_frames,
                                  qkd_counters* c, hipStream_t stream) {
    if (n_frames <= kCountersOneBlock) {
        hipLaunchKernelGGL(counters_one_kernel, dim3(1), dim3(1024), 0, stream, iters, sp, ko, (uint32_t)n_frames, c);
    } else {
        hipLaunchKernelGGL(counters_init_kernel, dim3(1), dim3(1), 0, stream, c);
        hipLaunchKernelGGL(counters_kernel, dim3((unsigned)((n_frames + 255) / 256)), dim3(256), 0, stream, iters, sp,
                           ko, (uint32_t)n_frames, c);
    }
    return hipGetLastError();
}

// The records of n ranks (one all-gather, qkd_ldpc_amd/dist.py) combined as the
// reference's one-process reduction would see all their frames
// (simulation.cpp:252-312): sums add, extrema take min / max. One wave; every
// record is read before `out` is written, so `out` may alias any of them.
__global__ __launch_bounds__(64) void counters_merge_kernel(const qkd_counters* recs, uint32_t n,
                                                            qkd_counters* out) {
    unsigned long long s[5] = {0, 0, 0, 0, 0};
    uint32_t mn = 0xffffffffu, mx = 0;
    for (uint32_t r = threadIdx.x; r < n; r += 64) {
        const qkd_counters c = recs[r];
        s[0] += c.frames;
        s[1] += c.sp_ok;
        s[2] += c.ldpc_ok;
        s[3] += c.sum_iters;
        s[4] += c.sum_iters_sq;
        mn = min(mn, c.min_iters);
        mx = max(mx, c.max_iters);
    }
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int k = 0; k < 5; ++k) s[k] += __shfl_xor(s[k], o);
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        out->frames = s[0];
        out->sp_ok = s[1];
        out->ldpc_ok = s[2];
        out->sum_iters = s[3];
        out->sum_iters_sq = s[4];
        out->min_iters = mn;
        out->max_iters = mx;
    }
}

// ---- launch plumbing --------------------------------------------------------


// Check-degree buckets: the in-check product reads DC values per lane.
template <int MODE, int RULE, bool CLAMP, bool GT>
static DecodeFn pick_decode_dc(int max_dc, int* dc) {
    if constexpr (GT) {                           // large codes: two buckets
        if (max_dc <= 16) { *dc = 16; return decode_kernel<MODE, RULE, 16, CLAMP, true>; }
        *dc = 64;
        return decode_kernel<MODE, RULE, 64, CLAMP, true>;
    } else {
        if (max_dc <= 4) { *dc = 4; return decode_kernel<MODE, RULE, 4, CLAMP, false>; }
        if (max_dc <= 6) { *dc = 6; return decode_kernel<MODE, RULE, 6, CLAMP, false>; }
        if (max_dc <= 8) { *dc = 8; return decode_kernel<MODE, RULE, 8, CLAMP, false>; }
        if (max_dc <= 16) { *dc = 16; return decode_kernel<MODE, RULE, 16, CLAMP, false>; }
        if constexpr (RULE == kRuleMinSumLds || RULE == kRuleMinSumLdsSc) {   // decode_ms_fits: degree <= 32
            *dc = 32;
            return decode_kernel<MODE, RULE, 32, CLAMP, false>;
        } else {
            *dc = 64;
            return decode_kernel<MODE, RULE, 64, CLAMP, false>;
        }
    }
}

template <int MODE, int RULE, bool GT>
static DecodeFn pick_decode_clamp(bool clamp, int max_dc, int* dc) {
    return clamp ? pick_decode_dc<MODE, RULE, true, GT>(max_dc, dc)
                 : pick_decode_dc<MODE, RULE, false, GT>(max_dc, dc);
}

template <int MODE, bool GT>
static DecodeFn pick_decode_rule(int rule, bool clamp, int max_dc, int* dc) {
    if (rule == kRuleSp32) return pick_decode_clamp<MODE, kRuleSp32, GT>(clamp, max_dc, dc);
    if (rule == kRuleMinSum) return pick_decode_clamp<MODE, kRuleMinSum, GT>(clamp, max_dc, dc);
    if constexpr (!GT)
        if (rule == kRuleMinSumLds) return pick_decode_clamp<MODE, kRuleMinSumLds, false>(clamp, max_dc, dc);
    if constexpr (!GT)
        if (rule == kRuleMinSumLdsSc) return pick_decode_clamp<MODE, kRuleMinSumLdsSc, false>(clamp, max_dc, dc);
    return pick_decode_clamp<MODE, kRuleSp64, GT>(clamp, max_dc, dc);
}

static DecodeFn pick_decode(int mode, int rule, bool clamp, int max_dc, bool gt, int* dc) {
    if (gt)
        return mode == kModeLlr ? pick_decode_rule<kModeLlr, true>(rule, clamp, max_dc, dc)
                                : pick_decode_rule<kModeKeys, true>(rule, clamp, max_dc, dc);
    return mode == kModeLlr ? pick_decode_rule<kModeLlr, false>(rule, clamp, max_dc, dc)
                            : pick_decode_rule<kModeKeys, false>(rule, clamp, max_dc, dc);
}

static int rule_of(uint32_t flags) {
    switch (flags & QKD_VARIANT_MASK) {
        case QKD_VARIANT_SP_F32: return kRuleSp32;
        case QKD_VARIANT_MINSUM: return kRuleMinSum;
        default: return kRuleSp64;
    }
}

static float minsum_scale_of(uint32_t flags) {
    const uint32_t q = (flags >> QKD_MINSUM_SCALE_SHIFT) & 0xffu;
    return q ? (float)q / 256.0f : (float)QKD_MINSUM_DEFAULT_SCALE;
}

static size_t decode_lds_bytes(const qkd_code* c, int dc, int tab2_entries, int rule, bool gt = false,
                               bool sc = false) {
    const int esz = rule == kRuleSp64 ? 8 : 4;
    const bool msl = rule == kRuleMinSumLds || rule == kRuleMinSumLdsSc;
    return DecodeLds(c->n_pad, (c->n + 63) / 64, c->m, dc, tab2_entries, gt ? 0 : esz,
                     msl ? c->m : 0, esz, msl && sc).bytes;
}

static constexpr size_t kLdsBytesMax = 160 * 1024;
// the split decoders' encoded slot words (qkd_decode.h encode_slot): a global
// slot's word, kSlotGlobalBase + offset, must be an LDS address past any
// allocation (its LDS access then reads 0 and drops the store)
static_assert(kLdsBytesMax <= kSlotGlobalBase, "global slot words must lie past the LDS");

static int dc_bucket(int max_dc) {
    return max_dc <= 4 ? 4 : max_dc <= 6 ? 6 : max_dc <= 8 ? 8 : max_dc <= 16 ? 16 : 64;
}

// Totals in LDS unless the code is too long for them (the large-code kernels).
static bool decode_needs_gt(const qkd_code* c, int rule, int tab2_entries) {
    return c->n > kMaxBitsLds || decode_lds_bytes(c, dc_bucket(c->max_dc), tab2_entries, rule) > kLdsBytesMax;
}

// The LDS-resident min-sum needs the check state (sign bits in one word:
// degree <= 32) and all of its LDS in one workgroup.
static bool decode_ms_fits(const qkd_code* c, bool sc) {
    if (c->max_dc > 32 || c->n > kMaxBitsLds) return false;
    const int dc = c->max_dc <= 4 ? 4 : c->max_dc <= 6 ? 6 : c->max_dc <= 8 ? 8 : c->max_dc <= 16 ? 16 : 32;
    return decode_lds_bytes(c, dc, 0, kRuleMinSumLds, false, sc) <= kLdsBytesMax;
}

// Resident workgroups of decode_kernel for this code on its device.
static qkd_status decode_grid(const qkd_code* c, DecodeFn fn, size_t lds, int* grid) {
    QKD_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int per_cu = 0;
    QKD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, kDecodeBlock, lds));
    if (per_cu < 1) return set_error(QKD_ERR_UNSUPPORTED, "decode kernel cannot be resident (LDS %zu B)", lds);
    *grid = per_cu * c->cu_count;
    return QKD_OK;
}

qkd_status ws_reserve_decode(qkd_workspace* ws, size_t slots) {
    const qkd_code* c = ws->code;
    if (!ws->counter) {
        QKD_HIP(hipMalloc(&ws->counter, 128));
        QKD_HIP(hipMemset(ws->counter, 0, 128));
    }
    if (ws->c2b_slots >= slots) return QKD_OK;
    if (ws->c2b) QKD_HIP(hipFree(ws->c2b));
    ws->c2b = nullptr;
    ws->c2b_slots = 0;
    // per slot: the c2b store (max_dv rows) and, at the end, a total row
    // (large codes keep their bit totals there)
    const size_t bytes = slots * ((size_t)c->max_dv + 1) * c->n_pad * sizeof(double);
    if (hipMalloc(&ws->c2b, bytes) != hipSuccess)
        return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate %zu B of c2b scratch", bytes);
    ws->c2b_slots = slots;
    return QKD_OK;
}

qkd_status ws_reserve_keys(qkd_workspace* ws, size_t frames, size_t low_words) {
    const qkd_code* c = ws->code;
    const size_t words = (size_t)(c->n + 63) / 64;
    if (ws->key_frames < frames) {
        if (ws->alice_w) QKD_HIP(hipFree(ws->alice_w));
        if (ws->bob_w) QKD_HIP(hipFree(ws->bob_w));
        if (ws->synw) QKD_HIP(hipFree(ws->synw));
        if (ws->zout) QKD_HIP(hipFree(ws->zout));
        ws->alice_w = ws->bob_w = ws->zout = nullptr;
        ws->synw = nullptr;
        ws->key_frames = 0;
        const size_t syn_words = 2 * (size_t)decode_m_words(c->m);
        if (hipMalloc(&ws->alice_w, frames * words * 8) != hipSuccess ||
            hipMalloc(&ws->bob_w, frames * words * 8) != hipSuccess ||
            hipMalloc(&ws->synw, frames * syn_words * 4) != hipSuccess ||
            hipMalloc(&ws->zout, frames * words * 8) != hipSuccess)
            return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate keys for %zu frames", frames);
        ws->key_frames = frames;
    }
    if (ws->low_words < low_words) {
        if (ws->low) QKD_HIP(hipFree(ws->low));
        ws->low = nullptr;
        ws->low_words = 0;
        if (hipMalloc(&ws->low, low_words * 4) != hipSuccess)
            return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate shuffle scratch");
        ws->low_words = low_words;
    }
    return QKD_OK;
}

static qkd_status ws_free(qkd_workspace* ws) {
    DeviceGuard g(ws->device);
    if (ws->c2b) (void)hipFree(ws->c2b);
    if (ws->counter) (void)hipFree(ws->counter);
    if (ws->alice_w) (void)hipFree(ws->alice_w);
    if (ws->bob_w) (void)hipFree(ws->bob_w);
    if (ws->synw) (void)hipFree(ws->synw);
    if (ws->zout) (void)hipFree(ws->zout);
    if (ws->low) (void)hipFree(ws->low);
    if (ws->ckpt) (void)hipFree(ws->ckpt);
    if (ws->win) (void)hipFree(ws->win);
    if (ws->ilv) (void)hipFree(ws->ilv);
    if (ws->fb_list) (void)hipFree(ws->fb_list);
    if (ws->spec_stat_ev) (void)hipEventSynchronize(ws->spec_stat_ev);
    if (ws->spec_stat_host) (void)hipHostFree(ws->spec_stat_host);
    if (ws->spec_stat_ev) (void)hipEventDestroy(ws->spec_stat_ev);
    if (ws->done) (void)hipEventDestroy(ws->done);
    for (hipEvent_t e : ws->dec_ev) (void)hipEventDestroy(e);
    return QKD_OK;
}

static std::mutex g_default_ws_mu;

qkd_workspace* resolve_ws(const qkd_code* code, qkd_workspace* ws) {
    if (ws) return ws;
    std::lock_guard<std::mutex> lk(g_default_ws_mu);
    if (!code->default_ws) {
        qkd_status s;
        const_cast<qkd_code*>(code)->default_ws = qkd_workspace_create(code, &s);
    }
    return code->default_ws;
}

// Serialise users of one workspace across streams: wait for the previous
// user's completion event, record ours after our launches.
struct WsSession {
    qkd_workspace* ws;
    hipStream_t stream;
    std::unique_lock<std::mutex> lk;
    WsSession(qkd_workspace* w, hipStream_t s) : ws(w), stream(s), lk(w->mu) {
        if (ws->done) (void)hipStreamWaitEvent(stream, ws->done, 0);
    }
    ~WsSession() {
        if (!ws->done) (void)hipEventCreateWithFlags(&ws->done, hipEventDisableTiming);
        if (ws->done) (void)hipEventRecord(ws->done, stream);
    }
};

static unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// qkd_debug_decoder_timing: one event recorded on the launch stream before
// and one after each decoder kernel while timing is on (events pooled per ws;
// at kDecEvPairsMax recorded pairs the finished ones are folded into a running
// total, so the pool stays bounded)
static constexpr size_t kDecEvPairsMax = 256;
static hipError_t decoder_events_fold(qkd_workspace* ws) {
    const size_t pairs = ws->dec_ev_used / 2;
    // summed locally and committed only once every pair has been read: a failure
    // part-way leaves the totals and the pool as they were (a retry folds the
    // same pairs once, not twice)
    double ms_sum = 0.0;
    for (size_t k = 0; k < pairs; ++k) {
        hipError_t r = hipEventSynchronize(ws->dec_ev[2 * k + 1]);
        float ms = 0.0f;
        if (r == hipSuccess) r = hipEventElapsedTime(&ms, ws->dec_ev[2 * k], ws->dec_ev[2 * k + 1]);
        if (r != hipSuccess) return r;
        ms_sum += ms;
    }
    ws->dec_ms_folded += ms_sum;
    ws->dec_pairs_folded += pairs;
    ws->dec_ev_used = 0;
    return hipSuccess;
}
// the start event of a launch (stop: decoder_event_close)
static hipError_t decoder_event(qkd_workspace* ws, hipStream_t stream) {
    if (!ws->time_decoder) return hipSuccess;
    if (ws->dec_ev_used >= 2 * kDecEvPairsMax) {
        const hipError_t r = decoder_events_fold(ws);
        if (r != hipSuccess) return r;
    }
    while (ws->dec_ev.size() < ws->dec_ev_used + 2) {
        hipEvent_t e = nullptr;
        const hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        ws->dec_ev.push_back(e);
    }
    const hipError_t r = hipEventRecord(ws->dec_ev[ws->dec_ev_used], stream);
    if (r == hipSuccess) ws->dec_ev_used++;
    return r;
}
// after the launch: its stop event, or, when the launch (`launch`) or the
// record failed, the start event taken back, so pairs stay (start, stop)
static hipError_t decoder_event_close(qkd_workspace* ws, hipStream_t stream, hipError_t launch) {
    if (!ws->time_decoder) return launch;
    hipError_t r = launch;
    if (r == hipSuccess) r = hipEventRecord(ws->dec_ev[ws->dec_ev_used], stream);
    if (r == hipSuccess) ws->dec_ev_used++;
    else ws->dec_ev_used--;
    return r;
}

// DeviceCode::plan_slot encoded for a split-kernel layout and check-degree
// bucket: slot words by encode_slot (binary64 slots), segment words by
// encode_seg; built on a layout's first launch and kept with the code
// esz 4 (the binary32 min-sum rules, every slot in LDS): the slot word is
// the slot's LDS byte address itself (no kSlotLds tag, no global form)
static qkd_status plan_for_layout(const qkd_code* c, const SplitLds& L, int dc, const uint2** out, int esz = 8) {
    std::lock_guard<std::mutex> lock(c->plan_mu);
    const auto key = std::make_pair(L.S, ((uint32_t)L.msg << 8) | (uint32_t)dc | (esz == 4 ? 0x80u : 0u));
    auto it = c->d_plan_enc.find(key);
    if (it == c->d_plan_enc.end()) {
        std::vector<uint2> enc(c->plan_slot_host);
        for (size_t k = 0; k < enc.size(); ++k) {
            uint2& w = enc[k];
            w.x = esz == 4 ? (uint32_t)L.msg + w.x * 4u : encode_slot(w.x, L.S, (uint32_t)L.msg, (uint32_t)sizeof(double));
            w.y = encode_seg(w.y & qkdp::kPlanChkMask, (w.y >> 20) & 63u, (w.y >> 26) + 1, (uint32_t)(k & 63),
                             (uint32_t)dc);
        }
        uint2* d = nullptr;
        if (hipMalloc(&d, enc.size() * sizeof(uint2)) != hipSuccess)
            return set_error(QKD_ERR_OUT_OF_MEMORY, "code: cannot allocate %zu B for an encoded plan",
                             enc.size() * sizeof(uint2));
        if (hipMemcpy(d, enc.data(), enc.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return set_error(QKD_ERR_DEVICE, "code: encoded plan upload failed");
        }
        it = c->d_plan_enc.emplace(key, d).first;
    }
    *out = it->second;
    return QKD_OK;
}

// The split kernels' encoded slot words are absolute LDS addresses: their
// dynamic LDS must start at address 0, i.e. no static LDS (checked once per
// kernel).
static qkd_status check_no_static_lds(DecodeFn fn) {
    static std::mutex mu;
    static std::map<const void*, size_t> seen;
    std::lock_guard<std::mutex> lock(mu);
    auto it = seen.find((const void*)fn);
    if (it == seen.end()) {
        hipFuncAttributes fa{};
        QKD_HIP(hipFuncGetAttributes(&fa, (const void*)fn));
        it = seen.emplace((const void*)fn, fa.sharedSizeBytes).first;
    }
    if (it->second != 0)
        return set_error(QKD_ERR_UNSUPPORTED, "split decoder with %zu B of static LDS (its slot words "
                                              "address LDS from 0)", it->second);
    return QKD_OK;
}

static qkd_status launch_decode(const qkd_code* c, qkd_workspace* ws, DecodeArgs& a, int mode,
                                uint32_t flags, hipStream_t stream) {
    int dc = 0;
    int rule = rule_of(flags);
    // QKD_MINSUM_STORE=global keeps the global-message-store min-sum (tests)
    // (QKD_MINSUM_STORE=lds keeps the LDS-state kernel: tests)
    const DbgOpt ms_store = debug_option(ws, "QKD_MINSUM_STORE");
    const bool ms_global = ms_store.is("global");
    const bool ms_lds = ms_store.is("lds");
    a.ms_sc = (flags & QKD_MINSUM_SELF_CORRECT) ? 1 : 0;
    const bool classic = debug_option(ws, "QKD_DECODE_KERNEL").is("classic");
    // min-sum: the split skeleton (every binary32 slot in LDS, the binary32
    // rule's bit phase over DeviceCode::bit_code) when it applies, else the
    // LDS-state kernel, else the global message store
    if (rule == kRuleMinSum && !ms_global && !ms_lds && !classic && !a.trace && c->d_bit_code &&
        c->n <= kMaxBitsSplit && c->m <= kMaxChecksSplit && c->max_dc <= 8) {
        // (check degree <= 8: the additive mask table, seg_weight_entries)
        const SplitLds Lm(c->n_pad, (c->n + 63) / 64, c->m, c->max_dv, c->max_dc <= 4 ? 4 : c->max_dc <= 6 ? 6 : 8,
                          0, a.ms_sc ? 2 * c->n_tasks + (c->n + 63) / 64 : 0, 4, kLdsBytesMax);
        if (Lm.S >= (uint32_t)((size_t)c->max_dv * c->n_pad) && Lm.bytes <= kLdsBytesMax)
            rule = a.ms_sc ? kRuleMinSumSplitSc : kRuleMinSumSplit;
    }
    if (rule == kRuleMinSum && !ms_global && decode_ms_fits(c, a.ms_sc != 0)) rule = kRuleMinSumLds;
    if (a.ms_sc && rule != kRuleMinSumLds && rule != kRuleMinSumSplitSc)
        return set_error(QKD_ERR_UNSUPPORTED, "self-corrected min-sum needs the split or the LDS-state min-sum "
                                              "kernel (check degree <= 32, its state in LDS)");
    if (a.ms_sc && rule == kRuleMinSumLds) rule = kRuleMinSumLdsSc;
    a.ms_scale = minsum_scale_of(flags);
    a.ms_offset = (float)((flags >> QKD_MINSUM_OFFSET_SHIFT) & 0xffu) / 64.0f;
    // The split-store kernel (decode_split.hip) for the sum-product rules
    // whenever its LDS layout fits; QKD_DECODE_KERNEL=classic keeps
    // decode_kernel (A/B measurements, tests). Trace mode records the classic
    // kernel's store.
    const bool msr = rule == kRuleMinSumSplit || rule == kRuleMinSumSplitSc;
    // codes past kMaxBitsSplit (up to kMaxBitsSplitLong): only the
    // frame-interleaved decoder and its exact hand-off kernel (LONG) take
    // them, on the keys path with the split view's arrays; otherwise the
    // classic kernel below
    const bool long_code = c->n > kMaxBitsSplit;
    const bool long_ok = rule == kRuleSp64 && mode == kModeKeys && c->n <= kMaxBitsSplitLong && c->d_ilv_slots &&
                         c->max_dc <= 16;
    if ((rule == kRuleSp64 || rule == kRuleSp32 || msr) && !classic && !a.trace && (!long_code || long_ok) &&
        c->m <= kMaxChecksSplit) {
        // (a long code falls back to the classic kernel with the arguments as given)
        const DecodeArgs a_in = a;
        int sdc = 0;
        DecodeFn sfn = long_code ? pick_split_long(a.clamp_on != 0, c->max_dc, &sdc)
                                 : pick_split_decode(mode, rule, a.clamp_on != 0, c->max_dc, &sdc);
        const int esz = rule == kRuleSp64 ? 8 : 4;
        // diagnostic: QKD_SPLIT_BUDGET lowers the LDS budget (fewer LDS slots)
        size_t budget = kLdsBytesMax;
        if (const DbgOpt b = debug_option(ws, "QKD_SPLIT_BUDGET")) budget = std::min(budget, (size_t)b.as_long());
        // the speculative kernel (interval iterations, qkd_spec.h, exact
        // replays in place) when it applies: QKD path with the folded first
        // iteration, binary64 rule, clamped messages, bit degree <= kDvUnroll
        // (the QKD path needs its folded first iteration; the LLR path starts from the LLRs)
        const bool spec = rule == kRuleSp64 && a.spec_cap > 0 && a.clamp_on &&
                          (mode == kModeLlr || a.first_table) && c->max_dv <= kDvUnroll && c->d_bit_code;
        const bool ckpt = spec && mode == kModeKeys && a.ckpt_unsat > 0;
        // its folded first iteration from a table (decode_split.hip fold_table_fill)
        // (at most kFoldTabMaxEntries: the table's LDS comes off the message slots)
        a.ftab_entries = (spec && !ckpt && mode == kModeKeys && a.tab2_entries &&
                          c->n_pat * kFoldTabPat <= kFoldTabMaxEntries)
                             ? c->n_pat * kFoldTabPat : 0;
        // (QKD_FOLD_TABLE=0: the per-bit form; tests compare the two)
        if (const DbgOpt e = debug_option(ws, "QKD_FOLD_TABLE")) if (e.as_int() == 0) a.ftab_entries = 0;
        if (debug_option(ws, "QKD_SPEC_POLICY").is("always")) a.spec_always = 1u;
        // (self-corrected min-sum: its previous-b2c ballot words and the
        // frame's Bob words in the ftab region)
        if (rule == kRuleMinSumSplitSc) a.ftab_entries = 2 * c->n_tasks + (c->n + 63) / 64;
        // (the long-code hand-off kernel: the frame's Bob words there)
        if (long_code) a.ftab_entries = std::max(a.ftab_entries, (c->n + 63) / 64);
        const SplitLds L(c->n_pad, (c->n + 63) / 64, c->m, c->max_dv, sdc, a.tab2_entries, a.ftab_entries, esz,
                         budget);
        // (the binary32 rule's kernel keeps every slot in LDS: SplitStore<float, true>)
        // (binary64: any share of the slots in LDS, the rest in the
        // workgroup's global region; long codes keep most of them there)
        const bool fits = rule != kRuleSp64 ? L.S >= (uint32_t)((size_t)c->max_dv * c->n_pad) : L.S >= 64;
        if (L.bytes <= kLdsBytesMax && fits) {
            int grid = 0;
            qkd_status s = decode_grid(c, sfn, L.bytes, &grid);
            if (s != QKD_OK) return s;
            grid = (int)std::min<size_t>((size_t)grid, a.n_frames);
            if (const DbgOpt g = debug_option(ws, "QKD_DECODE_GRID")) grid = std::max(1, std::min(grid, g.as_int()));
            s = ws_reserve_decode(ws, (size_t)grid);
            if (s != QKD_OK) return s;
            a.code = c->view_split();     // the internal bit order (host.cpp build_code)
            a.c2b = ws->c2b;
            a.plan_enc = nullptr;
            if (rule == kRuleSp64 || msr) {
                s = plan_for_layout(c, L, sdc, &a.plan_enc, esz);
                if (s != QKD_OK) return s;
            }
            const size_t slots = (size_t)c->max_dv * c->n_pad;
            // elements of the message type, plus kC2bPad: the workgroups' regions
            // start off a common alignment (measured: config 2 with the fold table
            // has a region of 13184 slots, 4 % slower than 13248;
            // QKD_C2B_PAD overrides the pad)
            // Default: the region rounded up to an ODD multiple of kC2bPad
            // slots (512 bytes), so consecutive regions never share an
            // alignment above 512 bytes (13248 = 207 x 64 is the measured
            // good case above); QKD_C2B_PAD adds a fixed pad instead.
            if (const DbgOpt e = debug_option(ws, "QKD_C2B_PAD")) {
                const size_t pad = std::min((size_t)e.as_long(), (size_t)c->n_pad);
                a.c2b_stride = ((slots - L.S + 31) & ~(size_t)31) + pad;
            } else {
                size_t st = (slots - L.S + kC2bPad - 1) / kC2bPad;
                if ((st & 1u) == 0) st++;
                a.c2b_stride = st * kC2bPad;
            }
            // an encoded global slot word (kSlotGlobalBase + byte offset) must
            // stay below kSlotLds, the LDS words' tag bit
            if (rule == kRuleSp64 && kSlotGlobalBase + a.c2b_stride * sizeof(double) >= kSlotLds)
                return set_error(QKD_ERR_UNSUPPORTED, "code too large for the split decoder's slot words "
                                                      "(%zu global slots per frame)", a.c2b_stride);
            a.lds_budget = (uint32_t)budget;
            a.counter = ws->counter;
            const bool timing = (bool)debug_option(ws, "QKD_PHASE_TIMING");
            a.phase = nullptr;
            if (timing) {
                a.phase = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws->counter) + 64);
                QKD_HIP(hipMemsetAsync(a.phase, 0, 64, stream));
            }
            a.replay_count = ws->counter + 1;
            a.spec_replays = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws->counter) + 120);
            if (spec) {
                // (a long code: the interleaved decoder speculates; no split speculation)
                if (!long_code) {
                    int xdc = 0, sgrid = 0;
                    DecodeFn xfn = pick_split_spec(mode, c->max_dc, ckpt, &xdc);
                    if (xdc != sdc)      // (the layout and the encoded plan are the bucket's)
                        return set_error(QKD_ERR_UNSUPPORTED, "speculative kernel bucket %d != %d", xdc, sdc);
                    s = decode_grid(c, xfn, L.bytes, &sgrid);
                    if (s != QKD_OK) return s;
                    sfn = xfn;
                    grid = std::min(sgrid, grid);
                }
                if (ckpt && !long_code) {
                    // one saved message store per resident workgroup
                    const size_t need = (size_t)grid * slots;
                    if (ws->ckpt_slots < need) {
                        if (ws->ckpt) QKD_HIP(hipFree(ws->ckpt));
                        ws->ckpt = nullptr;
                        ws->ckpt_slots = 0;
                        if (hipMalloc(&ws->ckpt, need * sizeof(double)) != hipSuccess)
                            return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate %zu B of checkpoints",
                                             need * sizeof(double));
                        ws->ckpt_slots = need;
                    }
                    a.ckpt = ws->ckpt;
                    a.ckpt_stride = (uint32_t)slots;
                }
            }
            a.win = nullptr;
            a.win_count = 0;
            if (spec) {
                // the in-launch policy's windows (zeroed below with the queue)
                a.win_shift = kSpecWinShift;
                a.win_lag = kSpecWinLag;
                a.win_count = (uint32_t)((a.n_frames + (1u << kSpecWinShift) - 1) >> kSpecWinShift);
                const size_t need = 2 * (size_t)a.win_count;
                if (ws->win_words < need) {
                    if (ws->win) QKD_HIP(hipFree(ws->win));
                    ws->win = nullptr;
                    ws->win_words = 0;
                    if (hipMalloc(&ws->win, need * sizeof(uint32_t)) != hipSuccess)
                        return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate the policy windows");
                    ws->win_words = need;
                }
                a.win = ws->win;
            }
            if (rule == kRuleSp64 || msr) {
                s = check_no_static_lds(sfn);
                if (s != QKD_OK) return s;
            }
            // Long codes (the split store keeps under a quarter of the slots
            // in LDS): the frame-interleaved decoder (decode_ilv.hip), its
            // hand-offs decoded by this split kernel from a frame list.
            // QKD_ILV=1 / 0 forces it on / off (tests, A/B).
            // (the target syndrome words in LDS when the three arrays fit, else
            // in global memory: measured 30 % slower at N = 40,000, where
            // they fit, and twice as fast as the split kernel at 60,000)
            // (then also the uncertainty words, for M past ~37,000)
            const bool tsg = IlvLds(c->m, false).bytes > kLdsBytesMax;
            const bool ug = tsg && IlvLds(c->m, true).bytes > kLdsBytesMax;
            const IlvLds IL(c->m, tsg, ug);
            bool ilv = mode == kModeKeys && spec && !ckpt && !a.bits_out && a.first_table && c->d_ilv_slots &&
                       IL.bytes <= kLdsBytesMax;
            bool ilv_forced = false;
            if (ilv) {
                const DbgOpt ie = debug_option(ws, "QKD_ILV");
                ilv_forced = (bool)ie;
                ilv = ie ? ie.as_int() != 0
                         : (size_t)L.S * 4 < slots && (size_t)a.n_frames * 2 >= (size_t)kIlvCols * c->cu_count;
            }
            DecodeFn ifn = nullptr;
            int igrid = 0;
            // (per workgroup: the message lines, the columns' key words, their
            // target syndrome words: (M + 1) / 2 words, in doubles)
            // rounded to 512 bytes: every workgroup's lines start on a cache
            // line (an unaligned stride splits each line access in two)
            // (and, ug, their uncertainty words as many again)
            const size_t istride = (slots * kIlvCols + (size_t)((c->n + 63) / 64) * kIlvCols * 2 +
                                    (ug ? 2 : 1) * (((size_t)(c->m + 1) / 2 + 1) / 2) + 63) & ~(size_t)63;
            if (ilv) {
                ifn = pick_ilv(c->ilv_rs, c->max_dc, tsg, ug);
                QKD_HIP(hipFuncSetAttribute((const void*)ifn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)IL.bytes));
                int per_cu = 0;
                QKD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)ifn, kIlvBlock, IL.bytes));
                if (per_cu < 1) return set_error(QKD_ERR_UNSUPPORTED, "interleaved decoder cannot be resident");
                igrid = per_cu * c->cu_count;
                igrid = (int)std::min<size_t>((size_t)igrid, ((size_t)a.n_frames + kIlvCols - 1) / kIlvCols);
                // (QKD_ILV_GRID caps the workgroups: tests take columns through several frames)
                if (const DbgOpt g = debug_option(ws, "QKD_ILV_GRID")) igrid = std::max(1, std::min(igrid, g.as_int()));
                const size_t need = (size_t)igrid * istride;
                if (ws->ilv_elems < need) {
                    if (ws->ilv) QKD_HIP(hipFree(ws->ilv));
                    ws->ilv = nullptr;
                    ws->ilv_elems = 0;
                    if (hipMalloc(&ws->ilv, need * sizeof(double)) != hipSuccess) {
                        // (one message region per resident workgroup: ~6 GB at N
                        // = 60,000. Unless forced, the split kernel, which needs
                        // far less, decodes the batch instead)
                        (void)hipGetLastError();
                        if (ilv_forced)
                            return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate %zu B of "
                                                                    "interleaved message lines", need * sizeof(double));
                        ilv = false;
                    } else {
                        ws->ilv_elems = need;
                    }
                }
            }
            // (a long code the interleaved decoder does not take: the classic kernel)
            if (long_code && !ilv) {
                a = a_in;
                goto classic_path;
            }
            if (ilv) {
                if (ws->fb_frames < a.n_frames) {
                    if (ws->fb_list) QKD_HIP(hipFree(ws->fb_list));
                    ws->fb_list = nullptr;
                    ws->fb_frames = 0;
                    if (hipMalloc(&ws->fb_list, (size_t)a.n_frames * sizeof(uint32_t)) != hipSuccess)
                        return set_error(QKD_ERR_OUT_OF_MEMORY, "workspace: cannot allocate the hand-off list");
                    ws->fb_frames = a.n_frames;
                }
            }
            // [0] frame queue, [1] replays: zeroed by frame_syn_kernel on the
            // keys path (it runs first on this stream: block 0 writes both
            // words), by a memset otherwise -- one branch, so a keys-mode
            // launch without frame_syn cannot exist. Every check that can fail
            // comes before it: frame_syn rewrites ws->alice_w / bob_w in place
            // in the internal bit order, and after it only the decoder (which
            // reads them in that order) may follow.
            if (mode == kModeKeys) {
                a.synw = ws->synw;
                a.zout = ws->zout;
                QKD_HIP(launch_frame_syn(a, stream, debug_option(ws, "QKD_SYN_SLICED").is("0"),
                                         debug_option(ws, "QKD_SYN_BYTES").is("0")));
            } else {
                QKD_HIP(hipMemsetAsync(ws->counter, 0, 8, stream));
                if (a.win) QKD_HIP(hipMemsetAsync(a.win, 0, 2 * (size_t)a.win_count * sizeof(uint32_t), stream));
            }
            QKD_HIP(decoder_event(ws, stream));
            if (ilv) {
                // [2] the hand-off queue, [3] the hand-off count
                QKD_HIP(hipMemsetAsync(ws->counter + 2, 0, 8, stream));
                DecodeArgs ai = a;
                ai.ilv_store = ws->ilv;
                ai.ilv_stride = istride;
                ai.fb_list = ws->fb_list;
                ai.fb_count = ws->counter + 3;
                hipLaunchKernelGGL(ifn, dim3(igrid), dim3(kIlvBlock), IL.bytes, stream, ai);
                // the hand-offs: the split kernel's exact iterations (their
                // intervals could not certify; speculating again measured 1.7x
                // slower), through the frame list
                DecodeArgs af = a;
                af.counter = ws->counter + 2;
                af.frame_list = ws->fb_list;
                af.frame_count = ws->counter + 3;
                af.spec_cap = 0;
                af.spec_always = 1;
                af.phase = nullptr;       // (QKD_PHASE_TIMING: the interleaved kernel's phases)
                int xdc = 0;
                DecodeFn ffn = long_code ? pick_split_long(a.clamp_on != 0, c->max_dc, &xdc)
                                         : pick_split_decode(mode, rule, a.clamp_on != 0, c->max_dc, &xdc);
                if (xdc != sdc)
                    return set_error(QKD_ERR_UNSUPPORTED, "exact split kernel bucket %d != %d", xdc, sdc);
                // (the interleaved launch's error is read once and carried to
                // decoder_event_close: a failed launch skips the hand-offs and
                // fails the call instead of leaving stale outputs)
                hipError_t le = hipGetLastError();
                if (le == hipSuccess) {
                    hipLaunchKernelGGL(ffn, dim3(grid), dim3(kDecodeBlock), L.bytes, stream, af);
                    le = hipGetLastError();
                }
                QKD_HIP(decoder_event_close(ws, stream, le));
            } else {
                hipLaunchKernelGGL(sfn, dim3(grid), dim3(kDecodeBlock), L.bytes, stream, a);
                QKD_HIP(decoder_event_close(ws, stream, hipGetLastError()));
            }
            if (mode == kModeKeys) QKD_HIP(launch_key_match(a, stream));
            return QKD_OK;
        }
    }
classic_path:
    const bool gt = decode_needs_gt(c, rule, a.tab2_entries);
    if (gt) {                                     // large code: no per-bit LDS tables
        a.first_table = 0;
        a.tab2_entries = 0;
    }
    DecodeFn fn = pick_decode(mode, rule, a.clamp_on != 0, c->max_dc, gt, &dc);
    const size_t lds = decode_lds_bytes(c, dc, a.tab2_entries, rule, gt, a.ms_sc != 0);
    int grid = 0;
    qkd_status s = decode_grid(c, fn, lds, &grid);
    if (s != QKD_OK) return s;
    grid = (int)std::min<size_t>((size_t)grid, a.n_frames);
    // diagnostic: QKD_DECODE_GRID caps the resident workgroups (frames in flight)
    if (const DbgOpt g = debug_option(ws, "QKD_DECODE_GRID")) grid = std::max(1, std::min(grid, g.as_int()));
    s = ws_reserve_decode(ws, (rule == kRuleMinSumLds || rule == kRuleMinSumLdsSc) ? 0 : (size_t)grid);   // no global messages
    if (s != QKD_OK) return s;
    a.code = c->view();
    // (byte keys: the classic kernel reads them packed, in the original order)
    if (mode == kModeKeys && a.alice_b) QKD_HIP(launch_pack_keys(a, stream));
    a.c2b = ws->c2b;
    a.c2b_stride = (size_t)c->max_dv * c->n_pad;
    // the workspace holds one total row per slot after all the message stores
    a.totals = gt ? ws->c2b + ws->c2b_slots * a.c2b_stride : nullptr;
    a.totals_stride = c->n_pad;
    a.counter = ws->counter;
    QKD_HIP(hipMemsetAsync(ws->counter, 0, 4, stream));
    const bool timing = (bool)debug_option(ws, "QKD_PHASE_TIMING");
    a.phase = nullptr;
    if (timing) {
        a.phase = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws->counter) + 64);
        QKD_HIP(hipMemsetAsync(a.phase, 0, 64, stream));
    }
    QKD_HIP(decoder_event(ws, stream));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kDecodeBlock), lds, stream, a);
    QKD_HIP(decoder_event_close(ws, stream, hipGetLastError()));
    return QKD_OK;
}

static qkd_status check_frames(size_t n_frames) {
    if (n_frames == 0) return set_error(QKD_ERR_INVALID_ARG, "n_frames must be > 0");
    if (n_frames > 0xffffffffull) return set_error(QKD_ERR_INVALID_ARG, "n_frames too large");
    return QKD_OK;
}

static qkd_status check_decode_params(uint32_t max_it, double thr, uint32_t flags) {
    if (max_it < 1) return set_error(QKD_ERR_INVALID_ARG, "max_iterations must be >= 1");
    const uint32_t known = QKD_FLAG_THRESHOLD | QKD_VARIANT_MASK | (0xffu << QKD_MINSUM_SCALE_SHIFT) |
                           (0xffu << QKD_MINSUM_OFFSET_SHIFT) | QKD_MINSUM_SELF_CORRECT;
    if (flags & ~known) return set_error(QKD_ERR_INVALID_ARG, "unknown flags 0x%x", flags);
    if ((flags & QKD_VARIANT_MASK) == QKD_VARIANT_MASK)
        return set_error(QKD_ERR_INVALID_ARG, "unknown decoder variant 0x%x", flags & QKD_VARIANT_MASK);
    if ((flags >> QKD_MINSUM_SCALE_SHIFT) && (flags & QKD_VARIANT_MASK) != QKD_VARIANT_MINSUM)
        return set_error(QKD_ERR_INVALID_ARG, "min-sum scale or offset given without QKD_VARIANT_MINSUM");
    if ((flags & QKD_FLAG_THRESHOLD) && !(thr > 0.0))
        return set_error(QKD_ERR_INVALID_ARG, "message threshold must be > 0");
    return QKD_OK;
}


}  // namespace qkd

using namespace qkd;

extern "C" {

qkd_workspace* qkd_workspace_create(const qkd_code* code, qkd_status* status) {
    if (!code) {
        if (status) *status = set_error(QKD_ERR_INVALID_ARG, "null code");
        return nullptr;
    }
    qkd_workspace* ws = new (std::nothrow) qkd_workspace();
    if (!ws) {
        if (status) *status = set_error(QKD_ERR_OUT_OF_MEMORY, "out of host memory");
        return nullptr;
    }
    ws->code = code;
    ws->device = code->device;
    if (status) *status = QKD_OK;
    return ws;
}

void qkd_workspace_destroy(qkd_workspace* ws) {
    if (!ws) return;
    ws_free(ws);
    delete ws;
}

qkd_status qkd_syndrome_batch(const qkd_code* c, const uint8_t* bits, size_t n_frames, uint8_t* syn,
                              void* stream) {
    clear_error();
    if (!c || !bits || !syn) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s != QKD_OK) return s;
    DeviceGuard g(c->device);
    const size_t total = n_frames * (size_t)c->m;
    hipLaunchKernelGGL(syndrome_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       c->view(), bits, (uint32_t)n_frames, syn);
    QKD_HIP(hipGetLastError());
    return QKD_OK;
}

// binary32 bound of a binary64 value: the largest float <= x (up: smallest >= x)
static float f32_bound(double x, bool up) {
    float f = (float)x;
    if (up && (double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    if (!up && (double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}

qkd_status qkd_decode_batch(const qkd_code* c, qkd_workspace* ws, const double* llr,
                            const uint8_t* syndrome, size_t n_frames, uint32_t max_iterations,
                            double msg_threshold, uint32_t flags, uint8_t* bits_out,
                            uint32_t* iterations, uint8_t* syndromes_match, void* stream) {
    clear_error();
    if (!c || !llr || !syndrome || !iterations || !syndromes_match)
        return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s == QKD_OK) s = check_decode_params(max_iterations, msg_threshold, flags);
    if (s != QKD_OK) return s;
    DeviceGuard g(c->device);
    ws = resolve_ws(c, ws);
    if (!ws) return set_error(QKD_ERR_OUT_OF_MEMORY, "no workspace");
    WsSession sess(ws, (hipStream_t)stream);
    DecodeArgs a{};
    a.pinf = std::numeric_limits<float>::infinity();
    a.n_frames = (uint32_t)n_frames;
    a.max_it = max_iterations;
    a.thr = msg_threshold;
    a.clamp_on = (flags & QKD_FLAG_THRESHOLD) ? 1 : 0;
    a.llr = llr;
    a.syn = syndrome;
    a.bits_out = bits_out;
    a.iters = iterations;
    a.sp_ok = syndromes_match;
    // speculative interval iterations (decode_split.hip, qkd_spec.h): binary64
    // rule with clamped messages; QKD_SPEC_CAP overrides how many (0: off)
    int cap = kSpecCapDefault;
    if (const DbgOpt e = debug_option(ws, "QKD_SPEC_CAP")) cap = std::max(0, e.as_int());
    a.spec_cap = (rule_of(flags) == kRuleSp64 && a.clamp_on) ? (uint32_t)cap : 0u;
    a.thr_dn = f32_bound(msg_threshold, false);
    a.thr_up = f32_bound(msg_threshold, true);
    return launch_decode(c, ws, a, kModeLlr, flags, (hipStream_t)stream);
}


// The speculation policy's per-QBER record (qkd_workspace::spec_clean). The
// map is bounded: a workspace fed ever new QBERs (a continuous-q pipeline, a
// sweep) forgets the records once there are kSpecCleanMax of them, which only
// resamples those QBERs' replay fractions.
static constexpr size_t kSpecCleanMax = 64;
static SpecClean& spec_clean_of(qkd_workspace* ws, double q) {
    if (ws->spec_clean.size() >= kSpecCleanMax && !ws->spec_clean.count(q)) ws->spec_clean.clear();
    return ws->spec_clean[q];
}

// Shared by qkd_qkd_ldpc_batch and qkd_trials_batch: keys already packed in ws.
static qkd_status decode_keys(const qkd_code* c, qkd_workspace* ws, size_t n_frames, double q,
                              uint32_t max_it, double thr, uint32_t flags, uint8_t* bits_out,
                              uint32_t* iters, uint8_t* sp_ok, uint8_t* key_ok, hipStream_t stream,
                              const uint8_t* alice_b = nullptr, const uint8_t* bob_b = nullptr) {
    DecodeArgs a{};
    a.alice_b = alice_b;
    a.bob_b = bob_b;
    a.pinf = std::numeric_limits<float>::infinity();
    a.n_frames = (uint32_t)n_frames;
    a.max_it = max_it;
    a.thr = thr;
    a.clamp_on = (flags & QKD_FLAG_THRESHOLD) ? 1 : 0;
    a.alice_w = ws->alice_w;
    a.bob_w = ws->bob_w;
    a.words = (uint32_t)((c->n + 63) / 64);
    a.log_p = std::log((1. - q) / q);          // host glibc log, qkd_ldpc_algorithm.cpp:400
    // first-iteration message magnitudes by check degree (first_check_phase)
    // (the binary32 rule folds on the device, decode_split_kernel; not at
    // log_p = 0, where Bob's 1 bits give -0.0, not negative)
    // (min-sum folds on the device too, decode_split_kernel)
    a.first_table = (c->max_dc <= kFirstTableDeg &&
                     (rule_of(flags) == kRuleSp64 ||
                      ((rule_of(flags) == kRuleSp32 || rule_of(flags) == kRuleMinSum) && a.log_p != 0.0)))
                        ? 1 : 0;
    if (a.first_table) {
        const double T = std::fabs(qkdm::tanh_flat(a.log_p / 2.0));
        double M = 1.0;
        a.first_c2b[0] = 0.0;
        for (int d = 1; d <= kFirstTableDeg; ++d) {
            M = M * T;
            double v = 2.0 * qkdm::atanh_flat(M / T);
            if (a.clamp_on) v = v > thr ? thr : (v < -thr ? -thr : v);
            a.first_c2b[d] = v;
        }
    }
    a.tab2_entries = (a.first_table && c->n_pat > 0 && rule_of(flags) == kRuleSp64)
                         ? c->n_pat * tab2_stride(c->max_dv) : 0;
    // speculative interval iterations (decode_split.hip, qkd_spec.h) ahead of
    // the exact ones, for the binary64 rule with clamped messages;
    // QKD_SPEC_CAP overrides how many (0: off)
    int cap = kSpecCapDefault;
    if (const DbgOpt e = debug_option(ws, "QKD_SPEC_CAP")) cap = std::max(0, e.as_int());
    a.spec_cap = (rule_of(flags) == kRuleSp64 && a.clamp_on && a.first_table) ? (uint32_t)cap : 0u;
    a.lp_dn = f32_bound(a.log_p, false);
    a.lp_up = f32_bound(a.log_p, true);
    a.thr_dn = f32_bound(thr, false);
    a.thr_up = f32_bound(thr, true);
    a.bits_out = bits_out;
    a.iters = iters;
    a.sp_ok = sp_ok;
    a.key_ok = key_ok;
    // across calls: the last speculative call's replay fraction, once its
    // count is back (never waits); above kSpecCkptSwitch the frames speculate
    // from a checkpoint instead, from that QBER up
    if (ws->spec_stat_pending && hipEventQuery(ws->spec_stat_ev) == hipSuccess) {
        ws->spec_stat_pending = false;
        const bool over = (double)*ws->spec_stat_host > kSpecCkptSwitch * (double)ws->spec_stat_frames;
        if (over) ws->spec_ckpt_q = std::min(ws->spec_ckpt_q, ws->spec_stat_q);
        SpecClean& sc = spec_clean_of(ws, ws->spec_stat_q);
        sc.clean = over ? 0 : sc.clean + 1;
    }
    // at and above that QBER: the checkpointed speculation (QKD_CKPT_UNSAT
    // overrides its trigger; 0: exact iterations only)
    a.ckpt = nullptr;
    a.ckpt_stride = 0;
    a.ckpt_unsat = 0;
    // (QKD_SPEC_CKPT=1: the checkpointed variant at every QBER; tests)
    const DbgOpt force_ck = debug_option(ws, "QKD_SPEC_CKPT");
    if (q >= ws->spec_ckpt_q || (force_ck && force_ck.as_int() == 1)) {
        int cu = kCkptUnsatDefault;
        if (const DbgOpt e = debug_option(ws, "QKD_CKPT_UNSAT")) cu = std::max(0, e.as_int());
        a.ckpt_unsat = (uint32_t)cu;
        if (cu == 0) a.spec_cap = 0;
    }
    qkd_status st = launch_decode(c, ws, a, kModeKeys, flags, stream);
    if (st != QKD_OK || a.spec_cap == 0 || a.ckpt_unsat || ws->spec_stat_pending) return st;
    // (a QBER whose last two samples stayed under the switch is sampled again
    // only every kSpecStatEvery calls: each sample is a device-to-host copy
    // and an event on the caller's stream)
    {
        SpecClean& sc = spec_clean_of(ws, q);
        if (sc.clean >= 2 && (++sc.skip % kSpecStatEvery) != 0) return st;
    }
    if (!ws->spec_stat_host) {
        if (hipHostMalloc(reinterpret_cast<void**>(&ws->spec_stat_host), 8, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ws->spec_stat_ev, hipEventDisableTiming) != hipSuccess)
            return QKD_OK;                        // no policy feedback, decoding is unaffected
    }
    if (hipMemcpyAsync(ws->spec_stat_host, ws->counter + 1, 4, hipMemcpyDeviceToHost, stream) == hipSuccess &&
        hipEventRecord(ws->spec_stat_ev, stream) == hipSuccess) {
        ws->spec_stat_pending = true;
        ws->spec_stat_q = q;
        ws->spec_stat_frames = n_frames;
    }
    return QKD_OK;
}

qkd_status qkd_qkd_ldpc_batch(const qkd_code* c, qkd_workspace* ws, const uint8_t* alice,
                              const uint8_t* bob, size_t n_frames, double qber, uint32_t max_iterations,
                              double msg_threshold, uint32_t flags, uint8_t* bits_out,
                              uint32_t* iterations, uint8_t* syndromes_match, uint8_t* keys_match,
                              void* stream) {
    clear_error();
    if (!c || !alice || !bob || !iterations || !syndromes_match)
        return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s == QKD_OK) s = check_decode_params(max_iterations, msg_threshold, flags);
    if (s != QKD_OK) return s;
    if (!(qber > 0.0 && qber < 1.0)) return set_error(QKD_ERR_INVALID_ARG, "QBER must be in (0,1)");
    DeviceGuard g(c->device);
    ws = resolve_ws(c, ws);
    if (!ws) return set_error(QKD_ERR_OUT_OF_MEMORY, "no workspace");
    WsSession sess(ws, (hipStream_t)stream);
    s = ws_reserve_keys(ws, n_frames, 1);
    if (s != QKD_OK) return s;
    // the byte keys go to the decode launch, which packs them (the split
    // path inside its frame-syndrome kernel, launch_frame_syn)
    return decode_keys(c, ws, n_frames, qber, max_iterations, msg_threshold, flags, bits_out, iterations,
                       syndromes_match, keys_match, (hipStream_t)stream, alice, bob);
}

static qkd_status keygen_into_ws(const qkd_code* c, qkd_workspace* ws, const uint64_t* seeds,
                                 uint64_t offset, size_t n_frames, double q_nom, double* exact_q,
                                 hipStream_t stream) {
    if (!(q_nom > 0.0 && q_nom <= 1.0)) return set_error(QKD_ERR_INVALID_ARG, "QBER must be in (0,1]");
    const uint64_t ne = qkdr::num_errors((uint32_t)c->n, q_nom);
    if (ne == 0)
        return set_error(QKD_ERR_QBER_TOO_SMALL, "Key size '%d' is too small for QBER.", c->n);
    qkd_status s = ws_reserve_keys(ws, n_frames, n_frames * ne);
    if (s != QKD_OK) return s;
    const uint32_t words = (uint32_t)((c->n + 63) / 64);
    // QKD_KEYGEN=serial forces the one-thread-per-frame kernel, QKD_KEYGEN=replay
    // the two-wave kernel's serial path for every frame, QKD_KEYGEN=lanes the
    // one-wave kernel (keygen_fast_kernel), QKD_KEYGEN=matrix that kernel with its
    // lane jumps as GF(2) matrix products instead of polynomials (tests of all).
    const DbgOpt mode = debug_option(ws, "QKD_KEYGEN");
    const bool serial = mode.is("serial");
    const uint32_t replay = mode.is("replay") ? 1u : 0u;
    const bool matrix = mode.is("matrix");
    const bool lanes = mode.is("lanes");
    // the two-wave generator (default; QKD_KEYGEN=replay forces its serial path)
    const size_t lds2 = (size_t)kKgSplitFrames * ((2 * (size_t)ne + 2 * (ne / 2 + 1)) * sizeof(uint32_t) +
                                                  2 * (size_t)words * sizeof(uint64_t));
    if (ne <= kKeygenFastMaxErrors && c->d_jpoly2 && !serial && !matrix && !lanes && lds2 <= kLdsBytesMax) {
        auto* const kg = c->n <= 65536 ? keygen_split_kernel<true> : keygen_split_kernel<false>;
        hipLaunchKernelGGL(kg, dim3((unsigned)((n_frames + kKgSplitFrames - 1) / kKgSplitFrames)), dim3(kKgBlock), lds2,
                           stream, seeds, offset, (uint32_t)c->n, words, (uint32_t)ne, c->kg_cb, c->kg_cs,
                           (uint32_t)n_frames, c->d_jpoly2, ws->alice_w, ws->bob_w, exact_q, replay);
        QKD_HIP(hipGetLastError());
        return QKD_OK;
    }
    // (the fast kernel's per-frame LDS times kKeygenFrames must fit a workgroup's LDS)
    const size_t lds = (size_t)kKeygenFrames * (2 * (size_t)ne * sizeof(uint32_t) + (ne / 2 + 1) * sizeof(uint2));
    if (ne <= kKeygenFastMaxErrors && c->d_jump && !serial && lds <= kLdsBytesMax) {
        auto* const kg = c->n <= 65536 ? keygen_fast_kernel<true> : keygen_fast_kernel<false>;
        hipLaunchKernelGGL(kg, dim3((unsigned)((n_frames + kKeygenFrames - 1) / kKeygenFrames)),
                           dim3(kKeygenBlock), lds, stream, seeds, offset, (uint32_t)c->n, words, (uint32_t)ne,
                           c->keygen_chunk, (uint32_t)n_frames, c->d_jump, matrix ? nullptr : c->d_jpoly,
                           ws->alice_w, ws->bob_w, exact_q, replay);
    } else {
        hipLaunchKernelGGL(keygen_kernel, dim3(blocks_for(n_frames, 64)), dim3(64), 0, stream, seeds, offset,
                           (uint32_t)n_frames, (uint32_t)c->n, words, (uint32_t)ne, ws->alice_w, ws->bob_w,
                           ws->low, exact_q);
    }
    QKD_HIP(hipGetLastError());
    return QKD_OK;
}

qkd_status qkd_keygen_batch(const qkd_code* c, qkd_workspace* ws, const uint64_t* seeds,
                            uint64_t seed_offset, size_t n_frames, double q_nominal, uint8_t* alice,
                            uint8_t* bob, double* exact_qber, void* stream) {
    clear_error();
    if (!c || !seeds || !alice || !bob) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s != QKD_OK) return s;
    DeviceGuard g(c->device);
    ws = resolve_ws(c, ws);
    if (!ws) return set_error(QKD_ERR_OUT_OF_MEMORY, "no workspace");
    WsSession sess(ws, (hipStream_t)stream);
    s = keygen_into_ws(c, ws, seeds, seed_offset, n_frames, q_nominal, exact_qber, (hipStream_t)stream);
    if (s != QKD_OK) return s;
    const uint32_t words = (uint32_t)((c->n + 63) / 64);
    const size_t nb = n_frames * (size_t)c->n;
    hipLaunchKernelGGL(unpack_kernel, dim3(blocks_for(nb, 256)), dim3(256), 0, (hipStream_t)stream,
                       ws->alice_w, (uint32_t)c->n, words, (uint32_t)n_frames, alice);
    hipLaunchKernelGGL(unpack_kernel, dim3(blocks_for(nb, 256)), dim3(256), 0, (hipStream_t)stream,
                       ws->bob_w, (uint32_t)c->n, words, (uint32_t)n_frames, bob);
    QKD_HIP(hipGetLastError());
    return QKD_OK;
}

// ---- interactive mode: one key stream across the QBER points ------------------
// QKD_LDPC_interactive_simulation (simulation.cpp:73-137) seeds ONE
// Xoshiro256PlusPlus(SIMULATION_SEED) (:95) and draws every point's Alice key
// and Bob errors from it in turn (:102-103), so point p starts where point p-1's
// shuffle stopped, Lemire rejections included. A handful of points per run and
// no throughput target: one thread walks the stream exactly as the reference
// does (the batch path's jump-ahead keygen needs independent seeds).
__global__ void keygen_stream_kernel(uint64_t sim_seed, uint32_t n, uint32_t words, uint32_t n_points,
                                     const uint32_t* ne, uint64_t* alice_w, uint64_t* bob_w, uint32_t* low) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    qkdr::Xoshiro256pp g;
    g.seed(sim_seed);
    for (uint32_t p = 0; p < n_points; ++p) {
        uint64_t* A = alice_w + (size_t)p * words;
        uint64_t* B = bob_w + (size_t)p * words;
        for (uint32_t w = 0; w < words; ++w) {
            const uint32_t nb = min(64u, n - w * 64);
            uint64_t v = 0;
            for (uint32_t b = 0; b < nb; ++b) v |= (g.next() >> 63) << b;
            A[w] = v;
            B[w] = v;
        }
        qkdr::shuffle_low_positions(g, n, ne[p], low);
        for (uint32_t k = 0; k < ne[p]; ++k) B[low[k] >> 6] ^= 1ull << (low[k] & 63);
    }
}

qkd_status qkd_interactive_batch(const qkd_code* c, qkd_workspace* ws, uint64_t simulation_seed, size_t n_points,
                                 const double* q_nominal, uint32_t max_iterations, double msg_threshold,
                                 uint32_t flags, uint32_t* iterations, uint8_t* syndromes_match,
                                 uint8_t* keys_match, double* exact_qber, uint32_t* errors, size_t* points_done) {
    clear_error();
    if (!c || !q_nominal || !iterations || !syndromes_match || !keys_match || !exact_qber || !errors || !points_done)
        return set_error(QKD_ERR_INVALID_ARG, "null argument");
    *points_done = 0;
    if (n_points == 0 || n_points > (1u << 20)) return set_error(QKD_ERR_INVALID_ARG, "bad point count");
    qkd_status s = check_decode_params(max_iterations, msg_threshold, flags);
    if (s != QKD_OK) return s;
    // the reference throws at the first point whose exact QBER is 0 (:105-111),
    // after running the points before it
    std::vector<uint32_t> ne;
    uint32_t max_ne = 1;
    size_t run = n_points;
    for (size_t p = 0; p < n_points; ++p) {
        // (decoded points: log((1 - q) / q) must be finite, as qkd_qkd_ldpc_batch requires)
        if (!(q_nominal[p] > 0.0 && q_nominal[p] < 1.0)) return set_error(QKD_ERR_INVALID_ARG, "QBER must be in (0,1)");
        const uint64_t e = qkdr::num_errors((uint32_t)c->n, q_nominal[p]);
        if (e == 0) {
            run = p;
            break;
        }
        ne.push_back((uint32_t)e);
        max_ne = std::max(max_ne, (uint32_t)e);
    }
    DeviceGuard g(c->device);
    ws = resolve_ws(c, ws);
    if (!ws) return set_error(QKD_ERR_OUT_OF_MEMORY, "no workspace");
    hipStream_t st = nullptr;
    if (run > 0) {
        WsSession sess(ws, st);
        s = ws_reserve_keys(ws, 1, 1);
        if (s != QKD_OK) return s;
        const uint32_t words = (uint32_t)((c->n + 63) / 64);
        uint64_t *d_a = nullptr, *d_b = nullptr;
        uint32_t *d_ne = nullptr, *d_low = nullptr, *d_it = nullptr;
        uint8_t* d_flags = nullptr;
        auto cleanup = [&]() {
            for (void* q : {(void*)d_a, (void*)d_b, (void*)d_ne, (void*)d_low, (void*)d_it, (void*)d_flags})
                if (q) (void)hipFree(q);
        };
        if (hipMalloc(&d_a, run * words * 8) != hipSuccess || hipMalloc(&d_b, run * words * 8) != hipSuccess ||
            hipMalloc(&d_ne, run * 4) != hipSuccess || hipMalloc(&d_low, (size_t)max_ne * 4) != hipSuccess ||
            hipMalloc(&d_it, run * 4) != hipSuccess || hipMalloc(&d_flags, run * 2) != hipSuccess) {
            cleanup();
            return set_error(QKD_ERR_OUT_OF_MEMORY, "interactive: cannot allocate");
        }
        hipError_t e = hipMemcpy(d_ne, ne.data(), run * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(keygen_stream_kernel, dim3(1), dim3(64), 0, st, simulation_seed, (uint32_t)c->n, words,
                               (uint32_t)run, d_ne, d_a, d_b, d_low);
            e = hipGetLastError();
        }
        for (size_t p = 0; p < run && e == hipSuccess && s == QKD_OK; ++p) {
            exact_qber[p] = (double)ne[p] / (double)c->n;
            errors[p] = ne[p];   // distinct positions: every flip is a differing bit (:115-119)
            e = hipMemcpyAsync(ws->alice_w, d_a + p * words, words * 8, hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipMemcpyAsync(ws->bob_w, d_b + p * words, words * 8, hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess)
                s = decode_keys(c, ws, 1, exact_qber[p], max_iterations, msg_threshold, flags, nullptr, d_it + p,
                                d_flags + p, d_flags + run + p, st);
        }
        if (e == hipSuccess && s == QKD_OK) e = hipMemcpy(iterations, d_it, run * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess && s == QKD_OK) e = hipMemcpy(syndromes_match, d_flags, run, hipMemcpyDeviceToHost);
        if (e == hipSuccess && s == QKD_OK) e = hipMemcpy(keys_match, d_flags + run, run, hipMemcpyDeviceToHost);
        cleanup();
        if (s != QKD_OK) return s;
        if (e != hipSuccess) return set_error(QKD_ERR_DEVICE, "interactive: %s", hipGetErrorString(e));
    }
    *points_done = run;
    if (run < n_points) {
        exact_qber[run] = 0.0;
        return set_error(QKD_ERR_QBER_TOO_SMALL, "Key size '%d' is too small for QBER.", c->n);
    }
    return QKD_OK;
}

__global__ void math_kernel(int which, const double* x, double* y, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (which) {
        case 0: y[i] = qkdm::tanh_flat(x[i]); break;
        case 1: y[i] = qkdm::atanh_flat(x[i]); break;
        case 2: y[i] = (double)RuleMath<kRuleSp32>::tanh_half((float)x[i]); break;   // signed psi(|x|)
        case 4:
        case 5: {
            // phi bounds over [x[2k], x[2k+1]] -> y[2k] = lo, y[2k+1] = hi
            // (4: qkds::phi_bounds, 5: qkds::phi_bounds_out); one thread per pair
            // phi_bounds gives psi = phi / ln 2 (returned scaled back to phi in
            // binary64); phi_bounds_out takes psi-unit sums (x = S / ln 2)
            if (i & 1) break;
            float lo, hi;
            if (which == 4) {
                qkds::phi_bounds((float)x[i], (float)x[i + 1], lo, hi);
                y[i] = (double)lo * 0.6931471805599453;
                y[i + 1] = (double)hi * 0.6931471805599453;
            } else {
                qkds::phi_bounds_out((float)x[i], (float)x[i + 1], lo, hi);
                y[i] = lo;
                y[i + 1] = hi;
            }
            break;
        }
        case 8:
        case 9: {
            // quadruples (a, b, s_lo, s_hi) -> (in lo, in hi, out lo, out hi),
            // raw binary32 results: 8 the packed qkds::phi_pair, 9 the scalar
            // phi_bounds (psi units) and phi_bounds_out; one thread per quadruple
            if (i & 3) break;
            qkds::f2 in, out;
            if (which == 8) {
                qkds::phi_pair((float)x[i], (float)x[i + 1], (float)x[i + 2], (float)x[i + 3], in, out);
            } else {
                in = qkds::phi_bounds((float)x[i], (float)x[i + 1]);
                out = qkds::phi_bounds_out((float)x[i + 2], (float)x[i + 3]);
            }
            y[i] = in.x;
            y[i + 1] = in.y;
            y[i + 2] = out.x;
            y[i + 3] = out.y;
            break;
        }
        case 10:
        case 11: {
            // pairs of exact b2c (x[2k], x[2k+1]) -> raw binary32 psi bounds
            // (lo, hi of each): 10 the packed qkds::psi_of_exact2, 11 the
            // scalar psi_of_exact twice; one thread per pair
            if (i & 1) break;
            qkds::f2 r0, r1;
            if (which == 10) {
                qkds::psi_of_exact2(x[i], x[i + 1], r0, r1);
            } else {
                r0 = qkds::psi_of_exact(x[i]);
                r1 = qkds::psi_of_exact(x[i + 1]);
            }
            y[i] = __builtin_bit_cast(double, r0);
            y[i + 1] = __builtin_bit_cast(double, r1);
            break;
        }
        case 12:
        case 13: {
            // pairs (x, S) -> (|tanh_half(x)|, two_atanh(S)) of the binary32 rule:
            // 12 the packed RuleMath<kRuleSp32>::pair, 13 the scalar forms
            if (i & 1) break;
            qkds::f2 r;
            if (which == 12) {
                r = RuleMath<kRuleSp32>::pair((float)x[i], (float)x[i + 1]);
            } else {
                r = qkds::f2{__builtin_fabsf(RuleMath<kRuleSp32>::tanh_half((float)x[i])),
                             RuleMath<kRuleSp32>::two_atanh((float)x[i + 1])};
            }
            y[i] = r.x;
            y[i + 1] = r.y;
            break;
        }
        case 14:
        case 15:
        case 16:
        case 17: {
            // quadruples (a lo, a hi, b lo, b hi) -> the bounds of both
            // intervals: 14 the packed phi_bounds2, 15 two scalar phi_bounds
            // (the interleaved decoder's input form); 16 the packed
            // phi_bounds_out2, 17 two scalar phi_bounds_out (its output form)
            if (i & 3) break;
            const qkds::f2 u{(float)x[i], (float)x[i + 1]}, v{(float)x[i + 2], (float)x[i + 3]};
            qkds::f2 ru, rv;
            if (which == 14) qkds::phi_bounds2(u, v, ru, rv);
            else if (which == 16) qkds::phi_bounds_out2(u, v, ru, rv);
            else if (which == 15) { ru = qkds::phi_bounds(u.x, u.y); rv = qkds::phi_bounds(v.x, v.y); }
            else { ru = qkds::phi_bounds_out(u.x, u.y); rv = qkds::phi_bounds_out(v.x, v.y); }
            y[i] = ru.x;
            y[i + 1] = ru.y;
            y[i + 2] = rv.x;
            y[i + 3] = rv.y;
            break;
        }
        case 6: y[i] = (double)__builtin_amdgcn_exp2f((float)x[i]); break;   // hardware v_exp_f32
        case 7: y[i] = (double)__builtin_amdgcn_logf((float)x[i]); break;    // hardware v_log_f32
        default: y[i] = (double)RuleMath<kRuleSp32>::two_atanh((float)x[i]); break;  // phi(S ln 2)
    }
}

qkd_status qkd_debug_math(int which, const double* x, double* y, size_t n, void* stream) {
    clear_error();
    if (!x || !y || which < 0 || which > 17) return set_error(QKD_ERR_INVALID_ARG, "bad argument");
    if (which >= 14 && (n & 3)) return set_error(QKD_ERR_INVALID_ARG, "packed phi bounds take quadruples");
    if ((which == 10 || which == 11) && (n & 1)) return set_error(QKD_ERR_INVALID_ARG, "psi pairs take n even");
    if ((which == 12 || which == 13) && (n & 1)) return set_error(QKD_ERR_INVALID_ARG, "rule pairs take n even");
    if ((which == 4 || which == 5) && (n & 1)) return set_error(QKD_ERR_INVALID_ARG, "phi bounds take pairs (n even)");
    if ((which == 8 || which == 9) && (n & 3))
        return set_error(QKD_ERR_INVALID_ARG, "paired phi bounds take quadruples (n % 4 == 0)");
    if (n == 0) return QKD_OK;
    hipLaunchKernelGGL(math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, which,
                       x, y, n);
    QKD_HIP(hipGetLastError());
    return QKD_OK;
}

// Exhaustive phi-bound sweep (qkd_debug_phi_sweep): one binary32 point per
// (thread, step), binary64 phi and |phi'| from OCML's exp / expm1 / log1p
// (about 1 ulp of binary64, 2^-32 of the 2^-20 allowance).
__device__ __forceinline__ void sweep_max(float v, uint32_t bits, uint32_t* mx, uint32_t* at) {
    const uint32_t b = __builtin_bit_cast(uint32_t, v);
    if (b > atomicMax(mx, b)) atomicExch(at, bits);
}

__global__ void phi_sweep_kernel(int which, uint32_t first, uint32_t last, unsigned long long* cnt,
                                 uint32_t* mx) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long pts = 0, bad_hi = 0, bad_lo = 0, bad_sl = 0;
    float e_max = 0.0f, s_max = 0.0f;
    uint32_t e_at = 0, s_at = 0;
    constexpr double R = 0x1.0p-20;
    for (uint64_t k = (uint64_t)first + blockIdx.x * blockDim.x + threadIdx.x; k <= last; k += stride) {
        const uint32_t bits = (uint32_t)k;
        const float a = __builtin_bit_cast(float, bits);
        double S, v, lo, hi, sl;       // S in nep units; v, lo, hi in the form's output units
        if (which == 4) {
            const float a1 = __builtin_amdgcn_fmed3f(a, 0.0f, qkds::kPhiHuge);
            const qkds::PhiVal e = qkds::phi_core<true, false>(a1, qkds::exp_neg(a1), __builtin_amdgcn_logf(a1));
            const qkds::f2 b = qkds::phi_bounds(a, a);
            S = a1;
            v = e.v * 0.6931471805599453;         // psi -> phi
            lo = b.x * 0.6931471805599453;
            hi = b.y * 0.6931471805599453;
            sl = e.slope;
        } else {
            const float at = __builtin_fminf(a, qkds::kPsiHuge);
            const qkds::PhiVal e = qkds::phi_core<false, true>(at * qkds::kLn2, __builtin_amdgcn_exp2f(-at),
                                                               __builtin_amdgcn_logf(at));
            const qkds::f2 b = qkds::phi_bounds_out(a, a);
            S = (double)at * 0.6931471805599453;
            v = e.v;
            lo = b.x;
            hi = b.y;
            sl = e.slope;
        }
        const double u = exp(-S), w = -expm1(-S);                    // e^-S, 1 - e^-S
        const double phi = log1p(2.0 * u / w);                       // -ln tanh(S / 2)
        const double dphi = 2.0 * u / (w * (1.0 + u));               // 1 / sinh(S)
        ++pts;
        bad_hi += hi < phi;
        bad_lo += lo > phi;
        bad_sl += sl * (1.0 + R) < dphi;
        // evaluation-error statistics over normal arguments (a subnormal a gives
        // rcp overflow and an infinite upper bound: sound, counted above)
        if (phi > 1e-30 && bits >= 0x00800000u && v < 3.0e38) {
            const float err = (float)(fabs(v / phi - 1.0) / R);
            if (err > e_max) { e_max = err; e_at = bits; }
        }
        const float sr = (float)(dphi / sl);
        if (sr > s_max && bits >= 0x00800000u) { s_max = sr; s_at = bits; }
    }
    atomicAdd(&cnt[0], pts);
    if (bad_hi) atomicAdd(&cnt[1], bad_hi);
    if (bad_lo) atomicAdd(&cnt[2], bad_lo);
    if (bad_sl) atomicAdd(&cnt[3], bad_sl);
    sweep_max(e_max, e_at, &mx[0], &mx[2]);
    sweep_max(s_max, s_at, &mx[1], &mx[3]);
}

qkd_status qkd_debug_phi_sweep(int which, uint32_t first_bits, uint32_t last_bits, uint64_t* result) {
    clear_error();
    if ((which != 4 && which != 5) || !result || first_bits > last_bits || last_bits >= 0x7f800000u)
        return set_error(QKD_ERR_INVALID_ARG, "bad argument");
    unsigned long long* d_cnt = nullptr;
    uint32_t* d_mx = nullptr;
    QKD_HIP(hipMalloc(&d_cnt, 4 * sizeof(unsigned long long)));
    if (hipMalloc(&d_mx, 4 * sizeof(uint32_t)) != hipSuccess) {
        (void)hipFree(d_cnt);
        return set_error(QKD_ERR_OUT_OF_MEMORY, "phi sweep: cannot allocate");
    }
    hipError_t e = hipMemset(d_cnt, 0, 4 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_mx, 0, 4 * sizeof(uint32_t));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(phi_sweep_kernel, dim3(4096), dim3(256), 0, nullptr, which, first_bits, last_bits, d_cnt,
                           d_mx);
        e = hipGetLastError();
    }
    unsigned long long cnt[4] = {0, 0, 0, 0};
    uint32_t mx[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(cnt, d_cnt, sizeof cnt, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(mx, d_mx, sizeof mx, hipMemcpyDeviceToHost);
    (void)hipFree(d_cnt);
    (void)hipFree(d_mx);
    if (e != hipSuccess) return set_error(QKD_ERR_DEVICE, "phi sweep: %s", hipGetErrorString(e));
    for (int k = 0; k < 4; ++k) result[k] = cnt[k];
    for (int k = 0; k < 4; ++k) result[4 + k] = mx[k];
    return QKD_OK;
}

qkd_status qkd_trace_decode(const qkd_code* c, const double* llr, const uint8_t* syndrome,
                            uint32_t max_iterations, double msg_threshold, uint32_t flags,
                            double* c2b_trace, double* total_trace, uint32_t* iterations,
                            uint8_t* syndrome_match) {
    clear_error();
    if (!c || !llr || !syndrome || !iterations || !syndrome_match)
        return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_decode_params(max_iterations, msg_threshold, flags);
    if (s != QKD_OK) return s;
    if ((flags & QKD_VARIANT_MASK) != QKD_VARIANT_SP_F64)
        return set_error(QKD_ERR_UNSUPPORTED, "trace is provided for the reference rule (QKD_VARIANT_SP_F64) only");
    DeviceGuard g(c->device);
    qkd_workspace* ws = qkd_workspace_create(c, &s);
    if (!ws) return s;
    const size_t stride = (size_t)c->max_dv * c->n_pad + c->n_pad;
    double *d_llr = nullptr, *d_tr = nullptr;
    uint8_t *d_syn = nullptr, *d_ok = nullptr;
    uint32_t* d_it = nullptr;
    auto cleanup = [&]() {
        for (void* p : {(void*)d_llr, (void*)d_tr, (void*)d_syn, (void*)d_ok, (void*)d_it})
            if (p) (void)hipFree(p);
        qkd_workspace_destroy(ws);
    };
    hipStream_t st = nullptr;
    if (hipMalloc(&d_llr, (size_t)c->n * 8) != hipSuccess || hipMalloc(&d_syn, (size_t)c->m) != hipSuccess ||
        hipMalloc(&d_ok, 1) != hipSuccess || hipMalloc(&d_it, 4) != hipSuccess ||
        hipMalloc(&d_tr, stride * max_iterations * 8) != hipSuccess) {
        cleanup();
        return set_error(QKD_ERR_OUT_OF_MEMORY, "trace: cannot allocate %zu B", stride * max_iterations * 8);
    }
    std::vector<uint8_t> syn01((size_t)c->m);
    for (int32_t j = 0; j < c->m; ++j) syn01[j] = syndrome[j] ? 1 : 0;
    hipError_t e = hipMemcpy(d_llr, llr, (size_t)c->n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_syn, syn01.data(), (size_t)c->m, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        cleanup();
        return set_error(QKD_ERR_DEVICE, "trace: %s", hipGetErrorString(e));
    }
    DecodeArgs a{};
    a.pinf = std::numeric_limits<float>::infinity();
    a.n_frames = 1;
    a.max_it = max_iterations;
    a.thr = msg_threshold;
    a.clamp_on = (flags & QKD_FLAG_THRESHOLD) ? 1 : 0;
    a.llr = d_llr;
    a.syn = d_syn;
    a.iters = d_it;
    a.sp_ok = d_ok;
    a.trace = d_tr;
    a.trace_stride = stride;
    s = launch_decode(c, ws, a, kModeLlr, flags, st);
    if (s == QKD_OK) {
        std::vector<double> tr(stride * max_iterations);
        e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipMemcpy(iterations, d_it, 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(syndrome_match, d_ok, 1, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(tr.data(), d_tr, tr.size() * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            s = set_error(QKD_ERR_DEVICE, "trace: %s", hipGetErrorString(e));
        } else {
            // bit-major jagged order of the reference's check_to_bit_msg rows
            const size_t nm = (size_t)c->max_dv * c->n_pad;
            for (uint32_t t = 0; t < *iterations; ++t) {
                const double* src = tr.data() + t * stride;
                if (c2b_trace)
                    for (int32_t i = 0; i < c->n; ++i)
                        for (int32_t k = 0; k < c->bit_ptr[i + 1] - c->bit_ptr[i]; ++k)
                            c2b_trace[(size_t)t * c->e + c->bit_ptr[i] + k] = src[(size_t)k * c->n_pad + i];
                if (total_trace)
                    for (int32_t i = 0; i < c->n; ++i) total_trace[(size_t)t * c->n + i] = src[nm + i];
            }
        }
    }
    cleanup();
    return s;
}

qkd_status qkd_debug_spec_replays(qkd_workspace* ws, uint64_t* replays, int reset) {
    if (!ws || !replays) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    *replays = 0;
    if (!ws->counter) return QKD_OK;
    DeviceGuard g(ws->device);
    QKD_HIP(hipDeviceSynchronize());
    char* p = reinterpret_cast<char*>(ws->counter) + 120;
    QKD_HIP(hipMemcpy(replays, p, 8, hipMemcpyDeviceToHost));
    if (reset) QKD_HIP(hipMemset(p, 0, 8));
    return QKD_OK;
}

qkd_status qkd_debug_decoder_timing(qkd_workspace* ws, int start, double* ms_total, uint64_t* launches) {
    if (!ws) return set_error(QKD_ERR_INVALID_ARG, "null workspace");
    DeviceGuard g(ws->device);
    std::lock_guard<std::mutex> lk(ws->mu);
    if (!start) QKD_HIP(decoder_events_fold(ws));
    if (ms_total) *ms_total = start ? 0.0 : ws->dec_ms_folded;
    if (launches) *launches = start ? 0 : ws->dec_pairs_folded;
    ws->dec_ev_used = 0;
    ws->dec_ms_folded = 0.0;
    ws->dec_pairs_folded = 0;
    ws->time_decoder = start != 0;
    return QKD_OK;
}

qkd_status qkd_debug_phase_cycles(qkd_workspace* ws, uint64_t* cycles7) {
    if (!ws || !cycles7) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    if (!ws->counter) return set_error(QKD_ERR_INVALID_ARG, "workspace has not decoded yet");
    DeviceGuard g(ws->device);
    QKD_HIP(hipDeviceSynchronize());
    QKD_HIP(hipMemcpy(cycles7, reinterpret_cast<char*>(ws->counter) + 64, 56, hipMemcpyDeviceToHost));
    return QKD_OK;
}

qkd_status qkd_counters_batch(const uint32_t* iterations, const uint8_t* syndromes_match,
                              const uint8_t* keys_match, size_t n_frames, qkd_counters* counters,
                              int device, void* stream) {
    clear_error();
    if (!iterations || !syndromes_match || !counters) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s != QKD_OK) return s;
    DeviceGuard g(device);
    QKD_HIP(launch_counters(iterations, syndromes_match, keys_match, n_frames, counters, (hipStream_t)stream));
    return QKD_OK;
}

qkd_status qkd_counters_merge(const qkd_counters* records, size_t n_records, qkd_counters* out, int device,
                              void* stream) {
    clear_error();
    if (!records || !out) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    if (n_records == 0 || n_records > 0xffffffffu) return set_error(QKD_ERR_INVALID_ARG, "bad record count");
    DeviceGuard g(device);
    hipLaunchKernelGGL(counters_merge_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, records,
                       (uint32_t)n_records, out);
    QKD_HIP(hipGetLastError());
    return QKD_OK;
}

qkd_status qkd_trials_batch(const qkd_code* c, qkd_workspace* ws, const uint64_t* seeds,
                            uint64_t seed_offset, size_t n_frames, double q_nominal,
                            uint32_t max_iterations, double msg_threshold, uint32_t flags,
                            uint32_t* iterations, uint8_t* syndromes_match, uint8_t* keys_match,
                            double* exact_qber, qkd_counters* counters, void* stream) {
    clear_error();
    if (!c || !seeds || !iterations || !syndromes_match)
        return set_error(QKD_ERR_INVALID_ARG, "null argument");
    qkd_status s = check_frames(n_frames);
    if (s == QKD_OK) s = check_decode_params(max_iterations, msg_threshold, flags);
    if (s != QKD_OK) return s;
    // (the keys are decoded: log((1 - q) / q) must be finite, as qkd_qkd_ldpc_batch requires)
    if (!(q_nominal > 0.0 && q_nominal < 1.0)) return set_error(QKD_ERR_INVALID_ARG, "QBER must be in (0,1)");
    DeviceGuard g(c->device);
    ws = resolve_ws(c, ws);
    if (!ws) return set_error(QKD_ERR_OUT_OF_MEMORY, "no workspace");
    WsSession sess(ws, (hipStream_t)stream);
    s = keygen_into_ws(c, ws, seeds, seed_offset, n_frames, q_nominal, exact_qber, (hipStream_t)stream);
    if (s != QKD_OK) return s;
    const double q = (double)qkdr::num_errors((uint32_t)c->n, q_nominal) / (double)c->n;
    s = decode_keys(c, ws, n_frames, q, max_iterations, msg_threshold, flags, nullptr, iterations,
                    syndromes_match, keys_match, (hipStream_t)stream);
    if (s != QKD_OK) return s;
    if (counters) QKD_HIP(launch_counters(iterations, syndromes_match, keys_match, n_frames, counters,
                                          (hipStream_t)stream));
    return QKD_OK;
}

}  // extern "C"
