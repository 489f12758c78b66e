// qkd_decode.h — device-side pieces shared by the decode kernels (decode.hip:
// the classic message store; decode_split.hip: the LDS/global split store):
// launch arguments, LDS helpers, wave-plan words, the per-edge check rule and
// the second-iteration table. Compiled with -ffp-contract=off (qkd_math.h).
#pragma once
#include <hip/hip_runtime.h>

#include "qkd_internal.h"
#include "qkd_math.h"
#include "qkd_plan.h"
#include "qkd_spec.h"

namespace qkd {


// Speculative interval iterations per frame before the exact fallback
// (decode_split.hip; QKD_SPEC_CAP overrides).
constexpr int kSpecCapDefault = 8;
constexpr int kCkptUnsatDefault = 128;    // checkpointed speculation trigger (unsatisfied checks)
// across calls: a QBER whose speculative call replayed more than this fraction
// of its frames switches to the checkpointed speculation (decode_keys)
constexpr double kSpecCkptSwitch = 1.0 / 16.0;
// Replay fraction above which speculation stops: within a launch for the
// frames still to start (decode_split.hip), across calls for that QBER and up.
constexpr double kSpecReplayMax = 1.0 / 6.0;
// the in-launch policy's frame windows (DecodeArgs::win): 256 frames, decided
// from the window 8 back (2048 frames earlier, ~8 frame-times at 256 resident
// workgroups: by then it has almost always completed; with the window 4 back
// the waits for a window's last slow frames cost 3.5 % per config-2 batch)
constexpr uint32_t kSpecWinShift = 8;
constexpr uint32_t kSpecWinLag = 8;
// decode_keys samples the replay count of a QBER that twice stayed under
// kSpecCkptSwitch only once every this many calls
constexpr uint64_t kSpecStatEvery = 64;

// Largest check degree the first-iteration table covers.
constexpr int kFirstTableDeg = 16;


enum DecodeMode : int {
    kModeLlr = 0,  // qkd_decode_batch: caller LLRs + syndrome bytes
    kModeKeys = 1  // QKD_LDPC path: packed alice/bob keys, LLR = +-log_p
};

// Check-node rule and message width (QKD_VARIANT_* in qkd_ldpc.h).
//   kRuleSp64   the reference's sum-product in binary64, bit-exact
//   kRuleSp32   the same schedule with binary32 messages and totals, the
//               check rule in Gallager's form with the hardware exp2 / log2
//               (a variant: not bit-exact to anything)
//   kRuleMinSum normalised min-sum in binary32: c2b = scale * sign * min|b2c|
//               over the other edges of the check (a variant, no transcendental)
//   kRuleMinSumLds  the same min-sum with the frame's whole message state in
//               LDS (per check: min1, min2, argmin, sign bits), no global
//               message store; used when the state fits (decode_ms_fits)
//   kRuleMinSumLdsSc  kRuleMinSumLds with Savin's self-correction
//               (QKD_MINSUM_SELF_CORRECT) compiled in: its own kernel
//               instantiation, so profiles attribute its time to it
//   kRuleMinSumSplit / kRuleMinSumSplitSc  the same min-sum rules (plain /
//               self-corrected) on the split decoder's skeleton: one binary32
//               slot per edge, all in LDS, edge-parallel check phase
//               (decode_split.hip ms_split_check_phase); used whenever that
//               store fits (the default for codes like the reference's)
enum DecodeRule : int {
    kRuleSp64 = 0, kRuleSp32 = 1, kRuleMinSum = 2, kRuleMinSumLds = 3, kRuleMinSumLdsSc = 4,
    kRuleMinSumSplit = 5, kRuleMinSumSplitSc = 6
};
template <int RULE> struct RuleMsg { using T = float; };
template <> struct RuleMsg<kRuleSp64> { using T = double; };

struct DecodeArgs {
    DeviceCode code;
    uint32_t n_frames;
    uint32_t max_it;
    double thr;
    int clamp_on;
    float ms_scale;    // kRuleMinSum normalisation
    float ms_offset;   // kRuleMinSum offset (subtracted after the scale, floored at 0)
    int ms_sc;         // kRuleMinSumLds: self-corrected (QKD_MINSUM_SELF_CORRECT)
    // kModeLlr
    const double* llr;
    const uint8_t* syn;
    // kModeKeys
    const uint64_t* alice_w;
    const uint64_t* bob_w;
    // qkd_qkd_ldpc_batch: the caller's byte keys (F x N, 0/1), packed into
    // alice_w / bob_w by the frame-syndrome kernel itself (the split path's
    // byte form) or by pack_kernel first (launch_pack_keys); nullptr when the
    // keys are packed already (device keygen)
    const uint8_t* alice_b;
    const uint8_t* bob_b;
    uint32_t words;
    double log_p;
    // First-iteration message table (kModeKeys): with every channel LLR equal
    // to +-log_p, the first check phase is a function of signs and degrees
    // only (see first_check_phase); first_c2b[d] = its message magnitude for
    // a check of degree d. Used when first_table != 0.
    int first_table;
    double first_c2b[kFirstTableDeg + 1];
    // Second-iteration tanh table (kModeKeys, needs first_table): entries,
    // 0 when off (see second_table_fill).
    int tab2_entries;
    // speculative kernel, QKD path: entries of the folded first iteration's
    // table (kFoldTabPat per degree pattern, decode_split.hip fold_table_fill),
    // 0 when off
    int ftab_entries;
    // outputs
    uint8_t* bits_out;
    uint32_t* iters;
    uint8_t* sp_ok;
    uint8_t* key_ok;
    // scratch
    double* c2b;
    size_t c2b_stride;
    uint32_t* counter;
    // diagnostics: per-phase shader-clock cycles summed over workgroups
    // (thread 0's view between barriers), or nullptr
    unsigned long long* phase;
    // qkd_trace_decode (binary64 rule, one frame): per executed iteration, the
    // c2b store (max_dv x n_pad) then the bit totals (n_pad), or nullptr
    double* trace;
    size_t trace_stride;
    // large codes (decode_kernel<..., GT = true>): the bit totals of each
    // workgroup's frame in global scratch, totals_stride doubles apart
    double* totals;
    size_t totals_stride;
    // decode_split_kernel: the LDS budget its layout was sized for (SplitLds)
    uint32_t lds_budget;
    // decode_split_kernel, binary64 rule: DeviceCode::plan_slot with the slot
    // field encoded for this launch's layout (encode_slot)
    const uint2* plan_enc;
    // decode_split_kernel, kModeKeys: per frame 2 * m_words syndrome words
    // from frame_syn_kernel (target s_A, then the first-product signs), and
    // the frame's last hard decision out as packed words (key_match_kernel
    // compares them with Alice's key and unpacks bits_out)
    const uint32_t* synw;
    uint64_t* zout;
    // decode_split_kernel, kModeKeys, binary64 rule: speculative interval
    // iterations (qkd_spec.h) before the exact ones; spec_cap = how many (0:
    // off), log_p and thr as binary32 bounds, spec_replays counts the frames
    // that fell back to the exact iterations
    uint32_t spec_cap;
    float lp_dn, lp_up, thr_dn, thr_up;
    float pinf;          // +inf (an operand the compiler cannot fold: decode_split.hip)
    unsigned long long* spec_replays;
    // frames replayed exactly in this launch (zeroed per launch): once they
    // pass a quarter of the frames started, later frames skip the speculation
    uint32_t* replay_count;
    // QKD_SPEC_POLICY=always (tests): the in-launch replay policy never turns
    // the speculation off
    uint32_t spec_always;
    // The in-launch replay policy over frame-index windows of 2^win_shift
    // frames (decode_split.hip spec_policy): 64-bit word w of win (2 *
    // win_count uint32) holds window w's completed frames (low half) and
    // replay events (high half), zeroed per launch by the frame-syndrome
    // kernel, or a memset. Frame f speculates iff window
    // f / W - win_lag replayed at most a sixth of its frames (windows below
    // win_lag: always) -- a function of the frames alone, not of the order in
    // which workgroups finish them.
    uint32_t* win;
    uint32_t win_count;
    uint32_t win_shift;
    uint32_t win_lag;
    // checkpointed speculation (SPEC 2, high QBER): once an exact iteration
    // leaves at most ckpt_unsat checks unsatisfied, the messages are saved to
    // ckpt (ckpt_stride elements per workgroup) and the iterations continue on
    // intervals; a frame they cannot certify resumes exactly from the save
    double* ckpt;
    uint32_t ckpt_stride;
    uint32_t ckpt_unsat;
    // the frame-interleaved decoder (decode_ilv.hip): its message lines
    // (ilv_stride doubles per workgroup) and the frames whose intervals could
    // not certify, for the split kernel (fb_list, fb_count entries)
    double* ilv_store;
    size_t ilv_stride;
    uint32_t* fb_list;
    uint32_t* fb_count;
    // decode_split_kernel: decode only frame_list[0 .. *frame_count) (the
    // interleaved decoder's hand-offs), or every frame when nullptr
    const uint32_t* frame_list;
    const uint32_t* frame_count;
};

// The frame-interleaved decoder (decode_ilv.hip): kIlvCols frames per
// workgroup in lockstep, one per lane of each 16-lane group; one message
// line = one slot of the kIlvCols frames (128 bytes).
constexpr int kIlvCols = 16;
constexpr int kIlvCtlWords = 64;
// its workgroup size (QKD_ILV_BLOCK; one workgroup per CU either way: its LDS)
#ifndef QKD_ILV_BLOCK
#define QKD_ILV_BLOCK 1024
#endif
constexpr int kIlvBlock = QKD_ILV_BLOCK;
// the check phase's index ring: per 16-lane group four stages of kRingStage
// words (a check's line indices, ~0 past its degree)
constexpr int kRingStage = 16;
// LDS: tsyn / xsyn / xunc, one word per check pair (check 2w in bits 0-15,
// 2w + 1 in bits 16-31, bit = column), the column control words, the
// first-iteration magnitudes by check degree.
struct IlvLds {
    size_t tsyn, xsyn, xunc, ctl, ctab, ring, bytes;
    // tsyn_global: the target syndrome words in the workgroup's global region
    // instead (decode_ilv_kernel's TG), for codes whose three arrays do not
    // fit; xunc_global (UG, with TG): the uncertainty words there too (M past
    // ~37,000: only the XOR-built syndrome stays in LDS)
    __host__ __device__ IlvLds(int m, bool tsyn_global, bool xunc_global = false) {
        const size_t mw2 = (size_t)(m + 1) / 2;
        const size_t k = tsyn_global ? 0 : 1;
        const size_t u = xunc_global ? 0 : 1;
        tsyn = 0;
        xsyn = k * mw2 * 4;
        xunc = (k + 1) * mw2 * 4;
        ctl = ((k + 1 + u) * mw2 * 4 + 15) & ~(size_t)15;
        ctab = ctl + (size_t)kIlvCtlWords * 4;
        ring = ctab + (size_t)(kFirstTableDeg + 1) * 8;
        bytes = ring + (size_t)(kIlvBlock / kIlvCols) * 4 * kRingStage * 4;
    }
};

// Phase-clock accumulation (diagnostic; a wave-uniform test when off). Each
// mark adds straight to the global slot, so nothing is indexed dynamically in
// registers (an accumulator array would live in scratch).
struct PhaseClock {
    unsigned long long* out;
    long long t = 0;
    __device__ explicit PhaseClock(unsigned long long* o) : out(threadIdx.x == 0 ? o : nullptr) {
        if (out) t = clock64();
    }
    __device__ __forceinline__ void mark(int k) {
        if (out) {
            const long long n = clock64();
            atomicAdd(out + k, (unsigned long long)(n - t));
            t = n;
        }
    }
    __device__ void flush() {}
};

template <typename T>
__device__ __forceinline__ T clamp_msg(T v, T thr) {
    // threshold_matrix_irregular (array_and_matrix_operations.cpp:508-524):
    // compare-based, so NaN passes through.
    return v > thr ? thr : (v < -thr ? -thr : v);
}

// Block-wide any(); flags[2] live in LDS and alternate between calls. Every
// call must be separated from the next by at least one __syncthreads().
__device__ __forceinline__ bool block_any(bool p, uint32_t* flags, uint32_t& k) {
    uint32_t* f = flags + (k & 1u);
    const bool wave_hit = __any(p);
    if (wave_hit && (threadIdx.x & 63) == 0) atomicOr(f, 1u);
    __syncthreads();
    const bool r = *f != 0;
    if (threadIdx.x == 0) flags[(k + 1) & 1u] = 0;
    k++;
    return r;
}


// Syndrome bit arrays hold whole 64-check groups (written by one ballot each).
__host__ __device__ inline int decode_m_words(int m) { return ((m + 63) / 64) * 2; }

// LDS layout of decode_kernel (bytes):
//   total  [n_pad]          bit totals (the reference's `total`, :256-267), message width
//   tsyn   [m_words]        target syndrome, one bit per check
//   xsyn   [m_words]        syndrome of the current hard decision (XOR-built)
//   qsyn   [m_words]        QKD path: sign of each check's first-iteration product
//   tval   [NW][64 + DC]    per-wave tanh values for the in-check products
//                           (prologue: the frame's Alice + Bob words)
//   ctab   [kFirstTableDeg+1] first-iteration message magnitudes by degree
//   tab2   [tab2_entries]   second-iteration tanh table
//   t2idx  [n_pad]          per-bit base index into tab2 (uint16)
//   ctl    [4]              frame index, block_any flags
//   cst    [m] (uint4)      kRuleMinSumLds: per-check min-sum state (ms_state)
struct DecodeLds {
    size_t tsyn, xsyn, qsyn, tval, ctab, tab2, t2idx, ctl, cst, czf, bytes;
    // total_esz: bytes per bit total in LDS (0: the totals live in global
    // memory, large codes); cst_checks: min-sum state of that many checks (16
    // bytes each, and with zf a word of zero flags each, self-corrected min-sum)
    __host__ __device__ DecodeLds(int n_pad, int n_words, int m, int dc, int tab2_entries, int total_esz,
                                  int cst_checks = 0, int row_esz = 0, bool zf = false) {
        const int m_words = decode_m_words(m);
        const int esz = row_esz ? row_esz : total_esz;
        tsyn = ((size_t)n_pad * total_esz + 15) & ~(size_t)15;
        xsyn = tsyn + (size_t)m_words * 4;
        qsyn = xsyn + (size_t)m_words * 4;
        tval = (qsyn + (size_t)m_words * 4 + 15) & ~(size_t)15;
        // the tanh rows double as the prologue's staging area for the frame's
        // Alice and Bob words
        const size_t rows = (size_t)(kDecodeBlock / 64) * (64 + dc) * esz;
        const size_t stage = (size_t)n_words * 16;
        ctab = (tval + (rows > stage ? rows : stage) + 15) & ~(size_t)15;
        tab2 = ctab + (size_t)(kFirstTableDeg + 1) * 8;
        t2idx = tab2 + (size_t)tab2_entries * 8;
        ctl = (t2idx + (tab2_entries ? (size_t)n_pad * 2 : 0) + 15) & ~(size_t)15;
        cst = ctl + 16;
        czf = cst + (size_t)cst_checks * 16;
        bytes = czf + (zf ? (size_t)cst_checks * 4 : 0);
    }
};

// Bit phase: message rows per bit loaded ahead of the ordered sum, and rounds
// (bits tid + r*kDecodeBlock) per load batch.
constexpr int kDvUnroll = 3;
// fold table entries per degree pattern: 2^(1 + kDvUnroll) sign codes x
// (kDvUnroll psi bounds + the hard decision)
constexpr int kFoldTabPat = (2 << kDvUnroll) * (kDvUnroll + 1);
constexpr int kBitChunk = 5;
#ifndef QKD_SPEC_EXACT_CHUNK
#define QKD_SPEC_EXACT_CHUNK 2
#endif
constexpr int kBitChunkSpec = QKD_SPEC_EXACT_CHUNK;     // the exact iterations inside the speculative kernel
// the second-iteration table index and the first-message fold read a bit's
// messages from the unrolled rows only
static_assert(kTab2MaxDv <= kDvUnroll, "tables need every row of their bits unrolled");
// Plan-walking loops outside the check phase load this many tasks' plan words
// per trip (the plan carries kPlanPadTasks >= kPlanGroup * NW idle tasks).
constexpr int kPlanGroup = 4;

// ---- wave-plan words (qkd_plan.h) ------------------------------------------
__device__ __forceinline__ uint32_t pw_bit(uint2 p) { return p.x & qkdp::kPlanBitMask; }
// DeviceCode::plan_slot's first word: the edge's message slot
__device__ __forceinline__ uint32_t pw_slot(uint2 p) { return p.x; }
__device__ __forceinline__ uint32_t pw_row(uint2 p) { return p.x >> 24; }
__device__ __forceinline__ uint32_t pw_chk(uint2 p) { return p.y & qkdp::kPlanChkMask; }
__device__ __forceinline__ int pw_start(uint2 p) { return (int)((p.y >> 20) & 63u); }
__device__ __forceinline__ int pw_deg(uint2 p) { return (int)(p.y >> 26) + 1; }
// Parity of the lanes of this lane's check (its segment) in a wave ballot.
__device__ __forceinline__ int seg_parity(uint64_t ballot, uint2 w) {
    // the segment's bits start at lane pw_start: shift them down, keep deg
    // (<= 64) of them, count
    const uint64_t sh = ballot >> pw_start(w);
    const int deg = pw_deg(w);
    // (v_bfe_u32 takes its width from 5 bits: a width of 32 would read as 0)
    if (deg < 32) return __popc(__builtin_amdgcn_ubfe((uint32_t)sh, 0, (uint32_t)deg)) & 1;
    const uint64_t m = deg == 64 ? ~0ull : ((1ull << deg) - 1ull);
    return __popcll(sh & m) & 1;
}
// The same for segments known to be shorter than 32 lanes (check-degree
// buckets up to 16; v_bfe_u32's width field has 5 bits).
__device__ __forceinline__ int seg_parity32(uint64_t ballot, uint2 w) {
    const uint32_t sh = (uint32_t)(ballot >> pw_start(w));
    return __popc(__builtin_amdgcn_ubfe(sh, 0, (uint32_t)pw_deg(w))) & 1;
}

// One edge of the check phase (qkd_ldpc_algorithm.cpp:220-249):
//   b2c = FIRST ? LLR_i : clamp(total_i - c2b)                  (:188, :303-316)
//   t   = tanh(b2c / 2)                                         (:224)
//   P   = (s_j ? -1 : 1) * t_0 * t_1 * ...  (ascending bits)    (:231-235)
//   c2b = clamp(2 * atanh(P / t))                               (:239-249)
// `row` is this wave's LDS row of tanh values (64 + DC doubles, so reads past
// a segment's end stay inside it and are discarded).
// Where a check phase takes its incoming tanh values from.
enum CheckSrc : int {
    kSrcGeneral = 0,   // tanh(clamp(total_i - c2b) / 2)
    kSrcFirst = 1,     // first iteration: tanh(LLR_i / 2)
    kSrcTable = 2      // second QKD iteration: looked up (second_table_index)
};

template <int RULE> struct RuleMath;
template <> struct RuleMath<kRuleSp64> {
    static __device__ __forceinline__ double tanh_half(double x) { return qkdm::tanh_flat(x / 2.0); }
    static __device__ __forceinline__ double two_atanh(double p) { return 2.0 * qkdm::atanh_flat(p); }
};
// The binary32 variant evaluates the check rule in Gallager's form,
//   c2b = sigma * phi(sum_{k != self} phi(|b2c_k|)),  phi(x) = -ln tanh(x / 2),
// sigma = s_j xor the other signs: the sum-product rule without the tanh
// domain's binary32 trouble (tanh(b2c / 2) rounds to 1 from |b2c| ~ 18 on,
// and P / t is 0 / 0 when a b2c cancels to 0). "tanh_half" publishes
// sign(b2c) * psi(|b2c|), psi = phi / ln 2, with |b2c| limited to [1e-30,
// 80] so psi is finite and positive (the sign survives); "two_atanh" maps a
// psi-unit sum S to phi(S ln 2) (S limited to 115).
//
// This is a decoder, not a certificate: phi only needs to be accurate to a
// few 1e-6 relative (tests/test_variants.py holds it to 5e-6 against binary64
// numpy), which needs far fewer operations than the certified bounds'
// qkds::phi_core (2^-20 with an exact argument split):
//   x < 1/32:      w = x (1 - x/2 + x^2/6)   (truncation < x^3/24 < 1.3e-6 of w)
//   1/32 <= x:     w = 1 - u, u = e^-x = 2^-(x log2 e) (no argument split:
//                  x log2 e rounds to 2^-24 relative, ~4e-6 of psi at x = 80)
//   x < 2:         phi = ln((2 - w) / w)     (argument >= 1.31: v_log_f32's
//                  absolute error stays ~1e-7 of the value)
//   x >= 2:        phi = 2u (1 + s/3 + s^2/5), s = u^2 <= e^-4 (truncation < 9e-7)
// Measured (numpy model of the same steps): 3.7e-6 relative worst case, ~1e-6
// for x < 20.
namespace sp32m {
template <bool PSI>
__device__ __forceinline__ float phi(float x, float u) {
    float t = __builtin_fmaf(x, 1.0f / 6.0f, -0.5f);
    t = __builtin_fmaf(x, t, 1.0f);
    const float w = x < 0.03125f ? x * t : 1.0f - u;
    const float lg = __builtin_amdgcn_logf((2.0f - w) * __builtin_amdgcn_rcpf(w));
    const float vlo = PSI ? lg : qkds::kLn2 * lg;
    const float s = u * u;
    float h = __builtin_fmaf(s, 0.2f, 1.0f / 3.0f);
    h = __builtin_fmaf(s, h, 1.0f);
    const float vhi = (u * (PSI ? 2.0f * qkds::kInvLn2 : 2.0f)) * h;
    return x < 2.0f ? vlo : vhi;
}
}  // namespace sp32m
template <> struct RuleMath<kRuleSp32> {
    static __device__ __forceinline__ float tanh_half(float x) {
        const float a = __builtin_amdgcn_fmed3f(__builtin_fabsf(x), 1.0e-30f, qkds::kPhiHuge);
        const float p = sp32m::phi<true>(a, __builtin_amdgcn_exp2f(a * -qkds::kInvLn2));
        return x < 0.0f ? -p : p;
    }
    static __device__ __forceinline__ float two_atanh(float s) {
        const float at = __builtin_fminf(s, qkds::kPsiHuge);
        return sp32m::phi<false>(at * qkds::kLn2, __builtin_amdgcn_exp2f(-at));
    }
    // |tanh_half(x)| (half 0) and two_atanh(s) (half 1) in one packed
    // evaluation: every operation is the scalar forms', so each half is bit
    // for bit their result (tests/test_variants.py compares them)
    static __device__ __forceinline__ qkds::f2 pair(float x, float s) {
        typedef qkds::f2 f2;
        const float a = __builtin_amdgcn_fmed3f(__builtin_fabsf(x), 1.0e-30f, qkds::kPhiHuge);
        const float at = __builtin_fminf(s, qkds::kPsiHuge);
        const f2 e = f2{a, at} * f2{-qkds::kInvLn2, -1.0f};
        const f2 u = f2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
        const f2 xx = f2{a, at * qkds::kLn2};
        f2 t = __builtin_elementwise_fma(xx, f2(1.0f / 6.0f), f2(-0.5f));
        t = __builtin_elementwise_fma(xx, t, f2(1.0f));
        const f2 ws = xx * t;
        const f2 wd = f2(1.0f) - u;
        const f2 w = f2{xx.x < 0.03125f ? ws.x : wd.x, xx.y < 0.03125f ? ws.y : wd.y};
        const f2 arg = (f2(2.0f) - w) * f2{__builtin_amdgcn_rcpf(w.x), __builtin_amdgcn_rcpf(w.y)};
        const float lg1 = __builtin_amdgcn_logf(arg.y);
        const f2 vlo = f2{__builtin_amdgcn_logf(arg.x), qkds::kLn2 * lg1};
        const f2 sq = u * u;
        f2 h = __builtin_elementwise_fma(sq, f2(0.2f), f2(1.0f / 3.0f));
        h = __builtin_elementwise_fma(sq, h, f2(1.0f));
        const f2 vhi = (u * f2{2.0f * qkds::kInvLn2, 2.0f}) * h;
        return f2{xx.x < 2.0f ? vlo.x : vhi.x, xx.y < 2.0f ? vlo.y : vhi.y};
    }
};

// A check-phase message store. (Non-temporal stores, which skip L2, measured
// 2x slower: the bit phase re-reads these lines shortly after.)
template <typename T>
__device__ __forceinline__ void msg_store(T* p, T v) {
    *p = v;
}

// Makes this wave's LDS row writes visible to its own lanes (no s_barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// First half of an edge: the value the lane publishes in its wave's LDS row.
//   sum-product: t = tanh(b2c / 2) (or the tabulated t), min-sum: b2c itself.
template <int SRC, bool CLAMP, int RULE, typename T>
__device__ __forceinline__ T edge_in(T x, T old, T thr) {
    if (SRC == kSrcGeneral) {
        x = x - old;
        if (CLAMP) x = clamp_msg(x, thr);
    }
    if constexpr (RULE == kRuleMinSum) return x;
    else return SRC == kSrcTable ? x : RuleMath<RULE>::tanh_half(x);
}

// Second half: the lane's message from the published row of its check
// (segment [start, start + deg) of `row`; the row has 64 + DC entries, so reads
// past a segment's end stay inside it and are discarded).
template <bool CLAMP, int DC, int RULE, typename T>
__device__ __forceinline__ T edge_out(T tv, uint2 w, uint32_t sbit, int lane, T thr, const T* row,
                                      float ms_scale, float ms_offset = 0.0f) {
    const int start = pw_start(w);
    const int deg = pw_deg(w);
    T o[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) o[k] = row[start + k];
    T v;
    if constexpr (RULE == kRuleMinSum) {
        // c2b = scale * (s_j ^ signs of the other b2c) * min over the other |b2c|
        uint32_t neg = sbit ^ (tv < 0 ? 1u : 0u);
        T mn = __builtin_inff();
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < deg) {
                neg ^= o[k] < 0 ? 1u : 0u;
                if (start + k != lane) mn = fminf(mn, fabsf(o[k]));
            }
        }
        v = (T)ms_scale * mn;
        if (ms_offset > 0.0f) v = fmaxf(v - (T)ms_offset, (T)0);
        v = neg ? -v : v;
    } else if constexpr (RULE == kRuleSp64) {
        // the reference's P = (s_j ? -1 : 1) * prod_k t_k, then 2 atanh(P / t_self) (:231-241)
        T P = sbit ? (T)-1 : (T)1;
        P = P * o[0];                         // every check has degree >= 1
#pragma unroll
        for (int k = 1; k < DC; ++k) P = k < deg ? P * o[k] : P;
        v = RuleMath<RULE>::two_atanh(P / tv);
    } else {
        // binary32 variant (Gallager form, RuleMath<kRuleSp32>): the extrinsic
        // psi sum over the other edges in ascending order and their sign parity
        T S = (T)0;
        uint32_t neg = sbit;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < deg && start + k != lane) {
                S = S + __builtin_fabsf(o[k]);
                neg ^= o[k] < (T)0 ? 1u : 0u;
            }
        }
        v = RuleMath<RULE>::two_atanh(S);
        v = neg ? -v : v;
    }
    if (CLAMP) v = clamp_msg(v, thr);
    return v;
}

// Second check phase of the QKD path. After the first iteration every message
// is +-C_d (first_check_phase), so bit i's total is
//   total_i = ((LLR_i + c_0) + c_1) + ...    c_k = sign_k * C_{d_k}   (:256-267)
// and its second-iteration incoming value for its k-th check is
//   t = tanh(clamp(total_i - c_k) / 2)                            (:303-316, :224)
// a function of (the degrees d_k of bit i's checks, bob_i, sign_0.., k). The
// table holds it for every degree pattern p, sign code and row k:
//   tab2[p * stride + code * max_dv + k],  code = bob_i | sign_k << (1 + k)
// computed with the same binary64 operations in the same order. The
// iteration-1 bit phase records each bit's base index (second_table_index).
template <bool CLAMP>
__device__ void second_table_fill(const DeviceCode& c, const double* ctab, double log_p, double thr,
                                  double* tab2, int entries) {
    const int dvm = c.max_dv;
    const int stride = tab2_stride(dvm);
    for (int e = threadIdx.x; e < entries; e += kDecodeBlock) {
        const int p = e / stride;
        const int r = e - p * stride;
        const int code = r / dvm;
        const int k = r - code * dvm;
        const uint8_t* degs = c.pat_deg + p * dvm;
        double total = (code & 1) ? -log_p : log_p;
        double ck = 0.0;
        int dv = 0;
        for (int m = 0; m < dvm; ++m) {
            if (degs[m] == 0) break;
            const double cm = ctab[degs[m]];
            const double v = ((code >> (1 + m)) & 1) ? -cm : cm;
            total = total + v;
            if (m == k) ck = v;
            dv = m + 1;
        }
        double y = 0.0;
        if (k < dv) {
            double b = total - ck;
            if (CLAMP) b = clamp_msg(b, thr);
            y = qkdm::tanh_flat(b / 2.0);
        }
        tab2[e] = y;
    }
    __syncthreads();
}

// ---- split message store (decode_split.hip) ----------------------------------
// LDS layout of decode_split_kernel (bytes):
//   tsyn, xsyn, qsyn [m_words]   target syndrome / XOR-built syndrome / first-product signs
//   xunc  [m_words]              speculative rounds: checks with an uncertain hard decision
//   zw    [n_pad / 64] uint64    hard decision of the last bit phase, one bit per bit
//   aw    [n_words] uint64       keys path: Alice's key words (the epilogue's compare)
//   tval  [NW][64 + DC] T        per-wave rows for the in-check products
//                                (prologue: the frame's Bob words)
//   ctab  [kFirstTableDeg + 1]   first-iteration message magnitudes by degree
//   tab2  [tab2_entries]         second-iteration tanh table
//   ftab  [ftab_entries]         speculative kernel: the folded first
//                                iteration's psi bounds and hard decisions
//   ctl   [12]                   [1] next frame, [4..5] round flags, [7] key mismatch (decode_split.hip)
//   wtab  [dc][dc][dc] float     extrinsic-sum weights by (degree, position, k) (dc <= 8)
//   msg   [S + 64] T             message slots 0 .. S-1 (slots S .. max_dv*n_pad-1
//                                live in the workgroup's global region), then
//                                one trash slot per lane
// S is as many slots as the budget leaves after the rest, in whole 64s.
// Weights of a check phase's extrinsic sums: lane at position p of a
// segment of degree deg sums row entry k with weight (k < deg && k != p).
// Buckets up to 8 read them from an LDS table (wtab[deg - 1][p][k], two
// per ds_read_b64) instead of extracting and converting mask bits per entry.
// Buckets DC <= 8 index their segment-weight rows by deg * 8 + p (encode_seg),
// so a lane's degree is one bit-field read of its plan word instead of a
// division by DC (rows of degree 0 and p >= DC unused; -3 VALU per check-phase
// task; with the check phases' select-free row entries -3.4 % per config-2
// batch, profiles/r06_ab.txt)
__host__ __device__ inline int seg_weight_entries(int dc) { return dc <= 8 ? 9 * 8 * dc : 0; }

struct SplitLds {
    size_t tsyn, xsyn, qsyn, xunc, zw, aw, tval, ctab, tab2, ftab, ctl, wtab, msg, bytes;
    uint32_t S;
    __host__ __device__ SplitLds(int n_pad, int n_words, int m, int max_dv, int dc, int tab2_entries,
                                 int ftab_entries, int esz, size_t budget) {
        const int m_words = decode_m_words(m);
        tsyn = 0;
        qsyn = tsyn + (size_t)m_words * 4;
        xsyn = qsyn + (size_t)m_words * 4;
        xunc = xsyn + (size_t)m_words * 4;
        zw = (xunc + (size_t)m_words * 4 + 15) & ~(size_t)15;
        // keys path: Alice's words of the frame, loaded with the prologue's
        // batch for the epilogue's key compare
        aw = (zw + (size_t)(n_pad / 64) * 8 + 15) & ~(size_t)15;
        tval = (aw + (size_t)n_words * 8 + 15) & ~(size_t)15;
        const size_t rows = (size_t)(kDecodeBlock / 64) * (64 + dc) * esz;
        const size_t stage = (size_t)n_words * 8;     // (the prologue stages Bob's words there)
        ctab = (tval + (rows > stage ? rows : stage) + 15) & ~(size_t)15;
        tab2 = ctab + (size_t)(kFirstTableDeg + 1) * 8;
        ftab = (tab2 + (size_t)tab2_entries * 8 + 15) & ~(size_t)15;
        ctl = (ftab + (size_t)ftab_entries * 8 + 15) & ~(size_t)15;
        wtab = ctl + 48;
        msg = (wtab + (size_t)seg_weight_entries(dc) * 4 + 15) & ~(size_t)15;
        const size_t slots = (size_t)max_dv * n_pad;
        // 64 trash slots follow the S message slots (decode_split.hip SplitStore)
        const size_t fit = budget > msg + 64 * (size_t)esz ? (budget - msg) / (size_t)esz - 64 : 0;
        // (a multiple of 64: with n_pad one too, a wave's 64 consecutive bits
        // of one row are all in LDS or all global, SplitStore::ld_row)
        S = (uint32_t)(slots < fit ? slots : fit) & ~63u;
        bytes = msg + ((size_t)S + 64) * esz;
    }
};

// Encoded message-slot words of the split decoder's check phases (its plan,
// DecodeArgs::plan_enc, one per LDS layout): slot x < S (in LDS) as
// kSlotLds | its byte address from the dynamic LDS base; a global slot as
// kSlotGlobalBase + its byte offset in the workgroup's region. The buffer
// descriptor of the region starts kSlotGlobalBase bytes early and spans
// kSlotGlobalBase + the region, so LDS words fail its range check (loads give
// 0, stores are dropped), and global words are LDS addresses past any
// allocation (the same there: tools/mb/lds_oob.hip measures it on gfx950).
constexpr uint32_t kSlotLds = 0x80000000u;
constexpr uint32_t kSlotGlobalBase = 0x40000u;
__host__ __device__ inline uint32_t encode_slot(uint32_t x, uint32_t S, uint32_t msg, uint32_t esz) {
    return x < S ? (kSlotLds | (msg + x * esz)) : (kSlotGlobalBase + (x - S) * esz);
}

// The encoded plan's second word (check-degree bucket DC), the lane's
// segment and its check's target bit pre-decoded for the check phases:
//   bits 0-4    j & 31: the target bit's position in its syndrome word (a
//               shift by the whole word uses these bits only)
//   bits 5-10   start: the segment's first lane
//   bits 11-18  wi: the row of the segment-weight table (SegWeights): DC <= 8:
//               deg * 8 + min(lane - start, DC - 1); DC = 16: (deg - 1) * DC +
//               min(lane - start, DC - 1); wider buckets: deg - 1
//   bits 19-31  (j >> 5) * 4: the byte offset of the check's syndrome word
// (needs M <= 65536: the split decoder's limit).
constexpr uint32_t kSegStartShift = 5, kSegWiShift = 11, kSegWordShift = 19;
__host__ __device__ inline uint32_t encode_seg(uint32_t j, uint32_t start, uint32_t deg, uint32_t lane, uint32_t dc) {
    const uint32_t p = lane - start;
    const uint32_t pc = p < dc - 1 ? p : dc - 1;
    const uint32_t wi = dc <= 8 ? deg * 8 + pc : dc <= 16 ? (deg - 1) * dc + pc : deg - 1;
    return (j & 31u) | (start << kSegStartShift) | (wi << kSegWiShift) | (((j >> 5) * 4u) << kSegWordShift);
}

using DecodeFn = void (*)(DecodeArgs);
// decode_split.hip: the split-store kernel for (mode, rule in {kRuleSp64,
// kRuleSp32}, clamp, check-degree bucket); *dc receives the bucket.
DecodeFn pick_split_decode(int mode, int rule, bool clamp, int max_dc, int* dc);
// the exact keys-path split kernel for codes past kMaxBitsSplit bits (up to
// kMaxBitsSplitLong; check degree <= 16): the interleaved decoder's hand-offs
DecodeFn pick_split_long(bool clamp, int max_dc, int* dc);
// The speculative kernel (binary64 rule, clamp on) for a mode; ckpt: the
// checkpointed variant (keys path: exact iterations first, interval ones from
// a checkpoint once few checks are unsatisfied).
DecodeFn pick_split_spec(int mode, int max_dc, bool ckpt, int* dc);
// the frame-interleaved decoder (decode_ilv.hip) for check-row stride rs (8 or 16)
DecodeFn pick_ilv(int rs, int max_dc, bool tsyn_global, bool xunc_global = false);
// decode_split.hip, kModeKeys: the kernels around the split decoder.
// Before: a.synw from the packed keys. After: key_ok / bits_out from a.zout.
// gather: the gather kernel instead of the bit-sliced one; pack_first: byte
// keys packed by pack_kernel first (the QKD_SYN_SLICED / QKD_SYN_BYTES options)
hipError_t launch_frame_syn(const DecodeArgs& a, hipStream_t stream, bool gather = false, bool pack_first = false);
// decode.hip: a.alice_b / a.bob_b -> a.alice_w / a.bob_w (original bit order)
hipError_t launch_pack_keys(const DecodeArgs& a, hipStream_t stream);
hipError_t launch_key_match(const DecodeArgs& a, hipStream_t stream);

}  // namespace qkd
