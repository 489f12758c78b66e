// decode_ilv.hip — the frame-interleaved decoder for long codes (keys path,
// the binary64 rule through the certified interval iterations of qkd_spec.h).
//
// The split decoder (decode_split.hip) gives each workgroup one frame and
// keeps what fits of its message slots in LDS. For long codes almost nothing
// fits (N = 40,000: 13 % of the slots), and the check phase's scattered
// 8-byte slot accesses each pull a whole cache line from the Infinity Cache,
// about 16 times the bytes they use. Here a workgroup
// decodes kIlvCols = 16 frames in lockstep and stores message slot x of its
// 16 frames in one 128-byte line: lane c of each 16-lane group works on the
// frame of column c, so every slot access of a group is one whole line and
// every fetched byte is used. The lines live in HBM (16 frames x 0.96 MB per
// workgroup for N = 40,000); the LDS holds per-check syndrome bits of the 16
// columns only.
//
// Per iteration (reference src/qkd_ldpc_algorithm.cpp:212-330):
//   check phase  lane (check j, column c): its edges' b2c intervals from the
//                lines of check j's slots, the extrinsic psi sums over the
//                check's other edges, the c2b intervals back (as
//                spec_check_phase_paired: the same bounds, qkd_spec.h)
//   bit phase    lane (bit i, column c): total = LLR + sum c2b (intervals),
//                the hard decision and its syndrome bits (one LDS atomic per
//                group and check: the 16 columns' bits at once), the key
//                compare, b2c_k = clamp(total - c2b_k) back
//   syndrome     per column: a check certainly unsatisfied, or uncertain
// A column's first iteration is the folded one: its messages are the exact
// +-C_d of first_check_phase, so the bit phase computes it in binary64 (as
// the split kernel's FOLD path) and the check phase skips the column.
//
// A column whose round cannot stand (a sign lost in the check phase, an
// uncertain outcome, or spec_cap interval iterations) hands its frame to the
// split kernel, which decodes it from the start (speculating, with exact
// replays): outputs are the reference's bit for bit either way. A column
// whose frame finished takes the next frame of the queue at once.
#include <hip/hip_runtime.h>

#include "qkd_decode.h"
#include "qkd_spec.h"

namespace qkd {

// checks of lines in flight per group while one computes (2 needs the
// registers of a 512-thread workgroup)
#ifndef QKD_ILV_AHEAD
#define QKD_ILV_AHEAD (QKD_ILV_BLOCK <= 512 ? 2 : 1)
#endif

namespace {

constexpr int kIlvGroups = kIlvBlock / kIlvCols;     // 16-lane groups per workgroup

// ctl words (IlvLds::ctl)
constexpr int kCtlFrame = 0;      // [16] frame of each column (n_frames: none)
constexpr int kCtlIt = 16;        // [16] the column's current iteration (0: the folded first)
constexpr int kCtlActive = 32;    // columns with a frame
constexpr int kCtlAbort = 33;     // this round: columns whose check phase lost a sign
constexpr int kCtlKeyMis = 34;    // this round: columns whose decision differs from Alice's key
constexpr int kCtlMis = 35;       // this round: columns with a check certainly unsatisfied
constexpr int kCtlUnc = 36;       // this round: columns with a check whose parity is uncertain
constexpr int kCtlRefill = 37;    // columns given a new frame (their target syndromes to load)
constexpr int kCtlIvl = 38;       // columns in an interval iteration (check phase runs)
constexpr int kCtlDrained = 39;   // the frame queue ran out
// at most this many columns still iterating once the queue is drained hand
// their frames off (QKD_ILV_TAIL; 0 keeps every frame to its end)
#ifndef QKD_ILV_TAIL
#define QKD_ILV_TAIL 4
#endif
constexpr int kIlvTail = QKD_ILV_TAIL;

__device__ __forceinline__ qkds::f2 neg_if(bool neg, qkds::f2 v) {
    return qkds::f2{neg ? -v.y : v.x, neg ? -v.x : v.y};
}

// the 16-bit column mask of a wave ballot: the OR of its four groups
__device__ __forceinline__ uint32_t fold_groups(uint64_t b) {
    return (uint32_t)(b | (b >> 16) | (b >> 32) | (b >> 48)) & 0xffffu;
}

}  // namespace

// RS: the row stride of DeviceCode::ilv_slots; DM: the largest check degree
// rounded up to even (the register arrays' size); TG: the target syndrome
// words in global memory (IlvLds: codes whose three LDS syndrome arrays would
// not fit); UG (with TG): the uncertainty words there too, after the target
// words (codes past M ~ 37,000: kept by L2 atomics, read and cleared by
// exchange)
template <int RS, int DM, bool TG, bool UG = false>
__global__ __launch_bounds__(kIlvBlock) void decode_ilv_kernel(DecodeArgs a) {
    static_assert(DM <= RS && DM % 2 == 0, "degree bucket");
    using qkds::f2;
    extern __shared__ __align__(16) unsigned char smem[];
    const DeviceCode& c = a.code;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t col = (uint32_t)tid & (kIlvCols - 1);
    const int grp = tid / kIlvCols;
    static_assert(TG || !UG, "global uncertainty words follow global target words");
    const IlvLds L(c.m, TG, UG);
    const uint32_t mw2 = (uint32_t)(c.m + 1) >> 1;
    uint32_t* xsyn = reinterpret_cast<uint32_t*>(smem + L.xsyn);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + L.ctl);
    double* ctab = reinterpret_cast<double*>(smem + L.ctab);
    uint32_t* ilv_ring = reinterpret_cast<uint32_t*>(smem + L.ring);
    const uint32_t m_words = (uint32_t)decode_m_words(c.m);
    const uint32_t n_pad = (uint32_t)c.n_pad;
    double* const lines = a.ilv_store + (size_t)blockIdx.x * a.ilv_stride;
    // after the lines: the columns' key words, interleaved ([word][column]
    // {bob, alice}), copied at each refill
    uint4* const keyi = reinterpret_cast<uint4*>(lines + (size_t)c.max_dv * n_pad * kIlvCols);
    // the columns' target syndrome bits (16 columns x 2 checks per word:
    // check j is bit ((j & 1) << 4) + column of word j >> 1): in LDS, or (TG)
    // after the key words in global memory, so the LDS holds only the
    // syndrome words the bit phase updates (codes up to M ~ 36,000; the check
    // phase then loads each check's word with its lines)
    uint32_t* const tsyn = TG ? reinterpret_cast<uint32_t*>(keyi + (size_t)a.words * kIlvCols)
                              : reinterpret_cast<uint32_t*>(smem + L.tsyn);
    // (the region rounds the target words up to whole doubles)
    uint32_t* const xunc = UG ? tsyn + ((mw2 + 1u) & ~1u) : reinterpret_cast<uint32_t*>(smem + L.xunc);
    // The lines through a buffer descriptor: a line index of ~0 (an edge past
    // the check's degree, a row past the bit's) gives an offset past the
    // region, which loads 0 and drops the store -- no branch around any
    // access (a branch there made the compiler wait for every load in flight
    // at the top of each pipelined loop)
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
        lines, (short)0, (int)((size_t)c.max_dv * n_pad * kIlvCols * sizeof(double)), 0x00020000);
    using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(lrs, 0, 0, 0));
    auto ld_line = [&](uint32_t x) -> double {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(lrs, (int)(x * 128u + col * 8u), 0, 0));
    };
    auto st_line = [&](uint32_t x, double v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, v), lrs, (int)(x * 128u + col * 8u), 0, 0);
    };
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;
    const double llr_p = a.log_p;

    for (int d = tid; d <= kFirstTableDeg; d += kIlvBlock) ctab[d] = a.first_c2b[d];
    for (uint32_t w = (uint32_t)tid; w < mw2; w += kIlvBlock) {
        tsyn[w] = 0;
        xsyn[w] = 0;
        if constexpr (UG)
            __hip_atomic_store(xunc + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            xunc[w] = 0;
    }
    if (tid < kIlvCtlWords) ctl[tid] = 0;
    __syncthreads();

    // wave 0: the columns in `need` take the next frames of the queue (one
    // atomic for all of them); the active and refill masks follow
    auto assign = [&](uint32_t need) {
        const uint32_t cnt = (uint32_t)__popc(need);
        uint32_t base = 0;
        if (lane == 0 && cnt) {
            base = atomicAdd(a.counter, cnt);
            if (base + cnt > a.n_frames) ctl[kCtlDrained] = 1;     // (some columns get no frame)
        }
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        bool got = false;
        if (lane < kIlvCols && ((need >> lane) & 1u)) {
            const uint32_t f = base + (uint32_t)__popc(need & ((1u << lane) - 1u));
            got = f < a.n_frames;
            ctl[kCtlFrame + lane] = got ? f : a.n_frames;
            ctl[kCtlIt + lane] = 0;
        }
        const uint32_t gm = (uint32_t)__ballot(got) & 0xffffu;
        if (lane == 0) {
            ctl[kCtlActive] = (ctl[kCtlActive] & ~need) | gm;
            ctl[kCtlRefill] = gm;
        }
    };
    // every thread: the target syndrome bits of the refilled columns
    // (frame_syn_kernel's words: check j is bit j & 31 of word j >> 5)
    auto refill = [&]() {
        const uint32_t rf = ctl[kCtlRefill];
        if (rf == 0) return;
        for (uint32_t w = (uint32_t)tid; w < mw2; w += kIlvBlock) {
            uint32_t v = tsyn[w];
            for (uint32_t r = rf; r != 0; r &= r - 1u) {
                const uint32_t cc = (uint32_t)__builtin_ctz(r);
                const uint32_t f = ctl[kCtlFrame + cc];
                const uint32_t sw = a.synw[(size_t)f * 2 * m_words + (w >> 4)];
                const uint32_t b0 = (sw >> ((2u * w) & 31u)) & 1u, b1 = (sw >> ((2u * w + 1u) & 31u)) & 1u;
                v = (v & ~(0x10001u << cc)) | (b0 << cc) | (b1 << (16u + cc));
            }
            tsyn[w] = v;
        }
        for (uint32_t r = rf; r != 0; r &= r - 1u) {
            const uint32_t cc = (uint32_t)__builtin_ctz(r);
            const uint32_t f = ctl[kCtlFrame + cc];
            for (uint32_t w = (uint32_t)tid; w < a.words; w += kIlvBlock) {
                const uint64_t b = a.bob_w[(size_t)f * a.words + w], al = a.alice_w[(size_t)f * a.words + w];
                keyi[(size_t)w * kIlvCols + cc] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)al,
                                                             (uint32_t)(al >> 32));
            }
        }
    };
    if (tid < 64) assign((1u << kIlvCols) - 1u);
    __syncthreads();
    refill();
    // QKD_PHASE_TIMING in a build with -DQKD_ILV_PHASES (thread 0's shader
    // clock, summed over workgroups): 0 check phase, 1 bit phase, 2 syndrome
    // test and outcomes, 3 refill. Not in the product build: the clock's
    // registers live across the frame loop and add spills.
#ifdef QKD_ILV_PHASES
    PhaseClock pc(a.phase);
#else
    struct {
        __device__ void mark(int) {}
    } pc;
#endif

    for (;;) {
        __syncthreads();
        pc.mark(3);
        const uint32_t active = ctl[kCtlActive];
        if (active == 0) break;
        const uint32_t f = ctl[kCtlFrame + col];
        const uint32_t it = ctl[kCtlIt + col];
        const bool act = (active >> col) & 1u;

        // ---- check phase (columns past their folded first iteration).
        // Software-pipelined over the group's checks t = 0, 1, ... (check j =
        // grp + t G): the lines of check t + 1 are in flight while check t
        // computes; each check's line indices go through a four-stage LDS
        // ring of the group (one copy per group instead of a register per
        // lane), loaded from global memory three checks ahead.
        bool bad = false;
        // (every lane of a group keeps the ring, whatever its column's state:
        // the lanes that write an index are fixed columns; lanes of columns
        // not in an interval iteration load and store nothing, ~0)
        const bool part = act && it != 0;
        if (__builtin_amdgcn_readfirstlane((int)ctl[kCtlIvl]) != 0) {
            uint32_t* ring = ilv_ring + grp * (4 * kRingStage);
            // lane col < DM: line index col of check jj (~0 past its degree,
            // DeviceCode::ilv_slots, and past the last check)
            // (a clamped, unconditional load and a select: a branch around a
            // load or store makes the compiler drain every load in flight)
            // (the raw load; the validity select waits until the commit a
            // step later, so nothing consumes the value right after its load)
            auto idx_issue = [&](int jj) -> uint32_t {
                const int jq = jj < c.m ? jj : c.m - 1;
                return c.ilv_slots[(size_t)jq * RS + (col < (uint32_t)DM ? col : 0u)];
            };
            auto idx_commit = [&](int t, uint32_t r) {
                const bool ok = grp + t * kIlvGroups < c.m;
                if (col < (uint32_t)DM) ring[(t & 3) * kRingStage + col] = ok ? r : ~0u;
            };
            // check t's lines, and its target syndrome word (a clamped check
            // index past the last: unused)
            struct LineSet {
                double v[DM];
                uint32_t sw;
            };
            auto lines_issue = [&](int t, LineSet& ls) {
                const uint32_t* st = ring + (t & 3) * kRingStage;
#pragma unroll
                for (int k = 0; k < DM; ++k) ls.v[k] = ld_line(part ? st[k] : ~0u);
                if constexpr (TG) {
                    const int jt = grp + t * kIlvGroups;
                    ls.sw = tsyn[(jt < c.m ? jt : c.m - 1) >> 1];
                }
            };
            const int nt = (c.m - grp + kIlvGroups - 1) / kIlvGroups;     // this group's checks
            // (memory operations complete in issue order for the waits: each
            // iteration issues the index load it commits next, then the lines
            // two checks ahead, then commits the indices loaded one iteration
            // earlier -- whose wait covers check t's lines only)
            idx_commit(0, idx_issue(grp));
            idx_commit(1, idx_issue(grp + kIlvGroups));
            idx_commit(2, idx_issue(grp + 2 * kIlvGroups));
            uint32_t rnext = idx_issue(grp + 3 * kIlvGroups);
            LineSet va, vb;
            lines_issue(0, va);
#if QKD_ILV_AHEAD == 2
            LineSet vc;
            lines_issue(1, vb);
#endif
            // one check: t's lines in `cur`, t + 1's issued into `ld`. The loop
            // runs it unrolled twice over two register sets, so no line value
            // is copied between iterations (a copy waits for the load it
            // copies, which would drain the pipeline every check; a third set
            // for two checks ahead spills at this occupancy)
            // (rc: the indices of check t + 3, loaded a step earlier; rl: those
            // of check t + 4, loaded now -- two registers alternating, no copy)
            auto step = [&](int t, const LineSet& cur, LineSet& ld, const uint32_t& rc, uint32_t& rl) -> bool {
                if (t >= nt) return false;
                const int j = grp + t * kIlvGroups;
                rl = idx_issue(j + 4 * kIlvGroups);
                lines_issue(t + QKD_ILV_AHEAD, ld);
                idx_commit(t + 3, rc);
                const uint32_t* st = ring + (t & 3) * kRingStage;
                uint32_t live = 0;          // bit k: edge k exists
#pragma unroll
                for (int k = 0; k < DM; ++k) live |= (st[k] != ~0u ? 1u : 0u) << k;
                // |b2c| bounds (psi units) and signs, two edges per packed
                // evaluation (spec_check_phase_paired's input bounds)
                f2 ph[DM];
                uint32_t negs = 0;
#pragma unroll
                for (int k = 0; k < DM; k += 2) {
                    const f2 b0 = qkds::unpack_iv(cur.v[k]), b1 = qkds::unpack_iv(cur.v[k + 1]);
                    const bool n0 = b0.y < 0.0f, n1 = b1.y < 0.0f;
                    const f2 a0 = neg_if(n0, b0), a1 = neg_if(n1, b1);
                    const bool ok0 = a0.x > 1.0e-30f, ok1 = a1.x > 1.0e-30f;
                    f2 r0, r1;
                    const bool in0 = (live >> k) & 1u, in1 = (live >> (k + 1)) & 1u;
                    qkds::phi_bounds2(a0, a1, r0, r1);
                    bad |= part && ((in0 && !ok0) || (in1 && !ok1));
                    negs |= (in0 && n0 ? 1u : 0u) << k;
                    negs |= (in1 && n1 ? 1u : 0u) << (k + 1);
                    ph[k] = (in0 && ok0) ? r0 : f2{0.0f, 0.0f};
                    ph[k + 1] = (in1 && ok1) ? r1 : f2{0.0f, 0.0f};
                }
                const uint32_t sbit = ((TG ? cur.sw : tsyn[j >> 1]) >> ((((uint32_t)j & 1u) << 4) + col)) & 1u;
                const uint32_t par = (uint32_t)__popc(negs) & 1u;
                // extrinsic sums over the other edges: prefix sums, then a
                // backward suffix (every term >= 0, zeros past the degree),
                // widened by the binary32 roundings and the reference's
                // binary64 ones (the split kernel's); the c2b bounds two edges
                // per packed evaluation, threshold_matrix (:246-249) on the
                // magnitude, then the sign
                f2 pre[DM];
                pre[0] = f2{0.0f, 0.0f};
#pragma unroll
                for (int k = 1; k < DM; ++k) pre[k] = pre[k - 1] + ph[k - 1];
                f2 suf = f2{0.0f, 0.0f};
                auto ext_of = [&](int k) -> f2 {
                    const f2 sum = pre[k] + suf;
                    suf = suf + ph[k];
                    const float mg = __builtin_fmaf(sum.y, (float)(DM + 2) * qkds::kSumRel, qkds::kRefSumAbs);
                    f2 e = sum + f2{-mg, mg};
                    e.x = e.x > 0.0f ? e.x : 0.0f;
                    bad |= part && ((live >> k) & 1u) && !(e.y < qkds::kPsiSumMax);
                    return e;
                };
#pragma unroll
                for (int k = DM - 1; k >= 1; k -= 2) {
                    const f2 e1 = ext_of(k);
                    const f2 e0 = ext_of(k - 1);
                    {
                        f2 m0, m1;
                        qkds::phi_bounds_out2(e0, e1, m0, m1);
                        m0.x = __builtin_amdgcn_fmed3f(m0.x, 0.0f, a.thr_dn);
                        m0.y = __builtin_amdgcn_fmed3f(m0.y, 0.0f, a.thr_up);
                        m1.x = __builtin_amdgcn_fmed3f(m1.x, 0.0f, a.thr_dn);
                        m1.y = __builtin_amdgcn_fmed3f(m1.y, 0.0f, a.thr_up);
                        const uint32_t s0 = sbit ^ par ^ ((negs >> (k - 1)) & 1u);
                        const uint32_t s1 = sbit ^ par ^ ((negs >> k) & 1u);
                        // (dropped past the degree: the ring holds ~0 there)
                        st_line(part ? st[k - 1] : ~0u, qkds::pack_iv(neg_if(s0 != 0u, m0)));
                        st_line(part ? st[k] : ~0u, qkds::pack_iv(neg_if(s1 != 0u, m1)));
                    }
                }
                return true;
            };
            uint32_t rb = 0;
#if QKD_ILV_AHEAD == 2
            // (three line sets and three index registers rotating: step t
            // computes set t % 3 and loads check t + 2 into set (t + 2) % 3)
            uint32_t rc2 = 0;
            for (int t = 0;; t += 3) {
                if (!step(t, va, vc, rnext, rb)) break;
                if (!step(t + 1, vb, va, rb, rc2)) break;
                if (!step(t + 2, vc, vb, rc2, rnext)) break;
            }
#else
            for (int t = 0;; t += 2) {
                if (!step(t, va, vb, rnext, rb)) break;
                if (!step(t + 1, vb, va, rb, rnext)) break;
            }
#endif
        }
        {
            const uint32_t bm = fold_groups(__ballot(bad));
            if (lane == 0 && bm) atomicOr(ctl + kCtlAbort, bm);
        }
        __syncthreads();
        pc.mark(0);

        // ---- bit phase, software-pipelined over the group's bits i, i + G,
        // ...: the next bit's code word, key words and lines are loaded
        // before this bit's arithmetic and stores
        const bool keep = it + 1 < a.max_it;
        const bool ivl = act && it != 0;
        uint32_t kmis = 0;
        struct BitIn {
            uint64_t bc;
            uint4 kw;
            double v[kDvUnroll];
            uint32_t qw[kDvUnroll];     // folded first iteration: the checks' first-product sign words
        };
        // (unconditional loads: a bit index past N reads bit N - 1's words,
        // unused; a row past the bit's degree or an inactive column reads
        // through the descriptor's out-of-range offset, 0)
        // bit ii's code word (two bits ahead), then its key words, lines and
        // fold words (one bit ahead, from the code word loaded a step
        // earlier: nothing waits on a load issued in the same step)
        auto bit_load_bc = [&](int ii, BitIn& b) { b.bc = c.bit_code[ii < c.n ? ii : c.n - 1]; };
        auto bit_load = [&](int ii, BitIn& b) {
            const int iq = ii < c.n ? ii : c.n - 1;
            b.kw = keyi[(size_t)(iq >> 6) * kIlvCols + col];
            // (every row's line, not just the bit's degree's: rows past the
            // degree are read and never used)
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) {
                b.v[k] = ld_line((ivl && k < c.max_dv) ? (uint32_t)k * n_pad + (uint32_t)iq : ~0u);
                // (word 0 of the array when not folding: one cached line for all)
                const uint32_t j = (uint32_t)(b.bc >> (16 * k)) & 0xffffu;
                b.qw[k] = a.synw[(act && it == 0) ? (size_t)f * 2 * m_words + m_words + (j >> 5) : 0];
            }
        };
        // one bit: `cur` holds bit i's inputs, the next bit's go into `ld`;
        // unrolled twice over two input sets (no copies, as the check phase)
        auto bstep = [&](int i, BitIn& cur, BitIn& ld) -> bool {
            if (i >= c.n) return false;
            bit_load(i + kIlvGroups, ld);
            const uint64_t bc = cur.bc;
            bit_load_bc(i + 2 * kIlvGroups, cur);
            const int deg = (int)(bc >> 48) & 3;
            int32_t jc[kDvUnroll];
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) jc[k] = (int32_t)(bc >> (16 * k)) & 0xffff;
            // (every lane computes, inactive columns' results masked: no
            // branch around the stores)
            bool z = false, unc = false, dif = false;
            {
                // (this column's Bob and Alice words of bit i, from the
                // workgroup's interleaved copy: one 256-byte run per group)
                const uint4 kw = cur.kw;
                const uint64_t bw = ((uint64_t)kw.y << 32) | kw.x, aw = ((uint64_t)kw.w << 32) | kw.z;
                const uint32_t bob = (uint32_t)(bw >> (i & 63)) & 1u;
                f2 bo[kDvUnroll];
                if (it == 0) {
                    // the folded first iteration (fold_first_message, :256-267,
                    // :303-316), exact as the split kernel's FOLD path
                    const uint32_t sgi = bob ^ lsign;
                    double acc = bob ? -llr_p : llr_p;
                    double cv[kDvUnroll];
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) {
                        const int j = jc[k];
                        const uint32_t sp = (cur.qw[k] >> (j & 31)) & 1u;
                        const double cm = ctab[((uint32_t)(bc >> (50 + 4 * k)) & 15u) + 1u];
                        cv[k] = k < deg ? ((sp ^ sgi) ? -cm : cm) : 0.0;
                    }
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) acc = k < deg ? acc + cv[k] : acc;
                    z = acc <= 0;
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) bo[k] = qkds::iv_of(clamp_msg(acc - cv[k], a.thr));
                } else {
                    // intervals (spec_bit_phase's general form)
                    const f2 L = bob ? f2{-a.lp_up, -a.lp_dn} : f2{a.lp_dn, a.lp_up};
                    const float pinf = a.pinf;
                    auto amax = [pinf](f2 x) { return __builtin_amdgcn_fmed3f(x.y, -x.x, pinf); };
                    f2 cs[kDvUnroll];
                    f2 T = L;
                    float mag = amax(L);
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) {
                        cs[k] = k < deg ? qkds::unpack_iv(cur.v[k]) : f2{0.0f, 0.0f};
                        T = T + cs[k];
                        mag = mag + amax(cs[k]);
                    }
                    const float mg = mag * ((float)(kDvUnroll + 2) * qkds::kSumRel) + 1.0e-30f;
                    T = T + f2{-mg, mg};
                    const bool z1 = T.y <= 0.0f;
                    unc = !(z1 || T.x > 0.0f);
                    z = z1;
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k) {
                        f2 e = L + f2{-mg, mg};
#pragma unroll
                        for (int m = 0; m < kDvUnroll; ++m)
                            if (m != k) e = e + cs[m];
                        bo[k] = f2{__builtin_amdgcn_fmed3f(e.x, -a.thr_up, a.thr_dn),
                                   __builtin_amdgcn_fmed3f(e.y, -a.thr_dn, a.thr_up)};
                    }
                }
                const uint32_t al = (uint32_t)(aw >> (i & 63)) & 1u;
                z = act && z;
                unc = act && unc;
                dif = act && (uint32_t)z != al;
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k)
                    st_line((act && keep && k < deg) ? (uint32_t)k * n_pad + (uint32_t)i : ~0u, qkds::pack_iv(bo[k]));
            }
            // the group's 16 columns' decisions: one syndrome atomic per check
            const uint32_t sh = (uint32_t)lane & 48u;
            const uint32_t zm = (uint32_t)(__ballot(z) >> sh) & 0xffffu;
            const uint32_t um = (uint32_t)(__ballot(unc) >> sh) & 0xffffu;
            kmis |= fold_groups(__ballot(dif));
            if (col == 0) {
#pragma unroll
                for (int k = 0; k < kDvUnroll; ++k) {
                    if (k < deg) {
                        const uint32_t s = ((uint32_t)jc[k] & 1u) << 4;
                        if (zm) atomicXor(xsyn + (jc[k] >> 1), zm << s);
                        if (um) atomicOr(xunc + (jc[k] >> 1), um << s);
                    }
                }
            }
            return true;
        };
        BitIn ba, bb;
        bit_load_bc(grp, ba);
        bit_load(grp, ba);
        bit_load_bc(grp + kIlvGroups, bb);
        for (int i = grp;; i += 2 * kIlvGroups) {
            if (!bstep(i, ba, bb)) break;
            if (!bstep(i + kIlvGroups, bb, ba)) break;
        }
        if (lane == 0 && kmis) atomicOr(ctl + kCtlKeyMis, kmis);
        __syncthreads();
        pc.mark(1);

        // ---- syndrome test (:285): per column, a check certainly unsatisfied
        // and a check whose parity is uncertain; xsyn / xunc cleared
        uint32_t mis = 0, un = 0;
        for (uint32_t w = (uint32_t)tid; w < mw2; w += kIlvBlock) {
            const uint32_t u = UG ? atomicExch(xunc + w, 0u) : xunc[w];
            const uint32_t d = (xsyn[w] ^ tsyn[w]) & ~u;
            mis |= d | (d >> 16);
            un |= u | (u >> 16);
            xsyn[w] = 0;
            if constexpr (!UG) xunc[w] = 0;
        }
        mis &= 0xffffu;
        un &= 0xffffu;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mis |= (uint32_t)__shfl_xor((int)mis, o);
            un |= (uint32_t)__shfl_xor((int)un, o);
        }
        if (lane == 0) {
            if (mis) atomicOr(ctl + kCtlMis, mis);
            if (un) atomicOr(ctl + kCtlUnc, un);
        }
        __syncthreads();

        // ---- outcomes (wave 0, lane = column), as decode_split_kernel's: a
        // round stands if no sign was lost and its outcome is certain
        if (tid < 64) {
            bool fin = false;
            if (lane < kIlvCols && ((active >> lane) & 1u)) {
                const uint32_t fc = ctl[kCtlFrame + lane];
                const uint32_t itc = ctl[kCtlIt + lane];
                const bool ab = (ctl[kCtlAbort] >> lane) & 1u;
                const bool mi = (ctl[kCtlMis] >> lane) & 1u;
                const bool un_c = (ctl[kCtlUnc] >> lane) & 1u;
                const bool km = (ctl[kCtlKeyMis] >> lane) & 1u;
                const bool last = itc + 1 >= a.max_it;
                // (a hand-off for an uncertified round counts as a replay, as
                // the split kernel's do: the cross-call policy, decode_keys,
                // and qkd_debug_spec_replays read these counts)
                if (itc != 0 && (ab || (un_c && (!mi || last)))) {
                    a.fb_list[atomicAdd(a.fb_count, 1u)] = fc;       // to the split kernel
                    atomicAdd(a.replay_count, 1u);
                    atomicAdd(a.spec_replays, 1ull);
                    fin = true;
                } else if (!mi || last) {
                    a.iters[fc] = mi ? a.max_it : itc + 1;
                    a.sp_ok[fc] = mi ? 0 : 1;
                    if (a.key_ok) a.key_ok[fc] = km ? 0 : 1;
                    fin = true;
                } else if (itc + 1 >= a.spec_cap) {
                    a.fb_list[atomicAdd(a.fb_count, 1u)] = fc;
                    atomicAdd(a.replay_count, 1u);
                    atomicAdd(a.spec_replays, 1ull);
                    fin = true;
                } else {
                    ctl[kCtlIt + lane] = itc + 1;
                }
            }
            uint32_t need = (uint32_t)__ballot(fin) & 0xffffu;
            // The workgroup's tail: once the queue is drained, a few columns
            // left iterating would cost whole lockstep rounds (every line is
            // fetched whatever the number of live columns) and hold the
            // launch open; their frames go to the split kernel instead
            // (decoded there from the start, exactly)
            const uint32_t remain = active & ~need;
            if (ctl[kCtlDrained] != 0 && remain != 0 && __popc(remain) <= kIlvTail) {
                if (lane < kIlvCols && ((remain >> lane) & 1u))
                    a.fb_list[atomicAdd(a.fb_count, 1u)] = ctl[kCtlFrame + lane];
                need |= remain;
            }
            if (lane == 0) {
                ctl[kCtlAbort] = 0;
                ctl[kCtlKeyMis] = 0;
                ctl[kCtlMis] = 0;
                ctl[kCtlUnc] = 0;
                ctl[kCtlRefill] = 0;
            }
            if (need) assign(need);
            // the columns whose next round is an interval one
            const bool iv = lane < kIlvCols && ((ctl[kCtlActive] >> lane) & 1u) && ctl[kCtlIt + lane] != 0;
            const uint32_t ivm = (uint32_t)__ballot(iv) & 0xffffu;
            if (lane == 0) ctl[kCtlIvl] = ivm;
        }
        __syncthreads();
        pc.mark(2);
        refill();
    }
}

template <bool TG, bool UG>
static DecodeFn pick_ilv_dc(int rs, int max_dc) {
    if (rs > 8) return decode_ilv_kernel<16, 16, TG, UG>;
    if (max_dc <= 4) return decode_ilv_kernel<8, 4, TG, UG>;
    if (max_dc <= 6) return decode_ilv_kernel<8, 6, TG, UG>;
    return decode_ilv_kernel<8, 8, TG, UG>;
}

DecodeFn pick_ilv(int rs, int max_dc, bool tsyn_global, bool xunc_global) {
    if (xunc_global) return pick_ilv_dc<true, true>(rs, max_dc);
    return tsyn_global ? pick_ilv_dc<true, false>(rs, max_dc) : pick_ilv_dc<false, false>(rs, max_dc);
}

}  // namespace qkd
