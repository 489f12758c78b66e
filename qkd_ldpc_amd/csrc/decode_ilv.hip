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

namespace {

constexpr int kIlvGroups = kDecodeBlock / kIlvCols;     // 16-lane groups per workgroup

// ctl words (IlvLds::ctl)
constexpr int kCtlFrame = 0;      // [16] frame of each column (n_frames: none)
constexpr int kCtlIt = 16;        // [16] the column's current iteration (0: the folded first)
constexpr int kCtlActive = 32;    // columns with a frame
constexpr int kCtlAbort = 33;     // this round: columns whose check phase lost a sign
constexpr int kCtlKeyMis = 34;    // this round: columns whose decision differs from Alice's key
constexpr int kCtlMis = 35;       // this round: columns with a check certainly unsatisfied
constexpr int kCtlUnc = 36;       // this round: columns with a check whose parity is uncertain
constexpr int kCtlRefill = 37;    // columns given a new frame (their target syndromes to load)

__device__ __forceinline__ qkds::f2 neg_if(bool neg, qkds::f2 v) {
    return qkds::f2{neg ? -v.y : v.x, neg ? -v.x : v.y};
}

// the 16-bit column mask of a wave ballot: the OR of its four groups
__device__ __forceinline__ uint32_t fold_groups(uint64_t b) {
    return (uint32_t)(b | (b >> 16) | (b >> 32) | (b >> 48)) & 0xffffu;
}

}  // namespace

// RS: the row stride of DeviceCode::ilv_slots; DM: the largest check degree
// rounded up to even (the register arrays' size)
template <int RS, int DM>
__global__ __launch_bounds__(kDecodeBlock) void decode_ilv_kernel(DecodeArgs a) {
    static_assert(DM <= RS && DM % 2 == 0, "degree bucket");
    using qkds::f2;
    extern __shared__ __align__(16) unsigned char smem[];
    const DeviceCode& c = a.code;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t col = (uint32_t)tid & (kIlvCols - 1);
    const int grp = tid / kIlvCols;
    const IlvLds L(c.m);
    const uint32_t mw2 = (uint32_t)(c.m + 1) >> 1;
    uint32_t* tsyn = reinterpret_cast<uint32_t*>(smem + L.tsyn);
    uint32_t* xsyn = reinterpret_cast<uint32_t*>(smem + L.xsyn);
    uint32_t* xunc = reinterpret_cast<uint32_t*>(smem + L.xunc);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + L.ctl);
    double* ctab = reinterpret_cast<double*>(smem + L.ctab);
    const uint32_t m_words = (uint32_t)decode_m_words(c.m);
    const uint32_t n_pad = (uint32_t)c.n_pad;
    double* const lines = a.ilv_store + (size_t)blockIdx.x * a.ilv_stride;
    // after the lines: the columns' key words, interleaved ([word][column]
    // {bob, alice}), copied at each refill
    uint4* const keyi = reinterpret_cast<uint4*>(lines + (size_t)c.max_dv * n_pad * kIlvCols);
    const uint32_t lsign = (uint32_t)qkdm::hi32(a.log_p) >> 31;
    const double llr_p = a.log_p;

    for (int d = tid; d <= kFirstTableDeg; d += kDecodeBlock) ctab[d] = a.first_c2b[d];
    for (uint32_t w = (uint32_t)tid; w < mw2; w += kDecodeBlock) {
        tsyn[w] = 0;
        xsyn[w] = 0;
        xunc[w] = 0;
    }
    if (tid < kIlvCtlWords) ctl[tid] = 0;
    __syncthreads();

    // wave 0: the columns in `need` take the next frames of the queue (one
    // atomic for all of them); the active and refill masks follow
    auto assign = [&](uint32_t need) {
        const uint32_t cnt = (uint32_t)__popc(need);
        uint32_t base = 0;
        if (lane == 0 && cnt) base = atomicAdd(a.counter, cnt);
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
        for (uint32_t w = (uint32_t)tid; w < mw2; w += kDecodeBlock) {
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
            for (uint32_t w = (uint32_t)tid; w < a.words; w += kDecodeBlock) {
                const uint64_t b = a.bob_w[(size_t)f * a.words + w], al = a.alice_w[(size_t)f * a.words + w];
                keyi[(size_t)w * kIlvCols + cc] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)al,
                                                             (uint32_t)(al >> 32));
            }
        }
    };
    if (tid < 64) assign((1u << kIlvCols) - 1u);
    __syncthreads();
    refill();

    for (;;) {
        __syncthreads();
        const uint32_t active = ctl[kCtlActive];
        if (active == 0) break;
        const uint32_t f = ctl[kCtlFrame + col];
        const uint32_t it = ctl[kCtlIt + col];
        const bool act = (active >> col) & 1u;

        // ---- check phase (columns past their folded first iteration).
        // Software-pipelined over the group's checks j, j + G, ...: the lines of
        // the next check are loaded while this one computes, its line indices
        // a check earlier still.
        bool bad = false;
        if (act && it != 0) {
            auto load_idx = [&](int jj, uint32_t (&x)[DM], int& deg) {
                deg = 0;
#pragma unroll
                for (int k = 0; k < DM; ++k) x[k] = 0;
                if (jj < c.m) {
                    deg = c.chk_deg[jj];
                    const uint2* sl = reinterpret_cast<const uint2*>(c.ilv_slots + (size_t)jj * RS);
#pragma unroll
                    for (int q = 0; q < DM / 2; ++q) {
                        const uint2 u = sl[q];
                        x[2 * q] = u.x;
                        x[2 * q + 1] = u.y;
                    }
                }
            };
            auto load_lines = [&](const uint32_t (&x)[DM], int deg, double (&v)[DM]) {
#pragma unroll
                for (int k = 0; k < DM; ++k) v[k] = k < deg ? lines[(size_t)x[k] * kIlvCols + col] : 0.0;
            };
            uint32_t xa[DM], xb[DM];
            int dega, degb;
            double va[DM];
            int j = grp;
            load_idx(j, xa, dega);
            load_lines(xa, dega, va);
            load_idx(j + kIlvGroups, xb, degb);
            while (j < c.m) {
                double vb[DM];
                load_lines(xb, degb, vb);
                uint32_t xc[DM];
                int degc;
                load_idx(j + 2 * kIlvGroups, xc, degc);
                // |b2c| bounds (psi units) and signs, two edges per packed
                // evaluation (spec_check_phase_paired's input bounds)
                f2 ph[DM];
                uint32_t negs = 0;
#pragma unroll
                for (int k = 0; k < DM; k += 2) {
                    const f2 b0 = qkds::unpack_iv(va[k]), b1 = qkds::unpack_iv(va[k + 1]);
                    const bool n0 = b0.y < 0.0f, n1 = b1.y < 0.0f;
                    const f2 a0 = neg_if(n0, b0), a1 = neg_if(n1, b1);
                    const bool ok0 = a0.x > 1.0e-30f, ok1 = a1.x > 1.0e-30f;
                    f2 r0 = f2{0.0f, 0.0f}, r1 = f2{0.0f, 0.0f};
                    if (k < dega) qkds::phi_bounds2(a0, a1, r0, r1);
                    const bool in0 = k < dega, in1 = k + 1 < dega;
                    bad |= (in0 && !ok0) || (in1 && !ok1);
                    negs |= (in0 && n0 ? 1u : 0u) << k;
                    negs |= (in1 && n1 ? 1u : 0u) << (k + 1);
                    ph[k] = (in0 && ok0) ? r0 : f2{0.0f, 0.0f};
                    ph[k + 1] = (in1 && ok1) ? r1 : f2{0.0f, 0.0f};
                }
                const uint32_t sbit = (tsyn[j >> 1] >> ((((uint32_t)j & 1u) << 4) + col)) & 1u;
                const uint32_t par = (uint32_t)__popc(negs) & 1u;
                // extrinsic sums over the other edges: prefix + suffix (every
                // term >= 0, zeros past the degree), widened by the binary32
                // roundings and the reference's binary64 ones (split kernel's)
                f2 ext[DM];
                ext[0] = f2{0.0f, 0.0f};
#pragma unroll
                for (int k = 1; k < DM; ++k) ext[k] = ext[k - 1] + ph[k - 1];
                f2 suf = f2{0.0f, 0.0f};
#pragma unroll
                for (int k = DM - 1; k >= 0; --k) {
                    const f2 sum = ext[k] + suf;
                    suf = suf + ph[k];
                    const float mg = __builtin_fmaf(sum.y, (float)(DM + 2) * qkds::kSumRel, qkds::kRefSumAbs);
                    f2 e = sum + f2{-mg, mg};
                    e.x = e.x > 0.0f ? e.x : 0.0f;
                    bad |= k < dega && !(e.y < qkds::kPsiSumMax);
                    ext[k] = e;
                }
                // the c2b bounds, two edges per packed evaluation; threshold_matrix
                // (:246-249) on the magnitude, then the sign
#pragma unroll
                for (int k = 0; k < DM; k += 2) {
                    if (k < dega) {
                        f2 m0, m1;
                        qkds::phi_bounds_out2(ext[k], ext[k + 1], m0, m1);
                        m0.x = __builtin_amdgcn_fmed3f(m0.x, 0.0f, a.thr_dn);
                        m0.y = __builtin_amdgcn_fmed3f(m0.y, 0.0f, a.thr_up);
                        m1.x = __builtin_amdgcn_fmed3f(m1.x, 0.0f, a.thr_dn);
                        m1.y = __builtin_amdgcn_fmed3f(m1.y, 0.0f, a.thr_up);
                        const uint32_t s0 = sbit ^ par ^ ((negs >> k) & 1u);
                        const uint32_t s1 = sbit ^ par ^ ((negs >> (k + 1)) & 1u);
                        lines[(size_t)xa[k] * kIlvCols + col] = qkds::pack_iv(neg_if(s0 != 0u, m0));
                        if (k + 1 < dega) lines[(size_t)xa[k + 1] * kIlvCols + col] = qkds::pack_iv(neg_if(s1 != 0u, m1));
                    }
                }
#pragma unroll
                for (int k = 0; k < DM; ++k) {
                    xa[k] = xb[k];
                    xb[k] = xc[k];
                    va[k] = vb[k];
                }
                dega = degb;
                degb = degc;
                j += kIlvGroups;
            }
        }
        {
            const uint32_t bm = fold_groups(__ballot(bad));
            if (lane == 0 && bm) atomicOr(ctl + kCtlAbort, bm);
        }
        __syncthreads();

        // ---- bit phase
        const bool keep = it + 1 < a.max_it;
        uint32_t kmis = 0;
        for (int i = grp; i < c.n; i += kIlvGroups) {
            const uint64_t bc = c.bit_code[i];
            const int deg = (int)(bc >> 48) & 3;
            int32_t jc[kDvUnroll];
#pragma unroll
            for (int k = 0; k < kDvUnroll; ++k) jc[k] = (int32_t)(bc >> (16 * k)) & 0xffff;
            bool z = false, unc = false, dif = false;
            if (act) {
                // (this column's Bob and Alice words of bit i, from the
                // workgroup's interleaved copy: one 256-byte run per group)
                const uint4 kw = keyi[(size_t)(i >> 6) * kIlvCols + col];
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
                        const uint32_t qw = a.synw[(size_t)f * 2 * m_words + m_words + ((uint32_t)j >> 5)];
                        const uint32_t sp = (qw >> (j & 31)) & 1u;
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
                        cs[k] = k < deg ? qkds::unpack_iv(lines[((size_t)k * n_pad + (uint32_t)i) * kIlvCols + col])
                                        : f2{0.0f, 0.0f};
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
                dif = (uint32_t)z != al;
                if (keep) {
#pragma unroll
                    for (int k = 0; k < kDvUnroll; ++k)
                        if (k < deg) lines[((size_t)k * n_pad + (uint32_t)i) * kIlvCols + col] = qkds::pack_iv(bo[k]);
                }
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
        }
        if (lane == 0 && kmis) atomicOr(ctl + kCtlKeyMis, kmis);
        __syncthreads();

        // ---- syndrome test (:285): per column, a check certainly unsatisfied
        // and a check whose parity is uncertain; xsyn / xunc cleared
        uint32_t mis = 0, un = 0;
        for (uint32_t w = (uint32_t)tid; w < mw2; w += kDecodeBlock) {
            const uint32_t u = xunc[w];
            const uint32_t d = (xsyn[w] ^ tsyn[w]) & ~u;
            mis |= d | (d >> 16);
            un |= u | (u >> 16);
            xsyn[w] = 0;
            xunc[w] = 0;
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
                if (itc != 0 && (ab || (un_c && (!mi || last)))) {
                    a.fb_list[atomicAdd(a.fb_count, 1u)] = fc;       // to the split kernel
                    fin = true;
                } else if (!mi || last) {
                    a.iters[fc] = mi ? a.max_it : itc + 1;
                    a.sp_ok[fc] = mi ? 0 : 1;
                    if (a.key_ok) a.key_ok[fc] = km ? 0 : 1;
                    fin = true;
                } else if (itc + 1 >= a.spec_cap) {
                    a.fb_list[atomicAdd(a.fb_count, 1u)] = fc;
                    fin = true;
                } else {
                    ctl[kCtlIt + lane] = itc + 1;
                }
            }
            const uint32_t need = (uint32_t)__ballot(fin) & 0xffffu;
            if (lane == 0) {
                ctl[kCtlAbort] = 0;
                ctl[kCtlKeyMis] = 0;
                ctl[kCtlMis] = 0;
                ctl[kCtlUnc] = 0;
                ctl[kCtlRefill] = 0;
            }
            if (need) assign(need);
        }
        __syncthreads();
        refill();
    }
}

DecodeFn pick_ilv(int rs, int max_dc) {
    if (rs > 8) return decode_ilv_kernel<16, 16>;
    if (max_dc <= 4) return decode_ilv_kernel<8, 4>;
    if (max_dc <= 6) return decode_ilv_kernel<8, 6>;
    return decode_ilv_kernel<8, 8>;
}

}  // namespace qkd
