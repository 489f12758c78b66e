// qkd_spec.h — certified interval arithmetic for speculative decoding.
//
// The speculative pass of decode_split_kernel (decode_split.hip) runs the
// reference's flooding sum-product iterations on binary32 INTERVALS instead
// of binary64 messages: every interval is guaranteed to contain the message
// the reference computes in binary64 (src/qkd_ldpc_algorithm.cpp:220-316,
// glibc tanh/atanh, its operation order and roundings). Whenever every hard
// decision's sign is certain, the hard decisions, the syndrome test and
// therefore the iteration count are exactly the reference's; the first time
// a sign is not certain the frame is decoded again with the exact binary64
// kernel path. Outputs are bit-exact either way; only the internal messages
// of the speculative pass are approximate.
//
// The check rule is evaluated in Gallager's form. For b2c values b_k (of
// known sign, magnitudes |b_k|) and target bit s_j, the reference's message
//   c2b = clamp(2 atanh(P / t_self)),  P = (s_j ? -1 : 1) prod_k tanh(b_k / 2)
// equals, in exact arithmetic, sigma * phi(sum_{k != self} phi(|b_k|)) with
//   phi(x) = -ln tanh(x / 2) = 2 atanh(e^-x)        (x > 0; decreasing, convex, phi(phi(x)) = x)
//   sigma  = s_j xor (sign bits of the other b_k)
// The reference's binary64 roundings (d glibc tanh calls of e_t ulp each,
// d - 1 products and one division of half an ulp, one atanh of e_a ulp) move
// the phi-domain sum by an ABSOLUTE (2 d e_t + d) 2^-53 + e_a 2^-52 at most,
// including a tanh that rounds to exactly 1; with e_t, e_a <= 3 ulp (glibc
// measures 2.15 / 1.62 against x87 80-bit, tests/test_spec_bounds.py) that is
// 1.3e-14 for d = 16, the largest check degree the kernel takes. It is absorbed
// by widening that sum by kRefSumAbs (2.8e-14 in the phi domain); this also covers the saturated cases where the reference's
// P / t is exactly +-1 (message +-inf, clamped to +-thr): the widened sum then
// reaches 0 and the upper bound becomes inf (then thr).
//
// binary32 evaluation errors: phi_core's value and slope are within a few ulp
// (hardware v_exp_f32 / v_log_f32 after an exact argument split); every bound
// is widened by kPhiRel (2^-20, ~8 ulp; measured use under a third of it)
// relative plus tiny absolute terms.
// tests/test_spec.py checks phi bounds against a binary64 phi on a dense sweep
// and reports the headroom.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qkds {

constexpr float kPhiRel = 0x1.0p-20f;      // relative error allowance of one phi bound (~8 ulp)
constexpr float kSumRel = 0x1.0p-23f;      // relative allowance per binary32 add (2^-24 is the rounding)
// The check rule sums psi = phi / ln 2 (the log2 domain): the input bounds are
// produced in it (no ln 2 scaling after the log) and the output evaluation
// takes 2^-S directly (no argument split).
constexpr float kLn2 = 0.693147180559945f;
constexpr float kInvLn2 = 1.44269504088896f;
constexpr float kRefSumAbs = 4.0e-14f;     // reference roundings (2.8e-14 in the phi domain), psi units
constexpr float kPhiHuge = 80.0f;          // phi evaluated at most here (e^-80: a normal binary32)
// phi_pair evaluates its input bound at no less than this: the check phase
// certifies only |b2c| > 1e-30, so the bounds of smaller inputs are never used
constexpr float kPhiTiny = 1.0e-30f;
constexpr float kPsiHuge = 115.0f;         // the same bound for psi-unit sums (115 ln 2 < 80)
constexpr float kPsiSumMax = 865.0f;       // 600 / ln 2: the reference's product would underflow

typedef float f2 __attribute__((ext_vector_type(2)));   // [lo, hi]; packed binary32 ops

// The two series of phi_core, for a binary32 value or a packed pair (every
// operation elementwise, so a pair's halves are bit for bit the scalar
// results), in Horner's form:
//   series_h(s) ~ atanh(sqrt s) / sqrt s    (2 atanh(u) = 2u h, s = u^2 <= e^-2)
//   series_g(y), below
// Degree-4 near-minimax fits with binary32 coefficients
// (tools/phi_poly_fit.py): series_h at most 7.2e-8 relative error including
// the binary32 Horner evaluation, below the Taylor degree-6 form it replaced
// (1.2e-7) with two operations fewer; 2^-20 (kPhiRel) bounds the whole
// evaluation, certified over every binary32 input on the GPU
// (tests/test_spec.py::test_phi_bounds_exhaustive).
// (Estrin's scheme, depth 2 for one more operation each, measured slower per
// config-2 batch at degree 6: DESIGN.md §4.3.)
template <typename V>
__device__ __forceinline__ V poly4(V z, float c0, float c1, float c2, float c3, float c4) {
    V p = __builtin_elementwise_fma(z, V(c4), V(c3));
    p = __builtin_elementwise_fma(z, p, V(c2));
    p = __builtin_elementwise_fma(z, p, V(c1));
    return __builtin_elementwise_fma(z, p, V(c0));
}
// g(y) = -ln(tanh(t) / t), t = sqrt(y) / 2: phi(x) = ln 2 - ln x + g(x^2)
// for x < 1 (y < 1; g(0) = 0, g < 0.081), degree 4 without a constant term,
// 1.3e-8 absolute at most with binary32 Horner evaluation (tools/phi_poly_fit.py)
template <typename V>
__device__ __forceinline__ V series_g(V y) {
    V p = __builtin_elementwise_fma(y, V(-0x1.6bf16ap-16f), V(0x1.627b52p-12f));
    p = __builtin_elementwise_fma(y, p, V(-0x1.3e8026p-8f));
    p = __builtin_elementwise_fma(y, p, V(0x1.555536p-4f));
    return y * p;
}
template <typename V>
__device__ __forceinline__ V series_h(V s) {
    return poly4(s, 1.0f, 0x1.55549p-2f, 0x1.9a05a2p-3f, 0x1.1b7792p-3f, 0x1.2e9afep-3f);
}
// phi's constant below x = 1 for a log taken of x / ln 2 (a psi-unit sum):
// phi = ln 2 - ln x + g = (ln 2 - ln ln 2) - ln 2 log2(x / ln 2) + g
constexpr float kPhiK = 1.05966010f;

// phi (PSI: phi / ln 2) and an upper bound of |phi'(x)| = 1 / sinh(x) at
// 0 < x <= kPhiHuge from u = e^-x (accurate), x (for g, the slope and the
// branch) and lg = log2 of the log's argument: of x itself (LGP false) or of
// P = x / ln 2, the psi-unit sum the output bound starts from (LGP true; x is
// then the rounded P ln 2, which only feeds g, the slope and the branch).
struct PhiVal {
    float v;
    float slope;
};

template <bool PSI, bool LGP>
__device__ __forceinline__ PhiVal phi_core(float x, float u, float lg) {
    static_assert(PSI != LGP, "psi values of a natural argument, or phi values of a psi-unit one");
    // x < 1: phi = ln 2 - ln x + g(x^2) (psi: 1 - log2 x + g / ln 2): one
    // log of the argument itself, off the polynomial's path (v_log_f32 is
    // accurate to ~2^-22 absolute near 1, under a quarter of kPhiRel there)
    const float g = series_g(x * x);
    const float t = __builtin_fmaf(PSI ? -1.0f : -kLn2, lg, PSI ? 1.0f : kPhiK);
    const float vlo = __builtin_fmaf(g, PSI ? kInvLn2 : 1.0f, t);
    // x >= 1: phi = 2 atanh(u) = 2u series_h(s), s = u^2 <= e^-2 (7.2e-8
    // relative at most, under 8 % of kPhiRel)
    const float s = u * u;
    const float h = series_h(s);
    const float vhi = (u * (PSI ? 2.0f * kInvLn2 : 2.0f)) * h;
    PhiVal o;
    o.v = x < 1.0f ? vlo : vhi;
    // |phi'(x)| = 1 / sinh(x): below x = 1 at most 1 / x (sinh x > x), from x
    // = 1 on 2u / (1 - u^2) <= 2u / (1 - e^-2) < 2.32 u (tangents need an
    // upper bound only)
    o.slope = x < 1.0f ? __builtin_amdgcn_rcpf(x) : 2.32f * u;
    return o;
}

// u = e^-x = 2^-(x log2 e), argument split so the reduction is exact to
// ~2^-48: p = fl(x * L), r = x * L - p (fma, exact) + x * L_lo, and
// 2^-(p + r) = 2^-p (1 - r ln2 + ...), |r| < 2^-17 (r ln2 formed directly)
__device__ __forceinline__ float exp_neg(float x) {
    const float L = 1.44269502162933349609375f;          // log2(e) rounded to binary32
    const float L_lo = 1.925963033500011079e-08f;        // log2(e) - L
    const float p = x * L;
    const float rl = __builtin_fmaf(__builtin_fmaf(x, L, -p), kLn2, x * (L_lo * kLn2));
    const float e2 = __builtin_amdgcn_exp2f(-p);
    return __builtin_fmaf(e2, -rl, e2);
}

// Bounds of psi = phi / ln 2 over [a, b], 0 < a <= b (finite or +inf):
// lo <= psi(x) <= hi. phi is decreasing and convex: phi(a) is the maximum,
// and the tangent at a lies below phi, so phi(a) - (b - a) / sinh(a) is a
// lower bound. Past kPhiHuge both come from a' = kPhiHuge <= a: phi(a')
// bounds phi(a) above, and the tangent at a' stays below phi on [a', b].
__device__ __forceinline__ f2 phi_bounds(float a, float b) {
    const float a1 = __builtin_amdgcn_fmed3f(a, 0.0f, kPhiHuge);     // min(a, kPhiHuge), a > 0
    const PhiVal e = phi_core<true, false>(a1, exp_neg(a1), __builtin_amdgcn_logf(a1));
    const float hi = __builtin_fmaf(e.v, kPhiRel, e.v) + 1.0e-37f;
    const float t = __builtin_fmaf(-e.slope * ((1.0f + 2.0f * kPhiRel) * kInvLn2), b - a1, e.v * (1.0f - kPhiRel));
    return f2{t > 0.0f ? t : 0.0f, hi};     // lo: also for b = inf (t = -inf) and NaN
}
__device__ __forceinline__ void phi_bounds(float a, float b, float& lo, float& hi) {
    const f2 r = phi_bounds(a, b);
    lo = r.x;
    hi = r.y;
}

// Bounds of phi(S) over psi-unit sums [P_lo, P_hi] (S = P ln 2), 0 <= P_lo
// <= P_hi: at P_lo = 0 (the widened sum reached zero) the maximum is +inf and
// the minimum is taken at P_hi; otherwise one evaluation at P_lo and its
// tangent (both clamped to kPsiHuge as in phi_bounds). u = 2^-P needs no
// argument split, the log is taken of P itself; x = P ln 2 (rounded) only
// feeds g, the slope and the branch.
__device__ __forceinline__ f2 phi_bounds_out(float s_lo, float s_hi) {
    const bool zero = !(s_lo > 0.0f);
    const float at = __builtin_fminf(zero ? s_hi : s_lo, kPsiHuge);
    const PhiVal e = phi_core<false, true>(at * kLn2, __builtin_amdgcn_exp2f(-at), __builtin_amdgcn_logf(at));
    const float vmax = __builtin_fmaf(e.v, kPhiRel, e.v) + 1.0e-37f;
    const float tan = __builtin_fmaf(-e.slope * ((1.0f + 2.0f * kPhiRel) * kLn2), s_hi - at, e.v * (1.0f - kPhiRel));
    return f2{tan > 0.0f ? tan : 0.0f, zero ? __builtin_inff() : vmax};
}
__device__ __forceinline__ void phi_bounds_out(float s_lo, float s_hi, float& lo, float& hi) {
    const f2 r = phi_bounds_out(s_lo, s_hi);
    lo = r.x;
    hi = r.y;
}

// phi_core twice, in the two halves of the packed binary32 unit: half 0
// phi_core<true, false> (psi values of a natural argument), half 1
// phi_core<false, true> (phi values of a psi-unit one), or, PSI1, both
// phi_core<true, false>; every operation is phi_core's, so each half is bit
// for bit its result.
struct PhiVal2 {
    f2 v;
    f2 slope;
};
template <bool PSI1 = false>   // half 1 in psi units of a natural argument too
__device__ __forceinline__ PhiVal2 phi_core_pair(f2 x, f2 u, f2 lg) {
    const f2 g = series_g(x * x);
    const f2 t = __builtin_elementwise_fma(f2{-1.0f, PSI1 ? -1.0f : -kLn2}, lg, f2{1.0f, PSI1 ? 1.0f : kPhiK});
    const f2 vlo = __builtin_elementwise_fma(g, f2{kInvLn2, PSI1 ? kInvLn2 : 1.0f}, t);
    const f2 s = u * u;
    const f2 h = series_h(s);
    const f2 vhi = (u * f2{2.0f * kInvLn2, PSI1 ? 2.0f * kInvLn2 : 2.0f}) * h;
    const f2 sh = f2(2.32f) * u;
    PhiVal2 o;
    o.v = f2{x.x < 1.0f ? vlo.x : vhi.x, x.y < 1.0f ? vlo.y : vhi.y};
    o.slope = f2{x.x < 1.0f ? __builtin_amdgcn_rcpf(x.x) : sh.x, x.y < 1.0f ? __builtin_amdgcn_rcpf(x.y) : sh.y};
    return o;
}

// phi_bounds and phi_bounds_out evaluated together, one in each half of the
// packed binary32 unit (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 issue at
// almost the cost of one scalar instruction for both halves): the check
// phase pairs the input bound of one task's edge (half 0, psi units) with the
// output bound of the previous task's edge (half 1). Every operation is the
// one the scalar forms above perform, so each half is bit for bit their
// result (tests/test_spec.py compares them); only the transcendentals, the
// selects and the argument split of half 0 stay scalar.
__device__ __forceinline__ void phi_pair(float a, float b, float s_lo, float s_hi, f2& in, f2& out) {
    // evaluation points: phi_bounds at a1 = min(a, kPhiHuge); phi_bounds_out
    // at P = min(s_lo, kPsiHuge) (s_hi when the sum reached zero), x = P ln 2
    // (at no less than kPhiTiny: an input the check phase does not certify,
    // a <= 1e-30, still gives finite bounds -- the dummy column's 0)
    const float a1 = __builtin_amdgcn_fmed3f(a, kPhiTiny, kPhiHuge);
    const bool zero = !(s_lo > 0.0f);
    const float P = __builtin_fminf(zero ? s_hi : s_lo, kPsiHuge);
    // u = e^-x: half 0 by exp_neg's argument split, half 1 = 2^-P
    const float L = 1.44269502162933349609375f;
    const float L_lo = 1.925963033500011079e-08f;
    const float p0 = a1 * L;
    const float rl = __builtin_fmaf(__builtin_fmaf(a1, L, -p0), kLn2, a1 * (L_lo * kLn2));
    const f2 e2 = f2{__builtin_amdgcn_exp2f(-p0), __builtin_amdgcn_exp2f(-P)};
    const f2 u = f2{__builtin_fmaf(e2.x, -rl, e2.x), e2.y};
    const PhiVal2 e = phi_core_pair(f2{a1, P * kLn2}, u, f2{__builtin_amdgcn_logf(a1), __builtin_amdgcn_logf(P)});
    const f2 v = e.v, slope = e.slope;
    // the bounds: phi(a) widened up; the tangent at the evaluation point, down
    const f2 hi = __builtin_elementwise_fma(v, f2(kPhiRel), v) + f2(1.0e-37f);
    // (the interval widths elementwise: two scalar subtractions straight into
    // the pair, where a packed one needs both operand pairs assembled first)
    // (each an empty asm's operand: left alone, the SLP vectorizer packs the
    // two into a v_pk_add_f32 whose operand pairs take two moves to build)
    float d0 = b - a1, d1 = s_hi - P;
    asm("" : "+v"(d0));
    asm("" : "+v"(d1));
    const f2 dd = f2{d0, d1};
    const f2 tn = __builtin_elementwise_fma(
        -slope * f2{(1.0f + 2.0f * kPhiRel) * kInvLn2, (1.0f + 2.0f * kPhiRel) * kLn2}, dd,
        v * f2(1.0f - kPhiRel));
    in = f2{tn.x > 0.0f ? tn.x : 0.0f, hi.x};
    out = f2{tn.y > 0.0f ? tn.y : 0.0f, zero ? __builtin_inff() : hi.y};
}

// An interval enclosing a finite binary64 value: its binary32 rounding
// widened by 2^-22 relative (twice the rounding error and the widening's own)
// and 1e-38 absolute (0 and subnormals give an interval containing 0).
__device__ __forceinline__ f2 iv_of(double x) {
    const float f = (float)x;
    const float a = __builtin_fabsf(f);
    return f2{__builtin_fmaf(a, -0x1.0p-22f, f) - 1.0e-38f, __builtin_fmaf(a, 0x1.0p-22f, f) + 1.0e-38f};
}

// The folded first bit phase's b2c are exact binary64 values: it stores, in
// place of their intervals, the psi bounds the next check phase would compute
// from those intervals (bit for bit the same), with the sign of b2c carried by
// the low word: [lo, hi] for b2c > 0, [-hi, -lo] for b2c < 0 (hi > 0, so the
// low word is negative exactly then); NaN for a b2c whose sign is not certain
// (0 or NaN: the check phase aborts the round).
__device__ __forceinline__ f2 psi_of_exact(double b) {
    const f2 iv = iv_of(b);
    const bool neg = iv.y < 0.0f;
    const f2 ab = neg ? -iv.yx : iv;
    const bool ok = (neg || iv.x > 0.0f) && ab.x > 1.0e-30f;
    const f2 ph = phi_bounds(ab.x, ab.y);
    return ok ? (neg ? -ph.yx : ph) : f2{__builtin_nanf(""), __builtin_nanf("")};
}

// psi_of_exact of two values in one packed evaluation (phi_bounds' operations
// in each half: bit for bit psi_of_exact of each).
__device__ __forceinline__ void psi_of_exact2(double b0, double b1, f2& r0, f2& r1) {
    const f2 i0 = iv_of(b0), i1 = iv_of(b1);
    const bool n0 = i0.y < 0.0f, n1 = i1.y < 0.0f;
    const f2 a0 = n0 ? -i0.yx : i0, a1 = n1 ? -i1.yx : i1;
    const bool ok0 = (n0 || i0.x > 0.0f) && a0.x > 1.0e-30f;
    const bool ok1 = (n1 || i1.x > 0.0f) && a1.x > 1.0e-30f;
    // phi_bounds(a.x, a.y) in both halves: exp_neg's argument split, phi_core
    const f2 x = f2{__builtin_amdgcn_fmed3f(a0.x, 0.0f, kPhiHuge), __builtin_amdgcn_fmed3f(a1.x, 0.0f, kPhiHuge)};
    const float L = 1.44269502162933349609375f;
    const float L_lo = 1.925963033500011079e-08f;
    const f2 p = x * f2(L);
    const f2 rl = __builtin_elementwise_fma(__builtin_elementwise_fma(x, f2(L), -p), f2(kLn2), x * f2(L_lo * kLn2));
    const f2 e2 = f2{__builtin_amdgcn_exp2f(-p.x), __builtin_amdgcn_exp2f(-p.y)};
    const f2 u = __builtin_elementwise_fma(e2, -rl, e2);
    const PhiVal2 e = phi_core_pair<true>(x, u, f2{__builtin_amdgcn_logf(x.x), __builtin_amdgcn_logf(x.y)});
    const f2 hi = __builtin_elementwise_fma(e.v, f2(kPhiRel), e.v) + f2(1.0e-37f);
    const f2 t = __builtin_elementwise_fma(-e.slope * f2((1.0f + 2.0f * kPhiRel) * kInvLn2), f2{a0.y, a1.y} - x,
                                           e.v * f2(1.0f - kPhiRel));
    const f2 ph0 = f2{t.x > 0.0f ? t.x : 0.0f, hi.x}, ph1 = f2{t.y > 0.0f ? t.y : 0.0f, hi.y};
    const float nan = __builtin_nanf("");
    r0 = ok0 ? (n0 ? -ph0.yx : ph0) : f2{nan, nan};
    r1 = ok1 ? (n1 ? -ph1.yx : ph1) : f2{nan, nan};
}

// phi_bounds of two intervals [a.x, a.y] and [b.x, b.y] in one packed
// evaluation (the operations of psi_of_exact2's core: each half bit for bit
// phi_bounds). The frame-interleaved check phase (decode_ilv.hip) pairs its
// edges with it.
__device__ __forceinline__ void phi_bounds2(f2 a, f2 b, f2& ra, f2& rb) {
    const f2 x = f2{__builtin_amdgcn_fmed3f(a.x, 0.0f, kPhiHuge), __builtin_amdgcn_fmed3f(b.x, 0.0f, kPhiHuge)};
    const float L = 1.44269502162933349609375f;
    const float L_lo = 1.925963033500011079e-08f;
    const f2 p = x * f2(L);
    const f2 rl = __builtin_elementwise_fma(__builtin_elementwise_fma(x, f2(L), -p), f2(kLn2), x * f2(L_lo * kLn2));
    const f2 e2 = f2{__builtin_amdgcn_exp2f(-p.x), __builtin_amdgcn_exp2f(-p.y)};
    const f2 u = __builtin_elementwise_fma(e2, -rl, e2);
    const PhiVal2 e = phi_core_pair<true>(x, u, f2{__builtin_amdgcn_logf(x.x), __builtin_amdgcn_logf(x.y)});
    const f2 hi = __builtin_elementwise_fma(e.v, f2(kPhiRel), e.v) + f2(1.0e-37f);
    const f2 t = __builtin_elementwise_fma(-e.slope * f2((1.0f + 2.0f * kPhiRel) * kInvLn2), f2{a.y, b.y} - x,
                                           e.v * f2(1.0f - kPhiRel));
    ra = f2{t.x > 0.0f ? t.x : 0.0f, hi.x};
    rb = f2{t.y > 0.0f ? t.y : 0.0f, hi.y};
}

// phi_bounds_out of two psi-unit sums [s.x, s.y] and [r.x, r.y] in one packed
// evaluation: phi_core<false, true>'s operations elementwise, each half bit
// for bit phi_bounds_out.
__device__ __forceinline__ void phi_bounds_out2(f2 s, f2 r, f2& os, f2& orr) {
    const bool z0 = !(s.x > 0.0f), z1 = !(r.x > 0.0f);
    const f2 at = f2{__builtin_fminf(z0 ? s.y : s.x, kPsiHuge), __builtin_fminf(z1 ? r.y : r.x, kPsiHuge)};
    const f2 x = at * f2(kLn2);
    const f2 u = f2{__builtin_amdgcn_exp2f(-at.x), __builtin_amdgcn_exp2f(-at.y)};
    const f2 lg = f2{__builtin_amdgcn_logf(at.x), __builtin_amdgcn_logf(at.y)};
    const f2 g = series_g(x * x);
    const f2 t = __builtin_elementwise_fma(f2(-kLn2), lg, f2(kPhiK));
    const f2 vlo = __builtin_elementwise_fma(g, f2(1.0f), t);
    const f2 h = series_h(u * u);
    const f2 vhi = (u * f2(2.0f)) * h;
    const f2 v = f2{x.x < 1.0f ? vlo.x : vhi.x, x.y < 1.0f ? vlo.y : vhi.y};
    const f2 sh = f2(2.32f) * u;
    const f2 slope = f2{x.x < 1.0f ? __builtin_amdgcn_rcpf(x.x) : sh.x, x.y < 1.0f ? __builtin_amdgcn_rcpf(x.y) : sh.y};
    const f2 vmax = __builtin_elementwise_fma(v, f2(kPhiRel), v) + f2(1.0e-37f);
    const f2 tn = __builtin_elementwise_fma(-slope * f2((1.0f + 2.0f * kPhiRel) * kLn2), f2{s.y, r.y} - at,
                                            v * f2(1.0f - kPhiRel));
    os = f2{tn.x > 0.0f ? tn.x : 0.0f, z0 ? __builtin_inff() : vmax.x};
    orr = f2{tn.y > 0.0f ? tn.y : 0.0f, z1 ? __builtin_inff() : vmax.y};
}

// An interval travels through the double-width message slots as its bits.
__device__ __forceinline__ double pack_iv(f2 v) { return __builtin_bit_cast(double, v); }
__device__ __forceinline__ f2 unpack_iv(double v) { return __builtin_bit_cast(f2, v); }
__device__ __forceinline__ double pack_iv(float lo, float hi) {
    return __builtin_bit_cast(double, ((uint64_t)__builtin_bit_cast(uint32_t, hi) << 32) |
                                          (uint64_t)__builtin_bit_cast(uint32_t, lo));
}
__device__ __forceinline__ float iv_lo(double v) {
    return __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(uint64_t, v));
}
__device__ __forceinline__ float iv_hi(double v) {
    return __builtin_bit_cast(float, (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32));
}

}  // namespace qkds
