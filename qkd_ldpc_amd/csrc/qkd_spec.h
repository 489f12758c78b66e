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
// The reference's binary64 roundings (tanh, the ordered product, the division,
// atanh: at most d + 3 roundings of relative size 2^-53, i.e. an ABSOLUTE
// perturbation of at most ~(d + 3) 1.2e-16 of the phi-domain sum, including a
// tanh that rounds to exactly 1) are absorbed by widening that sum by
// kRefSumAbs; this also covers the saturated cases where the reference's
// P / t is exactly +-1 (message +-inf, clamped to +-thr): the widened sum then
// reaches 0 and the upper bound becomes inf (then thr).
//
// binary32 evaluation errors: phi_eval's value and slope are within a few ulp
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
constexpr float kRefSumAbs = 1.0e-14f;     // reference roundings in the phi domain (absolute)
constexpr float kPhiHuge = 80.0f;          // phi evaluated at most here (e^-80: a normal binary32)

typedef float f2 __attribute__((ext_vector_type(2)));   // [lo, hi]; packed binary32 ops

// phi(x) and an upper bound of |phi'(x)| = 1 / sinh(x) (within a factor 2)
// for 0 < x <= kPhiHuge (the callers clamp).
struct PhiVal {
    float v;
    float slope;
};

__device__ __forceinline__ PhiVal phi_eval(float x) {
    // u = e^-x = 2^-(x log2 e), argument split so the reduction is exact to
    // ~2^-48: p = fl(x * L), r = x * L - p (fma, exact) + x * L_lo
    const float L = 1.44269502162933349609375f;          // log2(e) rounded to binary32
    const float L_lo = 1.925963033500011079e-08f;        // log2(e) - L
    const float p = x * L;
    const float r = __builtin_fmaf(x, L, -p) + x * L_lo;
    // 2^-(p + r) = 2^-p (1 - r ln2 + ...), |r| < 2^-17
    const float e2 = __builtin_amdgcn_exp2f(-p);
    const float u = __builtin_fmaf(e2, -r * 0.693147180559945f, e2);
    // w = 1 - u: direct for x >= 0.35 (u <= 0.705: the subtraction costs under
    // a bit), below it the series x (1 - x/2 + x^2/6 - ... + x^6/5040)
    // (truncation < x^7 / 40320 < 1.7e-8 relative)
    float t = __builtin_fmaf(x, 1.0f / 5040.0f, -1.0f / 720.0f);
    t = __builtin_fmaf(x, t, 1.0f / 120.0f);
    t = __builtin_fmaf(x, t, -1.0f / 24.0f);
    t = __builtin_fmaf(x, t, 1.0f / 6.0f);
    t = __builtin_fmaf(x, t, -0.5f);
    t = __builtin_fmaf(x, t, 1.0f);
    const float w = x < 0.35f ? x * t : 1.0f - u;
    const float w2 = 2.0f - w;
    const float rw = __builtin_amdgcn_rcpf(w);
    // x < 1: phi = ln((2 - w) / w) = ln 2 log2((2 - w) * rcp(w)); the
    // argument is >= 2.16 (v_log_f32 is accurate to ~2^-22 absolute near 1,
    // so the log is kept away from small results; rcp and the product add
    // 1.5 ulp of the argument)
    const float vlo = 0.693147180559945f * __builtin_amdgcn_logf(w2 * rw);
    // x >= 1: phi = 2 atanh(u) = 2u (1 + s/3 + s^2/5 + ... + s^6/13), s = u^2 <= e^-2
    // (truncation < s^7 / 15 (1 + s) < 6.4e-8 relative, under 7 % of kPhiRel)
    const float s = u * u;
    float h = __builtin_fmaf(s, 1.0f / 13.0f, 1.0f / 11.0f);
    h = __builtin_fmaf(s, h, 1.0f / 9.0f);
    h = __builtin_fmaf(s, h, 1.0f / 7.0f);
    h = __builtin_fmaf(s, h, 0.2f);
    h = __builtin_fmaf(s, h, 1.0f / 3.0f);
    h = __builtin_fmaf(s, h, 1.0f);
    const float vhi = (2.0f * u) * h;
    PhiVal o;
    o.v = x < 1.0f ? vlo : vhi;
    // |phi'(x)| = 1 / sinh(x) = 2u / (w (2 - w)) <= 2u / w (2 - w >= 1): an
    // upper bound within a factor 2, which is all the tangent below needs
    o.slope = (2.0f * u) * rw;
    return o;
}

// Bounds of phi over [a, b], 0 < a <= b (finite or +inf): lo <= phi(x) <= hi.
// phi is decreasing and convex: phi(a) is the maximum, and the tangent at a
// lies below phi, so phi(a) - (b - a) / sinh(a) is a lower bound. Past
// kPhiHuge both come from a' = kPhiHuge <= a: phi(a') bounds phi(a) above,
// and the tangent at a' stays below phi on [a', b].
__device__ __forceinline__ f2 phi_bounds(float a, float b) {
    const float a1 = __builtin_fminf(a, kPhiHuge);
    const PhiVal e = phi_eval(a1);
    const float hi = __builtin_fmaf(e.v, kPhiRel, e.v) + 1.0e-37f;
    const float t = __builtin_fmaf(-e.slope * (1.0f + 2.0f * kPhiRel), b - a1, e.v * (1.0f - kPhiRel));
    return f2{t > 0.0f ? t : 0.0f, hi};     // lo: also for b = inf (t = -inf) and NaN
}
__device__ __forceinline__ void phi_bounds(float a, float b, float& lo, float& hi) {
    const f2 r = phi_bounds(a, b);
    lo = r.x;
    hi = r.y;
}

// Bounds of phi over [S_lo, S_hi], 0 <= S_lo <= S_hi: at S_lo = 0 (the
// widened sum reached zero) the maximum is +inf and the minimum is taken at
// S_hi; otherwise one evaluation at S_lo and its tangent (both clamped to
// kPhiHuge as in phi_bounds).
__device__ __forceinline__ f2 phi_bounds_out(float s_lo, float s_hi) {
    const bool zero = !(s_lo > 0.0f);
    const float at = __builtin_fminf(zero ? s_hi : s_lo, kPhiHuge);
    const PhiVal e = phi_eval(at);
    const float vmax = __builtin_fmaf(e.v, kPhiRel, e.v) + 1.0e-37f;
    const float tan = __builtin_fmaf(-e.slope * (1.0f + 2.0f * kPhiRel), s_hi - at, e.v * (1.0f - kPhiRel));
    return f2{tan > 0.0f ? tan : 0.0f, zero ? __builtin_inff() : vmax};
}
__device__ __forceinline__ void phi_bounds_out(float s_lo, float s_hi, float& lo, float& hi) {
    const f2 r = phi_bounds_out(s_lo, s_hi);
    lo = r.x;
    hi = r.y;
}

// An interval enclosing a finite binary64 value: its binary32 rounding
// widened by 2^-22 relative (twice the rounding error and the widening's own)
// and 1e-38 absolute (0 and subnormals give an interval containing 0).
__device__ __forceinline__ f2 iv_of(double x) {
    const float f = (float)x;
    const float a = __builtin_fabsf(f);
    return f2{__builtin_fmaf(a, -0x1.0p-22f, f) - 1.0e-38f, __builtin_fmaf(a, 0x1.0p-22f, f) + 1.0e-38f};
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
