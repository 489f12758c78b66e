// qkd_math.h — bit-exact binary64 tanh / atanh for the sum-product kernels.
//
// The reference decoder calls glibc 2.35 `tanh` and `atanh` once per edge per
// half-iteration (reference src/qkd_ldpc_algorithm.cpp:224 and :241). Those are
// the fdlibm algorithms layered on glibc's `__expm1` / `__log1p`, whose
// polynomial tails glibc evaluates in a split (Estrin-like) order rather than
// fdlibm's Horner chain. ROCm's ocml tanh/atanh round differently, so the
// device cannot use them and still produce the reference's messages bit for
// bit. This header restates those published algorithms once, as straight-line
// binary64 code that compiles identically for the host (g++) and for gfx950
// (hipcc). Both builds MUST use -ffp-contract=off: a fused a*b+c rounds once
// and changes the last bit.
//
// Only round-to-nearest results matter here; floating-point exception flags
// (inexact/underflow side effects in the C library) are not modelled.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define QKD_HD __host__ __device__ __forceinline__
#else
#define QKD_HD inline
#endif

namespace qkdm {

QKD_HD uint64_t bits_of(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
}
QKD_HD double from_bits(uint64_t u) {
    double x;
    __builtin_memcpy(&x, &u, 8);
    return x;
}
QKD_HD int32_t hi32(double x) { return (int32_t)(bits_of(x) >> 32); }
QKD_HD uint32_t lo32(double x) { return (uint32_t)bits_of(x); }
// Replace the high 32 bits of x, keeping its low word.
QKD_HD double set_hi32(double x, uint32_t hi) {
    return from_bits(((uint64_t)hi << 32) | (bits_of(x) & 0xffffffffull));
}

// ---------------------------------------------------------------------------
// expm1(x) = e^x - 1.  fdlibm s_expm1.c argument reduction and reconstruction;
// the rational tail r1 is summed as (R1 + h2*R2) + h4*R3 (glibc dbl-64 order).
// ---------------------------------------------------------------------------
QKD_HD double expm1_ref(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;   // 0x3fe62e42 fee00000
    const double ln2_lo = 1.90821492927058770002e-10;   // 0x3dea39ef 35793c76
    const double invln2 = 1.44269504088896338700e+00;   // 0x3ff71547 652b82fe
    const double o_threshold = 7.09782712893383973096e+02;
    const double Q1 = -3.33333333333331316428e-02;
    const double Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05;
    const double Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;

    const uint32_t hword = (uint32_t)hi32(x);
    const bool neg = (hword & 0x80000000u) != 0;
    const uint32_t ahx = hword & 0x7fffffffu;

    if (ahx >= 0x4043687Au) {                 // |x| >= 56 ln2
        if (ahx >= 0x40862E42u) {             // |x| >= 709.78
            if (ahx >= 0x7ff00000u) {
                if (((ahx & 0xfffffu) | lo32(x)) != 0) return x + x;   // NaN
                return neg ? -1.0 : x;                                 // +-inf
            }
            if (x > o_threshold) return 1.0e300 * 1.0e300;             // +inf
        }
        if (neg) return 1.0e-300 - 1.0;       // rounds to -1
    }

    double hi, lo, c = 0.0;
    int k;
    if (ahx > 0x3fd62e42u) {                  // |x| > ln2/2
        if (ahx < 0x3FF0A2B2u) {              // |x| < 1.5 ln2
            if (!neg) { hi = x - ln2_hi; lo = ln2_lo;  k = 1; }
            else      { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int)(invln2 * x + (neg ? -0.5 : 0.5));
            const double t = (double)k;
            hi = x - t * ln2_hi;              // exact
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (ahx < 0x3c900000u) {           // |x| < 2^-54
        return x;
    } else {
        k = 0;
    }

    const double hfx = 0.5 * x;
    const double hxs = x * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    double t = 3.0 - r1 * hfx;
    double e = hxs * ((r1 - t) / (6.0 - x * t));
    if (k == 0) return x - (x * e - hxs);

    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5 * (x - e) - 0.5;
    if (k == 1) {
        if (x < -0.25) return -2.0 * (e - (x + 0.5));
        return 1.0 + 2.0 * (x - e);
    }
    double y;
    if (k <= -2 || k > 56) {                  // exp(x)-1 ~ exp(x)
        y = 1.0 - (e - x);
        if (k == 1024) {
            y = y * 2.0 * 0x1p1023;
        } else {
            y = set_hi32(y, (uint32_t)hi32(y) + ((uint32_t)k << 20));
        }
        return y - 1.0;
    }
    if (k < 20) {
        t = from_bits((uint64_t)(0x3ff00000u - (0x200000u >> k)) << 32);   // 1 - 2^-k
        y = t - (e - x);
    } else {
        t = from_bits((uint64_t)((uint32_t)(0x3ff - k) << 20) << 32);        // 2^-k
        y = x - (e + t);
        y += 1.0;
    }
    return set_hi32(y, (uint32_t)hi32(y) + ((uint32_t)k << 20));
}

// ---------------------------------------------------------------------------
// log1p(x) = ln(1 + x).  fdlibm s_log1p.c reduction; the Lp tail is summed as
// ((R1 + z2*R2) + z4*R3) + z6*R4 (glibc dbl-64 order).
// ---------------------------------------------------------------------------
QKD_HD double log1p_ref(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double two54 = 1.80143985094819840000e+16;
    const double Lp1 = 6.666666666666735130e-01;
    const double Lp2 = 3.999999999940941908e-01;
    const double Lp3 = 2.857142874366239149e-01;
    const double Lp4 = 2.222219843214978396e-01;
    const double Lp5 = 1.818357216161805012e-01;
    const double Lp6 = 1.531383769920937332e-01;
    const double Lp7 = 1.479819860511658591e-01;

    const int32_t hx = hi32(x);
    const int32_t ax = hx & 0x7fffffff;
    int32_t k = 1, hu = 0;
    double f = 0.0, c = 0.0;

    if (hx < 0x3FDA827A) {                    // x < 0.41422
        if (ax >= 0x3ff00000) {               // x <= -1
            if (x == -1.0) return -two54 / 0.0;   // -inf
            return (x - x) / (x - x);             // NaN
        }
        if (ax < 0x3e200000) {                // |x| < 2^-29
            if (ax < 0x3c900000) return x;
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec4) {   // -0.2929 < x < 0.41422
            k = 0; f = x; hu = 1;
        }
    } else if (hx >= 0x7ff00000) {
        return x + x;
    }
    if (k != 0) {
        double u;
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = hi32(u);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
            c /= u;
        } else {
            u = x;
            hu = hi32(u);
            k = (hu >> 20) - 1023;
            c = 0.0;
        }
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = set_hi32(u, (uint32_t)hu | 0x3ff00000u);   // u in [1, sqrt2)
        } else {
            k += 1;
            u = set_hi32(u, (uint32_t)hu | 0x3fe00000u);   // u/2
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    if (hu == 0) {                            // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += dk * ln2_lo;
            return dk * ln2_hi + c;
        }
        const double R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return dk * ln2_hi - ((R - (dk * ln2_lo + c)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

// ---------------------------------------------------------------------------
// tanh — fdlibm s_tanh.c on expm1_ref.
// ---------------------------------------------------------------------------
QKD_HD double tanh_ref(double x) {
    const int32_t jx = hi32(x);
    const int32_t ix = jx & 0x7fffffff;
    if (ix >= 0x7ff00000) {                   // inf or NaN
        return (jx >= 0) ? 1.0 / x + 1.0 : 1.0 / x - 1.0;
    }
    double z;
    if (ix < 0x40360000) {                    // |x| < 22
        if ((ix | (int32_t)lo32(x)) == 0) return x;      // +-0
        if (ix < 0x3c800000) return x * (1.0 + x);       // |x| < 2^-55
        const double ax = __builtin_fabs(x);
        if (ix >= 0x3ff00000) {               // |x| >= 1
            const double t = expm1_ref(2.0 * ax);
            z = 1.0 - 2.0 / (t + 2.0);
        } else {
            const double t = expm1_ref(-2.0 * ax);
            z = -t / (t + 2.0);
        }
    } else {
        z = 1.0;                              // 1 - tiny rounds to 1
    }
    return (jx >= 0) ? z : -z;
}

// ---------------------------------------------------------------------------
// atanh — glibc dbl-64 e_atanh.c structure on log1p_ref.
// ---------------------------------------------------------------------------
QKD_HD double atanh_ref(double x) {
    const double xa = __builtin_fabs(x);
    double t;
    if (xa < 0.5) {
        if (xa < 0x1.0p-28) return x;
        t = xa + xa;
        t = 0.5 * log1p_ref(t + t * xa / (1.0 - xa));
    } else if (xa < 1.0) {
        t = 0.5 * log1p_ref((xa + xa) / (1.0 - xa));
    } else {
        if (xa > 1.0) return (x - x) / (x - x);          // |x| > 1: NaN
        return x / 0.0;                                   // +-1: +-inf; NaN: NaN
    }
    return __builtin_copysign(t, x);
}


// ===========================================================================
// Branch-free ("flat") forms for the kernels.
//
// The functions above follow the published code path by path. On a 64-lane
// wavefront every value-dependent `if` whose lanes disagree executes both
// sides, and tanh/atanh each inline TWO copies of expm1/log1p (one per
// magnitude branch), so a divergent wave pays for four transcendentals per
// call. The forms below compute each result with the same sequence of
// binary64 operations on the same operands as the path the reference would
// take, but select operands and results instead of branching: one expm1 /
// log1p body per call, one division per quotient. Every select picks between
// values that the reference computes identically, so results are bitwise
// equal to tanh_ref / atanh_ref for every input (tests/native/math_check.cpp
// checks them against glibc and against the path-by-path forms).
// ===========================================================================

// a / b for operands the callers keep in the normal range: |a|, |b| and |a/b|
// in [2^-107, 2^64] (or a = +0 with b > 0). On gfx950 the compiler's IEEE
// division is v_div_scale x2, v_rcp, the Newton/Markstein fma chain,
// v_div_fmas and v_div_fixup; for such operands div_scale returns its input
// unchanged with VCC = 0, div_fmas is then a plain fma and div_fixup returns
// its first operand, so the chain below is the same sequence of roundings and
// the correctly rounded quotient, three instructions shorter. The host build
// divides.
QKD_HD double div_normal(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double r0 = __builtin_amdgcn_rcp(b);
    const double e0 = __builtin_fma(-b, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-b, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double q0 = a * r2;
    const double rem = __builtin_fma(-b, q0, a);
    return __builtin_fma(rem, r2, q0);
#else
    return a / b;
#endif
}

// expm1 restricted to the arguments tanh_flat feeds it:
//   a in (-2, 0]  (tanh of |x| < 1: expm1(-2|x|), tiny and zero included)
//   a in [2, 64]  (tanh of |x| >= 1: expm1(min(2|x|, 64)))
// On this domain the reference's expm1 takes only these paths:
//   k = 0 (|a| <= ln2/2; below 2^-54 it returns a, which the k = 0 formula
//   reproduces: a + a^2/2 rounds to a), k = -1 (ln2/2 < |a| < 1.5 ln2, a < 0),
//   general k in {-3,-2} or [3, 93]; no overflow, no k = 1, no k = 1024.
QKD_HD double expm1_tanh_domain(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double Q1 = -3.33333333333331316428e-02;
    const double Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05;
    const double Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;

    const uint32_t ahx = (uint32_t)hi32(x) & 0x7fffffffu;
    const bool red = ahx > 0x3fd62e42u;          // |x| > ln2/2: reduce
    const bool km1 = ahx < 0x3FF0A2B2u;          // |x| < 1.5 ln2 (negative side only here)
    // general k = (int)(invln2*x -+ 0.5)
    const int kg = (int)(invln2 * x + __builtin_copysign(0.5, x));
    const int k = red ? (km1 ? -1 : kg) : 0;
    // The reference's three reductions are one formula in t = (double)k:
    //   k = -1: hi = x + ln2_hi = x - (-1.0)*ln2_hi, lo = -ln2_lo = (-1.0)*ln2_lo
    //   k =  0: hi = x - 0.0 = x (also for -0), lo = +0, so xr = x and c = 0
    const double tk = (double)k;
    const double hi = x - tk * ln2_hi;
    const double lo = tk * ln2_lo;
    const double xr = hi - lo;
    const double c = (hi - xr) - lo;

    const double hfx = 0.5 * xr;
    const double hxs = xr * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t = 3.0 - r1 * hfx;
    const double e = hxs * div_normal(r1 - t, 6.0 - xr * t);   // ~ -2 / [5, 7]

    const double res0 = xr - (xr * e - hxs);                 // k == 0
    const double e2 = (xr * (e - c) - c) - hxs;              // k != 0
    const double resm1 = 0.5 * (xr - e2) - 0.5;              // k == -1
    const bool big = k <= -2 || k > 56;
    const int ks = (big || k > 31) ? 31 : (k < 0 ? 0 : k);
    // 1 - 2^-k for 2 <= k < 20; exactly 1.0 when big (the shift leaves 0)
    const double t1 = from_bits((uint64_t)(0x3ff00000u - (0x200000u >> ks)) << 32);
    const double t2 = from_bits((uint64_t)((uint32_t)(0x3ff - k) << 20) << 32);          // 2^-k
    const double a12 = t1 - (e2 - xr);                       // k <= -2 | k > 56 | 2 <= k < 20
    const double a3 = (xr - (e2 + t2)) + 1.0;                // 20 <= k <= 56
    const double a = (big || k < 20) ? a12 : a3;
    const double y = set_hi32(a, (uint32_t)hi32(a) + ((uint32_t)k << 20));
    const double resg = big ? y - 1.0 : y;
    return k == 0 ? res0 : (k == -1 ? resm1 : resg);
}

QKD_HD double tanh_flat(double x) {
    const uint32_t ix = (uint32_t)hi32(x) & 0x7fffffffu;
    const bool ge1 = ix >= 0x3ff00000u;
    // One expm1 argument for every input:
    //   |x| <  2^-55 (and +-0, subnormals): a = -2|x|; expm1's k = 0 branch then
    //     returns a exactly, q = |x| exactly, so the result is x, as the
    //     reference's x*(1+x) (1+x rounds to 1).
    //   |x| >= 22, +-inf, NaN: a = min(2|x|, 64) >= 44, so 2/(t+2) < 2^-54 and
    //     1 - q rounds to exactly 1.0, the reference's |x| >= 22 value (NaN is
    //     replaced below).
    const double aa = __builtin_fmin(2.0 * __builtin_fabs(x), 64.0);
    const double a = ge1 ? aa : -aa;
    const double t = expm1_tanh_domain(a);
    // 2/(t+2) or -t/(t+2); t+2 in [1.13, 2^93], numerator 2 or in [2^-55, 0.87]
    // (+0 for x = +-0; subnormal-range x divides a subnormal by exactly 2)
    const double q = div_normal(ge1 ? 2.0 : -t, t + 2.0);
    const double z = ge1 ? 1.0 - q : q;
    const double r = __builtin_copysign(z, x);
    return x != x ? x : r;
}

// log1p restricted to the arguments atanh feeds it: x in [2^-27, 2^54],
// finite and positive. Paths used: k = 0 (x < 0.41422), and k != 0 with
// u = 1 + x (x < 2^53) or u = x (x >= 2^53); either with |f| < 2^-20 tails.
QKD_HD double log1p_atanh_domain(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01;
    const double Lp2 = 3.999999999940941908e-01;
    const double Lp3 = 2.857142874366239149e-01;
    const double Lp4 = 2.222219843214978396e-01;
    const double Lp5 = 1.818357216161805012e-01;
    const double Lp6 = 1.531383769920937332e-01;
    const double Lp7 = 1.479819860511658591e-01;

    const int32_t hx = hi32(x);
    const bool k0 = hx < 0x3FDA827A;                          // x < 0.41422: k = 0, f = x
    const bool huge = hx >= 0x43400000;                       // x >= 2^53: u = x, c = 0
    const double u1 = 1.0 + x;
    double u = huge ? x : u1;
    int32_t hu = hi32(u);
    int32_t k = (hu >> 20) - 1023;
    double c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
    // c: the rounding error of 1 + x, 0 or a multiple of ulp(x) >= 2^-54; u in [1.41, 2^53]
    c = huge ? 0.0 : div_normal(c, u);
    hu &= 0x000fffff;
    const bool lowm = hu < 0x6a09e;
    u = set_hi32(u, (uint32_t)hu | (lowm ? 0x3ff00000u : 0x3fe00000u));
    k = lowm ? k : k + 1;
    hu = lowm ? hu : (0x00100000 - hu) >> 2;
    double f = u - 1.0;
    // k = 0 path (on the other path k >= 1: u = 1 + x >= sqrt 2 is halved)
    f = k0 ? x : f;
    k = k0 ? 0 : k;
    hu = k0 ? 1 : hu;
    c = k0 ? 0.0 : c;

    // The reference's k = 0 formulas equal its general ones at k = 0, c = 0:
    //   0*ln2_hi - ((A - (0*ln2_lo + 0)) - f) = -(A - f) = f - A  (rounding is
    //   symmetric under negation; the zero cases give +0 both ways), so one
    //   formula serves both.
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    const double cl = dk * ln2_lo + c;
    // |f| < 2^-20 tails (hu == 0)
    const double R0 = hfsq * (1.0 - 0.66666666666666666 * f);
    const double tail = f == 0.0 ? dk * ln2_hi + cl : dk * ln2_hi - ((R0 - cl) - f);
    // main
    const double s = div_normal(f, 2.0 + f);                  // f in [2^-54, 0.42], or 0
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    const double m = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + cl)) - f);
    return hu == 0 ? tail : m;
}

QKD_HD double atanh_flat(double x) {
    const double xa = __builtin_fabs(x);
    const bool small = xa < 0.5;
    const double t = xa + xa;
    // t*xa/(1-xa) or (xa+xa)/(1-xa): for 2^-28 <= xa < 1 numerator in [2^-55, 2),
    // 1 - xa in [2^-53, 1]; other lanes are replaced below
    const double q = div_normal(small ? t * xa : t, 1.0 - xa);
    const double arg = small ? t + q : q;
    // |x| >= 1 and NaN pass meaningless arguments through log1p (integer work
    // on bit patterns only: no traps, no undefined behaviour); replaced below
    const double r = 0.5 * log1p_atanh_domain(arg);
    const double res = __builtin_copysign(r, x);
    // +-1 -> +-inf; |x| > 1 and NaN -> NaN (payloads never reach an output)
    const double sp = xa == 1.0 ? __builtin_copysign(__builtin_inf(), x) : __builtin_nan("");
    return xa < 0x1.0p-28 ? x : (xa < 1.0 ? res : sp);
}

}  // namespace qkdm
