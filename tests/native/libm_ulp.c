/* Max error of glibc's binary64 tanh and atanh (the functions the reference calls,
 * src/qkd_ldpc_algorithm.cpp:224, :241) in ulps of the result, against the x87
 * 80-bit tanhl / atanhl (64-bit significand: 2^-11 ulp of binary64 resolution).
 * Feeds tests/test_spec_bounds.py's derivation of kRefSumAbs (qkd_spec.h).
 * Also the max RELATIVE error in units of 2^-52 (the unit the derivation of
 * kRefSumAbs and tests/test_spec_bounds.py's fdlibm error propagation use).
 *   libm_ulp <points>  ->  "tanh <max_ulp> <at_x>\natanh <max_ulp> <at_x>\n"
 *                          "tanh_rel <max>\natanh_rel <max>\n" */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static double ulp_of(long double y) {
    double d = (double)y;
    if (d == 0.0) return 0x1p-1074;
    int e;
    frexp(fabs(d), &e);
    return ldexp(1.0, e - 53);
}

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static double uni(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (double)(rng >> 11) * 0x1p-53;
}

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 2000000;
    double mt = 0, mt_x = 0, ma = 0, ma_x = 0, rt = 0, ra = 0;
    for (long k = 0; k < n; ++k) {
        /* tanh at x = b / 2 for |b| <= 100 (the clamp): log-uniform over [2^-40, 50] and uniform [0, 20] */
        double x = (k & 1) ? exp2(-40.0 + 45.64 * uni()) : 20.0 * uni();
        long double rx = tanhl((long double)x);
        double err = fabsl((long double)tanh(x) - rx) / ulp_of(rx);
        if (err > mt) { mt = err; mt_x = x; }
        double rel = (double)(fabsl(((long double)tanh(x) - rx) / rx) * 0x1p52L);
        if (rel > rt) rt = rel;
        /* atanh on (0, 1): log-uniform in x and in 1 - x */
        double y = (k & 1) ? exp2(-60.0 * uni()) : 1.0 - exp2(-53.0 * uni());
        if (y >= 1.0) continue;
        long double ry = atanhl((long double)y);
        err = fabsl((long double)atanh(y) - ry) / ulp_of(ry);
        if (err > ma) { ma = err; ma_x = y; }
        rel = (double)(fabsl(((long double)atanh(y) - ry) / ry) * 0x1p52L);
        if (rel > ra) ra = rel;
    }
    printf("tanh %.6f %.17g\natanh %.6f %.17g\ntanh_rel %.6f\natanh_rel %.6f\n", mt, mt_x, ma, ma_x, rt, ra);
    return 0;
}
