"""Soundness margins of the speculative iterations (qkd_ldpc_amd/csrc/qkd_spec.h),
derived rather than sampled.

kRefSumAbs: the binary32 intervals must contain the reference's binary64 messages,
so every phi-domain check sum is widened by the largest perturbation the
reference's own roundings can cause (src/qkd_ldpc_algorithm.cpp:220-249):
  * d tanh calls (glibc, e_t ulp each) and d - 1 products + 1 division (0.5 ulp
    each) change the extrinsic product P / t_self by a relative
    (2 d e_t + d) 2^-53 at most, an ABSOLUTE change of the same size of its
    phi-domain sum S = -ln|P / t_self|;
  * atanh (e_a ulp) changes c2b = phi(S) by a relative e_a 2^-52, i.e. S by at
    most e_a 2^-52 max_S phi(S) sinh(S) (computed below; < 1).
e_t and e_a are bounded two ways, and the derivation assumes 3 (relative
2^-52 units) for both:
  * derived (test_fdlibm_error_propagation): glibc 2.35's binary64 tanh and
    atanh are fdlibm's s_tanh.c / e_atanh.c formulas over expm1 / log1p
    (bit for bit: tests/native/math_check.cpp against our restatement,
    qkd_math.h), and fdlibm's s_expm1.c / s_log1p.c state "according to an
    error analysis, the error is always less than 1 ulp". Propagating that
    and each formula's own roundings through the formulas bounds tanh at 2.77
    and atanh at 2.25 relative units. (glibc's libm-test-ulps table is not in
    this image -- no network -- so the citation is fdlibm's published claim,
    not the table.)
  * measured against 80-bit x87 tanhl / atanhl (tests/native/libm_ulp.c): tanh
    2.15 ulp, atanh 1.62 ulp, both below the derived bounds in relative units.

The exhaustive binary32 sweep of the phi bounds themselves is a GPU test
(tests/test_spec.py::test_phi_bounds_exhaustive)."""
import os
import re
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEC_H = os.path.join(ROOT, "qkd_ldpc_amd", "csrc", "qkd_spec.h")


def spec_constant(name):
    m = re.search(rf"constexpr float {name} = ([0-9.eE+\-x]+)f;", open(SPEC_H).read())
    assert m, name
    v = m.group(1)
    return float.fromhex(v) if "x" in v else float(v)


def glibc_ulp_errors(tmp_path, points=4_000_000, relative=False):
    """Max errors of glibc tanh / atanh: in ulps of the result, or (relative=True)
    as relative errors in units of 2^-52."""
    exe = str(tmp_path / "libm_ulp")
    subprocess.check_call(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "tests", "native", "libm_ulp.c"), "-lm"])
    out = subprocess.check_output([exe, str(points)], text=True).split()
    return (float(out[7]), float(out[9])) if relative else (float(out[1]), float(out[4]))


# fdlibm's published accuracy of its expm1 and log1p (s_expm1.c, s_log1p.c header
# comments: "according to an error analysis, the error is always less than 1 ulp"),
# as a relative error in units of 2^-52 (1 ulp <= 2^-52 relative)
FDLIBM_EXPM1 = 1.0
FDLIBM_LOG1P = 1.0
RND = 0.5       # one correctly rounded binary64 operation: 2^-53 relative


def fdlibm_tanh_bound():
    """Relative error bound (units of 2^-52) of fdlibm's tanh (s_tanh.c), first order:
      |x| < 2^-55:       x * (1 + x)                     (error ~2^-55 relative)
      2^-55 <= |x| < 1:  t = expm1(-2|x|), z = -t / (t + 2)
      1 <= |x| < 22:     t = expm1(2|x|),  z = 1 - 2 / (t + 2)
      |x| >= 22:         z = 1 - tiny = 1                (error < 2^-53 relative)
    (2|x| is exact; the sign is applied exactly.)"""
    # branch 2: t in [e^-2 - 1, 0); d ln z / d ln t = 2 / (t + 2); then t + 2 and the
    # division round once each
    t = np.linspace(np.expm1(-2.0), -1e-12, 200001)
    b2 = float(np.max(2.0 / (t + 2.0))) * FDLIBM_EXPM1 + RND + RND
    # branch 3: t in [e^2 - 1, e^44 - 1]; w = 2 / (t + 2) has relative error
    # t / (t + 2) * e1 + two roundings; z = 1 - w: absolute error w * that, plus
    # the subtraction's rounding, relative to z
    t = np.geomspace(np.expm1(2.0), np.expm1(44.0), 200001)
    w = 2.0 / (t + 2.0)
    w_rel = (t / (t + 2.0)) * FDLIBM_EXPM1 + RND + RND
    b3 = float(np.max(w * w_rel / (1.0 - w))) + RND
    return max(b2, b3, RND, 2.0 ** -3)


def fdlibm_atanh_bound():
    """Relative error bound (units of 2^-52) of fdlibm's atanh (e_atanh.c), |x| < 1:
      |x| < 2^-28:       x                               (error x^2 / 3 relative)
      2^-28 <= x < 0.5:  0.5 * log1p(2x + 2x * x / (1 - x))
      0.5 <= x < 1:      0.5 * log1p(2x / (1 - x))       (1 - x exact: Sterbenz)
    log1p(u) turns a relative error of u into one at most as large (u / ((1 + u)
    ln(1 + u)) <= 1); 0.5 * and 2x are exact."""
    # x < 0.5: the second term 2x^2/(1-x) carries 3 roundings (x*t, 1-x, /); its
    # share of the (positive) sum is x; the sum rounds once; then log1p
    x = np.linspace(0.0, 0.5, 200001)
    arg = x * 3 * RND + RND
    b1 = float(np.max(arg)) * 1.0 + FDLIBM_LOG1P
    b2 = RND * 1.0 + FDLIBM_LOG1P
    return max(b1, b2)


def test_fdlibm_error_propagation(tmp_path):
    """The error bounds kRefSumAbs rests on, derived from fdlibm's published expm1 /
    log1p accuracy (see the module docstring), are within the 3 units the
    derivation assumes, and the measured glibc errors (relative, 2^-52 units) stay
    below them."""
    bt, ba = fdlibm_tanh_bound(), fdlibm_atanh_bound()
    rt, ra = glibc_ulp_errors(tmp_path, points=2_000_000, relative=True)
    print(f"derived: tanh <= {bt:.3f}, atanh <= {ba:.3f}; measured: tanh {rt:.3f}, atanh {ra:.3f} (2^-52 relative)")
    assert bt <= 3.0 and ba <= 3.0, (bt, ba)
    assert rt <= bt and ra <= ba, (rt, bt, ra, ba)


def max_phi_sinh():
    """max over S > 0 of phi(S) sinh(S), phi(S) = -ln tanh(S/2): the factor from a
    relative error of c2b to an absolute error of its phi-domain sum."""
    S = np.concatenate([np.geomspace(1e-12, 1.0, 200000), np.linspace(1.0, 700.0, 2000000)])
    u = np.exp(-S)
    phi = np.log1p(2 * u / -np.expm1(-S))
    return float(np.max(phi * np.sinh(S)))


def test_ref_sum_allowance_covers_reference_roundings(tmp_path, golden_code):
    e_t, e_a = glibc_ulp_errors(tmp_path)
    assert e_t <= 3.0 and e_a <= 3.0, (e_t, e_a)          # the bound the derivation assumes
    d = int(np.diff(golden_code["chk_off"]).max())           # max check degree of the code
    k = max_phi_sinh()
    assert 0.99 < k <= 1.0 + 1e-9, k
    # worst case of the reference's own rounding of one c2b, in nep units of S
    delta = (2 * d * e_t + d) * 2.0 ** -53 + e_a * 2.0 ** -52 * k
    # the same with the assumed 3-ulp bounds instead of the measured maxima
    delta_doc = (2 * d * 3.0 + d) * 2.0 ** -53 + 3.0 * 2.0 ** -52 * k
    allow = spec_constant("kRefSumAbs") * np.log(2.0)           # psi units -> nep
    print(f"glibc max error: tanh {e_t:.3f} ulp, atanh {e_a:.3f} ulp; degree {d}; "
          f"reference perturbation <= {delta:.3g} (3-ulp bounds {delta_doc:.3g}); "
          f"kRefSumAbs = {allow:.3g} nep: headroom x{allow / delta:.1f} (x{allow / delta_doc:.1f})")
    assert allow >= 2 * delta_doc


def test_ref_sum_allowance_in_kernel_degree_buckets():
    """The kernel keeps kRefSumAbs per check, independent of degree, so the bound must
    hold for the largest degree the speculative kernel accepts (DC = 16 at most)."""
    d = 16
    delta_doc = (2 * d * 3.0 + d) * 2.0 ** -53 + 3.0 * 2.0 ** -52
    assert spec_constant("kRefSumAbs") * np.log(2.0) >= 2 * delta_doc
